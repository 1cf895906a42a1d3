# The fast fbank mode as the contracted lane program (product library): the
# whole GPU suite, the fast-mode accuracy figures (-s prints them), C2 exact
# and fast, and the stress beside the GEMM streams.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05p
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05p/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r05p/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fbank_fast.py -m gpu -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider -k c2_set \
    > gpurun_out/r05p/fast_acc.log 2>&1 || { tail -20 gpurun_out/r05p/fast_acc.log; exit 1; }
grep "vs exact" gpurun_out/r05p/fast_acc.log
for rep in 1 2; do
  for m in exact fast; do
    timeout -k 10 200 python bench.py --workload c2 --fbank $m --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r05p/c2_$m.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05p/c2_$m.json')); print('c2 $m', l['value'], l['roofline']['frac'], l['checksum'])"
  done
done
for pcm in f32 s16; do
  timeout -k 10 120 python -u tools/experiments/lds_race_stress.py --fbank fast --pcm $pcm --seconds 20 > gpurun_out/r05p/stress_$pcm.log 2>&1 || { tail -5 gpurun_out/r05p/stress_$pcm.log; exit 1; }
  tail -1 gpurun_out/r05p/stress_$pcm.log | cut -c1-230
done
