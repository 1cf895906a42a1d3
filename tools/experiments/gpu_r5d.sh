# Round 5: the exact fbank with the register post-pass (fbank8_ops.h
# post_regs) against round 4's library on C2, after the fbank / int8 parity
# tests and the pipelined determinism check; then the C5 A/B (gpu_r5b.sh)
# and the bf16x6 ablations (gpu_r5c.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pcm16.py tests/test_gpu_determinism.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "fbank or cmvn or pcm or pipelined" \
    > gpurun_out/r05d/pytest.log 2>&1 || { tail -30 gpurun_out/r05d/pytest.log; exit 1; }
tail -1 gpurun_out/r05d/pytest.log
NEW=$R/catears_amd/lib/libcatears_hip.so
OLD=$R/catears_amd/lib/ab/libcatears_hip_r4.so
for i in 1 2 3; do
  for L in $NEW $OLD; do
    v=$(basename $L .so)
    CATEARS_HIP_LIB=$L timeout -k 10 200 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05d/c2_$v.$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05d/c2_$v.$i.json')); print('c2 $v', round(l['value']/1e9,4), 'G', l['roofline']['frac'], l.get('checksum'))"
  done
done
bash tools/experiments/gpu_r5b.sh || exit 1
bash tools/experiments/gpu_r5c.sh || exit 1
