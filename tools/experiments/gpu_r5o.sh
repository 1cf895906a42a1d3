# Fast fbank mode as the exact lane program with FMA contraction
# (kernels/fbank_fma.hip, CATEARS_FBANK_FAST_IMPL=fma) vs the four-step
# kernel: the fast-mode tests on the new kernel, C2 rates alternating
# (exact / four-step / fma), and the concurrency stress for the new kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05o
CATEARS_FBANK_FAST_IMPL=fma timeout -k 10 300 python -u -m pytest tests/test_gpu_fbank_fast.py tests/test_gpu_pcm16.py tests/test_gpu_determinism.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05o/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r05o/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in exact fast fma; do
    case $v in exact) A="--fbank exact"; E="";; fast) A="--fbank fast"; E="";; fma) A="--fbank fast"; E="fma";; esac
    CATEARS_FBANK_FAST_IMPL=$E timeout -k 10 200 python bench.py --workload c2 $A --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r05o/c2_$v.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05o/c2_$v.json')); print('c2 $v', l['value'], l['roofline']['frac'], l['checksum'])"
  done
done
CATEARS_FBANK_FAST_IMPL=fma timeout -k 10 120 python -u tools/experiments/lds_race_stress.py --fbank fast --seconds 20 > gpurun_out/r05o/stress.log 2>&1 || { tail -5 gpurun_out/r05o/stress.log; exit 1; }
tail -1 gpurun_out/r05o/stress.log | cut -c1-260
