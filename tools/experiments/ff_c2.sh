# (Historical: measures the four-step fast fbank kernel, kernels/fbank_fast.hip, removed
# in round 5 when the fast mode became the contracted exact lane program; kept as the
# record of DESIGN.md §8b.  It no longer builds against the current tree.)
# fast fbank: its GPU tests, then the C2 fast line (3 reps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/ff
timeout -k 10 300 python -u -m pytest tests/test_gpu_fbank_fast.py tests/test_gpu_pcm16.py -x -q -s --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/ff/pytest.log 2>&1 || { tail -30 gpurun_out/ff/pytest.log; exit 1; }
grep -E "vs exact|passed|failed" gpurun_out/ff/pytest.log
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --workload c2 --fbank fast --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ff/c2_$rep.json 2> gpurun_out/ff/c2_$rep.err || { tail -5 gpurun_out/ff/c2_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ff/c2_$rep.json')); print('C2 fast', round(d['value']/1e9,4), 'G', d['roofline']['frac'])"
done
