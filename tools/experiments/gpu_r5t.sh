# One fold launch pair per step (ce_gpu_sum_f64_many): fold tests, the fold
# probe, and the rank-0 rehearsal at 1 / 3 / 7 peers (C3 60 steps).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05t
timeout -k 10 400 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_c4.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05t/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r05t/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/probes/fold_cost.py 2>&1 | grep -v amdgpu.ids | head -3
for rep in 1 2; do
  for k in 0 1 3 7; do
    timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers $k > gpurun_out/r05t/k${k}_$rep.json 2>gpurun_out/r05t/k${k}_$rep.err || { tail -5 gpurun_out/r05t/k${k}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05t/k${k}_$rep.json')); print('peers $k', l['value'], l['ms_per_step'])"
  done
  CATEARS_REHEARSE_NOCOPY=1 timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers 7 > gpurun_out/r05t/k7nc_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05t/k7nc_$rep.json')); print('peers 7 folds only', l['value'], l['ms_per_step'])"
done
