# Latency-mode slice-rule sweep: per CATEARS_LAT_SLICES setting
# ("min_ktiles,max_slices,target_blocks"), the latency GPU tests and
# tools/latency.py.   RULES="6,8,64 3,16,128" bash tools/lat_sweep.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/latsw
for rule in ${RULES}; do
  CATEARS_LAT_SLICES=$rule timeout -k 10 300 python -u -m pytest tests/test_gpu_latency.py -q -x -m gpu --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/latsw/$rule.pytest.log 2>&1 \
      || { echo "tests $rule failed"; tail -20 gpurun_out/latsw/$rule.pytest.log; exit 1; }
  echo "rule $rule tests: $(tail -1 gpurun_out/latsw/$rule.pytest.log)"
  CATEARS_LAT_SLICES=$rule timeout -k 10 300 python tools/latency.py ${CALLS:-200} > gpurun_out/latsw/$rule.log 2>&1 \
      || { echo "latency $rule failed"; tail -5 gpurun_out/latsw/$rule.log; exit 1; }
  grep '^latency' gpurun_out/latsw/$rule.log
done
