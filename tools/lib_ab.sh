# A/B of alternative library builds (CATEARS_HIP_LIB) on the C3 bench, with a
# parity subset per build first:  LIBS="scratch/a.so scratch/b.so" bash tools/lib_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/libab
ARMS="base=X=1"
for L in ${LIBS}; do
  n=$(basename $L .so)
  CATEARS_HIP_LIB=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "test_am_s_vs_oracle or test_c3_full or test_am_xs_vs_oracle" \
      > gpurun_out/libab/$n.log 2>&1 || { echo "tests $n failed"; tail -20 gpurun_out/libab/$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/libab/$n.log)"
  ARMS="$ARMS;$n=CATEARS_HIP_LIB=$R/$L"
done
STEPS=${STEPS:-200} WARMUP=${WARMUP:-20} ARMS="$ARMS" REPS=${REPS:-2} bash tools/short_runs.sh
