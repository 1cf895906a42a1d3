# Parity + A/B of bf16x6 kernel variants (CATEARS_X6_VARIANT):
#   VARIANTS="60 61" [BASE=42] [SKIP_FULL=1] bash tools/x6m_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/x6m
if [ -z "$SKIP_FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/x6m/full.log 2>&1 || { echo "full gpu suite failed"; tail -30 gpurun_out/x6m/full.log; exit 1; }
  tail -2 gpurun_out/x6m/full.log
fi
for v in ${VARIANTS}; do
  CATEARS_X6_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 \
      --timeout-method thread -p no:cacheprovider \
      -k "test_am_s_vs_oracle and bf16x6 and not bf16x6p or test_c3_full or test_split_gemms or test_am_xs_vs_oracle and bf16x6 and not bf16x6p" \
      > gpurun_out/x6m/t$v.log 2>&1 || { echo "tests v$v failed"; tail -30 gpurun_out/x6m/t$v.log; exit 1; }
  echo "v$v parity: $(tail -1 gpurun_out/x6m/t$v.log)"
done
ARMS="base=CATEARS_X6_VARIANT=${BASE:-42}"
for v in ${VARIANTS}; do ARMS="$ARMS;v$v=CATEARS_X6_VARIANT=$v"; done
ARMS="$ARMS" REPS=${REPS:-2} STEPS=${STEPS:-200} bash tools/ab.sh
