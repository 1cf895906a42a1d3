# Warp-specialised bf16x6 variants: parity subset, per-layer serial times, C3 throughput A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/ws
for v in ${VARIANTS:-200 201 202 203}; do
  CATEARS_X6_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "test_am_s_vs_oracle or test_c3_full or test_am_xs_vs_oracle" \
      > gpurun_out/ws/p$v.log 2>&1 || { echo "parity $v failed"; tail -20 gpurun_out/ws/p$v.log; exit 1; }
  echo "v$v parity: $(tail -1 gpurun_out/ws/p$v.log)"
done
VARIANTS="160 ${VARIANTS:-200 201 202 203}" bash tools/x6_layers.sh || exit 1
ARMS="base=X=1"
for v in ${VARIANTS:-200 201 202 203}; do ARMS="$ARMS;v$v=CATEARS_X6_VARIANT=$v"; done
STEPS=200 REPS=2 ARMS="$ARMS" bash tools/ab.sh
