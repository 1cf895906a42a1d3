# Tune run for the split-plane GEMMs: C3 bench per kernel variant (plus the
# fp32-MFMA program for reference).
#   VARIANTS="0 1 2" [GEMM=f16x3|bf16x6] [NOTEST=1] [BENCH_ARGS=--serial] bash tools/x6_variants.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/x6var
O=gpurun_out/x6var
GEMM=${GEMM:-bf16x6}
case $GEMM in bf16x6) VAR=CATEARS_X6_VARIANT;; f16x3) VAR=CATEARS_X3_VARIANT;; *) echo "GEMM?"; exit 2;; esac
if [ -z "$NOFP32" ]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --gemm fp32 ${BENCH_ARGS} > $O/fp32.log 2>&1 || { echo "fp32 bench failed"; tail -5 $O/fp32.log; exit 1; }
fi
for v in ${VARIANTS:-0}; do
  if [ -z "$NOTEST" ]; then
    env $VAR=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "$GEMM or split_gemms" > $O/$GEMM.v$v.pytest.log 2>&1; rc=$?
    echo "$GEMM variant $v pytest rc=$rc $(tail -1 $O/$GEMM.v$v.pytest.log)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  fi
  env $VAR=$v timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --gemm $GEMM ${BENCH_ARGS} > $O/$GEMM.v$v.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "variant $v bench rc=$rc"; tail -5 $O/$GEMM.v$v.log; exit $rc; }
done
python - $GEMM ${VARIANTS:-0} <<'PY'
import json, os, sys
g = sys.argv[1]
names = (["fp32"] if os.path.exists("gpurun_out/x6var/fp32.log") and not os.environ.get("NOFP32") else []) + [f"{g}.v{a}" for a in sys.argv[2:]]
for v in names:
    d = json.loads(open(f"gpurun_out/x6var/{v}.log").read().strip().splitlines()[-1])
    st, r = d["stages"], d["roofline"]
    print(f"{v:12s}: {d['value']/1e6:.3f} M frames/s, {d['ms_per_step']} ms/step, gemm {r['achieved']} TF "
          f"(frac {r['frac']}), avg {st['gemm']['avg_ms']} ms, eff {r['effective_ms_per_launch']} ms, launches {r['launches']}; "
          f"finalize {st['finalize']['avg_ms']}, gather {st.get('gemm_gather', {}).get('avg_ms')}")
PY
