# Tune run: correctness + bench for every GEMM tile variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3 4}; do
  CATEARS_GEMM_VARIANT=$v timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "am_ or sgemm or score" > gpurun_out/var$v.pytest.log 2>&1; rc=$?
  echo "variant $v pytest rc=$rc $(tail -1 gpurun_out/var$v.pytest.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  CATEARS_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/var$v.bench.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/var$v.bench.log; exit $rc; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/var{v}.bench.log").read().strip().splitlines()[-1])
st = d["stages"]
print(f"variant {v}: {d['value']:.0f} frames/s, {d['ms_per_step']} ms/step, gemm {d['roofline']['achieved']} TF "
      f"({d['roofline']['frac']}), avg {st['gemm']['avg_ms']} ms, eff {d['roofline']['effective_ms_per_launch']} ms; cmvn {st['cmvn']['avg_ms']} ms, fbank {st['fbank']['avg_ms']} ms, finalize {st['finalize']['avg_ms']}, gather-gemm {st['gemm_gather']['avg_ms']}")
PY
done
