# int8 GEMM tile A/B (measurement library): parity per variant, the C5 line
# per variant (alternating), serial per-layer GEMM medians.
#   VARIANTS="15 40 41 44" bash tools/experiments/i8_tiles.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/i8t && export TMPDIR=/tmp
export CATEARS_HIP_LIB=catears_amd/lib/libcatears_hip_exp.so
V=${VARIANTS:-15 40 41 44}
for v in $V; do
  CATEARS_I8_GEMM=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/i8t/pytest$v.log 2>&1 || { echo "int8 tests failed under $v"; tail -30 gpurun_out/i8t/pytest$v.log; exit 1; }
  echo "int8 tests ($v): $(tail -1 gpurun_out/i8t/pytest$v.log)"
done
for rep in 1 2; do
  for v in $V; do
    CATEARS_I8_GEMM=$v timeout -k 10 300 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/i8t/b$v.$rep.json 2> gpurun_out/i8t/b$v.$rep.err || { tail -5 gpurun_out/i8t/b$v.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/i8t/b$v.$rep.json')); print('v$v rep $rep', round(d['value']/1e6,3), 'M', d['roofline']['frac'])"
  done
done
for v in $V; do
  rm -rf gpurun_out/i8t/run$v
  CATEARS_I8_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/i8t/run$v -o run -- \
      python3 bench.py --workload c5 --serial --steps 10 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/i8t/serial$v.log 2>&1 || { tail -5 gpurun_out/i8t/serial$v.log; exit 1; }
  python3 tools/trace_summary.py $(find gpurun_out/i8t/run$v -name '*kernel_trace.csv' | head -1) "C5 serial v$v" > gpurun_out/i8t/summary$v.txt
  grep gemm_i8 gpurun_out/i8t/summary$v.txt | head -4
done
