# int8 vectorised epilogue (CATEARS_I8_EPI=1, default) vs the column-store one (0):
# parity with each, serial per-layer GEMM medians, the C5 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/i8epi && export TMPDIR=/tmp
for e in 1 0; do
  CATEARS_I8_EPI=$e timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/i8epi/pytest$e.log 2>&1 || { echo "int8 tests failed with EPI=$e"; tail -30 gpurun_out/i8epi/pytest$e.log; exit 1; }
  echo "int8 tests (EPI=$e): $(tail -1 gpurun_out/i8epi/pytest$e.log)"
done
for e in 1 0; do
  rm -rf gpurun_out/i8epi/run$e
  CATEARS_I8_EPI=$e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/i8epi/run$e -o run -- \
      python3 bench.py --workload c5 --serial --steps 6 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/i8epi/serial$e.log 2>&1 || { tail -5 gpurun_out/i8epi/serial$e.log; exit 1; }
  python3 tools/trace_summary.py $(find gpurun_out/i8epi/run$e -name '*kernel_trace.csv' | head -1) "C5 serial EPI=$e" > gpurun_out/i8epi/summary$e.txt
  echo "EPI=$e $(grep 'gemm_i8' gpurun_out/i8epi/summary$e.txt | head -2 | awk '{print $(NF-5), $(NF-2)}' | tr '\n' ' ')"
done
for rep in 1 2; do
  for e in 1 0; do
    CATEARS_I8_EPI=$e timeout -k 10 300 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/i8epi/b$e.$rep.json 2> gpurun_out/i8epi/b$e.$rep.err || { tail -5 gpurun_out/i8epi/b$e.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/i8epi/b$e.$rep.json')); print('EPI=$e rep $rep', round(d['value']/1e6,3), 'M', d['roofline']['frac'])"
  done
done
