# Per-layer int8 GEMM durations (serial C5, rocprof kernel trace) for each
# CATEARS_I8_GEMM variant in VARIANTS.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in ${VARIANTS:-9 7 0}; do
  rm -rf gpurun_out/i8v$v
  CATEARS_I8_GEMM=$v timeout -k 10 300 python -m pytest tests/test_gpu_int8.py -q -m gpu -p no:cacheprovider > gpurun_out/i8v$v.pytest.log 2>&1; rc=$?
  echo "variant $v pytest rc=$rc $(tail -1 gpurun_out/i8v$v.pytest.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  CATEARS_I8_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/i8v$v -o run -- \
    python3 bench.py --workload c5 --serial --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > gpurun_out/i8v$v.log 2>&1 || { echo "v$v rc=$?"; tail -5 gpurun_out/i8v$v.log; exit 1; }
  echo "== variant $v: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/i8v$v.log') if l.startswith('{')][-1]); print(d['value'])")"
  python3 tools/trace_summary.py $(find gpurun_out/i8v$v -name '*kernel_trace.csv' | head -1) > gpurun_out/i8v$v.summary.txt
  python3 tools/dispatch_seq.py $(find gpurun_out/i8v$v -name '*kernel_trace.csv' | head -1) gemm_i8 14
done
