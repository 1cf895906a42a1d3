# GPU round-trip used during development: parity tests, bench, rocprof trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$PROF" -o run -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-profile > "$R/gpurun_out/$PROF.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; exit $rc
fi
