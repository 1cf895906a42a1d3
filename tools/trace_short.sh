# Kernel trace of the driver-shaped bench (--steps 20 --warmup 5) + timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/tl && export TMPDIR=/tmp
rm -rf gpurun_out/tl/run
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/run -o run -- \
    python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/tl/bench.log 2>&1 || { echo "failed"; tail -5 gpurun_out/tl/bench.log; exit 1; }
grep '^{' gpurun_out/tl/bench.log | cut -c1-250
python3 tools/timeline.py $(find gpurun_out/tl/run -name '*kernel_trace.csv' | head -1) ${BIN:-100} > gpurun_out/tl/timeline.txt
head -3 gpurun_out/tl/timeline.txt
