# Kernel trace of tools/latency.py (per-call latency of ce_gpu_nnet_propagate):
# shows the GPU busy time per call against the call-to-call interval.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/lat && export TMPDIR=/tmp
rm -rf gpurun_out/lat/run
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lat/run -o run -- \
    python3 tools/latency.py ${CALLS:-100} > gpurun_out/lat/latency.log 2>&1 || { echo "failed"; tail -5 gpurun_out/lat/latency.log; exit 1; }
cat gpurun_out/lat/latency.log | grep -v amdgpu.ids
cp $(find gpurun_out/lat/run -name '*kernel_trace.csv' | head -1) gpurun_out/lat/kernel_trace.csv
