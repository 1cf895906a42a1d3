# Round-4 measurements beside the round script: streaming latency (both
# modes), PMC counters of the int8 GEMM, and a kernel trace of the driver's
# C3 command (timeline).  Usage: bash tools/gpu_r4b.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4b
timeout -k 10 300 python tools/latency.py 200 > gpurun_out/r4b/latency.txt 2>&1 || { tail -20 gpurun_out/r4b/latency.txt; exit 1; }
cat gpurun_out/r4b/latency.txt | tail -12
KREGEX=gemm_i8 WORKLOAD=c5 OUT=r4b/pmc_i8 bash tools/pmc_kernel.sh || exit 1
