# GEMM packing of the pipelined C3 bench: kernel trace of 60 timed steps
# (tools/trace_short.sh), then tools/gemm_overlap.py over it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
STEPS=60 WARMUP=20 bash tools/trace_short.sh || exit 1
python3 tools/gemm_overlap.py $(find gpurun_out/tl/run -name '*kernel_trace.csv' | head -1) | tee gpurun_out/tl/overlap.txt
