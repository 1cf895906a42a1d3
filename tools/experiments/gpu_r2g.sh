R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/clk && export TMPDIR=/tmp
rm -rf gpurun_out/clk/*
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "gemm_bf16x6f" --output-format csv -d gpurun_out/clk/run -o run -- \
    python3 bench.py --steps 60 --warmup 1 --serial --no-cpu-baseline --no-profile > gpurun_out/clk/bench.log 2>&1 || { tail -5 gpurun_out/clk/bench.log; exit 1; }
ls -R gpurun_out/clk | head
