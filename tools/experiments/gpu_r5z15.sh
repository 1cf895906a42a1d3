# Final check of the committed tree: the GPU suite, smoke(), the driver's
# bench line x3 and the default 200-step line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z15
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z15/suite.log 2>&1 || { tail -30 gpurun_out/r05z15/suite.log; exit 1; }
tail -1 gpurun_out/r05z15/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05z15/smoke.log 2>&1 || { tail -5 gpurun_out/r05z15/smoke.log; exit 1; }
tail -1 gpurun_out/r05z15/smoke.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05z15/driver_$i.json 2>/dev/null || exit 1
  cut -c1-200 gpurun_out/r05z15/driver_$i.json
done
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z15/default.json 2>/dev/null || exit 1
cut -c1-160 gpurun_out/r05z15/default.json
