# Whole GPU suite, smoke() and the default bench line after the gather /
# fold / sink-share changes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05v
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05v/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r05v/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05v/smoke.log 2>&1 || { tail -5 gpurun_out/r05v/smoke.log; exit 1; }
tail -1 gpurun_out/r05v/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r05v/driver.json 2>gpurun_out/r05v/driver.err || { tail -5 gpurun_out/r05v/driver.err; exit 1; }
cut -c1-200 gpurun_out/r05v/driver.json
