# Final check after the int8 Quantize change: GPU suite, smoke, the driver's
# C3 line, and C5 once.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z22
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z22/suite.log 2>&1 || { tail -30 gpurun_out/r05z22/suite.log; exit 1; }
tail -1 gpurun_out/r05z22/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05z22/smoke.log 2>&1 || { tail -5 gpurun_out/r05z22/smoke.log; exit 1; }
tail -1 gpurun_out/r05z22/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05z22/driver.json 2>/dev/null || exit 1
cut -c1-160 gpurun_out/r05z22/driver.json
timeout -k 10 200 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/r05z22/c5.json 2>/dev/null || exit 1
python3 -c "import json; l=json.load(open('gpurun_out/r05z22/c5.json')); print('c5', l['value'], l['ms_per_step'], l['checksum'])"
