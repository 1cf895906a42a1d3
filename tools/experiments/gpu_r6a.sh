# Round-6 measurement of the tree (tools/round_gpu.sh: GPU suite, bench under
# rocprofv3 kernel stats with the timed-window markers, PMC traffic / MFMA /
# VALU passes, C2 and C5), then the streaming latency, the driver's flags
# (x2) and smoke.  Usage: T=r06a bash tools/experiments/gpu_r6a.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06a}
cd "$R" && mkdir -p gpurun_out/$T
TAG=$T bash tools/round_gpu.sh > gpurun_out/${T}_round.log 2>&1 || { tail -30 gpurun_out/${T}_round.log; exit 1; }
tail -32 gpurun_out/${T}_round.log
cd "$R" || exit 1
timeout -k 10 200 python tools/latency.py 200 > gpurun_out/$T/latency.txt 2>&1 || exit 1
grep "rows    70" gpurun_out/$T/latency.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/driver_$i.json 2>/dev/null || exit 1
  cut -c1-170 gpurun_out/$T/driver_$i.json
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
