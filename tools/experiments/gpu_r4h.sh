# The round-4 measurement again with bench.py's pre-warm (tools/round_gpu.sh,
# TAG=r04h), plus latency, the driver config and C4.  Usage: bash tools/experiments/gpu_r4h.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r04h
TAG=r04h bash tools/round_gpu.sh > gpurun_out/r04h_round.log 2>&1 || { tail -30 gpurun_out/r04h_round.log; exit 1; }
tail -32 gpurun_out/r04h_round.log
timeout -k 10 200 python tools/latency.py 200 > gpurun_out/r04h/latency.txt 2>&1 || exit 1
grep "rows" gpurun_out/r04h/latency.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04h/driver_$i.json 2>/dev/null || exit 1
  cut -c1-170 gpurun_out/r04h/driver_$i.json
done
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/r04h/c4.json 2> gpurun_out/r04h/c4.err || { tail -5 gpurun_out/r04h/c4.err; exit 1; }
cut -c1-300 gpurun_out/r04h/c4.json | tail -1
