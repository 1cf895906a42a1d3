# The round-4 measurement again with the aligned fbank mel table (tools/round_gpu.sh,
# TAG=r04i), plus latency, the driver config and C4.  Usage: bash tools/experiments/gpu_r4i.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r04i
TAG=r04i bash tools/round_gpu.sh > gpurun_out/r04i_round.log 2>&1 || { tail -30 gpurun_out/r04i_round.log; exit 1; }
tail -32 gpurun_out/r04i_round.log
timeout -k 10 200 python tools/latency.py 200 > gpurun_out/r04i/latency.txt 2>&1 || exit 1
grep "rows" gpurun_out/r04i/latency.txt
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04i/driver_$i.json 2>/dev/null || exit 1
  cut -c1-170 gpurun_out/r04i/driver_$i.json
done
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/r04i/c4.json 2> gpurun_out/r04i/c4.err || { tail -5 gpurun_out/r04i/c4.err; exit 1; }
cut -c1-300 gpurun_out/r04i/c4.json | tail -1
KREGEX=fbank WORKLOAD=c2 OUT=r04i/pmc_fb bash tools/pmc_kernel.sh > gpurun_out/r04i/pmc_fb.txt 2>&1 || exit 1
tail -30 gpurun_out/r04i/pmc_fb.txt
