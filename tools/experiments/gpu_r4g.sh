# CMVN / parity check, then the full round measurement (tools/round_gpu.sh,
# TAG=r04g) with the latency, driver-config, fbank PMC and C4 extras.  Usage: bash tools/experiments/gpu_r4g.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4f gpurun_out/r04g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "cmvn or score or c3" > gpurun_out/r4f/t.txt 2>&1 || { echo "CMVN parity FAILED"; tail -30 gpurun_out/r4f/t.txt; exit 1; }
tail -1 gpurun_out/r4f/t.txt
TAG=r04g bash tools/round_gpu.sh > gpurun_out/r04g_round.log 2>&1 || { tail -30 gpurun_out/r04g_round.log; exit 1; }
tail -32 gpurun_out/r04g_round.log
timeout -k 10 200 python tools/latency.py 200 > gpurun_out/r04g/latency.txt 2>&1 || exit 1
grep "rows" gpurun_out/r04g/latency.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04g/driver_$i.json 2>/dev/null || exit 1
  cut -c1-170 gpurun_out/r04g/driver_$i.json
done
KREGEX=fbank WORKLOAD=c2 OUT=r04g/pmc_fb bash tools/pmc_kernel.sh > gpurun_out/r04g/pmc_fb.txt 2>&1 || exit 1
tail -30 gpurun_out/r04g/pmc_fb.txt
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/r04g/c4.json 2> gpurun_out/r04g/c4.err || { tail -5 gpurun_out/r04g/c4.err; exit 1; }
cut -c1-300 gpurun_out/r04g/c4.json | tail -1
