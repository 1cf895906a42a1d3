# Round-5 final measurement of the tree (tools/round_gpu.sh, TAG=r05x: GPU
# suite, bench under rocprofv3 kernel stats, the PMC traffic / MFMA passes,
# C2 and C5), then the streaming latency, the driver's flags (x3), no
# pre-warm (x2), C4 with the stage profile, and the exact fbank's PMC
# counters.  Usage: bash tools/experiments/gpu_r5x.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r05x}
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
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms 0 > gpurun_out/$T/noprewarm_$i.json 2>/dev/null || exit 1
  cut -c1-120 gpurun_out/$T/noprewarm_$i.json
done
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --stage-profile > gpurun_out/$T/c4.json 2> gpurun_out/$T/c4.err || { tail -5 gpurun_out/$T/c4.err; exit 1; }
python3 -c "import json; l=json.load(open('gpurun_out/$T/c4.json')); print('c4', l['value'], l['roofline']['frac'], json.dumps(l.get('stages')))"
KREGEX=fbank WORKLOAD=c2 OUT=$T/pmc_fb bash tools/pmc_kernel.sh > gpurun_out/$T/pmc_fb.txt 2>&1 || { tail -20 gpurun_out/$T/pmc_fb.txt; exit 1; }
tail -30 gpurun_out/$T/pmc_fb.txt
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/$T/default.json 2>/dev/null || exit 1
cut -c1-120 gpurun_out/$T/default.json
timeout -k 10 200 python bench.py --workload c2 --fbank fast --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/$T/c2_fast.json 2>/dev/null || exit 1
cut -c1-120 gpurun_out/$T/c2_fast.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
KREGEX=fbank_fma WORKLOAD=c2 OUT=$T/pmc_fbf BENCH_ARGS="--fbank fast" bash tools/pmc_kernel.sh > gpurun_out/$T/pmc_fbf.txt 2>&1 || { tail -20 gpurun_out/$T/pmc_fbf.txt; exit 1; }
tail -14 gpurun_out/$T/pmc_fbf.txt
