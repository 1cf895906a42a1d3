# Round 5 check of the tree: the whole GPU suite, the new exact fbank's PMC
# counters (C2), C4 with the stage profile (the front stream's CMVN share),
# C3 at the driver's flags (x3), without the pre-warm (x2) and the default
# 200 steps, and the streaming latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05e
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05e/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r05e/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
KREGEX=fbank WORKLOAD=c2 OUT=r05e/pmc_fb bash tools/pmc_kernel.sh > gpurun_out/r05e/pmc_fb.txt 2>&1 || { tail -20 gpurun_out/r05e/pmc_fb.txt; exit 1; }
cat gpurun_out/r05e/pmc_fb.txt
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --stage-profile > gpurun_out/r05e/c4.json 2> gpurun_out/r05e/c4.err || { tail -5 gpurun_out/r05e/c4.err; exit 1; }
python3 -c "import json; l=json.load(open('gpurun_out/r05e/c4.json')); print('c4', l['value'], l['roofline']['frac'], json.dumps(l.get('stages')))"
for i in 1 2 3; do
  for ks in 2 1; do
    CATEARS_X6_KS=$ks timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05e/driver_ks${ks}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05e/driver_ks${ks}_$i.json')); print('driver ks$ks', l['value'], l['roofline']['frac'])"
  done
done
for ks in 2 1; do
  CATEARS_X6_KS=$ks VARIANTS=0 bash tools/x6_layers.sh | sed "s/^/ks$ks /"
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms 0 > gpurun_out/r05e/noprewarm_$i.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05e/noprewarm_$i.json')); print('no-prewarm', l['value'], l['roofline']['frac'])"
done
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05e/default.json 2>/dev/null || exit 1
python3 -c "import json; l=json.load(open('gpurun_out/r05e/default.json')); print('default-200', l['value'], l['roofline']['frac'])"
timeout -k 10 200 python tools/latency.py 200 > gpurun_out/r05e/latency.txt 2>&1 || exit 1
grep "rows    70" gpurun_out/r05e/latency.txt
