# Planes into the output layer only (CATEARS_X6_CHAIN=2: the 1024 x 3456
# layer's 14 unit tiles stop splitting the same activations; the layer
# before writes them split) against the fp32 chain: the variants test, then
# C3 at 200 steps and at the driver's flags, ABBA per round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z18
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6_variants.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z18/variants.log 2>&1 || { tail -30 gpurun_out/r05z18/variants.log; exit 1; }
tail -1 gpurun_out/r05z18/variants.log
for rep in 1 2 3; do
  i=0
  for c in 0 2 2 0; do
    i=$((i+1))
    CATEARS_X6_CHAIN=$c timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z18/c${c}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z18/c${c}_${rep}_$i.json')); print('chain=$c', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
