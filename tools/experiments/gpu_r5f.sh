# The gathered first layer with every K-tile's activations preloaded
# (CATEARS_X6_FIRST_PRE=1, default) against one tile ahead (0): the variant
# identity tests, serial per-layer times, C3 at the driver's flags alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05f
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6_variants.py tests/test_gpu_latency.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r05f/pytest.log 2>&1 || { tail -30 gpurun_out/r05f/pytest.log; exit 1; }
tail -1 gpurun_out/r05f/pytest.log
for pre in 1 0; do
  CATEARS_X6_FIRST_PRE=$pre VARIANTS=0 bash tools/x6_layers.sh | sed "s/^/pre$pre /"
done
for i in 1 2 3; do
  for pre in 1 0; do
    CATEARS_X6_FIRST_PRE=$pre timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05f/driver_pre${pre}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05f/driver_pre${pre}_$i.json')); print('driver pre$pre', l['value'], l['roofline']['frac'])"
  done
done
