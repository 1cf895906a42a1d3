# bf16x6 direct kernel: the next K-tile's three weight planes issued a full
# tile ahead (CATEARS_X6_WPF=1, double-buffered) vs the default; identity
# test, serial per-layer times, C3 at the driver's flags alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05i
timeout -k 10 300 python -u -m pytest tests/test_gpu_x6_variants.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05i/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r05i/pytest.log
[ $rc -eq 0 ] || exit $rc
for w in 1 0; do
  CATEARS_X6_WPF=$w VARIANTS=0 bash tools/x6_layers.sh | sed "s/^/wpf$w /"
done
for i in 1 2 3; do
  for w in 1 0; do
    CATEARS_X6_WPF=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05i/driver_w${w}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05i/driver_w${w}_$i.json')); print('driver wpf$w', l['value'], l['roofline']['frac'])"
  done
done
for w in 1 0; do
  CATEARS_X6_WPF=$w timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r05i/long_w${w}.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05i/long_w${w}.json')); print('200-step wpf$w', l['value'], l['roofline']['frac'])"
done
