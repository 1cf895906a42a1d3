# Round-4 latency rework + first-layer tile A/B.  Usage: bash tools/experiments/gpu_r4c.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4c
O=gpurun_out/r4c
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_latency.py \
  tests/test_gpu_x6_variants.py > $O/t8.txt 2>&1 || { tail -30 $O/t8.txt; exit 1; }
tail -2 $O/t8.txt
LAT_MODES=latency timeout -k 10 200 python tools/latency.py 200 > $O/lat_new.txt 2>&1 || exit 1
CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_r3fix.so LAT_MODES=latency timeout -k 10 200 \
  python tools/latency.py 200 > $O/lat_r3.txt 2>&1 || exit 1
LAT_MODES=latency timeout -k 10 200 python tools/latency.py 200 > $O/lat_new2.txt 2>&1 || exit 1
for f in lat_new lat_r3 lat_new2; do echo "== $f"; grep "latency " $O/$f.txt; done
for i in 1 2; do
  for t in 256 128; do
    CATEARS_X6_FIRST_TILE=$t timeout -k 10 200 python bench.py > $O/bench_t${t}_$i.json 2> $O/bench_t${t}_$i.err || exit 1
    echo "tile $t run $i: $(python -c "import json,sys; d=json.loads(open('$O/bench_t${t}_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o s -- \
  python bench.py --serial --steps 20 --warmup 3 > $O/serial.json 2> $O/serial.err || exit 1
CATEARS_X6_FIRST_TILE=128 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial128 -o s -- \
  python bench.py --serial --steps 20 --warmup 3 > $O/serial128.json 2> $O/serial128.err || exit 1
echo done
