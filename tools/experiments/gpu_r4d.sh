# Round-4 latency (round-3 split-K kernel + fused final reduce) A/B against
# the round-3 library, and the GPU tests it touches.  Usage: bash tools/experiments/gpu_r4d.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4d
O=gpurun_out/r4d
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_latency.py \
  tests/test_gpu_x6_variants.py tests/test_gpu_c4.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
for f in new r3 new2; do
  if [ $f = r3 ]; then export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_r3fix.so; else unset CATEARS_HIP_LIB; fi
  LAT_MODES=latency timeout -k 10 200 python tools/latency.py 200 > $O/lat_$f.txt 2>&1 || exit 1
  echo "== $f"; grep "latency " $O/lat_$f.txt
done
unset CATEARS_HIP_LIB
cd /tmp && export TMPDIR=/tmp && cd "$R"
LAT_MODES=latency LAT_ROWS=70 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o lat -- \
  python tools/latency.py 100 > $O/prof.txt 2>&1 || exit 1
echo done
