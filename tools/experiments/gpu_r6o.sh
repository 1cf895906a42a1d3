# Latency mode with the split-K fix-up (the tile's last slice block does the
# reduce; CATEARS_LAT_FIXUP=1, experiments library): the latency GPU tests on
# it, then tools/latency.py fix-up off (0) / on (1) ABBA x2 with the output
# hashes compared.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06o}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
CATEARS_LAT_FIXUP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_latency.py > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for rep in 1 2; do
  for f in 0 1 1 0; do
    CATEARS_LAT_FIXUP=$f LAT_MODES=latency LAT_ROWS=70,270,1018 timeout -k 10 200 python tools/latency.py 300 \
        > gpurun_out/$T/lat_f${f}_$rep.txt 2>&1 || { tail -5 gpurun_out/$T/lat_f${f}_$rep.txt; exit 1; }
    echo "fixup $f: $(grep -E 'rows ' gpurun_out/$T/lat_f${f}_$rep.txt | tr -s ' ' | cut -d' ' -f3,4,5,10,11 | tr '\n' ' ')"
  done
done
echo exit 0
