# Latency mode with fewer, longer split-K slices (CATEARS_LAT_TARGET 192 /
# 128 blocks per row tile against the default 256): 70-row TDNN-S chunk,
# tools/latency.py, order rotated, twice.  The knob is read by the
# experiments library only (push libcatears_hip_exp.so; it ran in the
# product library when measured, profiles/r05z16_lat_slices.txt).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z16
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2; do
  for t in ${TARGETS:-256 192 128 96}; do
    CATEARS_LAT_TARGET=$t LAT_MODES=latency LAT_ROWS=70,270 timeout -k 10 200 python tools/latency.py 300 > gpurun_out/r05z16/t${t}_$rep.txt 2>&1 || { tail -5 gpurun_out/r05z16/t${t}_$rep.txt; exit 1; }
    echo "target $t: $(grep 'rows' gpurun_out/r05z16/t${t}_$rep.txt | tr '\n' ' ')"
  done
done
