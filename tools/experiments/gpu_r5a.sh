# Round 5, first check after the packed-FP32 fix: the whole GPU suite, then
# the new library against round 4's (catears_amd/lib/ab/libcatears_hip_r4.so)
# on the driver's C3 config, C2 exact / fast, C5 and the streaming latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05a
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05a/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r05a/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
NEW=$R/catears_amd/lib/libcatears_hip.so
OLD=$R/catears_amd/lib/ab/libcatears_hip_r4.so
for i in 1 2; do
  for L in $NEW $OLD; do
    v=$(basename $L .so)
    CATEARS_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05a/c3_$v.$i.json 2>/dev/null || exit 1
    echo "c3 $v $(cut -c1-120 gpurun_out/r05a/c3_$v.$i.json)"
    for W in "c2" "c2 --fbank fast" "c5"; do
      n=$(echo $W | tr -d ' -')
      CATEARS_HIP_LIB=$L timeout -k 10 200 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05a/${n}_$v.$i.json 2>/dev/null || exit 1
      echo "$n $v $(cut -c1-120 gpurun_out/r05a/${n}_$v.$i.json)"
    done
    CATEARS_HIP_LIB=$L timeout -k 10 200 python tools/latency.py 100 > gpurun_out/r05a/lat_$v.$i.txt 2>&1 || exit 1
    echo "lat $v $(grep 'rows    70' gpurun_out/r05a/lat_$v.$i.txt | head -2 | tr '\n' ' ')"
  done
done
