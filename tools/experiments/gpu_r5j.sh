# CMVN without the alpha == 1 selects (new), and with 48-frame prefetch
# tiles (t48), against the r05 build (old): CMVN tests, then C4 with the
# stage profile and C3 at the driver's flags, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05j
timeout -k 10 600 python -u -m pytest tests -m gpu -k "cmvn or c4 or c3_full or determinism" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05j/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r05j/pytest.log
[ $rc -eq 0 ] || exit $rc
CATEARS_HIP_LIB=$PWD/abtmp/t48.so timeout -k 10 300 python -u -m pytest tests -m gpu -k "cmvn" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05j/pytest_t48.log 2>&1 || { tail -5 gpurun_out/r05j/pytest_t48.log; exit 1; }
tail -1 gpurun_out/r05j/pytest_t48.log
for rep in 1 2; do
  for v in old new t48; do
    CATEARS_HIP_LIB=$PWD/abtmp/$v.so timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --stage-profile > gpurun_out/r05j/c4_$v.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05j/c4_$v.json')); s=l['stages']; print('c4 $v', l['value'], 'cmvn', s['cmvn']['avg_ms'], s['cmvn']['share_of_wall'], s['cmvn']['share_of_front_busy'], 'fbank', s['fbank']['avg_ms'], 'front', s['front_stream']['share_of_wall'])"
    CATEARS_HIP_LIB=$PWD/abtmp/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05j/c3_$v.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05j/c3_$v.json')); print('c3 $v', l['value'])"
  done
done
