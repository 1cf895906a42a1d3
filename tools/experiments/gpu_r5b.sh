# C5: the fused fold + quantize (CATEARS_I8_QFOLD) and the non-temporal
# epilogue stores (CATEARS_I8_NT), alternating, after the int8 parity tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05b
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05b/pytest_i8.log 2>&1 || { tail -20 gpurun_out/r05b/pytest_i8.log; exit 1; }
tail -1 gpurun_out/r05b/pytest_i8.log
for i in 1 2; do
  for arm in "CATEARS_I8_QFOLD=0 CATEARS_I8_NT=1" "CATEARS_I8_QFOLD=1 CATEARS_I8_NT=1" "CATEARS_I8_QFOLD=1 CATEARS_I8_NT=0"; do
    n=$(echo $arm | tr -d ' =_' | sed 's/CATEARSI8//g')
    env $arm timeout -k 10 200 python bench.py --workload c5 --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline > gpurun_out/r05b/c5_$n.$i.json 2>/dev/null || exit 1
    python3 -c "
import json; l=json.load(open('gpurun_out/r05b/c5_$n.$i.json')); st=l['stages']
print('$n', round(l['value']/1e6,3), 'M', l['roofline']['frac'], {k: (v['avg_ms'], v['share_of_step']) for k, v in st.items()})"
  done
done
