# int8 GEMM variants: parity (tests/test_gpu_int8.py) then the C5 bench, per CATEARS_I8_GEMM value
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/i8ab
for v in ${VARIANTS:-15 20}; do
  CATEARS_I8_GEMM=$v timeout -k 10 300 python -m pytest tests/test_gpu_int8.py tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "int8 or u8" > gpurun_out/i8ab/v$v.pytest.log 2>&1; rc=$?
  echo "variant $v pytest rc=$rc $(tail -1 gpurun_out/i8ab/v$v.pytest.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  CATEARS_I8_GEMM=$v timeout -k 10 300 python bench.py --workload c5 --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline > gpurun_out/i8ab/v$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/i8ab/v$v.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/i8ab/v$v.log').read().strip().splitlines()[-1]); r=d['roofline']
print('i8 v$v', round(d['value']/1e6,3), 'M frames/s', r['achieved'], 'TOP/s', r['frac'])"
done
