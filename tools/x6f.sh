# fp32-in bf16x6 (CATEARS_X6_F32IN=1) vs the plane kernel: parity + bench per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/x6f
O=gpurun_out/x6f
for v in ${VARIANTS:-0}; do
  CATEARS_X6_F32IN=1 CATEARS_X6_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider -k "bf16x6 or split_gemms" > $O/f.v$v.pytest.log 2>&1; rc=$?
  echo "f32in variant $v pytest rc=$rc $(tail -1 $O/f.v$v.pytest.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  CATEARS_X6_F32IN=1 CATEARS_X6_VARIANT=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > $O/f.v$v.log 2>&1 || { echo "bench failed"; tail -5 $O/f.v$v.log; exit 1; }
  python -c "
import json; d=json.loads(open('$O/f.v$v.log').read().strip().splitlines()[-1]); r=d['roofline']
print('f32in v$v', round(d['value']/1e6,3), 'M frames/s', r['achieved'], 'TF', r['frac'])"
done
