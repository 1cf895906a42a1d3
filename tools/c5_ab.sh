# A/B of library builds on the C5 (int8) bench: int8 parity with the default
# library, then alternating bench runs per build.
#   LIBS="scratch/base.so scratch/new.so" bash tools/c5_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/c5ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/c5ab/pytest.log 2>&1 || { echo "int8 tests failed"; tail -20 gpurun_out/c5ab/pytest.log; exit 1; }
echo "int8 tests: $(tail -1 gpurun_out/c5ab/pytest.log)"
for rep in $(seq ${REPS:-2}); do
  for L in ${LIBS}; do
    n=$(basename $L .so)
    CATEARS_HIP_LIB=$R/$L timeout -k 10 300 python bench.py --workload c5 --steps ${STEPS:-60} --warmup ${WARMUP:-10} \
        --no-cpu-baseline > gpurun_out/c5ab/$n.$rep.log 2>&1 || { echo "bench $n failed"; tail -5 gpurun_out/c5ab/$n.$rep.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/c5ab/$n.$rep.log').read().strip().splitlines()[-1])
print('$n rep $rep', round(d['value']/1e6,3), 'M frames/s', d['ms_per_step'], 'ms/step', {k: v.get('avg_ms') for k, v in d.get('stages', {}).items()})"
  done
done
