# A/B of library builds on the C2 (batched fbank) bench and the C3 bench:
# fbank parity per build first, then alternating bench runs.
#   LIBS="scratch/base.so scratch/x.so" bash tools/c2_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/c2ab
for L in ${LIBS}; do
  n=$(basename $L .so)
  CATEARS_HIP_LIB=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "fbank or c3_full" > gpurun_out/c2ab/$n.pytest.log 2>&1 \
      || { echo "tests $n failed"; tail -20 gpurun_out/c2ab/$n.pytest.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/c2ab/$n.pytest.log)"
done
for rep in $(seq ${REPS:-2}); do
  for L in ${LIBS}; do
    n=$(basename $L .so)
    for W in ${WORKLOADS:-c2 c3}; do
      CATEARS_HIP_LIB=$R/$L timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-30} --warmup ${WARMUP:-5} \
          --no-cpu-baseline > gpurun_out/c2ab/$n.$W.$rep.log 2>&1 || { echo "bench $n $W failed"; tail -5 gpurun_out/c2ab/$n.$W.$rep.log; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/c2ab/$n.$W.$rep.log').read().strip().splitlines()[-1])
print('$n $W rep $rep', round(d['value']/1e6,3), 'M frames/s', d['ms_per_step'], 'ms/step', d['roofline'].get('avg_launch_ms'))"
    done
  done
done
