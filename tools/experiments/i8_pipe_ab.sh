# int8 GEMM: pipelined (16, default) vs round 3's (15) -- parity, then C5
# pipelined and serial (--serial: one stream, launch times are per layer).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/i8p
timeout -k 10 300 python -m pytest tests/test_gpu_int8.py -q -m gpu -p no:cacheprovider -x > gpurun_out/i8p/pytest.log 2>&1 \
  || { tail -30 gpurun_out/i8p/pytest.log; exit 1; }
tail -1 gpurun_out/i8p/pytest.log
for rep in 1 2; do
for v in ${VARIANTS:-15 16}; do
  for mode in pipe serial; do
    extra=""; [ $mode = serial ] && extra="--serial"
    CATEARS_I8_GEMM=$v timeout -k 10 300 python bench.py --workload c5 --steps ${STEPS:-60} --warmup 10 --no-cpu-baseline $extra \
      > gpurun_out/i8p/v$v.$mode.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/i8p/v$v.$mode.$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/i8p/v$v.$mode.$rep.log').read().strip().splitlines()[-1]); r=d['roofline']
print('i8 v$v $mode', round(d['value']/1e6,3), 'M frames/s', r['achieved'], 'TOP/s', r['frac'], 'avg launch ms', r['avg_launch_ms'])"
  done
done
done
