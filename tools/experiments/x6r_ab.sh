# bf16x6 default (0 = 300, direct weights + LDS activations) vs 400
# (register-direct, no LDS): C3 at the driver's step counts, alternating,
# then serial per-layer launch times.  Variant 400 lives in the experiments
# build only (`make EXPERIMENTS=1 lib`; remove its line from .gpurunignore
# for the call): both variants run from that library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
cd "$R" && mkdir -p gpurun_out/x6r
for rep in 1 2 3; do
  for v in 0 400; do
    CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup ${WARM:-5} --no-cpu-baseline \
      > gpurun_out/x6r/v$v.$rep.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/x6r/v$v.$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/x6r/v$v.$rep.log') if x.startswith('{')][0]); r=d['roofline']
print('x6 v$v', round(d['value']/1e6,3), 'M frames/s', r['achieved'], 'TF', r['frac'], 'checksum', d['checksum'])"
  done
done
for v in 0 400; do
  CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --steps 60 --warmup 10 --serial --no-cpu-baseline \
    > gpurun_out/x6r/serial.v$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/x6r/serial.v$v.log; exit 1; }
  python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/x6r/serial.v$v.log') if x.startswith('{')][0]); r=d['roofline']
print('x6 serial v$v', round(d['value']/1e6,3), 'M frames/s', r['achieved'], 'TF', 'avg launch ms', r['avg_launch_ms'])"
done
