# A/B of env settings on the C3 bench in one process sequence: ARMS="A=ENV1;B=ENV2" (ENV: space-separated K=V)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/ab
IFS=';' read -ra AR <<< "$ARMS"
for rep in $(seq ${REPS:-2}); do
  for arm in "${AR[@]}"; do
    name=${arm%%=*}; envs=${arm#*=}
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/$name.$rep.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ab/$name.$rep.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab/$name.$rep.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', $rep, round(d['value']/1e6,3), 'M frames/s', r['achieved'], 'TF')"
  done
done
