# The driver's bench shape (--steps 20 --warmup 5) repeated, beside longer runs:
#   ARMS="a=CATEARS_X6_VARIANT=42;b=CATEARS_X6_VARIANT=70|--no-profile" REPS=3 bash tools/short_runs.sh
# (arm = name=ENV ... [|extra bench args])
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/short
IFS=';' read -ra AR <<< "${ARMS:-base=X=1}"
for rep in $(seq ${REPS:-3}); do
  for arm in "${AR[@]}"; do
    name=${arm%%=*}; rest=${arm#*=}; envs=${rest%%|*}; xargs_=""; [[ "$rest" == *"|"* ]] && xargs_=${rest#*|}
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu-baseline ${BENCH_ARGS} $xargs_ \
        > gpurun_out/short/$name.$rep.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/short/$name.$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/short/$name.$rep.log').read().strip().splitlines()[-1])
print('$name', $rep, round(d['value']/1e6,3), 'M frames/s', d['ms_per_step'], 'ms/step', d['roofline']['achieved'], 'TF')"
  done
done
