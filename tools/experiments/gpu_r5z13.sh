# Two front streams (bench.py --front-streams 2: consecutive batches' fbank +
# CMVN on alternating streams, so the pipeline fills sooner) against one, at
# the driver's flags, ABBA per round; then 200 steps once each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z13
for rep in 1 2 3; do
  i=0
  for f in 1 2 2 1; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --front-streams $f > gpurun_out/r05z13/drv_f${f}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z13/drv_f${f}_${rep}_$i.json')); print('driver front=$f', l['value'], l['ms_per_step'])"
  done
done
for f in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --front-streams $f > gpurun_out/r05z13/def_f$f.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05z13/def_f$f.json')); print('200 steps front=$f', l['value'], l['ms_per_step'])"
done
