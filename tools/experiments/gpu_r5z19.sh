# What C5's int8 min / max + Quantize passes cost the pipelined step: the
# experiments library with CATEARS_SKIP=64 (those launches left out: wrong
# results, timing only) against it without, ABBA per round.  Needs
# libcatears_hip_exp.so pushed.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z19
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2 3; do
  i=0
  for k in 0 64 64 0; do
    i=$((i+1))
    CATEARS_SKIP=$k timeout -k 10 200 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/r05z19/s${k}_${rep}_$i.json 2>gpurun_out/r05z19/s${k}.err || { tail -5 gpurun_out/r05z19/s${k}.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05z19/s${k}_${rep}_$i.json')); print('skip=$k', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
