# Rank 0 at N = 8 rehearsed with its sink share: 7 peers' receives + folds
# every step, own batches on the share 1 - 0.054 * 7 = 0.622 (and 0.75, 1.0);
# C3 60 steps; ms per step should fall to the senders' ~0.61.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z2
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline > gpurun_out/r05z2/base_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05z2/base_$rep.json')); print('no peers', l['value'], l['ms_per_step'])"
  for sh in 1.0 0.75 0.622; do
    timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers 7 --sink-share $sh > gpurun_out/r05z2/s${sh}_$rep.json 2>gpurun_out/r05z2/s${sh}_$rep.err || { tail -5 gpurun_out/r05z2/s${sh}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05z2/s${sh}_$rep.json')); print('7 peers share $sh', l['value'], l['ms_per_step'])"
  done
done
