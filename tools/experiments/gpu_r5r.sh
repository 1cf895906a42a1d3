# Rank 0's receive-and-fold load at N = K+1 ranks, rehearsed on one GPU
# (bench.py --rehearse-peers K: K local copies of each batch plus K+1
# float64 folds on a stream of their own), C3 at the driver's flags and at
# 200 steps, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05r
for rep in 1 2; do
  for k in 0 1 3 7; do
    timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers $k > gpurun_out/r05r/k${k}_$rep.json 2>gpurun_out/r05r/k${k}_$rep.err || { tail -5 gpurun_out/r05r/k${k}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05r/k${k}_$rep.json')); print('peers $k', l['value'], l['ms_per_step'])"
  done
done
