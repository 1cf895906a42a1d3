# Two K-tiles per LDS stage (CATEARS_X6_KS=2: one block barrier per two
# K-tiles, same bits) against one, C3 at 200 steps, ABBA order per round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z11
for rep in 1 2 3; do
  i=0
  for k in 1 2 2 1; do
    i=$((i+1))
    CATEARS_X6_KS=$k timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z11/ks${k}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z11/ks${k}_${rep}_$i.json')); print('ks$k', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
