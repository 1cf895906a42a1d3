# Tile group of the 1024 x 3456 output layer (CATEARS_X6_GROUP_WIDE; default
# 2 like the hidden layers): serial per-layer times, then C3 at 60 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05n
for g in 2 1 4 7 14; do
  CATEARS_X6_GROUP_WIDE=$g VARIANTS=0 bash tools/x6_layers.sh | sed "s/^/g$g /"
done
for rep in 1 2; do
  for g in 2 1 4 7; do
    CATEARS_X6_GROUP_WIDE=$g timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline > gpurun_out/r05n/c3_g${g}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05n/c3_g${g}_$rep.json')); print('c3 g$g', l['value'], l['ms_per_step'])"
  done
done
