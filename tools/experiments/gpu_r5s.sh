# Rank-0 rehearsal at 7 peers: fold block count (CATEARS_SUM_BLOCKS) and
# folds without the receive copies (CATEARS_REHEARSE_NOCOPY), C3 60 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05s
run() {  # label, env..., peers
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers $K > gpurun_out/r05s/$label.json 2>gpurun_out/r05s/$label.err || { tail -5 gpurun_out/r05s/$label.err; exit 1; }
  python3 -c "import json; l=json.load(open('gpurun_out/r05s/$label.json')); print('$label', l['value'], l['ms_per_step'])"
}
for rep in 1 2; do
  K=0 run base_$rep X=1
  K=7 run k7_b1024_$rep CATEARS_SUM_BLOCKS=1024
  K=7 run k7_b128_$rep CATEARS_SUM_BLOCKS=128
  K=7 run k7_b32_$rep CATEARS_SUM_BLOCKS=32
  K=7 run k7_nocopy_b1024_$rep CATEARS_REHEARSE_NOCOPY=1 CATEARS_SUM_BLOCKS=1024
  K=7 run k7_nocopy_b128_$rep CATEARS_REHEARSE_NOCOPY=1 CATEARS_SUM_BLOCKS=128
done
