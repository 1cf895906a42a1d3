# Rank-0 rehearsal (7 peers) with the pipeline streams at high priority and
# the receive / fold stream at the default (CATEARS_PRIO_SPLIT=1), C3 60 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05w
for rep in 1 2; do
  for pr in 0 1; do
    for k in 0 7; do
      E=""; [ $pr = 1 ] && E="CATEARS_PRIO_SPLIT=1"
      env $E X=1 timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers $k > gpurun_out/r05w/p${pr}k${k}_$rep.json 2>gpurun_out/r05w/p${pr}k${k}_$rep.err || { tail -5 gpurun_out/r05w/p${pr}k${k}_$rep.err; exit 1; }
      python3 -c "import json; l=json.load(open('gpurun_out/r05w/p${pr}k${k}_$rep.json')); print('prio $pr peers $k', l['value'], l['ms_per_step'])"
    done
  done
done
