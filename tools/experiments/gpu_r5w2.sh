# Rank-0 rehearsal (7 peers) with the receive / fold stream at the lowest
# priority (CATEARS_COMM_LOW=1), pipeline at the default; C3 60 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05w
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for rep in 1 2; do
  for lo in 0 1; do
    for k in 0 7; do
      E="X=1"; [ $lo = 1 ] && E="CATEARS_COMM_LOW=1"
      env $E timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --rehearse-peers $k > gpurun_out/r05w/l${lo}k${k}_$rep.json 2>gpurun_out/r05w/l${lo}k${k}_$rep.err || { tail -5 gpurun_out/r05w/l${lo}k${k}_$rep.err; exit 1; }
      python3 -c "import json; l=json.load(open('gpurun_out/r05w/l${lo}k${k}_$rep.json')); print('low $lo peers $k', l['value'], l['ms_per_step'])"
    done
  done
done
