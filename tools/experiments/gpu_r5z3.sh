# A sender's local cost at N > 1 rehearsed (bench.py --rehearse-send: each
# batch read once more after it is scored); C3 60 steps, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z3
for rep in 1 2 3; do
  for m in base send; do
    A=""; [ $m = send ] && A="--rehearse-send"
    timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline $A > gpurun_out/r05z3/${m}_$rep.json 2>gpurun_out/r05z3/${m}_$rep.err || { tail -5 gpurun_out/r05z3/${m}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05z3/${m}_$rep.json')); print('$m', l['value'], l['ms_per_step'])"
  done
done
