# C5 (int8) and C4 (100 h, ragged batches, the round-6 bf16x6 default) over
# the nnet stream count; product library.  Usage: bash tools/experiments/gpu_r6i.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06i}
cd "$R" && mkdir -p gpurun_out/$T
for rep in 1 2; do
  for s in 3 4 6 8; do
    timeout -k 10 200 python bench.py --workload c5 --steps 40 --warmup 3 --no-cpu-baseline --back-streams $s \
        > gpurun_out/$T/c5_s${s}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c5_s${s}_$rep.json')); print('c5 streams $s', l['value'], l['ms_per_step'])"
  done
done
for s in 3 8; do
  timeout -k 10 400 python bench.py --workload c4 --no-cpu-baseline --back-streams $s > gpurun_out/$T/c4_s$s.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/$T/c4_s$s.json')); print('c4 streams $s', l['value'], l['ms_per_step'])"
done
