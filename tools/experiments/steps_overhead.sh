# Fixed per-run overhead of the C3 timed region: --steps 20 / 40 / 80 and
# --steps 20 without the per-launch GEMM events, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/steps
O=gpurun_out/steps
for i in 1 2; do
  for cfg in "20" "40" "80" "20 --no-profile"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 200 python bench.py --gpus 1 --steps $cfg --warmup 5 --no-cpu-baseline > $O/s_${tag}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/s_${tag}_$i.json').read().strip().splitlines()[-1]); print('steps $cfg', d['value'], d['ms_per_step'], round(d['ms_per_step']*d['steps'],3))"
  done
done
