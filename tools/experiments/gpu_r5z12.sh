# 128 x 128 tiles for the batches scored while the pipeline fills / drains
# (bench.py --wide-tiles last / ends) against none, at the driver's flags
# (--steps 20 --warmup 5), rotating order per round; then 200 steps once
# each.  First the variants test (wide tiles bit-identical).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z12
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6_variants.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z12/variants.log 2>&1 || { tail -30 gpurun_out/r05z12/variants.log; exit 1; }
tail -1 gpurun_out/r05z12/variants.log
for rep in 1 2 3 4; do
  case $rep in 1) ORD="none last ends";; 2) ORD="ends none last";; 3) ORD="last ends none";; 4) ORD="none ends last";; esac
  for w in $ORD; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --wide-tiles $w > gpurun_out/r05z12/drv_${w}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z12/drv_${w}_$rep.json')); print('driver $w', l['value'], l['ms_per_step'])"
  done
done
for w in none last; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --wide-tiles $w > gpurun_out/r05z12/def_$w.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05z12/def_$w.json')); print('200 steps $w', l['value'], l['ms_per_step'])"
done
