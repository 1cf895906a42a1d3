# CMVN issue priority (CATEARS_CMVN_PRIO=1: s_setprio 3 in the chain wave):
# C4 with the stage profile and C3 at the driver's flags, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05g
for i in 1 2; do
  for pr in 1 0; do
    CATEARS_CMVN_PRIO=$pr timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --stage-profile > gpurun_out/r05g/c4_p${pr}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05g/c4_p${pr}_$i.json')); st=l['stages']; print('c4 prio$pr', l['value'], 'cmvn', st['cmvn']['avg_ms'], st['cmvn']['share_of_wall'], st['cmvn']['share_of_front_busy'], 'front', st['front_stream']['share_of_wall'])"
    CATEARS_CMVN_PRIO=$pr timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05g/c3_p${pr}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05g/c3_p${pr}_$i.json')); print('c3 prio$pr', l['value'])"
  done
done
