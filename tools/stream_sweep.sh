# Bench 1 vs 2 vs 3 nnet streams back to back.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/streams"
cd "$R" || exit 1
for nb in ${NBLIST:-1 2 3}; do
  timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --back-streams $nb \
      > "gpurun_out/streams/nb$nb.log" 2>&1 || { echo "nb $nb failed"; tail -5 "gpurun_out/streams/nb$nb.log"; exit 1; }
  python - "$nb" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/streams/nb{sys.argv[1]}.log") if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["end_to_end_mfma_frac"])
PY
done
