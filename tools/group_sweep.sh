# Bench the GEMM tile-group width (CATEARS_GEMM_GROUP) back to back.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/group"
cd "$R" || exit 1
for g in ${GLIST:-1 2 4 8}; do
  CATEARS_GEMM_GROUP=$g timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline \
      > "gpurun_out/group/g$g.log" 2>&1 || { echo "group $g failed"; tail -5 "gpurun_out/group/g$g.log"; exit 1; }
  python - "$g" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/group/g{sys.argv[1]}.log") if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["stages"]["gemm_gather"]["avg_ms"])
PY
done
