# The driver's command (bench.py --steps 20 --warmup 5), ten times on one box,
# no profiler: the run-to-run spread the driver's single line falls in.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05y2
for i in $(seq 10); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05y2/d_$i.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05y2/d_$i.json')); print('driver', l['value'], l['roofline']['frac'])"
done
