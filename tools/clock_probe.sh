# Sample the GPU clock / power while a long bench runs (is the GEMM power-bound?)
#   ARGS="--steps 20000" MODES="pipe serial" bash tools/clock_probe.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/clk
for mode in ${MODES:-pipe serial}; do
  extra=""; [ "$mode" = serial ] && extra="--serial"
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --warmup 20 ${ARGS:---steps 20000} $extra \
      > gpurun_out/clk/$mode.log 2>&1 &
  pid=$!
  : > gpurun_out/clk/$mode.smi.txt
  while kill -0 $pid 2>/dev/null; do
    rocm-smi --showclocks --showpower >> gpurun_out/clk/$mode.smi.txt 2>&1
    sleep 0.3
  done
  wait $pid || { echo "$mode bench failed"; tail -5 gpurun_out/clk/$mode.log; exit 1; }
  echo "== $mode: $(grep '^{' gpurun_out/clk/$mode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  grep -h -i "sclk\|power (W)" gpurun_out/clk/$mode.smi.txt | sort | uniq -c | sort -rn | head -12
done
