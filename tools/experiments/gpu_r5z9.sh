# The GPU clock and power while the pipelined C3 bench runs (15000 steps,
# about 9 s): amd-smi samples every 0.2 s beside it, then the same during
# an idle second.  Reading the SMI changes no setting.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z9
timeout -k 10 60 amd-smi metric -g 0 > gpurun_out/r05z9/idle.txt 2>&1 || timeout -k 10 60 rocm-smi --showclocks --showpower > gpurun_out/r05z9/idle.txt 2>&1
timeout -k 10 200 python bench.py --steps 15000 --warmup 20 --no-cpu-baseline > gpurun_out/r05z9/bench.json 2> gpurun_out/r05z9/bench.err &
BP=$!
sleep 4
for i in $(seq 1 40); do
  kill -0 $BP 2>/dev/null || break
  echo "--- sample $i $(date +%s.%N)" >> gpurun_out/r05z9/load.txt
  timeout -k 5 20 amd-smi metric -g 0 --clock --power --usage >> gpurun_out/r05z9/load.txt 2>&1
  sleep 0.2
done
wait $BP; echo "bench rc=$?"
cut -c1-160 gpurun_out/r05z9/bench.json
grep -i -A3 "GFX_0\|SOCKET_POWER\|GFX_ACTIVITY\|CUR_FREQ\|clk:" gpurun_out/r05z9/load.txt | head -60
