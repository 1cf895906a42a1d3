# The int8 Quantize's corrected reciprocal product (CATEARS_I8_QDIV=1, a
# scratch/ build): hardware probe of the quotient against IEEE division,
# the int8 parity tests with that library, then C5 against the product
# library, ABBA per round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z21
timeout -k 10 120 ./tools/probes/qdp | tee gpurun_out/r05z21/probe.txt || exit 1
CATEARS_HIP_LIB=$R/scratch/libcatears_hip_qd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z21/int8.log 2>&1 || { tail -30 gpurun_out/r05z21/int8.log; exit 1; }
tail -1 gpurun_out/r05z21/int8.log
for rep in 1 2 3; do
  i=0
  for v in prod qd qd prod; do
    i=$((i+1))
    if [ $v = qd ]; then L=$R/scratch/libcatears_hip_qd.so; else L=$R/catears_amd/lib/libcatears_hip.so; fi
    CATEARS_HIP_LIB=$L timeout -k 10 200 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/r05z21/${v}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z21/${v}_${rep}_$i.json')); print('$v', l['value'], l['ms_per_step'], l['checksum'])"
  done
done
