# bf16x6 epilogue with non-temporal fp32 output stores (a build with
# X6FLAGS=-DCATEARS_X6_NT=1 in scratch/) against the product library, C3 at
# 200 steps, ABBA per round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z17
for rep in 1 2 3; do
  i=0
  for v in prod nt nt prod; do
    i=$((i+1))
    if [ $v = nt ]; then L=$R/scratch/libcatears_hip_nt.so; else L=$R/catears_amd/lib/libcatears_hip.so; fi
    CATEARS_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z17/${v}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z17/${v}_${rep}_$i.json')); print('$v', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
