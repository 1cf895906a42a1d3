# bf16x6 variants against the default 300 over the nnet stream count (3, 4,
# 6, 8; hardware queues = streams + 1): C3 at 200 steps, experiments library.
# Usage: VARS="507 508" bash tools/experiments/gpu_r6d.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06d}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for ns in ${STREAMS:-3 4 6 8}; do
  for v in 300 ${VARS:-507 508}; do
    CATEARS_HW_QUEUES=$(( ns + 1 > 4 ? ns + 1 : 4 )) CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --back-streams $ns > gpurun_out/$T/c3_v${v}_s$ns.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_v${v}_s$ns.json')); print('200 steps v$v streams $ns', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
# C5: the staggered int8 GEMM (CATEARS_I8_GEMM=17) against the default 16,
# ABBA, checksums compared (exact int32: the same bits)
for rep in 1 2; do
  i=0
  for g in 16 17 17 16; do
    i=$((i+1))
    CATEARS_I8_GEMM=$g timeout -k 10 200 python bench.py --workload c5 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/$T/c5_g${g}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c5_g${g}_${rep}_$i.json')); print('c5 gemm $g', l['value'], l['ms_per_step'], l['roofline']['frac'], l['checksum'])"
  done
done
