# int8 GEMM (variant 15) timing breakdown, measurement library, serial C5:
# 61 no DMA after the prologue, 62 no MFMAs, 64 no fragment reads,
# 65 neither DMA nor reads (MFMA only), 63 neither DMA nor MFMAs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/i8diag && export TMPDIR=/tmp
export CATEARS_HIP_LIB=catears_amd/lib/libcatears_hip_exp.so
for v in ${VARIANTS:-15 61 62 64 65 63}; do
  rm -rf gpurun_out/i8diag/run$v
  CATEARS_I8_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/i8diag/run$v -o run -- \
      python3 bench.py --workload c5 --serial --steps 6 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/i8diag/serial$v.log 2>&1 || { tail -5 gpurun_out/i8diag/serial$v.log; exit 1; }
  python3 tools/trace_summary.py $(find gpurun_out/i8diag/run$v -name '*kernel_trace.csv' | head -1) "C5 serial v$v" > gpurun_out/i8diag/summary$v.txt
  echo "v$v $(grep 'gemm_i8' gpurun_out/i8diag/summary$v.txt | head -2 | awk '{print $(NF-5), $(NF-2)}' | tr '\n' ' ')"
done
