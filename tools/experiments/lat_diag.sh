# Timing breakdown of the latency GEMM (70-row TDNN-S call) with the
# measurement library's diagnostic schedules (wrong results by design):
# 1 no weight loads, 2 no activation loads, 4 no MFMAs, 8 no stores.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/latdiag && export TMPDIR=/tmp
for d in 0 1 2 3 4; do
  rm -rf gpurun_out/latdiag/run
  CATEARS_HIP_LIB=catears_amd/lib/libcatears_hip_exp.so CATEARS_LAT_DIAG=$d LAT_MODES=latency LAT_ROWS=70 \
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/latdiag/run -o run -- \
    python3 tools/latency.py 50 > gpurun_out/latdiag/trace_$d.log 2>&1 || { tail -5 gpurun_out/latdiag/trace_$d.log; exit 1; }
  cp $(find gpurun_out/latdiag/run -name '*kernel_trace.csv' | head -1) gpurun_out/latdiag/kt_$d.csv
  echo "DIAG=$d  $(grep 'rows    70' gpurun_out/latdiag/trace_$d.log)"
  python3 tools/dispatch_seq.py gpurun_out/latdiag/kt_$d.csv "lat_gemm" 7
done
