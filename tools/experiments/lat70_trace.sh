# Latency mode: the per-call table with the weight source A/B (fp32 split in
# registers vs the fragment image: same output digests), then one 70-row
# call's kernel sequence.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/lat70 && export TMPDIR=/tmp
rm -rf gpurun_out/lat70/run
LAT_MODES=latency timeout -k 10 120 python3 tools/latency.py 200 2>&1 | grep -v amdgpu.ids || exit 1


LAT_MODES=latency LAT_ROWS=70 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lat70/run -o run -- \
    python3 tools/latency.py 50 > gpurun_out/lat70/trace.log 2>&1 || { tail -5 gpurun_out/lat70/trace.log; exit 1; }
cp $(find gpurun_out/lat70/run -name '*kernel_trace.csv' | head -1) gpurun_out/lat70/kernel_trace.csv
python3 tools/dispatch_seq.py gpurun_out/lat70/kernel_trace.csv "" 14
for rtb in 1 2 8; do
  echo "CATEARS_LAT_RTB=$rtb"
  CATEARS_LAT_RTB=$rtb LAT_MODES=latency LAT_ROWS=270,1018,4072 timeout -k 10 120 python3 tools/latency.py 100 2>&1 | grep "rows" || exit 1
done
