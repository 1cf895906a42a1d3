# C5 Quantize pass: wave-state counters of quantize_kernel (tools/pmc_kernel.sh)
# and the serial per-kernel durations of a C5 step (kernel trace, one stream).
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06k}
cd "$R" && mkdir -p gpurun_out/$T
PGROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE" \
  KREGEX=quantize_kernel WORKLOAD=c5 OUT=$T/pmc_q bash tools/pmc_kernel.sh > gpurun_out/$T/pmc_q.txt 2>&1 || { tail -20 gpurun_out/$T/pmc_q.txt; exit 1; }
tail -14 gpurun_out/$T/pmc_q.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/$T/serial" -o run -- \
    python "$R/bench.py" --workload c5 --serial --steps 20 --warmup 3 --no-cpu-baseline --no-profile \
    > "$R/gpurun_out/$T/serial.log" 2>&1 || { tail -5 "$R/gpurun_out/$T/serial.log"; exit 1; }
python3 "$R/tools/trace_summary.py" "$R/gpurun_out/$T/serial/run_kernel_trace.csv" "C5 serial" | head -16
# the fast quantize kernel (CATEARS_I8_QFAST 1 / 2 rows per wave) against
# quantize_kernel (0), C5 ABBA, checksums compared; experiments library
cd "$R"
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2; do
  for f in 0 1 2 2 1 0; do
    CATEARS_I8_QFAST=$f timeout -k 10 200 python bench.py --workload c5 --steps 40 --warmup 3 --no-cpu-baseline \
        > gpurun_out/$T/c5_q${f}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c5_q${f}_$rep.json')); print('c5 qfast $f', l['value'], l['ms_per_step'], l['checksum'], l['stages']['quantize']['avg_ms'] if 'quantize' in l.get('stages', {}) else '')"
  done
done
