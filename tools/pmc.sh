# PMC counter passes (one counter group per rocprofv3 run; never with tracing).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-pmc}
mkdir -p "$R/gpurun_out/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-gemm_f32|fbank|cmvn|finalize}" \
      --output-format csv -d "$R/gpurun_out/$OUT/p$i" -o run -- \
      python "$R/bench.py" --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-profile --serial \
      > "$R/gpurun_out/$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$R/gpurun_out/$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done
