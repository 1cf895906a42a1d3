# One GPU session: parity tests, the bench line under rocprofv3 kernel-trace
# stats (same command -> JSON + per-kernel durations), then the two PMC
# passes that give roofline.traffic.  Usage: TAG=r01x bash tools/round_gpu.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-run}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
timeout -k 10 1200 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$SKIP_BENCH" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python "$R/bench.py" --steps ${STEPS:-50} --warmup 5 ${BENCH_ARGS} > "$OUT/bench.log" 2>&1; rc=$?
echo "bench(rocprof) rc=$rc"; tail -2 "$OUT/bench.log"
[ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_PMC" ] && exit 0
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "gemm_|fbank|cmvn|finalize|splice" \
      --output-format csv -d "$OUT/pmc$i" -o run -- \
      python "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-profile --serial \
      > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc$i.log"; exit 1; }
  echo "pmc pass $i ok: $grp"
done
python "$R/tools/pmc_traffic.py" "$OUT/pmc1" "$OUT/pmc2" "$OUT/pmc_traffic.json" --layers 7
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "gemm_" \
    --output-format csv -d "$OUT/pmc3" -o run -- \
    python "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-profile --serial \
    > "$OUT/pmc3.log" 2>&1 || { echo "pmc pass 3 failed"; tail -20 "$OUT/pmc3.log"; exit 1; }
python "$R/tools/pmc_mfma.py" "$OUT/pmc3" "$OUT/pmc_mfma.json"
[ -n "$SKIP_EXTRA" ] && exit 0
# secondary workloads: C2 (batched fbank) and C5 (int8 nnet), same recipe
for W in c2 c5; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$W" -o run -- \
      python "$R/bench.py" --workload $W --steps ${STEPS_EXTRA:-30} --warmup 3 > "$OUT/bench_$W.log" 2>&1 || { echo "bench $W failed"; tail -20 "$OUT/bench_$W.log"; exit 1; }
  echo "bench $W ok"; grep '^{' "$OUT/bench_$W.log" | cut -c1-300
  case $W in c2) KRE="fbank";; c5) KRE="gemm_i8|quantize|minmax";; esac
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv -d "$OUT/pmc_${W}_$i" -o run -- \
        python "$R/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-profile --serial \
        > "$OUT/pmc_${W}_$i.log" 2>&1 || { echo "pmc $W $i failed"; tail -20 "$OUT/pmc_${W}_$i.log"; exit 1; }
  done
  python "$R/tools/pmc_traffic.py" "$OUT/pmc_${W}_1" "$OUT/pmc_${W}_2" "$OUT/pmc_traffic_$W.json"
  if [ $W = c2 ]; then
    # measured VALU occupancy of the fbank kernel (tools/pmc_valu.py): one pass, 7 SQ + 1 GRBM counters
    timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
        SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "fbank" \
        --output-format csv -d "$OUT/pmc_${W}_3" -o run -- \
        python "$R/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-profile --serial \
        > "$OUT/pmc_${W}_3.log" 2>&1 || { echo "pmc $W 3 failed"; tail -20 "$OUT/pmc_${W}_3.log"; exit 1; }
    timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
        SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "fbank" \
        --output-format csv -d "$OUT/pmc_${W}_4" -o run -- \
        python "$R/bench.py" --workload $W --fbank fast --steps 3 --warmup 1 --no-cpu-baseline --no-profile --serial \
        > "$OUT/pmc_${W}_4.log" 2>&1 || { echo "pmc $W 4 failed"; tail -20 "$OUT/pmc_${W}_4.log"; exit 1; }
    python "$R/tools/pmc_valu.py" "$OUT/pmc_valu_$W.json" "$OUT/pmc_${W}_3" "$OUT/pmc_${W}_4"
  fi
  if [ $W = c5 ]; then
    timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "gemm_" \
        --output-format csv -d "$OUT/pmc_${W}_3" -o run -- \
        python "$R/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-profile --serial \
        > "$OUT/pmc_${W}_3.log" 2>&1 || { echo "pmc $W 3 failed"; tail -20 "$OUT/pmc_${W}_3.log"; exit 1; }
    python "$R/tools/pmc_mfma.py" "$OUT/pmc_${W}_3" "$OUT/pmc_mfma_$W.json"
  fi
done
