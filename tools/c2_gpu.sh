# C2 (batched fbank) measurement: bench line under rocprofv3 stats, then the
# FETCH_SIZE / WRITE_SIZE passes for its traffic.  TAG=r01c2 bash tools/c2_gpu.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-c2}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python "$R/bench.py" --workload c2 --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS} > "$OUT/bench.log" 2>&1; rc=$?
echo "c2 bench rc=$rc"; grep '^{' "$OUT/bench.log" | cut -c1-600
[ $rc -eq 0 ] || { tail -20 "$OUT/bench.log"; exit $rc; }
[ -n "$SKIP_PMC" ] && exit 0
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "fbank" --output-format csv -d "$OUT/pmc$i" -o run -- \
      python "$R/bench.py" --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-profile \
      > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$OUT/pmc$i.log"; exit 1; }
done
python "$R/tools/pmc_traffic.py" "$OUT/pmc1" "$OUT/pmc2" "$OUT/pmc_traffic.json"
