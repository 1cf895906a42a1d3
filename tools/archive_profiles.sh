# Copies one tools/round_gpu.sh session (gpurun_out/$TAG) into profiles/ under
# the tag's name: bench JSON lines, rocprofv3 kernel stats, per-kernel
# summaries (tools/trace_summary.py --window: the timed steps only, checked
# against the bench line's roofline) and the PMC traffic files that bench.py
# reads for roofline.traffic.  Usage: bash tools/archive_profiles.sh r01g
set -e
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
S="$R/gpurun_out/$TAG"
P="$R/profiles"
[ -d "$S" ] || { echo "no $S"; exit 1; }
for W in "" _c2 _c5; do
  log="$S/bench${W}.log"; prof="$S/prof${W}"
  [ -f "$log" ] || continue
  grep '^{' "$log" | tail -1 > "$P/${TAG}${W}_bench.json"
  cp "$prof/run_kernel_stats.csv" "$P/${TAG}${W}_kernel_stats.csv"
  python "$R/tools/trace_summary.py" "$prof/run_kernel_trace.csv" --window --check "$log" \
    "rocprofv3 --kernel-trace --stats -- python bench.py ${W:+--workload ${W#_}}  (tools/round_gpu.sh, TAG=$TAG)
bench JSON line of the same command: profiles/${TAG}${W}_bench.json
" > "$P/${TAG}${W}_kernel_summary.txt"
  [ -f "$S/pmc_traffic${W}.json" ] && cp "$S/pmc_traffic${W}.json" "$P/${TAG}${W}_pmc_traffic.json"
  [ -f "$S/pmc_mfma${W}.json" ] && cp "$S/pmc_mfma${W}.json" "$P/${TAG}${W}_pmc_mfma.json"
  [ -f "$S/pmc_valu${W}.json" ] && cp "$S/pmc_valu${W}.json" "$P/${TAG}${W}_pmc_valu.json"
done
ls -la "$P" | grep "$TAG"
