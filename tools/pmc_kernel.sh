# PMC counter groups for one kernel of one bench workload (no tracing).
# KREGEX=fbank WORKLOAD=c2 OUT=pmcf [BENCH_ARGS="--fbank fast"] bash tools/pmc_kernel.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${OUT:-pmck}
mkdir -p "$R/gpurun_out/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
# PGROUPS (';'-separated counter groups) replaces the default groups.
DEFAULT_GROUPS="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES;SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY"
IFS=';' read -ra PG <<< "${PGROUPS:-$DEFAULT_GROUPS}"
for grp in "${PG[@]}" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-fbank}" --output-format csv \
      -d "$R/gpurun_out/$OUT/p$i" -o run -- \
      python "$R/bench.py" --workload ${WORKLOAD:-c2} --steps 3 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} \
      > "$R/gpurun_out/$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$R/gpurun_out/$OUT/p$i.log"; exit 1; }
done
python3 - "$R/gpurun_out/$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:28s} {sum(x) / len(x):16.0f}")
PY
