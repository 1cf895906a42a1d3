# Several PMC passes (one rocprofv3 run each) over the bf16x6 GEMM variants,
# serial C3 bench: VARIANTS="42 60" bash tools/pmc_x6_groups.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmcg"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
IFS=';' read -ra PG <<< "${PGROUPS:-$G1;$G2}"
for v in ${VARIANTS:-42}; do
  i=0
  for grp in "${PG[@]}"; do
    i=$((i+1))
    env ${VAR:-CATEARS_X6_VARIANT}=$v timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-gemm_bf16x6}" \
        --output-format csv -d "$OUT/v$v/p$i" -o run -- \
        python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --serial ${BENCH_ARGS} \
        > "$OUT/v$v.p$i.log" 2>&1 || { echo "variant $v pass $i failed"; tail -5 "$OUT/v$v.p$i.log"; exit 1; }
  done
done
python3 - "$OUT" ${VARIANTS:-42} <<'PY'
import csv, glob, sys, collections
for v in sys.argv[2:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{sys.argv[1]}/v{v}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("catears::", "").split("(")[0][-60:]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f"v{v} {k}")
        print("   " + "  ".join(f"{c}={sum(x)/len(x):.4g}" for c, x in sorted(d.items())))
PY
