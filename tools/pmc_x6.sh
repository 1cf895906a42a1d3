# PMC counters of the split GEMM per variant (C3 bench, no tracing).
#   VARIANTS="7 14" [VAR=CATEARS_X6_VARIANT] [KREGEX=gemm_bf16x6] bash tools/pmc_x6.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmcv"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CNT=${CNT:-"SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"}
for v in ${VARIANTS:-7}; do
  env ${VAR:-CATEARS_X6_VARIANT}=$v timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "${KREGEX:-gemm_bf16x6}" \
      --output-format csv -d "$OUT/v$v" -o run -- \
      python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-profile --serial ${BENCH_ARGS} \
      > "$OUT/v$v.log" 2>&1 || { echo "variant $v failed"; tail -5 "$OUT/v$v.log"; exit 1; }
done
python3 - "$OUT" ${VARIANTS:-7} <<'PY'
import csv, sys, collections
for v in sys.argv[2:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{sys.argv[1]}/v{v}/run_counter_collection.csv")):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("catears::", "").split("(")[0][-70:]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f"v{v} {k} n={len(next(iter(d.values())))}")
        print("   " + "  ".join(f"{c}={sum(x)/len(x):.4g}" for c, x in sorted(d.items())))
PY
