# Effective shader clock per GEMM dispatch (GRBM_GUI_ACTIVE / 8 XCDs / duration),
# serial bench:  VARIANTS="55 58" bash tools/pmc_clock.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/pclk && export TMPDIR=/tmp
for v in ${VARIANTS:-42}; do
  rm -rf gpurun_out/pclk/v$v
  CATEARS_X6_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "${KREGEX:-gemm_bf16x6}" \
      --output-format csv -d gpurun_out/pclk/v$v -o run -- \
      python3 bench.py --steps ${STEPS:-80} --warmup 1 --serial --no-cpu-baseline --no-profile ${BENCH_ARGS} > gpurun_out/pclk/v$v.log 2>&1 || { echo "v$v failed"; tail -5 gpurun_out/pclk/v$v.log; exit 1; }
  python3 - gpurun_out/pclk/v$v $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    k = int(r["Dispatch_Id"])
    d[k][r["Counter_Name"]] = float(r["Counter_Value"])
    d[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    d[k]["grid"] = int(r["Grid_Size"])
ks = sorted(d)[len(d) // 2:]
by = collections.defaultdict(list)
for k in ks:
    by[d[k]["grid"]].append(d[k])
for g, v in sorted(by.items()):
    clk = sorted(x["GRBM_GUI_ACTIVE"] / 8 / x["dur"] / 1e3 for x in v)
    dur = sorted(x["dur"] for x in v)
    print(f"v{sys.argv[2]} grid {g:7d} n {len(v):3d} dur {dur[len(dur)//2]:7.1f} us clk {clk[len(clk)//2]:.3f}")
PY
done
