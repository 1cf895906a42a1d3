# Per-layer durations of the fp32-operand bf16x6 GEMM variants, serial C3
# (one stream, so each launch runs alone): VARIANTS="42 43 40" bash tools/x6_layers.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/x6layers && export TMPDIR=/tmp
for v in ${VARIANTS:-42}; do
  rm -rf gpurun_out/x6layers/v$v
  CATEARS_X6_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/x6layers/v$v -o run -- \
    python3 bench.py --serial --steps 20 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/x6layers/v$v.log 2>&1 || { echo "v$v failed"; tail -5 gpurun_out/x6layers/v$v.log; exit 1; }
  python3 - gpurun_out/x6layers/v$v $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
seq = [r for r in csv.DictReader(open(f)) if "gemm_bf16x6" in r["Kernel_Name"]]
d = collections.defaultdict(list)
for i, r in enumerate(seq):
    d[i % 7].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("v" + sys.argv[2], " ".join(f"L{k + 1}:{sorted(v)[len(v) // 2]:.1f}" for k, v in sorted(d.items())),
      f"sum {sum(sorted(v)[len(v) // 2] for v in d.values()):.1f} us")
PY
done
