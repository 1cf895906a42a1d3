#!/bin/bash
# bf16x6 GEMM: static s_setprio 1 for the younger (1) or older (2) half of the
# waves (CATEARS_X6_PRIO) -- serial per-layer durations, then C3 at the driver's flags.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/x6prio && export TMPDIR=/tmp
for rep in 1 2; do
for v in 0 1 2; do
  rm -rf gpurun_out/x6prio/p$v
  CATEARS_X6_PRIO=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/x6prio/p$v -o run -- \
    python3 bench.py --serial --steps 20 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/x6prio/p$v.log 2>&1 || { echo "p$v failed"; tail -5 gpurun_out/x6prio/p$v.log; exit 1; }
  python3 - gpurun_out/x6prio/p$v $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
seq = [r for r in csv.DictReader(open(f)) if "gemm_bf16x6" in r["Kernel_Name"]]
d = collections.defaultdict(list)
for i, r in enumerate(seq):
    d[i % 7].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("prio" + sys.argv[2], " ".join(f"L{k + 1}:{sorted(v)[len(v) // 2]:.1f}" for k, v in sorted(d.items())),
      f"sum {sum(sorted(v)[len(v) // 2] for v in d.values()):.1f} us")
PY
done; done
for rep in 1 2; do
for v in 0 1 2; do
  CATEARS_X6_PRIO=$v timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/x6prio/c3_$v.out 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/x6prio/c3_$v.out').read().strip().splitlines()[-1]);print('c3 prio=$v',d['value'],d['ms_per_step'])"
done; done
