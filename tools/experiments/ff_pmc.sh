# (Historical: measures the four-step fast fbank kernel, kernels/fbank_fast.hip, removed
# in round 5 when the fast mode became the contracted exact lane program; kept as the
# record of DESIGN.md §8b.  It no longer builds against the current tree.)
# fast fbank instruction mix and stalls (two PMC passes over C2 fast, 3 steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/ffpmc && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  rm -rf gpurun_out/ffpmc/p$i
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "fbank" --output-format csv -d gpurun_out/ffpmc/p$i -o run -- \
      python3 bench.py --workload c2 --fbank fast --steps 3 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/ffpmc/p$i.log 2>&1 \
      || { echo "pass $i failed"; tail -5 gpurun_out/ffpmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/ffpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fbank" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:24s} {sum(v)/len(v):16.0f}  (n={len(v)})")
PY
