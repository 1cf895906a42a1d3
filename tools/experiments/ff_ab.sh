# (Historical: measures the four-step fast fbank kernel, kernels/fbank_fast.hip, removed
# in round 5 when the fast mode became the contracted exact lane program; kept as the
# record of DESIGN.md §8b.  It no longer builds against the current tree.)
# fast fbank: tests, C2 fast line x3, bank-conflict PMC pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/ff && export TMPDIR=/tmp
bash tools/experiments/ff_c2.sh || exit 1
rm -rf gpurun_out/ff/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-include-regex "fbank" --output-format csv -d gpurun_out/ff/pmc -o run -- \
    python3 bench.py --workload c2 --fbank fast --steps 3 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/ff/pmc.log 2>&1 || { tail -5 gpurun_out/ff/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/ff/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fbank" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:24s} {sum(v)/len(v):16.0f}")
PY
