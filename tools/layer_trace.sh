# Kernel trace of the bench for a given GEMM variant; prints per-dispatch-shape times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-13}; do
  CATEARS_GEMM_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/lt$v" -o run -- \
     python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-profile --serial > "$R/gpurun_out/lt$v.log" 2>&1 || exit 1
  python3 - "$R/gpurun_out/lt$v/run_kernel_trace.csv" "$v" <<'PY'
import csv, sys
from collections import defaultdict
d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'catears' not in r['Kernel_Name']: continue
    name = r['Kernel_Name'].split('(')[0].split('::')[-1][:40]
    d[(name, int(r['Grid_Size_X']))].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print("variant", sys.argv[2])
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = sorted(v)
    print(f"  {k[0]:40s} grid {k[1]:8d} n {len(v):3d} med {v[len(v)//2]:8.1f} us min {v[0]:8.1f}")
PY
done
