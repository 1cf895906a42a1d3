# int8 GEMM XCD tile-group width (CATEARS_I8_GROUP): serial hidden-layer
# time under rocprofv3 and C5 at 20 steps.
# (CATEARS_I8_GROUP was a measurement build's knob; the product library fixes the group at 8.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/i8g
O=gpurun_out/i8g
cd /tmp && export TMPDIR=/tmp && cd "$R"
for g in 8 1 2 4 16; do
  CATEARS_I8_GROUP=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/g$g -o s -- \
    python bench.py --workload c5 --serial --steps 10 --warmup 2 --no-cpu-baseline > $O/g$g.json 2>/dev/null || exit 1
  python - $O/g$g/s_kernel_trace.csv $g <<'PY'
import csv, sys, statistics
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in csv.DictReader(open(sys.argv[1]))
   if 'gemm_i8' in r['Kernel_Name'] and int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])==256]
d.sort(); h=d[len(d)//5:]  # hidden layers (drop the short first layer)
print('group', sys.argv[2], 'hidden-layer median us', round(statistics.median(h),2), 'n', len(h))
PY
done
for i in 1 2; do for g in 8 2; do
  CATEARS_I8_GROUP=$g timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_g${g}_$i.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/c5_g${g}_$i.json').read().strip().splitlines()[-1]); print('c5 group $g', d['value'], d['checksum'])"
done; done
