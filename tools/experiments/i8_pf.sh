# (variants 17 / 18 were a measurement build of round 4, not kept)
# int8 pipe kernel with L2 line touches PF tiles ahead (CATEARS_I8_GEMM 17:
# PF 2, 18: PF 3) against 16: serial hidden-layer time, C5 at 20 steps, bits.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/i8pf
O=gpurun_out/i8pf
cd /tmp && export TMPDIR=/tmp && cd "$R"
for v in 16 17 18; do
  CATEARS_I8_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/v$v -o s -- \
    python bench.py --workload c5 --serial --steps 10 --warmup 2 --no-cpu-baseline > $O/v$v.json 2>/dev/null || exit 1
  python - $O/v$v/s_kernel_trace.csv $v $O/v$v.json <<'PY'
import csv, sys, statistics, json
rows=list(csv.DictReader(open(sys.argv[1])))
d=sorted((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows
   if 'gemm_i8' in r['Kernel_Name'] and int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])==256)
l=sorted((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows
   if 'gemm_i8' in r['Kernel_Name'] and int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])==864)
b=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print('variant', sys.argv[2], 'hidden median', round(statistics.median(d[len(d)//5:]),2), 'last', round(statistics.median(l),2), 'checksum', b['checksum'])
PY
done
for i in 1 2; do for v in 16 17 18; do
  CATEARS_I8_GEMM=$v timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_${v}_$i.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/c5_${v}_$i.json').read().strip().splitlines()[-1]); print('c5 v$v', d['value'], d['checksum'])"
done; done
