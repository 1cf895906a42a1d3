# (CATEARS_X6_NT was a measurement build's switch, not kept.)
# Non-temporal stores for the last bf16x6 layer's logits (CATEARS_X6_NT,
# default 1) against normal stores: C3 at the driver config alternating, and
# serial last-layer + finalize times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/x6nt
O=gpurun_out/x6nt
for i in 1 2 3; do for nt in 1 0; do
  CATEARS_X6_NT=$nt timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_${nt}_$i.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/c3_${nt}_$i.json').read().strip().splitlines()[-1]); print('c3 nt=$nt', d['value'], d['checksum'])"
done; done
cd /tmp && export TMPDIR=/tmp && cd "$R"
for nt in 1 0; do
  CATEARS_X6_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/s$nt -o s -- \
    python bench.py --serial --steps 20 --warmup 3 --no-cpu-baseline > $O/s$nt.json 2>/dev/null || exit 1
  python - $O/s$nt/s_kernel_trace.csv $nt <<'PY'
import csv, sys, statistics
rows=list(csv.DictReader(open(sys.argv[1])))
def med(f): 
    d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if f(r)]
    return round(statistics.median(d),2) if d else None
last=med(lambda r: 'gemm_bf16x6d' in r['Kernel_Name'] and int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])==448)
fin=med(lambda r: 'finalize' in r['Kernel_Name'])
print('nt', sys.argv[2], 'last layer', last, 'finalize', fin)
PY
done
