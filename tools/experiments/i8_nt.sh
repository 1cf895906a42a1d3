# int8 epilogue with non-temporal 16-byte stores (libcatears_hip_nt.so, built
# from the -DCE_I8_NT variant of round 4, now the default)
# -DCE_I8_NT) against the default: serial hidden-layer time, C5 bits.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/i8nt
O=gpurun_out/i8nt
cd /tmp && export TMPDIR=/tmp && cd "$R"
for i in 1 2; do for L in def nt; do
  if [ $L = nt ]; then export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_nt.so; else unset CATEARS_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${L}_$i -o s -- \
    python bench.py --workload c5 --serial --steps 10 --warmup 2 --no-cpu-baseline > $O/${L}_$i.json 2>/dev/null || exit 1
  python - $O/${L}_$i/s_kernel_trace.csv $L $O/${L}_$i.json <<'PY'
import csv, sys, statistics, json
rows=list(csv.DictReader(open(sys.argv[1])))
d=sorted((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows
   if 'gemm_i8' in r['Kernel_Name'] and int(r['Grid_Size_X'])//int(r['Workgroup_Size_X'])==256)
q=sorted((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if 'quantize' in r['Kernel_Name'])
h=d[len(d)//5:]
b=json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[2], 'hidden median', round(statistics.median(h),2), 'quantize median', round(statistics.median(q),2), 'checksum', b['checksum'])
PY
done; done
