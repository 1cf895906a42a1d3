# bf16x6 direct-weight loop with s_setprio variants (331-335) against the
# default 300, in ABBA order per round (VARIANTS overrides the order);
# experiments library, C3 at 200 steps.  Needs libcatears_hip_exp.so pushed.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z8
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2 3; do
  i=0
  for v in ${VARIANTS:-300 331 331 300}; do
    i=$((i+1))
    CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z8/v${v}_${rep}_$i.json 2>gpurun_out/r05z8/v${v}_$rep.err || { tail -5 gpurun_out/r05z8/v${v}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05z8/v${v}_${rep}_$i.json')); print('v$v', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
