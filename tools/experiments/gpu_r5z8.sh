# bf16x6 direct-weight loop with s_setprio around its load issues (the
# default since r05z8; 330 = without it) or its MFMA regions (332);
# experiments library, C3 alternating (200 steps).  Needs libcatears_hip_exp.so pushed.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z8
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2 3; do
  for v in ${VARIANTS:-330 0 332}; do
    CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z8/v${v}_$rep.json 2>gpurun_out/r05z8/v${v}_$rep.err || { tail -5 gpurun_out/r05z8/v${v}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05z8/v${v}_$rep.json')); print('v$v', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
