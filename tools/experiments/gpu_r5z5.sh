# The bf16x6 DIAG ablations of gpu_r5c.sh, but in the pipelined C3 bench
# (three nnet streams, the chip full): does any removed part give back more
# under the full-load clock than in the serial runs?  Experiments library,
# wrong results, timing only.  Needs catears_amd/lib/libcatears_hip_exp.so
# pushed (drop it from .gpurunignore).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z5
for rep in 1 2; do
  for v in ${VARIANTS:-300 310 312 313 314 316}; do
    CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so CATEARS_X6_VARIANT=$v timeout -k 10 200 \
      python bench.py --no-cpu-baseline > gpurun_out/r05z5/v${v}_$rep.json 2> gpurun_out/r05z5/v${v}_$rep.err || { tail -5 gpurun_out/r05z5/v${v}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/r05z5/v${v}_$rep.json')); print('v$v', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
