# C3: the gathered first layer on 256 x 128 tiles (CATEARS_X6_FIRST_TILE=256)
# against the default 128 x 128, now that 8 nnet streams keep more batches in
# flight; experiments library, the driver's flags, A B B A x2.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06q}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2 3; do
  for f in 128 256 256 128; do
    CATEARS_X6_FIRST_TILE=$f timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline \
        > gpurun_out/$T/c3_f${f}_$rep.json 2>gpurun_out/$T/c3_f${f}_$rep.err || { tail -5 gpurun_out/$T/c3_f${f}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_f${f}_$rep.json')); print('c3 first tile $f', round(l['value']/1e6, 4), 'M frames/s', l['ms_per_step'], l['roofline']['frac'])"
  done
done
for f in 128 256; do
  CATEARS_X6_FIRST_TILE=$f timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline \
      > gpurun_out/$T/c3_f${f}_100.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_f${f}_100.json')); print('c3 first tile $f, 100 steps', round(l['value']/1e6, 4), 'M frames/s', l['ms_per_step'])"
done
echo exit 0
