# C2 exact fbank with phase A's lane-dependent twiddle cases removed (timing
# only, wrong results: kernels/fbank_nocase.hip, CATEARS_FB_NOCASE=1) against
# the exact kernel, ABBA x2 on the experiments library: the most a
# wave-uniform residue mapping of phase A could give.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06p}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2; do
  for f in 0 1 1 0; do
    CATEARS_FB_NOCASE=$f timeout -k 10 200 python bench.py --workload c2 --steps 60 --warmup 5 --no-cpu-baseline \
        > gpurun_out/$T/c2_n${f}_$rep.json 2>gpurun_out/$T/c2_n${f}_$rep.err || { tail -5 gpurun_out/$T/c2_n${f}_$rep.err; exit 1; }
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c2_n${f}_$rep.json')); print('c2 nocase $f', round(l['value']/1e9, 4), 'G frames/s', l['ms_per_step'], 'ms/step', l.get('checksum'))"
  done
done
echo exit 0
