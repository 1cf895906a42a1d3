# Pipelined-vs-serial bit identity of the C3 bench (bench.py --verify-serial)
# for several product libraries, alternating: LIBS = paths under the repo
# (default: round 3's library, round 3's fbank kernel without its forced
# occupancy, the in-tree build).  Each run scores warmup+steps batches through
# the four-stream pipeline and re-scores every batch serially in the same
# process.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/det
LIBS=${LIBS:-"catears_amd/lib/libcatears_hip_r3.so catears_amd/lib/libcatears_hip_r3fix.so catears_amd/lib/libcatears_hip.so"}
ARGS="--steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --verify-serial ${EXTRA}"
for k in $(seq ${RUNS:-4}); do
  for L in $LIBS; do
    v=$(basename $L .so)
    CATEARS_HIP_LIB=$R/$L timeout -k 10 200 python bench.py $ARGS > gpurun_out/det/$v.$k.log 2>&1 || { tail -20 gpurun_out/det/$v.$k.log; exit 1; }
    python3 -c "import json,sys; l=json.loads([x for x in open('gpurun_out/det/$v.$k.log') if x.startswith('{')][0]); v=l['verify']; print('$v.$k', l['value'], l['checksum'], v['batches'], v['differing'], json.dumps(v['detail'][:3]))"
  done
done
