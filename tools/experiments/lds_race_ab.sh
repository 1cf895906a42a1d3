# A/B of the intra-wave LDS hand-off: the round-4 library (wavefront fence +
# wave_barrier, no wait) against the in-tree one (s_waitcnt lgkmcnt(0)), under
# tools/experiments/lds_race_stress.py, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/race
OLD=${OLD:-catears_amd/lib/ab/libcatears_hip_r4.so}
NEW=${NEW:-catears_amd/lib/libcatears_hip.so}
S=${SECS:-15}
for k in $(seq ${RUNS:-2}); do
  for mode in ${MODES:-fast exact}; do
    for L in $OLD $NEW; do
      v=$(basename $L .so)
      CATEARS_HIP_LIB=$R/$L timeout -k 10 $((S + 90)) python -u tools/experiments/lds_race_stress.py --fbank $mode \
          --seconds $S > gpurun_out/race/$v.$mode.$k.log 2>&1 || { tail -20 gpurun_out/race/$v.$mode.$k.log; exit 1; }
      tail -1 gpurun_out/race/$v.$mode.$k.log
    done
  done
done
