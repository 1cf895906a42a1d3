# (Historical: measures the four-step fast fbank kernel, kernels/fbank_fast.hip, removed
# in round 5 when the fast mode became the contracted exact lane program; kept as the
# record of DESIGN.md §8b.  It no longer builds against the current tree.)
# Fast-fbank run-to-run difference: the stress (lds_race_stress.py) over the
# FF_DIAG builds of fbank_fast.hip (make lib OBJ=build/obj_ffdN
# LIB=catears_amd/lib/ab/libffdN.so FFDIAG=-DFF_DIAG=N).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/ffd
S=${SECS:-10}
for L in ${LIBS:-catears_amd/lib/libcatears_hip.so catears_amd/lib/ab/libffd1.so catears_amd/lib/ab/libffd2.so catears_amd/lib/ab/libffd3.so}; do
  v=$(basename $L .so)
  CATEARS_HIP_LIB=$R/$L timeout -k 10 $((S + 90)) python -u tools/experiments/lds_race_stress.py --fbank ${MODE:-fast} \
      --seconds $S ${EXTRA} > gpurun_out/ffd/$v.log 2>&1 || { tail -20 gpurun_out/ffd/$v.log; exit 1; }
  python3 -c "
import json; l=json.loads(open('gpurun_out/ffd/$v.log').read().strip().splitlines()[-1])
print('$v', l['iterations'], l['differing_iterations'], l['row_mod4'], json.dumps(l['captured'][:2]))"
done
