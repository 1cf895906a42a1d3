# One-wave-per-SIMD bf16x6 kernels (variants 500-503, experiments library)
# against the default 300: bits on TDNN-S, serial per-layer times, then C3 at
# 200 steps with 3 and 5 nnet streams.  Usage: bash tools/experiments/gpu_r6b.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06b}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.')
from catears_amd import synth
synth.write_model('/tmp/${T}_m', 'tdnn-s')" || exit 1
CFG=$(ls /tmp/${T}_m/*.conf | head -1)
for v in 300 ${VARS:-500 501 502 503}; do
  CATEARS_X6_VARIANT=$v PYTHONPATH=$R timeout -k 10 200 python tools/experiments/x6_child.py $CFG /tmp/${T}_v$v.npy || exit 1
  python3 -c "
import numpy as np
a=np.load('/tmp/${T}_v300.npy'); b=np.load('/tmp/${T}_v$v.npy')
print('v$v bits equal to 300:', a.shape, np.array_equal(a.view(np.uint32), b.view(np.uint32)), float(np.abs(a-b).max()))"
done
VARIANTS="300 ${VARS:-500 501 502 503}" bash tools/x6_layers.sh 2>&1 | tail -6 || exit 1
for ns in 3 5; do
  for v in 300 ${VARS:-500 501 502 503}; do
    CATEARS_HW_QUEUES=$(( ns > 3 ? 8 : 4 )) CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --back-streams $ns > gpurun_out/$T/c3_v${v}_s$ns.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_v${v}_s$ns.json')); print('200 steps v$v streams $ns', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
