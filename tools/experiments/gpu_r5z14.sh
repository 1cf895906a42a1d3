# bf16x6 direct-weight tiles of 256 units x 64 frames as 4-wave blocks, two
# per CU (variant 340: block barriers over four waves) against the default
# 300 (256 x 128, 8 waves); experiments library; bits against the default,
# then C3 at 200 steps and at the driver's flags, ABBA per round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z14
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.')
from catears_amd import synth
synth.write_model('/tmp/r05z14_m', 'tdnn-s')" || exit 1
CFG=$(ls /tmp/r05z14_m/*.conf | head -1)
for v in 300 340; do
  CATEARS_X6_VARIANT=$v PYTHONPATH=$R timeout -k 10 200 python tools/experiments/x6_child.py $CFG /tmp/r05z14_v$v.npy || exit 1
done
python3 -c "
import numpy as np
a=np.load('/tmp/r05z14_v300.npy'); b=np.load('/tmp/r05z14_v340.npy')
print('bits equal:', a.shape, np.array_equal(a.view(np.uint32), b.view(np.uint32)))"
for rep in 1 2 3; do
  i=0
  for v in 300 340 340 300; do
    i=$((i+1))
    CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z14/def_v${v}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z14/def_v${v}_${rep}_$i.json')); print('200 steps v$v', l['value'], l['ms_per_step'], l['roofline']['frac'])"
  done
done
