# bf16x6 direct-weight tiles as 8 waves of 32 units x 128 frames (variant
# 320: no weight fragment loaded by two waves; activation fragment reads 4x)
# against the default 300 (4 x 2 waves of 64 x 64).  Experiments library;
# bits checked against the default, then C3 alternating (200 steps and the
# driver's flags).  Needs libcatears_hip_exp.so pushed.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z7
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
cat > gpurun_out/r05z7/child.py <<'PY'
import sys, numpy as np, torch
from catears_amd import gpu
ctx = gpu.Context(0)
model = gpu.Model(ctx, sys.argv[1])
x = np.random.default_rng(750).normal(9.0, 3.0, size=(3000, 40)).astype(np.float32)
np.save(sys.argv[2], gpu.nnet_propagate(ctx, model, torch.from_numpy(x).to("cuda:0")).cpu().numpy())
PY
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from catears_amd import synth
synth.write_model('/tmp/r05z7_m', 'tdnn-s')" || exit 1
CFG=$(ls /tmp/r05z7_m/*.conf | head -1)
for v in 300 320; do
  CATEARS_X6_VARIANT=$v PYTHONPATH=$R timeout -k 10 200 python gpurun_out/r05z7/child.py $CFG /tmp/r05z7_v$v.npy || exit 1
done
python3 -c "
import numpy as np
a=np.load('/tmp/r05z7_v300.npy'); b=np.load('/tmp/r05z7_v320.npy')
print('bits equal:', a.shape, np.array_equal(a.view(np.uint32), b.view(np.uint32)))"
for rep in 1 2 3; do
  for v in 300 320; do
    CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z7/def_v${v}_$rep.json 2>/dev/null || exit 1
    CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05z7/drv_v${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json
a=json.load(open('gpurun_out/r05z7/def_v${v}_$rep.json')); b=json.load(open('gpurun_out/r05z7/drv_v${v}_$rep.json'))
print('v$v', '200 steps', a['value'], a['ms_per_step'], a['roofline']['frac'], '| driver', b['value'], b['ms_per_step'])"
  done
done
