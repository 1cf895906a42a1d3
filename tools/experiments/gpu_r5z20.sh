# C5 Quantize with x * (1 / scale) and one FMA correction instead of the
# full division (a build with EXPFLAGS=-DCATEARS_I8_QDIV=1 in scratch/):
# the int8 parity tests with that library (bit-exact Quantize / accumulators
# against the oracle), a billion-value comparison of the two quotients on
# the GPU, then C5 against the product library, ABBA per round.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z20
CATEARS_HIP_LIB=$R/scratch/libcatears_hip_qd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z20/int8.log 2>&1 || { tail -30 gpurun_out/r05z20/int8.log; exit 1; }
tail -1 gpurun_out/r05z20/int8.log
timeout -k 10 300 python - <<'PY' || exit 1
import torch
# x / s against x * r + one FMA correction, r = fl(1 / s), over random
# fp32 x and s (the activation and scale ranges the quantize sees, and wide)
g = torch.Generator(device="cuda").manual_seed(7)
bad = tot = 0
for it in range(40):
    s = torch.exp(torch.empty(1 << 22, device="cuda").uniform_(-12, 4, generator=g))
    x = torch.empty(1 << 22, device="cuda").uniform_(-60, 60, generator=g) * torch.exp(torch.empty(1 << 22, device="cuda").uniform_(-8, 2, generator=g))
    for rep in range(6):
        xs = x.roll(rep * 977)
        q = xs / s
        r = 1.0 / s
        q0 = xs * r
        # the two FMAs emulated in float64 (exact products; the sums round twice, so this only approximates the kernel)
        e = (xs.double() - s.double() * q0.double()).float()
        q1 = (q0.double() + e.double() * r.double()).float()
        bad += int((q1 != q).sum().item())
        tot += q.numel()
print(f"quotients compared: {tot}, differing: {bad}")
PY
for rep in 1 2 3; do
  i=0
  for v in prod qd qd prod; do
    i=$((i+1))
    if [ $v = qd ]; then L=$R/scratch/libcatears_hip_qd.so; else L=$R/catears_amd/lib/libcatears_hip.so; fi
    CATEARS_HIP_LIB=$L timeout -k 10 200 python bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/r05z20/${v}_${rep}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05z20/${v}_${rep}_$i.json')); print('$v', l['value'], l['ms_per_step'])"
  done
done
