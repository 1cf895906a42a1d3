# The bf16x6 plane chain (CATEARS_X6_CHAIN=1: each layer's output split once
# in its epilogue, read as planes by the next): parity (the variants file,
# then the whole GPU suite with the chain on), then C3 alternating with the
# fp32 chain at the driver's flags and at 200 steps.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05z6
timeout -k 10 600 python -u -m pytest tests/test_gpu_x6_variants.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z6/variants.log 2>&1 || { tail -30 gpurun_out/r05z6/variants.log; exit 1; }
tail -2 gpurun_out/r05z6/variants.log
CATEARS_X6_CHAIN=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z6/suite_chain.log 2>&1 || { tail -30 gpurun_out/r05z6/suite_chain.log; exit 1; }
tail -2 gpurun_out/r05z6/suite_chain.log
for rep in 1 2 3; do
  for c in 0 1; do
    CATEARS_X6_CHAIN=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05z6/drv_c${c}_$rep.json 2>/dev/null || exit 1
    CATEARS_X6_CHAIN=$c timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r05z6/def_c${c}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json
a=json.load(open('gpurun_out/r05z6/drv_c${c}_$rep.json')); b=json.load(open('gpurun_out/r05z6/def_c${c}_$rep.json'))
print('chain=$c', 'driver', a['value'], a['ms_per_step'], a['roofline']['frac'], '| 200 steps', b['value'], b['ms_per_step'], b['roofline']['frac'])"
  done
done
