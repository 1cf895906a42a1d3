# Tests touched by the latency / first-tile / quantize changes, C5 and C3
# short benches.  Usage: bash tools/experiments/gpu_r4e.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r4e
O=gpurun_out/r4e
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_latency.py \
  tests/test_gpu_x6_variants.py tests/test_gpu_int8.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 > $O/c5_$i.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/c5_$i.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], d['stages'].get('quantize'))"
  for nb in 3 2; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --back-streams $nb > $O/c3_nb${nb}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/c3_nb${nb}_$i.json').read().strip().splitlines()[-1]); print('c3 nb $nb', d['value'], d['ms_per_step'], d['checksum'])"
  done
done
# exact fbank frame stride in LDS (FB8_STRIDE): bit-exactness and C2
for st in 268 260; do
  CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_s$st.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_parity.py -k "fbank" > $O/fb_s$st.txt 2>&1 || { echo "stride $st parity FAIL"; tail -20 $O/fb_s$st.txt; exit 1; }
  echo "stride $st parity: $(tail -1 $O/fb_s$st.txt)"
done
for i in 1 2; do
  for st in 264 268 260; do
    if [ $st = 264 ]; then unset CATEARS_HIP_LIB; else export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_s$st.so; fi
    timeout -k 10 200 python bench.py --workload c2 --steps 30 --warmup 3 --no-cpu-baseline > $O/c2_s${st}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/c2_s${st}_$i.json').read().strip().splitlines()[-1]); print('c2 stride $st', d['value'])"
  done
done
