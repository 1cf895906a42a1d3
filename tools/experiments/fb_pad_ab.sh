# Exact fbank transposes with the 64-point padding (tpos) against the
# previous layout (libcatears_hip_prevfb.so): parity, C2 alternating, PMC.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/fbpad
O=gpurun_out/fbpad
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_pcm16.py -k "fbank or cmvn or score or c3" > $O/t.txt 2>&1 || { echo "parity FAILED"; tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for i in 1 2 3; do
  for L in new prev; do
    if [ $L = prev ]; then export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_prevfb.so; else unset CATEARS_HIP_LIB; fi
    timeout -k 10 200 python bench.py --workload c2 --steps 30 --warmup 3 --no-cpu-baseline > $O/c2_${L}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('$O/c2_${L}_$i.json').read().strip().splitlines()[-1]); print('c2 $L', d['value'], d['checksum'])"
  done
done
unset CATEARS_HIP_LIB
KREGEX=fbank WORKLOAD=c2 OUT=fbpad/pmc bash tools/pmc_kernel.sh > $O/pmc.txt 2>&1 || exit 1
tail -14 $O/pmc.txt
