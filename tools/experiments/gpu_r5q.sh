# ce_gpu_sum_f64 for the gather / C4 folds: the whole GPU suite, the fold
# cost probe, C4 (one process) and C3 at the driver's flags.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05q
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05q/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r05q/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/probes/fold_cost.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline --stage-profile > gpurun_out/r05q/c4.json 2> gpurun_out/r05q/c4.err || { tail -5 gpurun_out/r05q/c4.err; exit 1; }
python3 -c "import json; l=json.load(open('gpurun_out/r05q/c4.json')); print('c4', l['value'], l['roofline']['frac'], l['checksum'])"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05q/c3_$i.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/r05q/c3_$i.json')); print('c3', l['value'])"
done
