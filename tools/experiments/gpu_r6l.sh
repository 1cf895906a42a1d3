# C5: the next layer's int8 parameters folded into the GEMM's last block
# (gemm_i8_pipe_kernel<..., FOLD>) -- the int8 / parity GPU tests on the
# product library, the serial per-kernel trace, then fold on (1) / off (0)
# ABBA on the experiments library with the checksums compared.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06l}
cd "$R" && mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_int8.py tests/test_gpu_parity.py > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/$T/serial" -o run -- \
    python "$R/bench.py" --workload c5 --serial --steps 20 --warmup 3 --no-cpu-baseline --no-profile \
    > "$R/gpurun_out/$T/serial.log" 2>&1 || { tail -5 "$R/gpurun_out/$T/serial.log"; exit 1; }
python3 "$R/tools/trace_summary.py" "$R/gpurun_out/$T/serial/run_kernel_trace.csv" "C5 serial, fold" > "$R/gpurun_out/$T/serial.txt"
head -16 "$R/gpurun_out/$T/serial.txt"
cd "$R"
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
for rep in 1 2; do
  for f in 0 1 1 0; do
    CATEARS_I8_FOLD=$f timeout -k 10 200 python bench.py --workload c5 --steps 40 --warmup 3 --no-cpu-baseline \
        > gpurun_out/$T/c5_f${f}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/$T/c5_f${f}_$rep.json')); print('c5 fold $f', l['value'], l['ms_per_step'], l['checksum'])"
  done
done
unset CATEARS_HIP_LIB
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 > gpurun_out/$T/c5_driver_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/$T/c5_driver_$rep.json')); print('c5 product driver flags', l['value'], l['ms_per_step'], l['checksum'], l['roofline']['frac'])"
done
echo exit 0
