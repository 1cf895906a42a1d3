# Round-3 GPU check: every -m gpu test, then the driver-config C3 line and a
# full 100 h C4 pass on one GPU.  Usage: STAGE="tests bench c4" bash tools/gpu_r3.sh
set -o pipefail
mkdir -p gpurun_out/r3
cd "$(dirname "$0")/.."
for st in ${STAGE:-tests bench c4}; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/r3/pytest.log 2>&1 || { tail -40 gpurun_out/r3/pytest.log; exit 1; }
      tail -3 gpurun_out/r3/pytest.log ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3/bench.json 2> gpurun_out/r3/bench.err \
        || { tail -20 gpurun_out/r3/bench.err; exit 1; }
      cat gpurun_out/r3/bench.json ;;
    c4)
      timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/r3/c4.json 2> gpurun_out/r3/c4.err \
        || { tail -20 gpurun_out/r3/c4.err; exit 1; }
      cat gpurun_out/r3/c4.json ;;
    c2)
      for m in exact fast; do
        timeout -k 10 300 python bench.py --workload c2 --fbank $m --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3/c2_$m.json 2> gpurun_out/r3/c2_$m.err \
          || { tail -20 gpurun_out/r3/c2_$m.err; exit 1; }
        cat gpurun_out/r3/c2_$m.json
      done ;;
    fast)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_fbank_fast.py tests/test_gpu_pcm16.py -x -v -s --timeout 120 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/r3/pytest_fast.log 2>&1 || { tail -40 gpurun_out/r3/pytest_fast.log; exit 1; }
      grep -E "vs exact|passed|failed" gpurun_out/r3/pytest_fast.log ;;
    layers)
      # serial per-layer durations: direct-weight default (0) vs round-2 default (160)
      VARIANTS="${VARIANTS:-0 160}" bash tools/x6_layers.sh || exit 1 ;;
    prof)
      # the driver's C3 command under rocprofv3 kernel-trace (+ stats), PMC
      # traffic and MFMA busy of the GEMMs on a serial run, C2 fast likewise
      TAG=${TAG:-r03a}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
          python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
      grep '^{' $OUT/bench.log | cut -c1-200
      python3 tools/trace_summary.py $(ls $OUT/prof/*/*kernel_trace.csv $OUT/prof/*kernel_trace.csv 2>/dev/null | head -1) "C3 --steps 20 --warmup 5" > $OUT/kernel_summary.txt
      head -30 $OUT/kernel_summary.txt
      i=0
      for grp in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "gemm_|fbank|cmvn|finalize|splice" \
            --output-format csv -d $OUT/pmc$i -o run -- \
            python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile --serial > $OUT/pmc$i.log 2>&1 \
            || { echo "pmc $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
      done
      python3 tools/pmc_traffic.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc_traffic.json
      timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "gemm_" \
          --output-format csv -d $OUT/pmc3 -o run -- \
          python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-profile --serial > $OUT/pmc3.log 2>&1 \
          || { echo "pmc 3 failed"; tail -5 $OUT/pmc3.log; exit 1; }
      python3 tools/pmc_mfma.py $OUT/pmc3 $OUT/pmc_mfma.json
      cat $OUT/pmc_mfma.json | head -30
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- \
          python3 bench.py --workload c2 --fbank fast --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c2.log 2>&1 || { tail -5 $OUT/bench_c2.log; exit 1; }
      grep '^{' $OUT/bench_c2.log | cut -c1-200
      # both fbank modes' kernels in one summary (runs under one parent dir)
      i=0
      for grp in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        for m in exact fast; do
          timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "fbank" --output-format csv -d $OUT/pmc_c2_$i/$m -o run -- \
              python3 bench.py --workload c2 --fbank $m --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $OUT/pmc_c2_$i.$m.log 2>&1 \
              || { echo "pmc c2 $i $m failed"; tail -5 $OUT/pmc_c2_$i.$m.log; exit 1; }
        done
      done
      python3 tools/pmc_traffic.py $OUT/pmc_c2_1 $OUT/pmc_c2_2 $OUT/pmc_traffic_c2.json
      cat $OUT/pmc_traffic_c2.json | head -20
      # C5 (int8): kernel trace + stats of the pipelined line, PMC traffic and
      # MFMA busy of its GEMMs on a serial run
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- \
          python3 bench.py --workload c5 --steps 60 --warmup 10 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || { tail -5 $OUT/bench_c5.log; exit 1; }
      grep '^{' $OUT/bench_c5.log | cut -c1-200
      i=0
      for grp in FETCH_SIZE WRITE_SIZE; do
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "gemm_|quantize|minmax|finalize" --output-format csv -d $OUT/pmc_c5_$i -o run -- \
            python3 bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline --no-profile --serial > $OUT/pmc_c5_$i.log 2>&1 \
            || { echo "pmc c5 $i failed"; tail -5 $OUT/pmc_c5_$i.log; exit 1; }
      done
      python3 tools/pmc_traffic.py $OUT/pmc_c5_1 $OUT/pmc_c5_2 $OUT/pmc_traffic_c5.json
      timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "gemm_" \
          --output-format csv -d $OUT/pmc_c5_3 -o run -- \
          python3 bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline --no-profile --serial > $OUT/pmc_c5_3.log 2>&1 \
          || { echo "pmc c5 3 failed"; tail -5 $OUT/pmc_c5_3.log; exit 1; }
      python3 tools/pmc_mfma.py $OUT/pmc_c5_3 $OUT/pmc_mfma_c5.json
      head -20 $OUT/pmc_mfma_c5.json ;;
    lat)
      CALLS=${CALLS:-100} bash tools/trace_latency.sh || exit 1
      python3 tools/trace_summary.py gpurun_out/lat/kernel_trace.csv "latency.py trace" > gpurun_out/lat/kernel_summary.txt
      head -40 gpurun_out/lat/kernel_summary.txt ;;
    c4s16)
      timeout -k 10 300 python bench.py --workload c4 --pcm s16 --no-cpu-baseline > gpurun_out/r3/c4s16.json 2> gpurun_out/r3/c4s16.err \
        || { tail -20 gpurun_out/r3/c4s16.err; exit 1; }
      cat gpurun_out/r3/c4s16.json ;;
  esac
done
