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
    c4s16)
      timeout -k 10 300 python bench.py --workload c4 --pcm s16 --no-cpu-baseline > gpurun_out/r3/c4s16.json 2> gpurun_out/r3/c4s16.err \
        || { tail -20 gpurun_out/r3/c4s16.err; exit 1; }
      cat gpurun_out/r3/c4s16.json ;;
  esac
done
