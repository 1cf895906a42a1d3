# Round-4 GPU steps.  Usage: STAGE="det tests c2 bench" bash tools/gpu_r4.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4; mkdir -p $O
for st in ${STAGE:-tests bench}; do
  case $st in
    det)
      RUNS=${RUNS:-3} bash tools/experiments/determinism_ab.sh || exit 1 ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider ${TESTS:-} > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
      tail -3 $O/pytest.log ;;
    fbtests)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pcm16.py tests/test_dropin.py -m gpu -x -v \
        --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_fb.log 2>&1 || { tail -60 $O/pytest_fb.log; exit 1; }
      tail -3 $O/pytest_fb.log ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
        || { tail -20 $O/bench.err; exit 1; }
      cut -c1-400 $O/bench.json ;;
    c2)
      for m in exact fast; do
        timeout -k 10 300 python bench.py --workload c2 --fbank $m --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_$m.json 2> $O/c2_$m.err \
          || { tail -20 $O/c2_$m.err; exit 1; }
        cut -c1-300 $O/c2_$m.json
      done ;;
  esac
done
