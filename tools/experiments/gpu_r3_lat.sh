# Latency-mode check: the latency / drop-in / parity GPU tests, then the
# latency table A/B and one 70-row call's kernel sequence.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_latency.py tests/test_dropin.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3/pytest_lat.log 2>&1 || { tail -30 gpurun_out/r3/pytest_lat.log; exit 1; }
tail -2 gpurun_out/r3/pytest_lat.log
bash tools/experiments/lat70_trace.sh
