# The C3 sink share (rank 0 scores a share of the steps): the C3/C4 rank
# tests (2 gloo ranks on device 0) and the fold tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05u
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_fold.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05u/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r05u/pytest.log | tail -20
exit $rc
