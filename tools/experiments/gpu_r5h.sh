# Exact fbank with the LDS tables ahead of the frames (immediate table
# offsets) and a uniform last-frame clamp: fbank GPU tests, then C2 A/B
# against the previous build (abtmp/old.so vs abtmp/new.so, alternating).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05h
timeout -k 10 600 python -u -m pytest tests -m gpu -k "fbank or c2 or pcm16 or determinism or dropin" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05h/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05h/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/experiments/c2_lib_ab.sh
