# Round 2 re-entry check: GPU suite, driver-shaped bench lines, bf16x6 variant timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1; rc=$?; tail -3 gpurun_out/full.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/full.log | head -20; exit $rc; }
ARMS="drv=X=1;long=X=1|--steps 200 --warmup 20" REPS=2 bash tools/short_runs.sh || exit 1
STEPS=100 WARMUP=10 ARMS="v42=CATEARS_X6_VARIANT=42;v60=CATEARS_X6_VARIANT=60;v61=CATEARS_X6_VARIANT=61;v62=CATEARS_X6_VARIANT=62;v63=CATEARS_X6_VARIANT=63;v70=CATEARS_X6_VARIANT=70;v71=CATEARS_X6_VARIANT=71;v40=CATEARS_X6_VARIANT=40" REPS=1 bash tools/short_runs.sh
