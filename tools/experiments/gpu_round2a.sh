timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full.log 2>&1; rc=$?; tail -3 gpurun_out/full.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/full.log | head -20; exit $rc; }
ARMS="p=X=1;noprof=X=1|--no-profile;long=X=1|--steps 200 --warmup 20" REPS=2 bash tools/short_runs.sh && bash tools/trace_short.sh
