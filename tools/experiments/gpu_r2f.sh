R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 python tools/probes/blas_calib.py || exit 1
ARMS="drv=X=1;drvnp=X=1|--no-profile;w100=X=1|--warmup 100;s60=X=1|--steps 60" REPS=2 bash tools/short_runs.sh || exit 1
bash tools/trace_short.sh
