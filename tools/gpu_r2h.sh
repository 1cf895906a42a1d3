R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
SKIP_FULL=1 VARIANTS="58" REPS=1 STEPS=100 bash tools/x6m_ab.sh || exit 1
VARIANTS="55 58" bash tools/x6_layers.sh || exit 1
ARMS="v55b3=CATEARS_X6_VARIANT=55;v58b3=CATEARS_X6_VARIANT=58;v58b2=CATEARS_X6_VARIANT=58|--back-streams 2;v58b1=CATEARS_X6_VARIANT=58|--back-streams 1;v55b2=CATEARS_X6_VARIANT=55|--back-streams 2" REPS=2 bash tools/short_runs.sh
STEPS=200 WARMUP=20 ARMS="Lv55b3=CATEARS_X6_VARIANT=55;Lv58b3=CATEARS_X6_VARIANT=58;Lv58b2=CATEARS_X6_VARIANT=58|--back-streams 2" REPS=1 bash tools/short_runs.sh
