ARMS="w5s20=X=1;w100s20=X=1|--warmup 100;w5s200=X=1|--steps 200;w5s60=X=1|--steps 60" REPS=2 bash tools/short_runs.sh
