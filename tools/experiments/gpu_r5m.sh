# Stress of the final tree's fbank kernels (exact f32, exact s16, fast) beside
# three TDNN-S streams (tools/experiments/lds_race_stress.py): every launch
# bit-compared with the same launch made alone.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05m
for spec in "exact f32" "exact s16" "fast f32"; do
  set -- $spec
  timeout -k 10 120 python -u tools/experiments/lds_race_stress.py --fbank $1 --pcm $2 --seconds 20 \
      > gpurun_out/r05m/$1_$2.log 2>&1 || { tail -20 gpurun_out/r05m/$1_$2.log; exit 1; }
  echo "$1 $2 $(tail -1 gpurun_out/r05m/$1_$2.log | cut -c1-200)"
done
