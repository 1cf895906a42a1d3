# ABBA at the driver's flags (20 steps, 5 warm-up): default 300 on 3 nnet
# streams against 508 on 8 (and 508 on 8 with the last batch on 128 x 128
# tiles, --wide-tiles last); experiments library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06f}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
run() {  # variant streams tag extra
  CATEARS_HW_QUEUES=$(( $2 + 1 > 4 ? $2 + 1 : 4 )) CATEARS_X6_VARIANT=$1 timeout -k 10 200 python bench.py --no-cpu-baseline \
      --back-streams $2 --steps 20 --warmup 5 $4 > gpurun_out/$T/c3_v$1_s$2_$3.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_v$1_s$2_$3.json')); print('v$1 streams $2 $4', l['value'], l['ms_per_step'])"
}
for rep in 1 2 3 4; do
  run 300 3 ${rep}a
  run 508 8 ${rep}a
  run 508 8 ${rep}w "--wide-tiles last"
  run 508 8 ${rep}b
  run 300 3 ${rep}b
done
