# Variant 508 (512 x 128 bf16x6 tiles, 8 waves of 128 x 64) over more nnet
# streams, at 200 steps and at the driver's flags (20 steps, 5 warm-up),
# against the default 300 on 3 streams; experiments library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06e}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
run() {  # variant streams steps warmup tag
  CATEARS_HW_QUEUES=$(( $2 + 1 > 4 ? $2 + 1 : 4 )) CATEARS_X6_VARIANT=$1 timeout -k 10 200 python bench.py --no-cpu-baseline \
      --back-streams $2 --steps $3 --warmup $4 > gpurun_out/$T/c3_v$1_s$2_n$3_$5.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_v$1_s$2_n$3_$5.json')); print('v$1 streams $2 steps $3', l['value'], l['ms_per_step'], l['roofline']['frac'])"
}
for s in 6 8 10 12; do run 508 $s 200 5 a; done
run 300 3 200 5 a
for rep in 1 2; do
  run 300 3 20 5 $rep
  for s in 6 8 10; do run 508 $s 20 5 $rep; done
done
