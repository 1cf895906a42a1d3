# At the driver's flags (20 steps, 5 warm-up), ABC CBA on one box:
# A = the rounds 3-5 default (variant 300 on 3 nnet streams, no wide tiles),
# B = the round-6 default (512 x 128 tiles, 8 streams, last batch wide) with
# XCD tile groups of 1 column tile, C = the same with groups of 2; then the
# PMC traffic of B and C (serial); experiments library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${T:-r06h}
cd "$R" && mkdir -p gpurun_out/$T
export CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so
run() {  # tag extra-env... -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 ${BARGS} \
      > gpurun_out/$T/c3_${tag}.json 2>/dev/null || exit 1
  python3 -c "import json; l=json.load(open('gpurun_out/$T/c3_${tag}.json')); print('$tag', l['value'], l['ms_per_step'])"
}
for rep in 1 2; do
  BARGS="--back-streams 3 --wide-tiles none" run A${rep}a CATEARS_X6_VARIANT=300
  BARGS="" run B${rep}a CATEARS_X6W_GROUP=1
  BARGS="" run C${rep}a CATEARS_X6W_GROUP=2
  BARGS="" run C${rep}b CATEARS_X6W_GROUP=2
  BARGS="" run B${rep}b CATEARS_X6W_GROUP=1
  BARGS="--back-streams 3 --wide-tiles none" run A${rep}b CATEARS_X6_VARIANT=300
done
cd /tmp && export TMPDIR=/tmp
for g in 1 2; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    CATEARS_X6W_GROUP=$g timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "gemm_" --output-format csv \
        -d "$R/gpurun_out/$T/pmc_g${g}_$i" -o run -- python "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline \
        --no-profile --serial > "$R/gpurun_out/$T/pmc_g${g}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/$T/pmc_g${g}_$i.log"; exit 1; }
  done
  python "$R/tools/pmc_traffic.py" "$R/gpurun_out/$T/pmc_g${g}_1" "$R/gpurun_out/$T/pmc_g${g}_2" "$R/gpurun_out/$T/pmc_traffic_g$g.json" --layers 7 | head -7
done
