# Price each C3 stage by its absence: CATEARS_SKIP (measurement library only,
# wrong results) leaves out the first GEMM layer (1), the finalize (2), the
# fbank (4), CMVN (8), the last GEMM layer (16), the hidden layers (32);
# C3 at 60 timed steps after 20 warm-up, two rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out/r05k
for rep in 1 2; do
  for sk in 0 1 2 4 8 12 16 32; do
    CATEARS_HIP_LIB=$PWD/catears_amd/lib/libcatears_hip_exp.so CATEARS_SKIP=$sk timeout -k 10 200 python bench.py --steps 60 --warmup 20 --no-cpu-baseline > gpurun_out/r05k/skip${sk}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; l=json.load(open('gpurun_out/r05k/skip${sk}_$rep.json')); print('skip $sk', l['value'], l['ms_per_step'])"
  done
done
