# Direct-weight GEMM tile variants (measurement library): serial per-layer
# durations, then the driver-config C3 line per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out/dvar
export CATEARS_HIP_LIB=catears_amd/lib/libcatears_hip_exp.so
VARIANTS="${VARIANTS:-300 303 302 304}" bash tools/x6_layers.sh || exit 1
for v in ${VARIANTS:-300 303 302 304}; do
  CATEARS_X6_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dvar/b$v.json 2> gpurun_out/dvar/b$v.err || { tail -5 gpurun_out/dvar/b$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/dvar/b$v.json')); print('v$v', d['value'], d['roofline']['frac'])"
done
