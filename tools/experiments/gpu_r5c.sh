# Where the direct-weight bf16x6 GEMM's time goes: serial per-layer medians
# (tools/x6_layers.sh) of the default 300 and its DIAG ablations 310-316 in
# the experiments library (wrong results, timing only).  Needs
# catears_amd/lib/libcatears_hip_exp.so pushed (drop it from .gpurunignore).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
CATEARS_HIP_LIB=$R/catears_amd/lib/libcatears_hip_exp.so VARIANTS="${VARIANTS:-300 310 311 312 313 314 315 316}" bash tools/x6_layers.sh
