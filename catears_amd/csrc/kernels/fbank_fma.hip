// fbank_fma.hip -- the fast fbank mode (CE_GPU_FBANK_FAST): kernels/fbank.hip's
// lane program (eight lanes per frame, the reference's split-radix FFT in
// registers, fbank8_ops.h) built with FMA contraction (Makefile:
// -ffp-contract=fast for this file) and the pre-emphasis as one float FMA
// instead of the reference's double product.  Not bit-exact by design: every
// mul/add pair the compiler fuses rounds once instead of twice, so the
// results stay as close to the exact float64 result as the reference's own
// fp32 order (tests/test_gpu_fbank_fast.py), with fewer instructions.
#define FB8_FMA 1
#include "fbank.hip"
