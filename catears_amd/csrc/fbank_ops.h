// fbank_ops.h -- scalar helpers of the exact fbank kernel's lane program
// (fbank8_ops.h), shared by the device kernel and the CPU emulator in tests.
//
// Every expression keeps the reference's operation order and roundings; the
// translation units that include this header are compiled with
// -ffp-contract=off so no multiply-add is fused (the reference runs on x86-64
// without FMA).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define CE_HD __host__ __device__ __forceinline__
#else
#define CE_HD static inline
#endif

namespace catears {
namespace fb {

// Pre-emphasis of one sample in double (src/fbank.cc:57-61: PK_PREEMPH_COEFF
// is the double literal 0.97, `x[i] -= 0.97 * x[i-1]` on a float lvalue).
CE_HD float preemph(float cur, float prev) {
  const double p = 0.97 * (double)prev;
  return (float)((double)cur - p);
}

CE_HD int bitrev8(int k) {
  int r = 0;
  for (int b = 0; b < 8; ++b) r |= ((k >> b) & 1) << (7 - b);
  return r;
}

}  // namespace fb
}  // namespace catears
