// ref_harness.cc -- TEST INFRASTRUCTURE.  A C-ABI shim over the parts of the
// reference that compile from their own sources in this image:
//   * pocketkaldi::SRFFT        (/root/reference/src/srfft.cc, standalone)
//   * gemmlowp EightBitIntGemm  (/root/reference/src/gemmlowp/eight_bit_int_gemm/
//                                eight_bit_int_gemm.cc, vendored, standalone)
// The rest of the hot path (fbank.cc, cmvn.cc, nnet.cc, am.cc) links matrix.cc,
// which needs <cblas.h>; the image has none, so that part is unbuildable here and
// is pinned by the reference's golden fixtures instead ("Oracle").
// Built by oracle/Makefile into oracle/_ref/libref.so; only tests load it.
#include <stdint.h>
#include "srfft.h"
#include "eight_bit_int_gemm/eight_bit_int_gemm.h"

extern "C" {

void *ref_srfft_new(int real_len) { return new pocketkaldi::SRFFT(real_len); }

void ref_srfft_free(void *f) { delete static_cast<pocketkaldi::SRFFT *>(f); }

// Forward real FFT in place (src/srfft.cc:370-459); buf holds >= real_len floats.
void ref_srfft_forward(void *f, float *data, int real_len, float *buf) {
  static_cast<pocketkaldi::SRFFT *>(f)->Compute(data, real_len, true, buf, real_len);
}

// n forward transforms back to back (timing, tools/cpu_calibrate.py)
void ref_srfft_forward_n(void *f, float *data, int n, int real_len, float *buf) {
  for (int i = 0; i < n; ++i)
    static_cast<pocketkaldi::SRFFT *>(f)->Compute(data + (long)i * real_len, real_len, true, buf, real_len);
}

// MatMat_U8U8F32 (src/matrix.cc:389-420): row-major A (m x k), B (k x n), C (m x n).
void ref_gemm_u8u8f32(int m, int n, int k, const uint8_t *a, float sa, int32_t zpa,
                      const uint8_t *b, float sb, int32_t zpb, float *c) {
  gemmlowp::eight_bit_int_gemm::EightBitIntGemm(
      true, true, true, m, n, k, a, -zpa, k, b, -zpb, n, c, sa * sb, n,
      gemmlowp::eight_bit_int_gemm::BitDepthSetting::A8B8);
}

}  // extern "C"
