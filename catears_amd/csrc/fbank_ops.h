// fbank_ops.h -- per-lane arithmetic of the fbank kernel, shared verbatim by
// the device kernel (kernels/fbank.hip) and the CPU schedule emulator used in
// tests (tests/native/emu_fbank.cc), so the emulator proves on a CPU that the
// lane decomposition reproduces the reference's float operations exactly.
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

// LDS placement of complex point i in the re / im arrays: a bijective XOR
// swizzle (i ^ ((i >> 2) & 63)) that spreads the split-radix generations'
// strided lane accesses and the bit-reversed post-pass reads over the 64 LDS
// banks (simulated conflict passes 266 -> 146 per frame; 114 is the floor).
// Pure placement: values and arithmetic are unchanged.
CE_HD int sw(int i) { return i ^ ((i >> 2) & 63); }

// One lane op of the split-radix generation schedule (src/srfft.cc:124-265),
// from its precomputed descriptor (tables.cc build_fft_lanes):
//   addr  the op's four LDS slots, already swizzled, 8 bits each (slot j in
//         bits 8j..8j+7): points base+n, +q, +h, +h+q of a node of length
//         m = 2^lg (q = m/4, h = m/2); base..base+3 of a length-4 node;
//         base, base+1 of a length-2 node
//   meta  kind (bits 0-1: 0 none, 1 node, 2 length-4, 3 length-2) | twiddle
//         case (bits 2-3: 0 none (n == 0), 1 the n == m/8 rotation, 2 table)
//   tw    the node's six table twiddles for this n (table case)
CE_HD void fft_lane_op(uint32_t addr, uint32_t meta, const float *tw, float *re, float *im) {
  const uint32_t kind = meta & 3u;
  if (kind == 0u) return;
  const int p0 = (int)(addr & 255u), p1 = (int)((addr >> 8) & 255u);
  const int p2 = (int)((addr >> 16) & 255u), p3 = (int)(addr >> 24);
  float t1, t2;
  // every kind reads and writes its four slots here, so a generation that
  // mixes kinds issues one set of LDS accesses (a length-2 op's slots are
  // p0 p1 p0 p1: it writes its two results twice, the same values)
  float ar = re[p0], ai = im[p0], br = re[p1], bi = im[p1];
  float cr = re[p2], ci = im[p2], dr = re[p3], di = im[p3];
  // The kinds share their steps (same operations, same order per value):
  // a length-4 node is the general node's first two steps followed by the
  // (a, b) butterfly instead of twiddles; a length-2 node is that butterfly
  // alone.  Sharing them keeps a mixed generation's divergent paths short.
  if (kind != 3u) {
    // general node step 1 / length-4 (srfft.cc:163-205, points a b c d =
    // 0 1 2 3): butterflies (n, n+h) and (n+q, n+q+h)
    t1 = ar + cr; cr = ar - cr; ar = t1;
    t1 = ai + ci; ci = ai - ci; ai = t1;
    t1 = br + dr; dr = br - dr; br = t1;
    t1 = bi + di; di = bi - di; bi = t1;
    // step 2: (h+n, h+q+n) / the length-4 node's (c, d) rotation
    t1 = cr + di;
    t2 = ci + dr;
    ci = ci - dr;
    dr = cr - di;
    cr = t1;
    di = t2;
  }
  if (kind != 1u) {
    // (a, b) butterfly of a length-4 node, or a length-2 node (srfft.cc:206-216)
    t1 = ar + br; br = ar - br; ar = t1;
    t1 = ai + bi; bi = ai - bi; ai = t1;
    if (kind == 3u) cr = ar, ci = ai, dr = br, di = bi;
  } else {
    // steps 3 & 4: twiddles for n >= 1
    const uint32_t twc = (meta >> 2) & 3u;
    if (twc == 1u) {
      const float sq = (float)0.70710678118654752440;
      t1 = sq * (cr + ci);
      ci = sq * (ci - cr);
      cr = t1;
      t2 = sq * (di - dr);
      di = -sq * (dr + di);
      dr = t2;
    } else if (twc == 2u) {
      t2 = tw[0] * (cr + ci);
      t1 = tw[1] * cr + t2;
      cr = tw[2] * ci + t2;
      ci = t1;
      t2 = tw[3] * (dr + di);
      t1 = tw[4] * dr + t2;
      dr = tw[5] * di + t2;
      di = t1;
    }
  }
  re[p0] = ar; im[p0] = ai; re[p1] = br; im[p1] = bi;
  re[p2] = cr; im[p2] = ci; re[p3] = dr; im[p3] = di;
}

CE_HD int bitrev8(int k) {
  int r = 0;
  for (int b = 0; b < 8; ++b) r |= ((k >> b) & 1) << (7 - b);
  return r;
}

// Real-FFT post-processing for one k in 1..128 (src/srfft.cc:382-438) fused
// with the power spectrum (src/fbank.cc:193-211).  re/im hold the complex FFT
// before its bit-reversal permutation, so B_k is read at bitrev(k).  Writes
// power[k] and power[256-k].
// a, b: LDS slots of B_k and B_{256-k}, i.e. sw(bitrev8(k)), sw(bitrev8(256-k)).
CE_HD void post_power_ab(int k, int a, int b, const float *re, const float *im, float kr, float ki,
                         float *power) {
  const int kk = 256 - k;
  const float xr = re[a], xi = im[a], yr = re[b], yi = im[b];
  // 0.5 * (float sum) in double then back to float == exact halving
  const float c_re = (float)(0.5 * (double)(xr + yr));
  const float c_im = (float)(0.5 * (double)(xi - yi));
  const float d_re = (float)(0.5 * (double)(xi + yi));
  const float d_im = (float)(-0.5 * (double)(xr - yr));
  float o_re = c_re, o_im = c_im;
  o_re += kr * d_re - ki * d_im;
  o_im += kr * d_im + ki * d_re;
  power[k] = o_re * o_re + o_im * o_im;
  if (kk != k) {
    float p_re = c_re, p_im = -c_im;
    p_re += (-kr) * d_re - ki * (-d_im);
    p_im += (-kr) * (-d_im) + ki * d_re;
    power[kk] = p_re * p_re + p_im * p_im;
  }
}

CE_HD void post_power(int k, const float *re, const float *im, const float *kn, float *power) {
  post_power_ab(k, sw(bitrev8(k)), sw(bitrev8((256 - k) & 255)), re, im, kn[2 * k], kn[2 * k + 1], power);
}

// DC / Nyquist bins (src/srfft.cc:446-451 then fbank.cc:203-204).
CE_HD void edge_power(const float *re, const float *im, float *power) {
  const float z = re[sw(0)] + im[sw(0)], nyq = re[sw(0)] - im[sw(0)];
  power[0] = z * z;
  power[256] = nyq * nyq;
}

// Melbanks::Compute for one bin: sequential float dot (src/vector.cc:81-92).
CE_HD float mel_dot(const float *w, const float *p, int len) {
  float e = 0.0f;
  for (int i = 0; i < len; ++i) e += w[i] * p[i];
  return e;
}


}  // namespace fb
}  // namespace catears
