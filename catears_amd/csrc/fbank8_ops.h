// fbank8_ops.h -- per-lane program of the exact fbank kernel (kernels/fbank.hip):
// eight lanes per frame, eight frames per wave, the frame's 256-point complex
// FFT held in registers.  Shared verbatim by the device kernel and the CPU
// emulator in tests (tests/native/emu_fbank.cc), which runs the eight lanes
// of a frame one after another between the same synchronisation points and
// checks the result against the oracle bit for bit.
//
// The float operations are the reference's, in the reference's order
// (src/fbank.cc:44-100, 165-245; src/srfft.cc:124-265, 370-459); only the
// assignment of operations to lanes differs.  A split-radix DIF node of
// length m = 2^lg at `base` touches points base+n, +m/4, +m/2, +3m/4
// (n < m/4), and every node of length L starts at a multiple of L, so:
//   phase A: lane r owns the points p = r + 8j (j = 0..31).  Every op of the
//            nodes of length 256, 128, 64 and 32 touches points 8 apart or
//            more, all of one residue mod 8: 23 node ops per lane, no data
//            exchange;
//   phase B: after one transpose through LDS, lane q owns two aligned
//            16-point blocks; every remaining node (length 16, 8, 4, 2) lies
//            inside one block;
//   then the FFT output goes back to LDS, and the real-FFT post-pass, the
//   power spectrum and the mel dots read it from there.
// Compiled with -ffp-contract=off (no fused multiply-add, as the x86-64
// reference).
#pragma once

#include <stdint.h>

#include "fbank_ops.h"

// every loop over a lane's register arrays is unrolled (a rolled loop would
// index them at run time, which puts them in scratch memory)
#if defined(__HIPCC__)
#define CE_UNROLL _Pragma("unroll")
#define CE_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define CE_UNROLL
#define CE_SCHED_FENCE()
#endif

namespace catears {
namespace fb8 {

constexpr int kLanes = 8;    // lanes per frame
constexpr int kPts = 32;     // complex points per lane
constexpr int kSamp = 25;    // sample pairs per lane (400 samples / 8 lanes / 2)
// Floats per frame in LDS: 256 points + 8 (the phase A -> B transpose puts
// 4 floats of padding after point 127, tpos_a).  264 = 8 mod 32: the four
// frames of a 32-lane group start 8 banks apart, so the phase-A stores (8
// consecutive lanes of a frame) and the power-spectrum stores (8 lanes on 8
// consecutive bins) of a group fill the 32 banks exactly once
// (tools/fb_bank_model2.py).  Any value >= 260 that is a multiple of 4 gives
// the same bits (load_b and mel_window use 16-byte LDS accesses at
// region-relative offsets).
#ifndef FB8_STRIDE
#define FB8_STRIDE 264
#endif
constexpr int kStride = FB8_STRIDE;
static_assert(kStride % 4 == 0 && kStride >= 260, "frame regions: 16-byte aligned, room for 257 bins + padding");
constexpr int kOpsA = 23;    // phase-A node ops per lane
constexpr int kTwA = 8;      // floats per phase-A twiddle record (6 used)

// LDS: every address of the lane program is a per-lane base plus a
// compile-time offset, so the frame loop keeps no per-access address
// registers.  Bank spread comes from the lane -> point assignment instead.

// Phase-B blocks (16 points each) of lane q: the first is always an X block
// (a length-16 node and its subtree), the second a Y block (two length-8
// nodes) for q < 5 and an X block otherwise.  Of the 16 blocks, Y are
// 1, 5, 7, 9, 13: the second halves of the five length-32 nodes.  DIF block
// b holds the natural FFT indices k = 16 m + brev4(b) (the points of a block
// are one residue class r = brev4(b) mod 16), and the blocks are paired so
// that lane q holds the classes r and 16 - r (lane 0: 0 and 8): both
// operands of every real-FFT post-pass pair (k, 256 - k) then sit in the
// lane's own registers, and the post-pass needs no LDS exchange at all.
constexpr int kBlk1[kLanes] = {0, 4, 10, 6, 14, 8, 12, 2};
constexpr int kBlk2[kLanes] = {1, 7, 13, 5, 9, 15, 11, 3};
// the same tables as nibbles, for a run-time lane index (shift and mask
// instead of an indexed load): kBlk1, kBlk2 and the class brev4(kBlk1[q])
constexpr uint32_t kBlk1N = 0x2C8E6A40u, kBlk2N = 0x3BF95D71u, kClassN = 0x43176520u;
CE_HD int nib(uint32_t v, int q) { return (int)((v >> (4 * q)) & 15u); }
CE_HD bool second_is_x(int q) { return q >= 5; }

// Mel slots: lane q forms band mel_band(c, q) = 8c + perm_c(q) in slot c
// over a window of kMelW[c] bins starting at a multiple of 4 (weights zero
// outside the band, so the sum is the reference's sequential dot: 0 * p
// adds +0).  The permutations put the eight lanes' window starts on banks
// the four frames of a ds_read_b128 lane group share least: 92 extra passes
// per 8-frame group instead of 170 with perm_c(q) = q
// (tools/fb_bank_model2.py, exhaustive per slot).
constexpr int kMelSlots = 5;
constexpr int kMelW[kMelSlots] = {8, 12, 16, 24, 32};
constexpr int kMelWBase[kMelSlots] = {0, 8, 20, 36, 60};
constexpr int kMelWTot = 92;  // lane q's windows back to back at q * kMelWTot
constexpr uint32_t kMelPermN[kMelSlots] = {0x76543210u, 0x54327610u, 0x76534210u, 0x75316420u, 0x75436210u};
CE_HD int mel_band(int c, int q) { return 8 * c + (int)((kMelPermN[c] >> (4 * q)) & 15u); }

// ----------------------------------------------------------- node ops --

// step 1 + step 2 of a general node on points a b c d (srfft.cc:163-205)
CE_HD void node12(float &ar, float &ai, float &br, float &bi, float &cr, float &ci, float &dr, float &di) {
  float t1, t2;
  t1 = ar + cr; cr = ar - cr; ar = t1;
  t1 = ai + ci; ci = ai - ci; ai = t1;
  t1 = br + dr; dr = br - dr; br = t1;
  t1 = bi + di; di = bi - di; bi = t1;
  t1 = cr + di;
  t2 = ci + dr;
  ci = ci - dr;
  dr = cr - di;
  cr = t1;
  di = t2;
}

// steps 3 & 4, the n == m/8 rotation (srfft.cc:232-239)
CE_HD void node_sq(float &cr, float &ci, float &dr, float &di) {
  const float sq = (float)0.70710678118654752440;
  float t1 = sq * (cr + ci);
  ci = sq * (ci - cr);
  cr = t1;
  float t2 = sq * (di - dr);
  di = -sq * (dr + di);
  dr = t2;
}

// steps 3 & 4 from the tables (srfft.cc:240-249): tw = c, -(s+c), s-c for n
// and for 3n
CE_HD void node_tw(float &cr, float &ci, float &dr, float &di, const float *tw) {
  float t2 = tw[0] * (cr + ci);
  float t1 = tw[1] * cr + t2;
  cr = tw[2] * ci + t2;
  ci = t1;
  t2 = tw[3] * (dr + di);
  t1 = tw[4] * dr + t2;
  dr = tw[5] * di + t2;
  di = t1;
}

// One node op on register points J, J+D, J+2D, J+3D of a lane's arrays.
// Lane condition: z (n == 0: no twiddle), s (n == m/8: the rotation), else
// the table twiddles tw.  TW / Z / S: which of the three the op's lanes may
// take (compile time); a lane-dependent choice is made by selects, not
// branches, so the whole phase stays one straight-line block.
template <int J, int D, bool TW, bool Z, bool S>
CE_HD void node_op(float *re, float *im, bool z, bool s, const float *tw) {
  float ar = re[J], ai = im[J], br = re[J + D], bi = im[J + D];
  float cr = re[J + 2 * D], ci = im[J + 2 * D], dr = re[J + 3 * D], di = im[J + 3 * D];
  node12(ar, ai, br, bi, cr, ci, dr, di);
  float tcr = cr, tci = ci, tdr = dr, tdi = di;
  if (TW) node_tw(tcr, tci, tdr, tdi, tw);
  if (S) {
    float scr = cr, sci = ci, sdr = dr, sdi = di;
    node_sq(scr, sci, sdr, sdi);
    tcr = s ? scr : tcr, tci = s ? sci : tci, tdr = s ? sdr : tdr, tdi = s ? sdi : tdi;
  }
  if (Z && (TW || S)) {
    tcr = z ? cr : tcr, tci = z ? ci : tci, tdr = z ? dr : tdr, tdi = z ? di : tdi;
  }
  re[J] = ar; im[J] = ai; re[J + D] = br; im[J + D] = bi;
  re[J + 2 * D] = tcr; im[J + 2 * D] = tci; re[J + 3 * D] = tdr; im[J + 3 * D] = tdi;
}

// (a, b) butterfly (srfft.cc:206-216)
template <int J>
CE_HD void leaf2(float *re, float *im) {
  float t = re[J] + re[J + 1]; re[J + 1] = re[J] - re[J + 1]; re[J] = t;
  t = im[J] + im[J + 1]; im[J + 1] = im[J] - im[J + 1]; im[J] = t;
}

// length-4 node (srfft.cc:136-178): (0,2) (1,3) butterflies, (0,1)
// butterfly, (2,3) rotation
template <int J>
CE_HD void leaf4(float *re, float *im) {
  float ar = re[J], ai = im[J], br = re[J + 1], bi = im[J + 1];
  float cr = re[J + 2], ci = im[J + 2], dr = re[J + 3], di = im[J + 3];
  node12(ar, ai, br, bi, cr, ci, dr, di);
  float t = ar + br; br = ar - br; ar = t;
  t = ai + bi; bi = ai - bi; ai = t;
  re[J] = ar; im[J] = ai; re[J + 1] = br; im[J + 1] = bi;
  re[J + 2] = cr; im[J + 2] = ci; re[J + 3] = dr; im[J + 3] = di;
}

// length-8 node at J (n = 0: no twiddle, n = 1: the rotation)
template <int J>
CE_HD void node8(float *re, float *im) {
  node_op<J, 2, false, true, false>(re, im, true, false, nullptr);
  node_op<J + 1, 2, false, false, true>(re, im, false, true, nullptr);
}

// length-16 node at J: n = 0 none, 1 table, 2 rotation, 3 table (tw16 =
// the six twiddles of n = 1, then of n = 3)
template <int J>
CE_HD void node16(float *re, float *im, const float *tw16) {
  node_op<J, 4, false, true, false>(re, im, true, false, nullptr);
  node_op<J + 1, 4, true, false, false>(re, im, false, false, tw16);
  node_op<J + 2, 4, false, false, true>(re, im, false, true, nullptr);
  node_op<J + 3, 4, true, false, false>(re, im, false, false, tw16 + 6);
}

// ------------------------------------------------------------- phase A --

// Lane r's 23 node ops; twa = the lane's twiddle records (kTwA floats each,
// in op order; n == 0 and n == m/8 records unused).  Op order respects the
// recursion: a node's ops come after its parent's.
template <class TwFn>
CE_HD void phase_a(float *re, float *im, int r, TwFn tw) {
#ifdef FB8_NOCASE  // timing only (kernels/fbank_nocase.hip): every lane takes the table path
  (void)r;
  constexpr bool r0 = false, r4 = false;
#else
  const bool r0 = r == 0;
#endif
  // length 256 (m/8 = 32: n = r + 8i)
  node_op<0, 8, true, true, false>(re, im, r0, false, tw(0));
  CE_SCHED_FENCE();
  node_op<1, 8, true, false, false>(re, im, false, false, tw(1));
  CE_SCHED_FENCE();
  node_op<2, 8, true, false, false>(re, im, false, false, tw(2));
  CE_SCHED_FENCE();
  node_op<3, 8, true, false, false>(re, im, false, false, tw(3));
  CE_SCHED_FENCE();
  node_op<4, 8, true, false, true>(re, im, false, r0, tw(4));
  CE_SCHED_FENCE();
  node_op<5, 8, true, false, false>(re, im, false, false, tw(5));
  CE_SCHED_FENCE();
  node_op<6, 8, true, false, false>(re, im, false, false, tw(6));
  CE_SCHED_FENCE();
  node_op<7, 8, true, false, false>(re, im, false, false, tw(7));
  CE_SCHED_FENCE();
  // length 128 at 0 (m/8 = 16)
  node_op<0, 4, true, true, false>(re, im, r0, false, tw(8));
  CE_SCHED_FENCE();
  node_op<1, 4, true, false, false>(re, im, false, false, tw(9));
  CE_SCHED_FENCE();
  node_op<2, 4, true, false, true>(re, im, false, r0, tw(10));
  CE_SCHED_FENCE();
  node_op<3, 4, true, false, false>(re, im, false, false, tw(11));
  CE_SCHED_FENCE();
  // length 64 at 0, 128, 192 (m/8 = 8)
  node_op<0, 2, true, true, false>(re, im, r0, false, tw(12));
  CE_SCHED_FENCE();
  node_op<1, 2, true, false, true>(re, im, false, r0, tw(13));
  CE_SCHED_FENCE();
  node_op<16, 2, true, true, false>(re, im, r0, false, tw(14));
  CE_SCHED_FENCE();
  node_op<17, 2, true, false, true>(re, im, false, r0, tw(15));
  CE_SCHED_FENCE();
  node_op<24, 2, true, true, false>(re, im, r0, false, tw(16));
  CE_SCHED_FENCE();
  node_op<25, 2, true, false, true>(re, im, false, r0, tw(17));
  CE_SCHED_FENCE();
  // length 32 at 0, 64, 96, 128, 192 (m/8 = 4: n = r)
#ifndef FB8_NOCASE
  const bool r4 = r == 4;
#endif
  node_op<0, 1, true, true, true>(re, im, r0, r4, tw(18));
  CE_SCHED_FENCE();
  node_op<8, 1, true, true, true>(re, im, r0, r4, tw(19));
  CE_SCHED_FENCE();
  node_op<12, 1, true, true, true>(re, im, r0, r4, tw(20));
  CE_SCHED_FENCE();
  node_op<16, 1, true, true, true>(re, im, r0, r4, tw(21));
  CE_SCHED_FENCE();
  node_op<24, 1, true, true, true>(re, im, r0, r4, tw(22));
  CE_SCHED_FENCE();
}

// (lg, n) of lane r's phase-A op t -- for the host table builder
inline void phase_a_op(int t, int r, int *lg, int *n) {
  if (t < 8) *lg = 8, *n = r + 8 * t;
  else if (t < 12) *lg = 7, *n = r + 8 * (t - 8);
  else if (t < 18) *lg = 6, *n = r + 8 * ((t - 12) & 1);
  else *lg = 5, *n = r;
}

// ------------------------------------------------------------- phase B --

// Lane q's two blocks: re/im[0..15] block kBlk1[q] (X), [16..31] block
// kBlk2[q] (Y for q < 5, else X).  A length-16 node's children: a length-8
// node at 0 and length-4 nodes at 8 and 12; a length-8 node's: a length-4
// node at 0 and length-2 nodes at 4 and 6.
CE_HD void phase_b(float *re, float *im, int q, const float *tw16) {
  node16<0>(re, im, tw16);
  node8<0>(re, im);
  leaf4<0>(re, im);
  leaf2<4>(re, im);
  leaf2<6>(re, im);
  leaf4<8>(re, im);
  leaf4<12>(re, im);
  const bool x = second_is_x(q);
  if (x) node16<16>(re, im, tw16);
  node8<16>(re, im);
  if (!x) node8<24>(re, im);
  leaf4<16>(re, im);
  leaf2<20>(re, im);
  leaf2<22>(re, im);
  leaf4<24>(re, im);
  if (x) {
    leaf4<28>(re, im);
  } else {
    leaf2<28>(re, im);
    leaf2<30>(re, im);
  }
}

// point held in register j of lane q in phase B
CE_HD int phase_b_point(int q, int j) { return 16 * (j < 16 ? nib(kBlk1N, q) : nib(kBlk2N, q)) + (j & 15); }

// ------------------------------------------------ real-FFT post + power --

CE_HD int brev4(int v) { return ((v & 1) << 3) | ((v & 2) << 1) | ((v >> 1) & 2) | ((v >> 3) & 1); }

// power[k] and power[256 - k] from B_k = (xr, xi), B_{256-k} = (yr, yi)
// (srfft.cc:394-438 then fbank.cc:201-208); the float halving is exact, as
// the reference's 0.5 * (double) product rounded to float
CE_HD void post_pair(float xr, float xi, float yr, float yi, float kr, float ki, float *pk, float *pkk) {
  const float c_re = 0.5f * (xr + yr);
  const float c_im = 0.5f * (xi - yi);
  const float d_re = 0.5f * (xi + yi);
  const float d_im = -(0.5f * (xr - yr));
  float o_re = c_re, o_im = c_im;
  o_re += kr * d_re - ki * d_im;
  o_im += kr * d_im + ki * d_re;
  *pk = o_re * o_re + o_im * o_im;
  float p_re = c_re, p_im = -c_im;
  p_re += (-kr) * d_re - ki * (-d_im);
  p_im += (-kr) * (-d_im) + ki * d_re;
  *pkk = p_re * p_re + p_im * p_im;
}

// The real-FFT post-pass and power spectrum of lane q's sixteen pairs, from
// its phase-B registers (B_k of point p = 16 b + j in register j of its block)
// into pw[0..256] (the frame's LDS region, reused).  Slot t = 0..15, c =
// brev4(t):
//   c <= 7: k = A + 16 c (A = r, lane 0: 8), B_k in register t (lane 0:
//           16 + t), B_{256-k} in register 31 - t;
//   c >= 8: k = (16 - r) + 16 (15 - c), B_k in register 31 - t (lane 0:
//           brev4(16 - c)), B_{256-k} in register t.
// So k runs over 1..128 once per frame (lane 0 takes the classes 8 and 0,
// with k = 128 pairing with itself), always the reference's k <= 128 form
// of the pair; every LDS address is a per-lane base plus a constant; for a
// given slot the eight lanes store to eight consecutive bins.  The k = 128
// pair's second value is stored first and then overwritten by the first, as
// the reference's loop leaves it.  DC and Nyquist (B_0, lane 0) are the
// caller's.
CE_HD void post_regs(int q, const float *re, const float *im, const float *kn, float *pw) {
  const bool z = q == 0;
  const int r = nib(kClassN, q);
  const int a = z ? 8 : r;
  const float *ka = kn + 2 * a, *kc = kn + 2 * (16 - r);
  float *pa = pw + a, *pak = pw + (256 - 112) - a, *pc = pw + (16 - r), *pd = pw + r;
  CE_UNROLL
  for (int t = 0; t < 16; ++t) {
    const int c = brev4(t);
    float pk, pkk;
    if (c <= 7) {
      const float xr = z ? re[16 + t] : re[t], xi = z ? im[16 + t] : im[t];
      post_pair(xr, xi, re[31 - t], im[31 - t], ka[32 * c], ka[32 * c + 1], &pk, &pkk);
      pak[112 - 16 * c] = pkk;  // pw[256 - k]
      pa[16 * c] = pk;          // pw[k]
    } else {
      const int j0 = brev4((16 - c) & 15);
      const float xr = z ? re[j0] : re[31 - t], xi = z ? im[j0] : im[31 - t];
      post_pair(xr, xi, re[t], im[t], kc[32 * (15 - c)], kc[32 * (15 - c) + 1], &pk, &pkk);
      pd[16 * c] = pkk;         // pw[256 - k]
      pc[16 * (15 - c)] = pk;   // pw[k]
    }
    if (t % 4 == 3) CE_SCHED_FENCE();
  }
}

// ------------------------------------------------ samples, DC, window --

// Lane r's samples of a frame: pairs (16j + 2r, 16j + 2r + 1), j = 0..24.
// lane_sum returns the lane's partial sum, exact for integer-valued PCM
// (every partial sum of <= 400 int16 values is an integer below 2^24), so
// the frame sum does not depend on the order the lanes combine it in.
template <typename Sample>
CE_HD float lane_sum(const Sample *src, int r) {
  float part = 0.0f;
  CE_UNROLL
  for (int j = 0; j < kSamp; ++j) {
    part += (float)src[16 * j + 2 * r];
    part += (float)src[16 * j + 2 * r + 1];
  }
  return part;
}

// DC removal, pre-emphasis (in double) and the Hamming window of lane r's
// samples (src/fbank.cc:48-71), packed as the complex points p = r + 8j:
// re = even sample 2p, im = odd sample 2p + 1 (srfft.cc:318-324); points
// 200..255 are the zero padding.  The samples are read again here (cache
// hits), each pair with the sample before it (the pre-emphasis neighbour; for
// sample 0 itself, as src/fbank.cc:61), so no lane holds all 75 at once.
template <typename Sample>
CE_HD void lane_window(const Sample *src, float mean, int r, const float *win, float *re, float *im) {
  CE_UNROLL
  for (int j = 0; j < kSamp; ++j) {
    const int e = 16 * j + 2 * r;
    const float de = (float)src[e] - mean, dod = (float)src[e + 1] - mean;
    const float dp = (float)src[e > 0 ? e - 1 : 0] - mean;
#ifdef FB8_FMA
    // fast mode: 0.97f and one fused rounding instead of the double product;
    // the loads in groups of five pairs (all 75 samples' loads hoisted ahead
    // took the kernel past 128 registers)
    re[j] = __builtin_fmaf(-0.97f, dp, de) * win[e];
    im[j] = __builtin_fmaf(-0.97f, de, dod) * win[e + 1];
    if (j % 5 == 4) CE_SCHED_FENCE();
#else
    re[j] = fb::preemph(de, dp) * win[e];
    im[j] = fb::preemph(dod, de) * win[e + 1];
#endif
  }
  CE_UNROLL
  for (int j = kSamp; j < kPts; ++j) re[j] = im[j] = 0.0f;
}

// ------------------------------------------------------- LDS exchanges --

// LDS position of FFT point p during the phase A -> B transpose: four
// floats of padding after point 127.  With the 264-float frame stride this
// gives the load_b reads 64 extra passes per 8-frame group instead of 96
// (tools/fb_bank_model2.py).  Points 0..255 -> 0..259.
CE_HD constexpr int tpos_a(int p) { return p + 4 * (p >> 7); }

// phase A -> LDS: lane r's point r + 8j from register j
CE_HD void store_a(const float *v, int r, float *fbuf) {
  CE_UNROLL
  for (int j = 0; j < kPts; ++j) fbuf[r + 8 * j + (j >= 16 ? 4 : 0)] = v[j];
}

// four floats at a 16-byte aligned LDS address (one ds_read/write_b128)
struct alignas(16) F4 {
  float x, y, z, w;
};

// LDS -> phase B registers: whole aligned groups of four points, block
// bases per lane (tpos_a's padding is a constant per block)
CE_HD void load_b(int q, const float *fbuf, float *v) {
  const int b1 = nib(kBlk1N, q), b2 = nib(kBlk2N, q);
  const float *s1 = fbuf + tpos_a(16 * b1), *s2 = fbuf + tpos_a(16 * b2);
  CE_UNROLL
  for (int j = 0; j < kPts; j += 4) {
    const F4 t = *reinterpret_cast<const F4 *>((j < 16 ? s1 : s2) + (j & 15));
    v[j] = t.x, v[j + 1] = t.y, v[j + 2] = t.z, v[j + 3] = t.w;
  }
}

// ------------------------------------------------------------------ mel --

// Lane q's band of slot c over its window: w = the slot's zero-padded
// weights, p = the power spectrum from the window's first bin.
template <int W>
CE_HD float mel_window(const float *w, const float *p) {
  float e = 0.0f;
  CE_UNROLL
  for (int i = 0; i < W; i += 4) {
    const F4 a = *reinterpret_cast<const F4 *>(w + i), b = *reinterpret_cast<const F4 *>(p + i);
    e += a.x * b.x;
    e += a.y * b.y;
    e += a.z * b.z;
    e += a.w * b.w;
    // (at most two quads' loads ahead of their products: hoisting every
    // window's loads would hold 184 values in registers)
    if (i % 8 == 4) CE_SCHED_FENCE();
  }
  return e;
}

}  // namespace fb8
}  // namespace catears
