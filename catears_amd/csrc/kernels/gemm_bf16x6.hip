// gemm_bf16x6.hip -- the TDNN layers' fp32 GEMM on the bf16 matrix cores.
//
// Same contraction as gemm_f32.hip (Splice + Narrow + LinearLayer + bias /
// ReLU / BatchNorm, src/nnet.cc:22-43,50-75,106-117,149-160,182-202;
// MatMat -> cblas_sgemm, src/matrix.cc:300-323), computed to fp32 accuracy
// with v_mfma_f32_16x16x32_bf16:
//
//   every fp32 operand x is stored as three bf16 planes x = x0 + x1 + x2
//   (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1); each
//   subtraction is exact, and 3 x 8 significand bits plus the signs cover
//   fp32's 24, so the split is exact for every normal fp32 value), and
//
//   w . x = w0x0 + w0x1 + w1x0 + w1x1 + w0x2 + w2x0  (+ w1x2 + w2x1 + w2x2)
//
// The six kept products are exact in the MFMA (8 x 8 significand bits) and
// accumulate in fp32; the three dropped ones are below 2^-25 |w x| each,
// under the 2^-24 rounding of a single fp32 multiply.  So the result is an
// fp32 GEMM with a different (blocked) summation order -- the same status as
// the fp32-MFMA kernel -- at 6 bf16 MFMAs per fp32 MAC block: the bf16 rate
// is 16x the fp32 MFMA rate on gfx950, i.e. 2.7x the fp32 ceiling.
//
// Layout (HBM):
//   weights  n x ldw bf16, row j = [plane0 | plane1 | plane2], plane stride pw
//            (= kpad, zero padded), uploaded once (capi.cc split_weights)
//   acts     rows x ldx bf16, row r = [plane0 | plane1 | plane2], stride px;
//            written split by the previous layer's epilogue (or by
//            splice_pad_split for the first layer)
//   output   split bf16 (a hidden layer) or fp32 (the last layer, which
//            finalize reads)
//
// The MFMA's A operand is the weights (M = output units), B the activations
// (N = frames): the accumulator then holds four consecutive units of one
// frame per lane, so the epilogue reads bias/BN as float4 and stores 8 bytes
// per plane (16 for fp32) per lane.
//
// Tiling: BW units x BF frames per block, K-tile 32 (one MFMA k-step, 64 B
// per row per plane), 4 waves of (BW/2) x (BF/2).  Operands travel global ->
// LDS by LDS-DMA (global_load_lds_dwordx4: one wave instruction = 16 rows x
// 64 B of one plane), STAGES-deep ring, one barrier per K-tile, counted
// vmcnt (same protocol as gemm_f32_glds_kernel).  Bank spread: 16-B chunk c
// of tile row r is stored at chunk c ^ (2 * ((r >> 3) & 1)), applied on the
// source address; each of ds_read_b128's four 16-lane groups ({0-3,12-15,
// 20-27}, {4-11,16-19,28-31}, +32) then hits 16 distinct bank slots
// (MI355X_MICROARCH.md, LDS; the plain (r >> 2) & 3 swizzle is 2-way there).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "../internal.h"
#include "../tile_order.h"

namespace catears {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct X6Args {
  const uint16_t *w;  // weights, n x ldw, plane stride pw (elements)
  const uint16_t *x;  // activations, rows x ldx, plane stride px
  const float *wf, *xf;  // or fp32 operands (gemm_bf16x6f_kernel; ldw / ldx in floats)
  const float *bias, *bn_scale, *bn_offset;
  float *y32;         // fp32 output (ldy floats per row), or
  uint16_t *y16;      // split output (ldy elements per row, plane stride py)
  int ldw, pw, ldx, px, ldy, py;
  int m, n, kpad, din;
  uint64_t off_packed;  // splice offset of segment s in signed byte s
  int post[4];
  int npost, post_mode;
  int tiles_m, tiles_n, group;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void glds16(const char *src, char *lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                   (__attribute__((address_space(3))) void *)lds_dst, 16, 0, 0);
}

__device__ __forceinline__ uint16_t bf16_bits(__bf16 b) { return __builtin_bit_cast(uint16_t, b); }

// v = h + m + l in bf16 (round-to-nearest-even at each step, v_cvt_pk_bf16_f32)
__device__ __forceinline__ void split3(float v, uint16_t *h, uint16_t *m, uint16_t *l) {
  const __bf16 b0 = (__bf16)v;
  const float r1 = v - (float)b0;
  const __bf16 b1 = (__bf16)r1;
  const float r2 = r1 - (float)b1;
  *h = bf16_bits(b0);
  *m = bf16_bits(b1);
  *l = bf16_bits((__bf16)r2);
}

// split3 for two values at once, packed (low half = a): one
// v_cvt_pk_bf16_f32 per plane, the bf16 -> f32 widenings as a shift / mask.
// Bit-identical to split3 on each value (the same RNE conversions and exact
// subtractions).
struct Planes2 {
  uint32_t h, m, l;
};
__device__ __forceinline__ Planes2 split3_pair(float a, float b) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  auto cvt = [](float x, float y) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2));
  };
  auto lo = [](uint32_t u) { return __builtin_bit_cast(float, u << 16); };
  auto hi = [](uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); };
  const uint32_t p0 = cvt(a, b);
  const float ra = a - lo(p0), rb = b - hi(p0);
  const uint32_t p1 = cvt(ra, rb);
  const float sa = ra - lo(p1), sb = rb - hi(p1);
  return Planes2{p0, p1, cvt(sa, sb)};
}

template <int BW_, int BF_, int WGW_, int WGF_, int STAGES_>
struct X6Cfg {
  static constexpr int BW = BW_, BF = BF_, WGW = WGW_, WGF = WGF_, STAGES = STAGES_;
  static constexpr int NW = WGW * WGF, NT = 64 * NW;
  static constexpr int TW = BW / WGW / 16, TF = BF / WGF / 16;  // 16 x 16 fragments per wave
  static constexpr int QW = 3 * BW / 16, QF = 3 * BF / 16;       // DMA instructions per stage
  static constexpr int NQW = QW / NW, NQF = QF / NW;
  static constexpr int NQM = (QW + QF) / NW;                      // pieces per wave, mixed
  static constexpr int STAGE = 3 * (BW + BF) * 64;                // bytes per stage
  static_assert(TW >= 1 && TF >= 1 && (QW + QF) % NW == 0, "bad bf16x6 tile");
  static_assert(STAGES == 2 || STAGES == 3, "2 or 3 LDS stages");
  static_assert(STAGES * STAGE <= 160 * 1024, "LDS");
};

// Epilogue: lane holds units n .. n+3 of frame f for each fragment pair.
// + bias, post chain in model order with the reference's roundings; an
// absent bias adds -0 (identity).  Requires n % 4 == 0 (host-checked).
template <int TW, int TF, bool OUT16>
__device__ __forceinline__ void x6_epilogue(const X6Args &p, const f32x4 (&acc)[TW][TF], int nw0, int fw0, int lane) {
  with_post_mode(p.post_mode, [&](auto M) {
#pragma unroll
    for (int i = 0; i < TW; ++i) {
      const int n = nw0 + i * 16 + 4 * (lane >> 4);
      if (n >= p.n) continue;
      const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
      const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
      const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        const int f = fw0 + j * 16 + (lane & 15);
        if (f >= p.m) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_post<decltype(M)::value>(acc[i][j][e] + bias[e], sc[e], of[e], p.post, p.npost);
        if constexpr (OUT16) {
          uint16_t h[4], m[4], l[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) split3(v[e], &h[e], &m[e], &l[e]);
          uint16_t *dst = p.y16 + (int64_t)f * p.ldy + n;
          typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
          *reinterpret_cast<u16x4 *>(dst) = u16x4{h[0], h[1], h[2], h[3]};
          *reinterpret_cast<u16x4 *>(dst + p.py) = u16x4{m[0], m[1], m[2], m[3]};
          *reinterpret_cast<u16x4 *>(dst + 2 * p.py) = u16x4{l[0], l[1], l[2], l[3]};
        } else {
          *reinterpret_cast<f32x4 *>(p.y32 + (int64_t)f * p.ldy + n) = v;
        }
      }
    }
  });
}

// DIAG (ablation builds, wrong results; not dispatched by the library -- the
// measurements they gave are recorded in DESIGN.md §8): 1 = DMAs and
// fragment reads without the MFMAs, 2 = fragment reads and MFMAs without the
// DMAs, 3/4 = DMA shape / L2-resident-tile ablations.
template <class C, bool OUT16, int DIAG = 0>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF;
  constexpr int NQW = C::NQW, NQF = C::NQF, STAGES = C::STAGES, STAGE = C::STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  if (DIAG == 4) tm = tn = 0;  // every block loads tile (0, 0): L2-resident operands
  const int f0 = tm * BF, n0 = tn * BW;

  // DMA lane geometry: lane -> (row lane/4 of the instruction's 16, chunk lane%4)
  // DIAG 3/4: the same bytes fetched as 8 rows x 128 B per instruction
  constexpr bool FULL = DIAG == 3 || DIAG == 4;
  const int lrow = FULL ? lane >> 3 : lane >> 2, lch = FULL ? lane & 7 : lane & 3;
  constexpr int RPQ = FULL ? 8 : 16;
  uint32_t woff[NQW];
#pragma unroll
  for (int i = 0; i < NQW; ++i) {
    const int q = wave * NQW + i, plane = q / (BW / 16), row = (q % (BW / 16)) * RPQ + lrow;
    woff[i] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + plane * p.pw + 8 * (lch ^ swz(row))) * 2);
  }
  uint32_t xoff[NQF];
  int cur_seg = -1;

  auto issue = [&](int kt) {
    const int k0 = FULL ? min(kt * 32, p.kpad - 64) : kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
      for (int i = 0; i < NQF; ++i) {
        const int q = wave * NQF + i, plane = q / (BF / 16), row = (q % (BF / 16)) * RPQ + lrow;
        const int src = clampi(f0 + row + shift, 0, p.m - 1);
        xoff[i] = (uint32_t)((src * p.ldx + plane * p.px + 8 * (lch ^ swz(row))) * 2);
      }
    }
    char *st = smem + (kt % STAGES) * STAGE;
    const char *wbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 2;
    const char *xbase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 2;
#pragma unroll
    for (int i = 0; i < NQW; ++i) glds16(wbase + woff[i], st + (wave * NQW + i) * 1024);
#pragma unroll
    for (int i = 0; i < NQF; ++i) glds16(xbase + xoff[i], st + 3 * BW * 64 + (wave * NQF + i) * 1024);
  };

  // fragment read: lane reads row (lane & 15) of the 16-row fragment, logical
  // chunk lane >> 4 (k = 8 (lane >> 4) .. +7), stored at chunk ^ swz(row)
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;

  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  const int ktiles = p.kpad / 32;
  if (DIAG != 2) issue(0);
  if (DIAG != 2 && STAGES == 3 && ktiles > 1) issue(1);
  for (int kt = 0; kt < ktiles; ++kt) {
    if (DIAG != 2 && STAGES == 3 && kt + 1 < ktiles)
      wait_vmcnt<NQW + NQF>();  // leave tile kt+1's DMAs in flight
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (DIAG != 2 && kt + STAGES - 1 < ktiles) issue(kt + STAGES - 1);
    const char *st = smem + (kt % STAGES) * STAGE;
    bf16x8 a[3][TW], b[3][TF];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < TW; ++i)
        a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
      for (int j = 0; j < TF; ++j)
        b[pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
    }
    if constexpr (DIAG == 1 || DIAG == 3 || DIAG == 4) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      u32x4 x = {0, 0, 0, 0};
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < TW; ++i) x ^= __builtin_bit_cast(u32x4, a[pl][i]);
#pragma unroll
        for (int j = 0; j < TF; ++j) x ^= __builtin_bit_cast(u32x4, b[pl][j]);
      }
      acc[0][0][0] += (float)((x[0] ^ x[1] ^ x[2] ^ x[3]) & 1u);
      continue;
    }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
      }
  }

  x6_epilogue<TW, TF, OUT16>(p, acc, n0 + wrow, f0 + frow, lane);
}

// Phased schedule (3 LDS stages): each K-tile's MFMAs run in three groups
// by the plane they first need -- w0x0 | w0x1 w1x0 w1x1 | w0x2 w2x0 -- and
// the fragment reads of the next plane are issued before each group, so LDS
// latency hides under MFMAs.  The one barrier per K-tile sits before the last
// group; after it the DMAs of tile kt+2 are issued and tile kt+1's plane-0
// fragments are read (into the other of two plane-0 register sets) under
// that group.
//   WAR: tile kt+2 goes to stage (kt-1) % 3, whose every read fed an MFMA
//   that each wave issued before this barrier.
//   RAW: tile kt+1 is read only after the barrier that follows every wave's
//   vmcnt(0) -- its DMAs, issued one tile earlier, are the only ones
//   outstanding there.
template <class C, bool OUT16, bool PRIO>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6p_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF;
  constexpr int NQW = C::NQW, NQF = C::NQF, STAGE = C::STAGE;
  static_assert(C::STAGES == 3, "the phased schedule needs three LDS stages");
  __shared__ __attribute__((aligned(1024))) char smem[3 * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;

  const int lrow = lane >> 2, lch = lane & 3;
  uint32_t woff[NQW];
#pragma unroll
  for (int i = 0; i < NQW; ++i) {
    const int q = wave * NQW + i, plane = q / (BW / 16), row = (q % (BW / 16)) * 16 + lrow;
    woff[i] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + plane * p.pw + 8 * (lch ^ swz(row))) * 2);
  }
  uint32_t xoff[NQF];
  int cur_seg = -1;
  auto issue = [&](int kt) {
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
      for (int i = 0; i < NQF; ++i) {
        const int q = wave * NQF + i, plane = q / (BF / 16), row = (q % (BF / 16)) * 16 + lrow;
        const int src = clampi(f0 + row + shift, 0, p.m - 1);
        xoff[i] = (uint32_t)((src * p.ldx + plane * p.px + 8 * (lch ^ swz(row))) * 2);
      }
    }
    char *st = smem + (kt % 3) * STAGE;
    const char *wbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 2;
    const char *xbase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 2;
#pragma unroll
    for (int i = 0; i < NQW; ++i) glds16(wbase + woff[i], st + (wave * NQW + i) * 1024);
#pragma unroll
    for (int i = 0; i < NQF; ++i) glds16(xbase + xoff[i], st + 3 * BW * 64 + (wave * NQF + i) * 1024);
  };

  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;
  auto rd = [&](const char *st, int pl, bf16x8 *a, bf16x8 *b) {
#pragma unroll
    for (int i = 0; i < TW; ++i) a[i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
    for (int j = 0; j < TF; ++j)
      b[j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
  };
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  auto mm = [&](const bf16x8 *a, const bf16x8 *b) {
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  };

  const int ktiles = p.kpad / 32;
  bf16x8 a0[2][TW], b0[2][TF], a1[TW], b1[TF], a2[TW], b2[TF];
  issue(0);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  if (ktiles > 1) issue(1);
  rd(smem, 0, a0[0], b0[0]);

  auto body = [&](int kt, auto cc) {
    constexpr int c = decltype(cc)::value;
    const char *st = smem + (kt % 3) * STAGE;
    rd(st, 1, a1, b1);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
    mm(a0[c], b0[c]);
    rd(st, 2, a2, b2);
    mm(a0[c], b1);
    mm(a1, b0[c]);
    mm(a1, b1);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < ktiles) {
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < ktiles) issue(kt + 2);
      rd(smem + ((kt + 1) % 3) * STAGE, 0, a0[c ^ 1], b0[c ^ 1]);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(1);
    mm(a0[c], b2);
    mm(a2, b0[c]);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  for (int kt = 0; kt < ktiles; kt += 2) {
    body(kt, std::integral_constant<int, 0>());
    if (kt + 1 < ktiles) body(kt + 1, std::integral_constant<int, 1>());
  }

  x6_epilogue<TW, TF, OUT16>(p, acc, n0 + wrow, f0 + frow, lane);
}

// Phased schedule, branch-free loop body.  Same three plane groups and LDS
// ring as gemm_bf16x6p_kernel, but every K-tile step runs the same
// straight-line code: the barrier, the DMA issue (clamped to the last tile:
// a dummy refetch into the free stage once the tail is reached) and the next
// tile's plane-0 fragment reads are unconditional, and the splice row
// offsets are recomputed per issue (no cached-segment branch).  One basic
// block per step lets the waitcnt pass count outstanding LDS reads exactly
// (lgkmcnt(N) instead of the lgkmcnt(0) a control-flow merge forces), so
// fragment reads of the next group stay in flight under this group's MFMAs.
// SCHED 1 additionally pins the last group's interleave: two MFMAs per DMA
// piece / fragment read.
template <class C, bool OUT16, int SCHED>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6q_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF;
  constexpr int STAGE = C::STAGE, NQ = C::NQM, QW = C::QW;
  constexpr int S = C::STAGES;  // 2 or 3
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;

  // DMA pieces: the stage's QW weight pieces then QF activation pieces (one
  // piece = 16 rows x 64 B of one plane, stored at stage + 1 KB * piece).
  // Balanced when both kinds divide over the waves (each wave NQW weight +
  // NQF activation pieces: measured faster than giving some waves only one
  // kind); otherwise wave w issues pieces w NQ .. w NQ + NQ - 1 (wave-uniform
  // selects, no branch).
  constexpr bool BAL = C::QW % C::NW == 0 && C::QF % C::NW == 0;
  const int lrow = lane >> 2, lch = lane & 3;
  bool isw[NQ];
  int piece[NQ];
  uint32_t pconst[NQ];  // weight: byte offset at K-tile 0; activation: plane / chunk offset
  int xrow[NQ];         // activation tile row
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    int q;
    if constexpr (BAL) {
      isw[i] = i < C::NQW;
      q = isw[i] ? wave * C::NQW + i : QW + wave * C::NQF + (i - C::NQW);
    } else {
      q = wave * NQ + i;
      isw[i] = q < QW;
    }
    piece[i] = q;
    if (isw[i]) {
      const int plane = q / (BW / 16), row = (q % (BW / 16)) * 16 + lrow;
      pconst[i] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + plane * p.pw + 8 * (lch ^ swz(row))) * 2);
      xrow[i] = 0;
    } else {
      const int q2 = q - QW, plane = q2 / (BF / 16), row = (q2 % (BF / 16)) * 16 + lrow;
      pconst[i] = (uint32_t)((plane * p.px + 8 * (lch ^ swz(row))) * 2);
      xrow[i] = f0 + row;
    }
  }
  const int ktiles = p.kpad / 32;
  auto issue = [&](int kt) {
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
    char *st = smem + (kt % S) * STAGE;
    const char *wbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 2;
    const char *xbase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 2;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const uint32_t xo = (uint32_t)(clampi(xrow[i] + shift, 0, p.m - 1) * p.ldx * 2) + pconst[i];
      const char *src = isw[i] ? wbase + pconst[i] : xbase + xo;
      glds16(src, st + piece[i] * 1024);
    }
  };
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;
  auto rd = [&](const char *st, int pl, bf16x8 *a, bf16x8 *b) {
#pragma unroll
    for (int i = 0; i < TW; ++i) a[i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
    for (int j = 0; j < TF; ++j)
      b[j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
  };
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  auto mm = [&](const bf16x8 *a, const bf16x8 *b) {
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  };

  bf16x8 a0[2][TW], b0[2][TF], a1[TW], b1[TF], a2[TW], b2[TF];
#pragma unroll
  for (int t = 0; t < S; ++t) issue(t);
  wait_vmcnt<(S - 1) * NQ>();
  __builtin_amdgcn_s_barrier();
  rd(smem, 0, a0[0], b0[0]);

  // Step kt reads stage kt % S: planes 1 and 2 before its barrier (plane 0
  // was read at the end of step kt-1), so once every wave has drained its
  // LDS reads (lgkmcnt(0)) and passed the barrier the stage is free and tile
  // kt+S is issued into it -- S-1 steps ahead of its first read.  RAW: tile
  // kt+1 is read (plane 0) right after the barrier; every wave's
  // vmcnt((S-2) NQ) before it retired all but the newest S-2 issues (tiles
  // kt+2 .. kt+S-1), i.e. tile kt+1.
  // In the last steps the issued tile is clamped to ktiles-1: a refetch of
  // the last tile into the stage it already occupies, writing the bytes it
  // holds, so any read of that stage sees the same values; it keeps one
  // issue per step, which the vmcnt count relies on.  The plane-0 read of
  // the nonexistent tile ktiles is never used.
  auto body = [&](int kt, auto cc) {
    constexpr int c = decltype(cc)::value;
    const char *st = smem + (kt % S) * STAGE;
    rd(st, 1, a1, b1);
    mm(a0[c], b0[c]);
    rd(st, 2, a2, b2);
    mm(a0[c], b1);
    mm(a1, b0[c]);
    mm(a1, b1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vmcnt<(S - 2) * NQ>();
    __builtin_amdgcn_s_barrier();
    issue(kt + S);
    rd(smem + ((kt + 1) % S) * STAGE, 0, a0[c ^ 1], b0[c ^ 1]);
    mm(a0[c], b2);
    mm(a2, b0[c]);
    if constexpr (SCHED == 1) {
      // the last group: 16 MFMAs; interleave the NQ DMA pieces and the
      // TW + TF plane-0 reads between them
#pragma unroll
      for (int g = 0; g < NQ; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      }
#pragma unroll
      for (int g = 0; g < TW + TF; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * TW * TF - NQ - TW - TF, 0);
    }
  };
  int kt = 0;
  for (; kt + 1 < ktiles; kt += 2) {
    body(kt, std::integral_constant<int, 0>());
    body(kt + 1, std::integral_constant<int, 1>());
  }
  if (kt < ktiles) body(kt, std::integral_constant<int, 0>());
  wait_vmcnt<0>();  // drain the tail refetches before the block ends

  x6_epilogue<TW, TF, OUT16>(p, acc, n0 + wrow, f0 + frow, lane);
}

// Staggered two-group schedule.  Each K-tile is three phases of 2 TW TF
// MFMAs (w0x0 + w0x1 | w1x0 + w1x1 | w0x2 + w2x0); a phase is
//   R: its fragment reads (+ up to half the wave's DMA pieces), barrier,
//   M: lgkmcnt(0), the MFMAs at raised priority, barrier.
// Waves 0-3 (group A) and 4-7 (group B, one of each per SIMD) run one
// section apart: B passes one extra barrier before its first phase (A one
// after its last), so while A multiplies B reads and issues DMAs and vice
// versa -- the two waves of a SIMD alternate between the MFMA pipe and the
// memory pipes instead of waiting on the same barrier for the same thing.
//
// Barrier instances (the joint prologue barrier = 0): A's phase q ends its R
// section at instance 2q+1 and its M section at 2q+2; B's at 2q+2 and 2q+3.
// A wave's reads of phase q are complete at the end of its M section
// (lgkmcnt(0) there).  K-tile j = phases 3j .. 3j+2, all reading stage j % 3.
//   WAR: stage (j-1) % 3 is last read in phase 3j-1, complete for A at
//        instance 6j, for B at 6j+1.  Its refill (tile j+2) is issued in the
//        R sections of phases 3j+1 and 3j+2, which start after instance
//        6j+2 (A) / 6j+3 (B).
//   RAW: tile j+1 is first read in phase 3j+3 (A: after instance 6j+6).
//        Every wave retires its own pieces of tile j+1 at the end of the R
//        section of phase 3j+2 (vmcnt: all but tile j+2's pieces), which is
//        instance 6j+5 (A) / 6j+6 (B): before A's read, and B reads after
//        6j+7.
// Tiles past the end are clamped to the last one (a refetch of identical
// bytes into the stage that holds it), so every step issues the same number
// of pieces, which the vmcnt count relies on.
template <class C, bool OUT16>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6z_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF;
  constexpr int STAGE = C::STAGE, NQ = C::NQM, QW = C::QW;
  static_assert(C::NW == 8 && C::STAGES == 3, "two groups of four waves, three stages");
  static_assert(C::QW % C::NW == 0 && C::QF % C::NW == 0, "balanced pieces");
  constexpr int NQ1 = (NQ + 1) / 2;  // pieces issued in phase 1, the rest in phase 2
  __shared__ __attribute__((aligned(1024))) char smem[3 * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool groupB = wave >= 4;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;

  const int lrow = lane >> 2, lch = lane & 3;
  bool isw[NQ];
  int piece[NQ];
  uint32_t pconst[NQ];
  int xrow[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    isw[i] = i < C::NQW;
    const int q = isw[i] ? wave * C::NQW + i : QW + wave * C::NQF + (i - C::NQW);
    piece[i] = q;
    if (isw[i]) {
      const int plane = q / (BW / 16), row = (q % (BW / 16)) * 16 + lrow;
      pconst[i] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + plane * p.pw + 8 * (lch ^ swz(row))) * 2);
      xrow[i] = 0;
    } else {
      const int q2 = q - QW, plane = q2 / (BF / 16), row = (q2 % (BF / 16)) * 16 + lrow;
      pconst[i] = (uint32_t)((plane * p.px + 8 * (lch ^ swz(row))) * 2);
      xrow[i] = f0 + row;
    }
  }
  const int ktiles = p.kpad / 32;
  // pieces lo .. hi-1 of tile kt (clamped)
  auto issue = [&](int kt, auto lo_c, auto hi_c) {
    constexpr int lo = decltype(lo_c)::value, hi = decltype(hi_c)::value;
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
    char *st = smem + (kt % 3) * STAGE;
    const char *wbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 2;
    const char *xbase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 2;
#pragma unroll
    for (int i = lo; i < hi; ++i) {
      const uint32_t xo = (uint32_t)(clampi(xrow[i] + shift, 0, p.m - 1) * p.ldx * 2) + pconst[i];
      const char *src = isw[i] ? wbase + pconst[i] : xbase + xo;
      glds16(src, st + piece[i] * 1024);
    }
  };

  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;
  auto rda = [&](const char *st, int pl, bf16x8 *a) {
#pragma unroll
    for (int i = 0; i < TW; ++i) a[i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
  };
  auto rdb = [&](const char *st, int pl, bf16x8 *b) {
#pragma unroll
    for (int j = 0; j < TF; ++j)
      b[j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
  };
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  auto mm = [&](const bf16x8 *a, const bf16x8 *b) {
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  };
  auto msect = [&](auto f) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    f();
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  bf16x8 a0[TW], a1[TW], a2[TW], b0[TF], b1[TF], b2[TF];
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, NQ1>;
  using I2 = std::integral_constant<int, NQ>;
  issue(0, I0(), I2());
  issue(1, I0(), I2());
  wait_vmcnt<NQ>();
  __builtin_amdgcn_s_barrier();           // instance 0
  if (groupB) __builtin_amdgcn_s_barrier();  // B: one section behind

  for (int kt = 0; kt < ktiles; ++kt) {
    const char *st = smem + (kt % 3) * STAGE;
    // phase 0: w0x0 + w0x1
    rda(st, 0, a0);
    rdb(st, 0, b0);
    rdb(st, 1, b1);
    __builtin_amdgcn_s_barrier();
    msect([&] { mm(a0, b0); mm(a0, b1); });
    // phase 1: w1x0 + w1x1; first half of tile kt+2's pieces
    rda(st, 1, a1);
    issue(kt + 2, I0(), I1());
    __builtin_amdgcn_s_barrier();
    msect([&] { mm(a1, b0); mm(a1, b1); });
    // phase 2: w0x2 + w2x0; the rest of tile kt+2, then retire tile kt+1
    rda(st, 2, a2);
    rdb(st, 2, b2);
    issue(kt + 2, I1(), I2());
    wait_vmcnt<NQ>();
    __builtin_amdgcn_s_barrier();
    msect([&] { mm(a0, b2); mm(a2, b0); });
  }
  if (!groupB) __builtin_amdgcn_s_barrier();  // A: match B's extra barrier
  wait_vmcnt<0>();

  x6_epilogue<TW, TF, OUT16>(p, acc, n0 + wrow, f0 + frow, lane);
}

// fp32-in schedule: operands stay fp32 in HBM (4 B per element instead of
// the planes' 6) and are split into the three bf16 planes on their way into
// LDS.  The split/plane kernels above are bound by the bytes the L2 can move
// into LDS (f16x3's 4 B per element runs at 6/4 of their fp32-FLOP rate with
// half the MFMA work), so the fill carries fp32 and the VALU pays for the
// split, interleaved with the MFMAs.  Per K-tile each thread loads 8
// consecutive floats of one weight row and of one activation row (one 128-B
// line per row across 4 threads; global_load_dwordx4 x 2), splits them with
// the same split3 as the epilogue (so the planes -- and the results -- are
// bit-identical to the plane path), and writes 16 B per plane with
// ds_write_b128 into the layout the fragment reads expect.  Two LDS stages,
// registers one tile ahead:
//   step kt: write tile kt+1 (loaded during step kt-1) into stage (kt+1) % 2,
//            load tile kt+2 into registers, fragment reads + MFMAs of stage
//            kt % 2, lgkmcnt(0), raw s_barrier (no vmcnt: the loads stay in
//            flight across it).
//   WAR: stage (kt+1) % 2 was read in step kt-1, whose reads all fed MFMAs
//        before that step's barrier.  RAW: the writes of tile kt+1 are
//        drained before step kt's barrier; step kt+1 reads after it.
// Tiles past the end are clamped to the last one (written to a stage no
// later step reads), so the body is one basic block.
// DIAG (ablation builds of the SCHED >= 4 loop, wrong results; timing only,
// DESIGN.md §8): bit 1 = no split (raw fp32 bits as the three planes),
// 2 = no global loads after the prologue, 4 = no MFMAs, 8 = no fragment
// reads after the first tile, 16 = no K-tile barrier, 32 = no plane writes
// after the prologue.
template <class C, int SCHED, int DIAG = 0>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6f_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT, STAGE = C::STAGE;
  constexpr int RPP = NT / 4;  // rows per pass (4 threads x 32 B per row)
  static_assert(BW % RPP == 0 && BF % RPP == 0, "rows per pass");
  constexpr int NPW = BW / RPP, NPX = BF / RPP;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;
  const int prow = tid >> 2, pch = tid & 3;

  typedef const __attribute__((address_space(1))) f32x4v gvec;
  uint32_t wsrc[NPW];  // float offset of this thread's weight row at k = 0
#pragma unroll
  for (int i = 0; i < NPW; ++i) wsrc[i] = (uint32_t)(min(n0 + prow + i * RPP, p.n - 1) * p.ldw + 8 * pch);
  const int ktiles = p.kpad / 32;
  f32x4v rw0[NPW], rw1[NPW], rx0[NPX], rx1[NPX];
  auto load = [&](int kt) {
    if constexpr ((DIAG & 2) != 0) {
      if (kt > 1) return;
    }
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
    gvec *wb = (gvec *)(p.wf + k0);
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      rw0[i] = wb[wsrc[i] / 4];
      rw1[i] = wb[wsrc[i] / 4 + 1];
    }
    gvec *xb = (gvec *)(p.xf + col0 + 8 * pch);
#pragma unroll
    for (int i = 0; i < NPX; ++i) {
      const int src = clampi(f0 + prow + i * RPP + shift, 0, p.m - 1);
      const uint32_t o = (uint32_t)(src * p.ldx) / 4;
      rx0[i] = xb[o];
      rx1[i] = xb[o + 1];
    }
  };
  // 8 floats -> three 16-B plane chunks at row r of the plane block `base`
  auto put = [&](char *base, int nrows, int r, f32x4v v0, f32x4v v1) {
    Planes2 q0, q1, q2, q3;
    if constexpr ((DIAG & 1) != 0) {
      auto raw = [](float a) { const uint32_t u = __builtin_bit_cast(uint32_t, a); return Planes2{u, u, u}; };
      q0 = raw(v0.x), q1 = raw(v0.z), q2 = raw(v1.x), q3 = raw(v1.z);
    } else {
      q0 = split3_pair(v0.x, v0.y), q1 = split3_pair(v0.z, v0.w);
      q2 = split3_pair(v1.x, v1.y), q3 = split3_pair(v1.z, v1.w);
    }
    const int off = r * 64 + ((pch ^ swz(r)) * 16);
    *reinterpret_cast<u32x4 *>(base + off) = u32x4{q0.h, q1.h, q2.h, q3.h};
    *reinterpret_cast<u32x4 *>(base + nrows * 64 + off) = u32x4{q0.m, q1.m, q2.m, q3.m};
    *reinterpret_cast<u32x4 *>(base + 2 * nrows * 64 + off) = u32x4{q0.l, q1.l, q2.l, q3.l};
  };
  auto store = [&](int kt) {
    if constexpr ((DIAG & 32) != 0) {
      if (kt > 1) return;
    }
    char *st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < NPW; ++i) put(st, BW, prow + i * RPP, rw0[i], rw1[i]);
#pragma unroll
    for (int i = 0; i < NPX; ++i) put(st + 3 * BW * 64, BF, prow + i * RPP, rx0[i], rx1[i]);
  };

  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  load(0);
  store(0);
  load(1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (SCHED >= 4) {
    // Staggered roles: each SIMD holds one wave of each half of the block
    // (waves w and w + NW/2).  After the K-tile barrier the first half
    // splits tile kt+1 into LDS (VALU + ds_write) and then runs the MFMAs of
    // tile kt; the second half runs its MFMAs first and splits afterwards.
    // So on every SIMD one wave's split VALU issues in the gaps of its
    // partner's MFMAs, instead of both waves splitting at once with the
    // matrix pipe idle (the SCHED 0 loop: one phase for all waves).  Same
    // barrier count and LDS protocol:
    //   WAR: stage (kt+1) % 2 was last read in tile kt-1, before the
    //        barrier that closed it;
    //   RAW: every wave's writes of stage kt+1 precede the barrier that
    //        closes tile kt.
    bf16x8 a[3][TW], b[3][TF];
    auto mfma_tile = [&](int kt) {
      const char *st = smem + (kt & 1) * STAGE;
      if ((DIAG & 8) == 0 || kt == 0) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < TW; ++i)
            a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
          for (int j = 0; j < TF; ++j)
            b[pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
        }
      }
      if constexpr ((DIAG & 4) != 0) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
          for (int i = 0; i < TW; ++i) asm volatile("" ::"v"(a[pl][i]));
#pragma unroll
          for (int j = 0; j < TF; ++j) asm volatile("" ::"v"(b[pl][j]));
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
        }
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
        }
    };
    if constexpr (SCHED == 8) {
      // Region-scheduled loop (sched_barrier between regions; the compiler
      // interleaves inside each): plane 0 and 1 fragment reads + the 16
      // plane-0 MFMAs + the weight-row split of tile kt+1 and the weight
      // loads of tile kt+2 | half the plane-1 MFMAs + activation row 0's
      // split and loads | the other half + row 1 + plane-2 reads | the 32
      // plane-2 MFMAs.  Each load is issued as soon as the split has freed
      // its registers, about one iteration before its data is split.
      static_assert(NPW == 1 && NPX == 2 && TW % 2 == 0, "SCHED 8 geometry");
      auto read_plane = [&](const char *st, int pl) {
#pragma unroll
        for (int i = 0; i < TW; ++i)
          a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
        for (int j = 0; j < TF; ++j)
          b[pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
      };
      auto kpos = [&](int kt, int *k0, int *col0, int *shift) {
        kt = min(kt, ktiles - 1);
        *k0 = kt * 32;
        const int seg = *k0 / p.din;
        *col0 = *k0 - seg * p.din;
        *shift = (int)(signed char)(p.off_packed >> (8 * seg));
      };
      auto load_w = [&](int kt) {
        int k0, col0, shift;
        kpos(kt, &k0, &col0, &shift);
        gvec *wb = (gvec *)(p.wf + k0);
        rw0[0] = wb[wsrc[0] / 4];
        rw1[0] = wb[wsrc[0] / 4 + 1];
      };
      auto load_x = [&](int kt, int i) {
        int k0, col0, shift;
        kpos(kt, &k0, &col0, &shift);
        gvec *xb = (gvec *)(p.xf + col0 + 8 * pch);
        const int src = clampi(f0 + prow + i * RPP + shift, 0, p.m - 1);
        const uint32_t o = (uint32_t)(src * p.ldx) / 4;
        rx0[i] = xb[o];
        rx1[i] = xb[o + 1];
      };
      for (int kt = 0; kt < ktiles; ++kt) {
        const char *st = smem + (kt & 1) * STAGE;
        char *sn = smem + ((kt + 1) & 1) * STAGE;
        read_plane(st, 0);
        read_plane(st, 1);
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
          for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        put(sn, BW, prow, rw0[0], rw1[0]);
        load_w(kt + 2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int i = h * TW / 2; i < (h + 1) * TW / 2; ++i)
#pragma unroll
            for (int j = 0; j < TF; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
            }
          put(sn + 3 * BW * 64, BF, prow + h * RPP, rx0[h], rx1[h]);
          load_x(kt + 2, h);
          if (h == 1) read_plane(st, 2);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < TW; ++i)
#pragma unroll
          for (int j = 0; j < TF; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      x6_epilogue<TW, TF, false>(p, acc, n0 + wrow, f0 + frow, lane);
      return;
    }
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    // SCHED 6: every wave in the second half's order (MFMAs of tile kt,
    // then the split of tile kt+1, which the compiler interleaves into the
    // MFMA stream)
    if (SCHED >= 6 || wv >= C::NW / 2) {
      if constexpr (SCHED == 5) __builtin_amdgcn_s_setprio(1);
      for (int kt = 0; kt < ktiles; ++kt) {
        mfma_tile(kt);
        store(kt + 1);
        load(kt + 2);
        if constexpr (SCHED == 7) {
          // explicit interleave: the split of tile kt+1 in the first third
          // of the MFMA stream, then the loads of tile kt+2 (so they have
          // two thirds of this iteration and the next barrier to land), then
          // the plane writes; fragment reads of planes 1 / 2 spread early
          constexpr int NMM = 6 * TW * TF, NRD = 3 * (TW + TF), NR0 = TW + TF;
          constexpr int NV = 5, NSPL = NMM / 3;
          __builtin_amdgcn_sched_group_barrier(0x100, NR0, 0);
#pragma unroll
          for (int g = 0; g < NSPL; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
            if (g % 2 == 0 && g / 2 < NRD - NR0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x020, 2 * (NPW + NPX), 0);
#pragma unroll
          for (int g = 0; g < 3 * (NPW + NPX); ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, NMM - NSPL - 3 * (NPW + NPX), 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr ((DIAG & 16) == 0) __builtin_amdgcn_s_barrier();
      }
    } else {
      for (int kt = 0; kt < ktiles; ++kt) {
        store(kt + 1);
        load(kt + 2);
        mfma_tile(kt);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x6_epilogue<TW, TF, false>(p, acc, n0 + wrow, f0 + frow, lane);
    return;
  }
  for (int kt = 0; kt < ktiles; ++kt) {
    store(kt + 1);
    load(kt + 2);
    const char *st = smem + (kt & 1) * STAGE;
    bf16x8 a[3][TW], b[3][TF];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < TW; ++i)
        a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
      for (int j = 0; j < TF; ++j)
        b[pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
    }
    if constexpr (SCHED == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
      }
    if constexpr (SCHED == 3) __builtin_amdgcn_s_setprio(0);
    if constexpr (SCHED == 2) {
      // all fragment reads of stage kt first, so their latency hides under
      // the split of tile kt+1 (VALU + plane writes) and the next loads;
      // then the MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * (TW + TF), 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 512, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 3 * (NPW + NPX), 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 2 * (NPW + NPX), 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 6 * TW * TF, 0);
    }
    if constexpr (SCHED == 1) {
      // interleave: plane-0 fragment reads first, then one MFMA per step
      // with two VALU (the split of tile kt+1) and the remaining fragment
      // reads / plane writes / next loads spread between the MFMAs
      constexpr int NFR = TW + TF, NMM = 6 * TW * TF;
      __builtin_amdgcn_sched_group_barrier(0x100, NFR, 0);
#pragma unroll
      for (int g = 0; g < NMM / 2; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        if (g < 2 * NFR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        else if (g < 2 * NFR + 3 * (NPW + NPX)) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        else if (g < 2 * NFR + 3 * (NPW + NPX) + 2 * (NPW + NPX)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NMM / 2, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  x6_epilogue<TW, TF, false>(p, acc, n0 + wrow, f0 + frow, lane);
}

// Weights in LDS, activations in registers (gemm_bf16x6w_kernel).  The
// block's 8 waves all span the tile's BW units and split its BF frames (BF/8
// per wave), so each activation element feeds exactly one wave: the wave
// loads its own rows straight into registers in the MFMA B-operand layout
// (lane l: frame l % 16, k = 8 (l / 16) .. +8 -- 32 contiguous bytes of one
// row, one 128-B line per row over 4 lanes) and splits them into the three
// bf16 planes in registers.  Only the weight planes go through LDS (written
// once per block, read by all 8 waves), so the LDS write traffic per K-tile
// drops from (BW + BF) to BW rows x 192 B: the plane writes were the largest
// single overhead of the fp32-operand kernel (ablation: -21 % time without
// them).  Same split, same products, same accumulation order
// per output as gemm_bf16x6f_kernel: bit-identical results.
template <int BW_, int BF_, int NW_>
struct X6WCfg {
  static constexpr int BW = BW_, BF = BF_, NW = NW_, NT = 64 * NW;
  static constexpr int TW = BW / 16, TF = BF / NW / 16;  // 16 x 16 fragments per wave
  static constexpr int STAGE = 3 * BW * 64;               // weight planes per K-tile (bytes)
  static constexpr int RPP = NT / 4;                      // weight rows per pass
  static constexpr int NPW = BW / RPP < 1 ? 1 : BW / RPP;
  static_assert(TF >= 1 && BF % (NW * 16) == 0, "bad X6W tile");
};

template <class C, int SCHED>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6w_kernel(X6Args p) {
  constexpr int BW = C::BW, TW = C::TW, TF = C::TF, NPW = C::NPW, RPP = C::RPP, STAGE = C::STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4v gvec;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * C::BF, n0 = tn * BW;
  const int prow = tid >> 2, pch = tid & 3;
  const bool wload = BW >= RPP || prow < BW;  // threads that stage weight rows
  const int ktiles = p.kpad / 32;

  uint32_t wsrc[NPW];  // float offset of this thread's weight row at k = 0
#pragma unroll
  for (int i = 0; i < NPW; ++i) wsrc[i] = (uint32_t)(min(n0 + min(prow + i * RPP, BW - 1), p.n - 1) * p.ldw + 8 * pch);
  const int fw = f0 + wave * (TF * 16);  // this wave's first frame
  const int kq = (lane >> 4) * 8;
  f32x4v rw0[NPW], rw1[NPW], rx0[TF], rx1[TF];

  auto load_w = [&](int kt) {
    kt = min(kt, ktiles - 1);
    gvec *wb = (gvec *)(p.wf + kt * 32);
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      rw0[i] = wb[wsrc[i] / 4];
      rw1[i] = wb[wsrc[i] / 4 + 1];
    }
  };
  auto load_x = [&](int kt) {
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
    gvec *xb = (gvec *)(p.xf + col0 + kq);
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const int src = clampi(fw + j * 16 + (lane & 15) + shift, 0, p.m - 1);
      const uint32_t o = (uint32_t)(src * p.ldx) / 4;
      rx0[j] = xb[o];
      rx1[j] = xb[o + 1];
    }
  };
  auto put_w = [&](int kt) {
    if (!wload) return;
    char *st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int r = prow + i * RPP;
      const Planes2 q0 = split3_pair(rw0[i].x, rw0[i].y), q1 = split3_pair(rw0[i].z, rw0[i].w);
      const Planes2 q2 = split3_pair(rw1[i].x, rw1[i].y), q3 = split3_pair(rw1[i].z, rw1[i].w);
      const int off = r * 64 + ((pch ^ swz(r)) * 16);
      *reinterpret_cast<u32x4 *>(st + off) = u32x4{q0.h, q1.h, q2.h, q3.h};
      *reinterpret_cast<u32x4 *>(st + BW * 64 + off) = u32x4{q0.m, q1.m, q2.m, q3.m};
      *reinterpret_cast<u32x4 *>(st + 2 * BW * 64 + off) = u32x4{q0.l, q1.l, q2.l, q3.l};
    }
  };
  auto split_x = [&](bf16x8 (&b)[3][TF]) {
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const Planes2 q0 = split3_pair(rx0[j].x, rx0[j].y), q1 = split3_pair(rx0[j].z, rx0[j].w);
      const Planes2 q2 = split3_pair(rx1[j].x, rx1[j].y), q3 = split3_pair(rx1[j].z, rx1[j].w);
      b[0][j] = __builtin_bit_cast(bf16x8, (u32x4{q0.h, q1.h, q2.h, q3.h}));
      b[1][j] = __builtin_bit_cast(bf16x8, (u32x4{q0.m, q1.m, q2.m, q3.m}));
      b[2][j] = __builtin_bit_cast(bf16x8, (u32x4{q0.l, q1.l, q2.l, q3.l}));
    }
  };

  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  if constexpr (SCHED == 1) {
    // activations split one K-tile ahead (b planes double-buffered in
    // registers): the split of tile kt+1 and the loads of tile kt+2 run
    // under the MFMAs of tile kt; the loop is unrolled by two so the two
    // plane sets alternate without register copies
    bf16x8 bA[3][TF], bB[3][TF];
    load_w(0);
    load_x(0);
    put_w(0);
    load_w(1);
    split_x(bA);
    load_x(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    auto step = [&](int kt, bf16x8 (&b)[3][TF], bf16x8 (&bn)[3][TF]) {
      const char *st = smem + (kt & 1) * STAGE;
      bf16x8 a[3][TW];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int i = 0; i < TW; ++i) a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + i * 16) * 64 + foff);
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
        }
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
        }
      split_x(bn);
      load_x(kt + 2);
      put_w(kt + 1);
      load_w(kt + 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    int kt = 0;
    for (; kt + 1 < ktiles; kt += 2) {
      step(kt, bA, bB);
      step(kt + 1, bB, bA);
    }
    if (kt < ktiles) step(kt, bA, bB);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x6_epilogue<TW, TF, false>(p, acc, n0, fw, lane);
    return;
  }
  load_w(0);
  load_x(0);
  put_w(0);
  load_w(1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < ktiles; ++kt) {
    const char *st = smem + (kt & 1) * STAGE;
    bf16x8 a[3][TW], b[3][TF];
    split_x(b);
    load_x(kt + 1);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int i = 0; i < TW; ++i) a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + i * 16) * 64 + foff);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
      }
    put_w(kt + 1);
    load_w(kt + 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x6_epilogue<TW, TF, false>(p, acc, n0, fw, lane);
}

// Weight planes by LDS-DMA, activations in registers (gemm_bf16x6v_kernel):
// the X6W geometry, but the weights arrive as the load-time bf16 planes
// (GemmLayer::wsplit, n x 3 kpad) by global_load_lds into a 4-stage ring
// issued three K-tiles ahead -- no VGPRs, no VALU, no ds_write for them --
// and every wave's activation rows are loaded two K-tiles ahead into a
// register double buffer and split in registers.  One barrier per K-tile,
// at its top: this wave's pieces of tile kt and its rows of tile kt have
// landed (counted vmcnt), so after the barrier every wave's have, and every
// wave has finished reading the stage the next DMA overwrites.
// Same products and accumulation order: bit-identical to the other kernels.
template <class C>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6v_kernel(X6Args p) {
  constexpr int BW = C::BW, TW = C::TW, TF = C::TF, NW = C::NW, STAGE = C::STAGE;
  constexpr int NS = 4;                    // weight stages (DMA three K-tiles ahead)
  constexpr int PIECES = 3 * (BW / 16);    // 1-KB DMA pieces per K-tile (16 rows x 64 B of one plane)
  constexpr int PPW = PIECES / NW;         // pieces per wave
  constexpr int XOPS = 2 * TF;             // activation loads per lane and K-tile
  static_assert(PIECES % NW == 0, "pieces per wave");
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4v gvec;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * C::BF, n0 = tn * BW;
  const int ktiles = p.kpad / 32;
  const int fw = f0 + wave * (TF * 16);
  const int kq = (lane >> 4) * 8;

  // this lane's source byte offset (at k = 0) and LDS offset for each of its
  // wave's DMA pieces; chunk swizzle c ^ 2((r >> 3) & 1) on the source side
  uint32_t dsrc[PPW];
  int ddst[PPW];
#pragma unroll
  for (int t = 0; t < PPW; ++t) {
    const int q = wave * PPW + t, plane = q / (BW / 16), rg = q % (BW / 16);
    const int row = rg * 16 + (lane >> 2), chunk = (lane & 3) ^ (((row >> 3) & 1) << 1);
    dsrc[t] = (uint32_t)((min(n0 + row, p.n - 1) * 3 * p.pw + plane * p.pw + chunk * 8) * 2);
    ddst[t] = (plane * BW + rg * 16) * 64;
  }
  auto dma_w = [&](int kt) {
    const int kc = min(kt, ktiles - 1);
    char *st = smem + (kt % NS) * STAGE;
    const char *wb = reinterpret_cast<const char *>(p.w) + kc * 64;
#pragma unroll
    for (int t = 0; t < PPW; ++t) glds16(wb + dsrc[t], st + ddst[t]);
  };
  const int din = p.din, mlast = p.m - 1, ldx = p.ldx;
  const uint64_t offs = p.off_packed;
  const float *xf = p.xf;
  auto load_x = [&](int kt, f32x4v (&r0)[TF], f32x4v (&r1)[TF]) {
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / din, col0 = k0 - seg * din;
    const int shift = (int)(signed char)(offs >> (8 * seg));
    gvec *xb = (gvec *)(xf + col0 + kq);
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const int src = clampi(fw + j * 16 + (lane & 15) + shift, 0, mlast);
      const uint32_t o = (uint32_t)(src * ldx) / 4;
      r0[j] = xb[o];
      r1[j] = xb[o + 1];
    }
  };
  auto split_x = [&](const f32x4v (&r0)[TF], const f32x4v (&r1)[TF], bf16x8 (&b)[3][TF]) {
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const Planes2 q0 = split3_pair(r0[j].x, r0[j].y), q1 = split3_pair(r0[j].z, r0[j].w);
      const Planes2 q2 = split3_pair(r1[j].x, r1[j].y), q3 = split3_pair(r1[j].z, r1[j].w);
      b[0][j] = __builtin_bit_cast(bf16x8, (u32x4{q0.h, q1.h, q2.h, q3.h}));
      b[1][j] = __builtin_bit_cast(bf16x8, (u32x4{q0.m, q1.m, q2.m, q3.m}));
      b[2][j] = __builtin_bit_cast(bf16x8, (u32x4{q0.l, q1.l, q2.l, q3.l}));
    }
  };

  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  f32x4v xa0[TF], xa1[TF], xb0[TF], xb1[TF];
  // issue order DMA(0) DMA(1) X(0) DMA(2) X(1), then per step DMA(kt+3)
  // X(kt+2): before every step the ops issued after X(kt) are one DMA group
  // and one row group, so one counted wait covers W(kt) and X(kt)
  dma_w(0);
  dma_w(1);
  load_x(0, xa0, xa1);
  dma_w(2);
  load_x(1, xb0, xb1);
  auto step = [&](int kt, f32x4v (&r0)[TF], f32x4v (&r1)[TF]) {
    wait_vmcnt<PPW + XOPS>();
    __builtin_amdgcn_s_barrier();
    bf16x8 b[3][TF];
    split_x(r0, r1, b);
    // keep the DMA issue behind the split (the compiler would hoist it and
    // then wait for it with vmcnt(0) before the split)
    __builtin_amdgcn_sched_barrier(0);
    dma_w(kt + 3);
    load_x(kt + 2, r0, r1);
    const char *st = smem + (kt % NS) * STAGE;
    bf16x8 a[3][TW];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int i = 0; i < TW; ++i) a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + i * 16) * 64 + foff);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
      }
  };
  int kt = 0;
  for (; kt + 1 < ktiles; kt += 2) {
    step(kt, xa0, xa1);
    step(kt + 1, xb0, xb1);
  }
  if (kt < ktiles) step(kt, xa0, xa1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x6_epilogue<TW, TF, false>(p, acc, n0, fw, lane);
}

// Register-staged schedule: operands travel global -> VGPR (plain
// global_load_dwordx4) -> LDS (ds_write_b128) instead of LDS-DMA.  An LDS-DMA
// piece costs its wave 60-185 issue cycles (MI355X_MICROARCH.md, constants
// table), which with 48 pieces per K-tile per CU is of the order of the
// K-tile's MFMA time itself; a plain load + LDS write is a few issue slots.
// Two LDS stages; tile kt+1 is loaded into registers while tile kt is
// computed, written to the other stage after it, one barrier per K-tile:
//   WAR: stage (kt+1) % 2 was last read in tile kt-1, before the barrier
//        that closed it;
//   RAW: the barrier after the writes.
template <class C, bool OUT16>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6r_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT;
  constexpr int STAGE = C::STAGE;
  constexpr int CHUNKS = 3 * (BW + BF) * 4;  // 16-B chunks per stage
  static_assert(CHUNKS % NT == 0, "chunks per thread");
  constexpr int NC = CHUNKS / NT;
  constexpr int NCW = 3 * BW * 4 / NT;       // of which weight chunks (whole per thread)
  static_assert((3 * BW * 4) % NT == 0, "weight chunks per thread");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;

  // thread -> chunks tid + i NT: row q / 4 of the stage (3 BW weight rows,
  // plane-major, then 3 BF activation rows), chunk q % 4
  uint32_t goff[NC];  // byte offset in the operand, K-tile 0, segment 0
  uint32_t soff[NC];  // byte offset in the stage
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int q = tid + i * NT, row = q >> 2, ch = q & 3;
    soff[i] = row * 64 + ((ch ^ swz(row)) * 16);
    if (i < NCW) {
      const int plane = row / BW, r = row % BW;
      goff[i] = (uint32_t)((min(n0 + r, p.n - 1) * p.ldw + plane * p.pw + 8 * ch) * 2);
    }
  }
  uint32_t xoff[NC - NCW];
  int cur_seg = -1;
  u32x4 stg[NC];
  auto load = [&](int kt) {
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
      for (int i = NCW; i < NC; ++i) {
        const int q = tid + i * NT, row = (q >> 2) - 3 * BW, ch = q & 3;
        const int plane = row / BF, r = row % BF;
        const int src = clampi(f0 + r + shift, 0, p.m - 1);
        xoff[i - NCW] = (uint32_t)((src * p.ldx + plane * p.px + 8 * ch) * 2);
      }
    }
    const char *wbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 2;
    const char *xbase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 2;
#pragma unroll
    for (int i = 0; i < NCW; ++i) stg[i] = *reinterpret_cast<const u32x4 *>(wbase + goff[i]);
#pragma unroll
    for (int i = NCW; i < NC; ++i) stg[i] = *reinterpret_cast<const u32x4 *>(xbase + xoff[i - NCW]);
  };
  auto store = [&](int kt) {
    char *st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < NC; ++i) *reinterpret_cast<u32x4 *>(st + soff[i]) = stg[i];
  };

  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  const int ktiles = p.kpad / 32;
  load(0);
  store(0);
  if (ktiles > 1) load(1);
  __syncthreads();
  for (int kt = 0; kt < ktiles; ++kt) {
    const char *st = smem + (kt & 1) * STAGE;
    bf16x8 a[3][TW], b[3][TF];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < TW; ++i)
        a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 16) * 64 + foff);
#pragma unroll
      for (int j = 0; j < TF; ++j)
        b[pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 16) * 64 + foff);
    }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
      }
    if (kt + 1 < ktiles) {
      store(kt + 1);
      if (kt + 2 < ktiles) load(kt + 2);
      __syncthreads();
    }
  }

  x6_epilogue<TW, TF, OUT16>(p, acc, n0 + wrow, f0 + frow, lane);
}

// 32x32 schedule: the fp32-in kernel's data flow on v_mfma_f32_32x32x16_bf16.
// Why: a 16x16x32 MFMA holds its SIMD's instruction issue for 8 of its 16
// cycles, a 32x32x16 for 8 of its 32 (MI355X_MICROARCH.md, issue costs).
// With the split VALU (11 instructions per pair of operand values) and the
// LDS traffic of the in-kernel split, the 16x16 kernel's issue demand per
// SIMD is about its MFMA time, so the MFMA pipe idles half the time; the
// 32x32 shape frees 768 issue cycles per SIMD and K-tile at the same tile.
//
// Fragments (bf16): lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h ..
// 8h+7] and B[k = 8h ..][col r] -- 16 B of one 64-B LDS row per plane and
// k-substep s (chunk 2s + h).  Chunk c of tile row r is stored at
// c ^ ((r >> 2) & 3): each 16-lane group of ds_read_b128 ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, +32) then hits 16 distinct 16-B bank slots.
// Accumulator: col = frame l & 31, rows = units 8g + 4h + (0..3) in registers
// 4g .. 4g+3 -- the same "4 consecutive units of one frame" per register
// quad as the 16x16 epilogue.
// WPL: weights read as the three bf16 planes split at load time
// (GemmLayer::wsplit) instead of fp32 (no VALU for them; 6 B per element
// through L2 instead of 4).
template <int BW_, int BF_, int WGW_, int WGF_>
struct X6MCfg {
  static constexpr int BW = BW_, BF = BF_, WGW = WGW_, WGF = WGF_;
  static constexpr int NW = WGW * WGF, NT = 64 * NW;
  static constexpr int TW = BW / WGW / 32, TF = BF / WGF / 32;  // 32 x 32 blocks per wave
  static constexpr int STAGE = 3 * (BW + BF) * 64;
  static_assert(TW >= 1 && TF >= 1, "bad bf16x6m tile");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
};

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <class C, bool WPL>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6m_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT, STAGE = C::STAGE;
  constexpr int RPP = NT / 4;  // rows per pass (4 threads x 32 B of fp32, or x 16 B per plane)
  static_assert(BW % RPP == 0 && BF % RPP == 0 && RPP % 16 == 0, "rows per pass");
  constexpr int NPW = BW / RPP, NPX = BF / RPP;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;
  const int prow = tid >> 2, pch = tid & 3;
  // every row this thread writes has the same (row >> 2) & 3 (RPP % 16 == 0)
  const int soff = prow * 64 + ((pch ^ ((prow >> 2) & 3)) * 16);

  typedef const __attribute__((address_space(1))) f32x4v gvec;
  typedef const __attribute__((address_space(1))) u32x4 gvecu;
  uint32_t wsrc[NPW];  // element offset of this thread's weight row at k = 0
  const int ldw = WPL ? 3 * p.pw : p.ldw;  // plane rows: [plane0 | plane1 | plane2]
#pragma unroll
  for (int i = 0; i < NPW; ++i) wsrc[i] = (uint32_t)(min(n0 + prow + i * RPP, p.n - 1) * ldw + 8 * pch);
  const int ktiles = p.kpad / 32;
  f32x4v rw0[NPW], rw1[NPW], rx0[NPX], rx1[NPX];
  u32x4 rwp[WPL ? 3 * NPW : 1];
  auto load = [&](int kt) {
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
    if constexpr (WPL) {
      gvecu *wb = (gvecu *)(p.w + k0);
#pragma unroll
      for (int i = 0; i < NPW; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) rwp[3 * i + pl] = wb[(wsrc[i] + pl * p.pw) / 8];
    } else {
      gvec *wb = (gvec *)(p.wf + k0);
#pragma unroll
      for (int i = 0; i < NPW; ++i) {
        rw0[i] = wb[wsrc[i] / 4];
        rw1[i] = wb[wsrc[i] / 4 + 1];
      }
    }
    gvec *xb = (gvec *)(p.xf + col0 + 8 * pch);
#pragma unroll
    for (int i = 0; i < NPX; ++i) {
      const int src = clampi(f0 + prow + i * RPP + shift, 0, p.m - 1);
      const uint32_t o = (uint32_t)(src * p.ldx) / 4;
      rx0[i] = xb[o];
      rx1[i] = xb[o + 1];
    }
  };
  auto put = [&](char *base, int nrows, int r, f32x4v v0, f32x4v v1) {
    const Planes2 q0 = split3_pair(v0.x, v0.y), q1 = split3_pair(v0.z, v0.w);
    const Planes2 q2 = split3_pair(v1.x, v1.y), q3 = split3_pair(v1.z, v1.w);
    const int off = r * 64 + soff;
    *reinterpret_cast<u32x4 *>(base + off) = u32x4{q0.h, q1.h, q2.h, q3.h};
    *reinterpret_cast<u32x4 *>(base + nrows * 64 + off) = u32x4{q0.m, q1.m, q2.m, q3.m};
    *reinterpret_cast<u32x4 *>(base + 2 * nrows * 64 + off) = u32x4{q0.l, q1.l, q2.l, q3.l};
  };
  auto store = [&](int kt) {
    char *st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      if constexpr (WPL) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<u32x4 *>(st + (pl * BW + i * RPP) * 64 + soff) = rwp[3 * i + pl];
      } else {
        put(st, BW, i * RPP, rw0[i], rw1[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < NPX; ++i) put(st + 3 * BW * 64, BF, i * RPP, rx0[i], rx1[i]);
  };

  const int lr = lane & 31, lh = lane >> 5;
  const int foff0 = lr * 64 + (((0 + lh) ^ ((lr >> 2) & 3)) * 16);
  const int foff1 = lr * 64 + (((2 + lh) ^ ((lr >> 2) & 3)) * 16);
  const int wrow = ww * TW * 32, frow = wf * TF * 32;
  f32x16 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  load(0);
  store(0);
  load(1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < ktiles; ++kt) {
    store(kt + 1);
    load(kt + 2);
    const char *st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int foff = s ? foff1 : foff0;
      bf16x8 a[3][TW], b[3][TF];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < TW; ++i)
          a[pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * 32) * 64 + foff);
#pragma unroll
        for (int j = 0; j < TF; ++j)
          b[pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * 32) * 64 + foff);
      }
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: register quad g of block (i, j) = units 8g + 4h .. +3 of frame lr
  with_post_mode(p.post_mode, [&](auto M) {
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wrow + i * 32 + 8 * g + 4 * lh;
        if (n >= p.n) continue;
        const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
        const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
        const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          const int f = f0 + frow + j * 32 + lr;
          if (f >= p.m) continue;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = apply_post<decltype(M)::value>(acc[i][j][4 * g + e] + bias[e], sc[e], of[e], p.post, p.npost);
          *reinterpret_cast<f32x4 *>(p.y32 + (int64_t)f * p.ldy + n) = v;
        }
      }
  });
}

// Chunked schedule: the fp32-in data flow with the split of tile kt+1
// spread through tile kt's MFMAs.  Left to itself hipcc emits the whole
// split (about 130 VALU per thread and K-tile) and the plane writes first,
// then the MFMAs; both waves of a SIMD reach that VALU block together after
// the barrier, so the MFMA pipe idles through it (PMC: 61 % MFMA-busy per
// active SIMD).  Here each K-tile is NC chunks fenced by sched_barrier(0):
// chunk c = split of one pair of operand values (+ that row's three plane
// writes and its next-tile loads when the row is done), then NM / NC MFMAs.
// MF = 32: v_mfma_f32_32x32x16_bf16 (two k-substeps per K-tile), MF = 16:
// v_mfma_f32_16x16x32_bf16.  WPL: weights from the load-time planes.
template <int BW_, int BF_, int WGW_, int WGF_, int MF_>
struct X6CCfg {
  static constexpr int BW = BW_, BF = BF_, WGW = WGW_, WGF = WGF_, MF = MF_;
  static constexpr int NW = WGW * WGF, NT = 64 * NW;
  static constexpr int TW = BW / WGW / MF, TF = BF / WGF / MF;  // MF x MF blocks per wave
  static constexpr int SUB = MF == 32 ? 2 : 1;                  // k-substeps per K-tile
  static constexpr int STAGE = 3 * (BW + BF) * 64;
  static_assert(TW >= 1 && TF >= 1, "bad bf16x6c tile");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
};

// DIAG (ablation builds, wrong results; variants 80-83 only): 1 = no MFMAs,
// 2 = no split / plane writes / next-tile loads in the loop, 3 = MFMAs and
// barriers only (no fragment reads either).
template <class C, bool WPL, int DIAG = 0>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6c_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT, STAGE = C::STAGE, MF = C::MF,
                SUB = C::SUB;
  constexpr int RPP = NT / 4;
  static_assert(BW % RPP == 0 && BF % RPP == 0 && RPP % 16 == 0, "rows per pass");
  constexpr int NPW = BW / RPP, NPX = BF / RPP;
  constexpr int NSR = (WPL ? 0 : NPW) + NPX;  // rows this thread splits per K-tile
  constexpr int NC = 4 * NSR;                 // chunks = value pairs split
  constexpr int NB = TW * TF;                 // accumulator blocks
  constexpr int NM = SUB * 6 * NB;            // MFMAs per K-tile
  static_assert(NM % NC == 0, "MFMAs per chunk");
  constexpr int MPC = NM / NC;
  using AccT = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;
  const int prow = tid >> 2, pch = tid & 3;
  // chunk swizzle of a tile row: conflict-free ds_read_b128 for the fragment
  // shape (32x32: c ^ ((r >> 2) & 3); 16x16: c ^ 2((r >> 3) & 1)); every row
  // this thread writes has the same value (RPP % 16 == 0)
  auto swz = [](int r) { return MF == 32 ? ((r >> 2) & 3) : (((r >> 3) & 1) << 1); };
  const int soff = prow * 64 + ((pch ^ swz(prow)) * 16);

  typedef const __attribute__((address_space(1))) f32x4v gvec;
  typedef const __attribute__((address_space(1))) u32x4 gvecu;
  const int ldw = WPL ? 3 * p.pw : p.ldw;
  uint32_t wsrc[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) wsrc[i] = (uint32_t)(min(n0 + prow + i * RPP, p.n - 1) * ldw + 8 * pch);
  const int ktiles = p.kpad / 32;
  // split rows: [W rows (fp32 weights)] [X rows]; two float4 each
  f32x4v r0[NSR], r1[NSR];
  u32x4 rwp[WPL ? 3 * NPW : 1];
  auto load_row = [&](int kt, int q) {  // the fp32 source of split row q, tile kt
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    if (!WPL && q < NPW) {
      gvec *wb = (gvec *)(p.wf + k0);
      r0[q] = wb[wsrc[q] / 4];
      r1[q] = wb[wsrc[q] / 4 + 1];
    } else {
      const int i = WPL ? q : q - NPW;
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
      gvec *xb = (gvec *)(p.xf + col0 + 8 * pch);
      const int src = clampi(f0 + prow + i * RPP + shift, 0, p.m - 1);
      const uint32_t o = (uint32_t)(src * p.ldx) / 4;
      r0[q] = xb[o];
      r1[q] = xb[o + 1];
    }
  };
  auto load_wpl = [&](int kt) {
    if constexpr (WPL) {
      kt = min(kt, ktiles - 1);
      gvecu *wb = (gvecu *)(p.w + kt * 32);
#pragma unroll
      for (int i = 0; i < NPW; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) rwp[3 * i + pl] = wb[(wsrc[i] + pl * p.pw) / 8];
    }
  };
  // LDS byte offset of split row q's plane-0 chunk within a stage
  auto row_base = [&](int q) {
    if (!WPL && q < NPW) return (q * RPP) * 64 + soff;
    const int i = WPL ? q : q - NPW;
    return 3 * BW * 64 + (i * RPP) * 64 + soff;
  };
  auto row_pstride = [&](int q) { return (!WPL && q < NPW) ? BW * 64 : BF * 64; };

  const int lr = lane & (MF - 1), lh = MF == 32 ? lane >> 5 : lane >> 4;
  int foff[SUB];
#pragma unroll
  for (int s = 0; s < SUB; ++s) {
    const int c = MF == 32 ? 2 * s + lh : lh;
    foff[s] = lr * 64 + ((c ^ swz(lr)) * 16);
  }
  const int wrow = ww * TW * MF, frow = wf * TF * MF;
  AccT acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j)
#pragma unroll
      for (int e = 0; e < (MF == 32 ? 16 : 4); ++e) acc[i][j][e] = 0.0f;

  // prologue: tile 0 split into stage 0, tile 1 in registers
  {
#pragma unroll
    for (int q = 0; q < NSR; ++q) load_row(0, q);
    load_wpl(0);
#pragma unroll
    for (int q = 0; q < NSR; ++q) {
      const Planes2 a = split3_pair(r0[q].x, r0[q].y), b = split3_pair(r0[q].z, r0[q].w);
      const Planes2 c = split3_pair(r1[q].x, r1[q].y), d = split3_pair(r1[q].z, r1[q].w);
      char *dst = smem + row_base(q);
      *reinterpret_cast<u32x4 *>(dst) = u32x4{a.h, b.h, c.h, d.h};
      *reinterpret_cast<u32x4 *>(dst + row_pstride(q)) = u32x4{a.m, b.m, c.m, d.m};
      *reinterpret_cast<u32x4 *>(dst + 2 * row_pstride(q)) = u32x4{a.l, b.l, c.l, d.l};
    }
    if constexpr (WPL) {
#pragma unroll
      for (int i = 0; i < NPW; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<u32x4 *>(smem + (pl * BW + i * RPP) * 64 + soff) = rwp[3 * i + pl];
    }
#pragma unroll
    for (int q = 0; q < NSR; ++q) load_row(1, q);
    load_wpl(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  constexpr int PA[6] = {0, 0, 1, 1, 0, 2}, PB[6] = {0, 1, 0, 1, 2, 0};
  bf16x8 a[SUB][3][TW], b[SUB][3][TF];
  for (int kt = 0; kt < ktiles; ++kt) {
    const char *st = smem + (kt & 1) * STAGE;
    char *nx = smem + ((kt + 1) & 1) * STAGE;
    auto rd = [&](int s) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < TW; ++i)
          a[s][pl][i] = *reinterpret_cast<const bf16x8 *>(st + (pl * BW + wrow + i * MF) * 64 + foff[s]);
#pragma unroll
        for (int j = 0; j < TF; ++j)
          b[s][pl][j] = *reinterpret_cast<const bf16x8 *>(st + 3 * BW * 64 + (pl * BF + frow + j * MF) * 64 + foff[s]);
      }
    };
    if (DIAG != 3 || kt == 0) rd(0);
    if (DIAG == 3 && SUB == 2 && kt == 0) rd(1);
    if constexpr (WPL && DIAG < 2) {
      // the weight planes of tile kt+1 need no split: write them now, then
      // fetch tile kt+2's
#pragma unroll
      for (int i = 0; i < NPW; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<u32x4 *>(nx + (pl * BW + i * RPP) * 64 + soff) = rwp[3 * i + pl];
      load_wpl(kt + 2);
    }
    uint32_t ph[4], pm[4], plo[4];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      __builtin_amdgcn_sched_barrier(0);
      const int q = c / 4, e = c % 4;
      const f32x4v &v = e < 2 ? r0[q] : r1[q];
      if constexpr (DIAG < 2) {
      const Planes2 pp = (e & 1) ? split3_pair(v.z, v.w) : split3_pair(v.x, v.y);
      ph[e] = pp.h, pm[e] = pp.m, plo[e] = pp.l;
      }
      if (DIAG < 2 && e == 3) {
        char *dst = nx + row_base(q);
        *reinterpret_cast<u32x4 *>(dst) = u32x4{ph[0], ph[1], ph[2], ph[3]};
        *reinterpret_cast<u32x4 *>(dst + row_pstride(q)) = u32x4{pm[0], pm[1], pm[2], pm[3]};
        *reinterpret_cast<u32x4 *>(dst + 2 * row_pstride(q)) = u32x4{plo[0], plo[1], plo[2], plo[3]};
        load_row(kt + 2, q);
      }
      if (DIAG != 3 && SUB == 2 && c == NC / 4) rd(1);
#pragma unroll
      for (int t = 0; t < MPC; ++t) {
        const int m = c * MPC + t;
        const int s = m / (6 * NB), r = m % (6 * NB), pr = r / NB, blk = r % NB;
        const int i = blk / TF, j = blk % TF;
        if constexpr (DIAG == 1)
          asm volatile("" ::"v"(a[s][PA[pr]][i]), "v"(b[s][PB[pr]][j]));
        else if constexpr (MF == 32)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s][PA[pr]][i], b[s][PB[pr]][j], acc[i][j], 0, 0, 0);
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][PA[pr]][i], b[s][PB[pr]][j], acc[i][j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  with_post_mode(p.post_mode, [&](auto M) {
    constexpr int NG = MF == 32 ? 4 : 1;  // register quads per block
#pragma unroll
    for (int i = 0; i < TW; ++i)
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int n = n0 + wrow + i * MF + (MF == 32 ? 8 * g + 4 * lh : 4 * lh);
        if (n >= p.n) continue;
        const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
        const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
        const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          const int f = f0 + frow + j * MF + lr;
          if (f >= p.m) continue;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = apply_post<decltype(M)::value>(acc[i][j][4 * g + e] + bias[e], sc[e], of[e], p.post, p.npost);
          *reinterpret_cast<f32x4 *>(p.y32 + (int64_t)f * p.ldy + n) = v;
        }
      }
  });
}

// First layer: the spliced, zero-padded block (splice_pad_kernel's output)
// written directly as three bf16 planes.  out row r = [plane0 | plane1 |
// plane2], each `po` wide; columns nseg*din .. po-1 are zero.
struct SpliceIdx8 {
  int v[8];
};

__global__ __launch_bounds__(256) void splice_pad_split_kernel(const float *__restrict__ in, int ld_in, int rows,
                                                               int din, int nseg, SpliceIdx8 idx,
                                                               const int *__restrict__ row_map,
                                                               uint16_t *__restrict__ out, int po) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  uint16_t *o = out + (int64_t)r * 3 * po;
  for (int c = lane; c < po; c += 64) {
    const int s = c / din;
    float v = 0.0f;
    if (s < nseg) {
      int src = clampi(r + idx.v[s], 0, rows - 1);
      if (row_map) src = row_map[src];
      v = in[(int64_t)src * ld_in + (c - s * din)];
    }
    uint16_t h, m, l;
    split3(v, &h, &m, &l);
    o[c] = h;
    o[po + c] = m;
    o[2 * po + c] = l;
  }
}

template <class C, int DIAG = 0>
int launch_cfg(hipStream_t s, X6Args p, bool out16) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  if (out16)
    hipLaunchKernelGGL((gemm_bf16x6_kernel<C, true, DIAG>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16x6_kernel<C, false, DIAG>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C, bool PRIO = false>
int launch_phased(hipStream_t s, X6Args p, bool out16) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  if (out16)
    hipLaunchKernelGGL((gemm_bf16x6p_kernel<C, true, PRIO>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16x6p_kernel<C, false, PRIO>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C, int SCHED>
int launch_q(hipStream_t s, X6Args p, bool out16) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  if (out16)
    hipLaunchKernelGGL((gemm_bf16x6q_kernel<C, true, SCHED>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16x6q_kernel<C, false, SCHED>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C>
int launch_z(hipStream_t s, X6Args p, bool out16) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  if (out16)
    hipLaunchKernelGGL((gemm_bf16x6z_kernel<C, true>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16x6z_kernel<C, false>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C, int SCHED = 0, int DIAG = 0>
int launch_f(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6f_kernel<C, SCHED, DIAG>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C, int SCHED = 0>
int launch_w(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6w_kernel<C, SCHED>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C>
int launch_v(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6v_kernel<C>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C, bool WPL>
int launch_m(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6m_kernel<C, WPL>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C, bool WPL, int DIAG = 0>
int launch_c(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6c_kernel<C, WPL, DIAG>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C>
int launch_reg(hipStream_t s, X6Args p, bool out16) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  if (out16)
    hipLaunchKernelGGL((gemm_bf16x6r_kernel<C, true>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16x6r_kernel<C, false>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int x6_variant() {
  static int v = [] {
    const char *e = getenv("CATEARS_X6_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

}  // namespace

int launch_gemm_bf16x6(hipStream_t s, const X6Gemm &a) {
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  if (a.kpad % 32 != 0 || a.din % 32 != 0 || a.nseg < 1 || a.nseg > 8 || a.nseg * a.din > a.kpad)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6: bad K geometry");
  if (a.n % 4 != 0 || a.ldy % 4 != 0 || (a.y16 && a.py % 4 != 0))
    return fail(CE_GPU_EINVAL, "gemm_bf16x6: output width must be a multiple of 4");
  const bool f32in = a.xf != nullptr;
  if (f32in) {
    if (!a.wf || !a.y32 || a.ldw % 4 || a.ldx % 4 || (reinterpret_cast<uintptr_t>(a.wf) & 15) ||
        (reinterpret_cast<uintptr_t>(a.xf) & 15))
      return fail(CE_GPU_EINVAL, "gemm_bf16x6: fp32 operands must be 16-byte aligned, output fp32");
    // the kernel forms row * ld element offsets in 32 bits
    if ((int64_t)a.n * a.ldw >= ((int64_t)1 << 31) || (int64_t)a.m * a.ldx >= ((int64_t)1 << 31) ||
        (int64_t)a.m * a.ldy >= ((int64_t)1 << 31))
      return fail(CE_GPU_EINVAL, "gemm_bf16x6: operand beyond 2^31 elements");
  } else {
    if (a.ldw % 8 || a.pw % 8 || a.ldx % 8 || a.px % 8 || (reinterpret_cast<uintptr_t>(a.w) & 15) ||
        (reinterpret_cast<uintptr_t>(a.x) & 15))
      return fail(CE_GPU_EINVAL, "gemm_bf16x6: operands must be 16-byte aligned");
    if ((int64_t)a.n * a.ldw * 2 >= ((int64_t)1 << 32) || (int64_t)a.m * a.ldx * 2 >= ((int64_t)1 << 32))
      return fail(CE_GPU_EINVAL, "gemm_bf16x6: operand beyond 4 GiB");
  }
  if (a.npost > 4) return fail(CE_GPU_EINVAL, "gemm_bf16x6: too many post ops");
  X6Args p;
  p.w = a.w;
  p.x = a.x;
  p.wf = a.wf;
  p.xf = a.xf;
  p.bias = a.bias;
  p.bn_scale = a.bn_scale;
  p.bn_offset = a.bn_offset;
  p.y32 = a.y32;
  p.y16 = a.y16;
  p.ldw = a.ldw;
  p.pw = a.pw;
  p.ldx = a.ldx;
  p.px = a.px;
  p.ldy = a.ldy;
  p.py = a.py;
  p.m = a.m;
  p.n = a.n;
  p.kpad = a.kpad;
  p.din = a.din;
  p.off_packed = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (a.off[i] < -128 || a.off[i] > 127) return fail(CE_GPU_ENOTSUP, "gemm_bf16x6: splice offset beyond +-127");
    p.off_packed |= (uint64_t)(uint8_t)(int8_t)a.off[i] << (8 * i);
  }
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.post_mode = post_mode(a.post, a.npost);
  p.group = 8;
  const bool out16 = a.y16 != nullptr;
  if (f32in) {
    switch (x6_variant()) {
      case 40:
        return launch_f<X6Cfg<128, 128, 4, 2, 2>>(s, p);
      case 41:
        return launch_f<X6Cfg<128, 128, 2, 4, 2>>(s, p);
      case 43:
        return launch_f<X6Cfg<256, 128, 4, 2, 2>>(s, p);
      case 44:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 1>(s, p);
      case 45:
        return launch_f<X6Cfg<256, 128, 4, 2, 2>, 1>(s, p);
      case 46:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 2>(s, p);
      case 50:  // raised priority around the MFMAs
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 3>(s, p);
      case 48:  // 4 waves of 128 x 64
        return launch_f<X6Cfg<256, 128, 2, 2, 2>>(s, p);
      case 49:  // 4 waves of 64 x 128
        return launch_f<X6Cfg<128, 256, 2, 2, 2>>(s, p);
      case 47:
        return launch_f<X6Cfg<256, 128, 4, 2, 2>, 2>(s, p);
      // staggered split / MFMA roles per SIMD (SCHED 4; 5: + static priority for the second half)
      case 51:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 4>(s, p);
      case 52:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 5>(s, p);
      case 53:
        return launch_f<X6Cfg<128, 128, 2, 4, 2>, 4>(s, p);
      case 54:
        return launch_f<X6Cfg<256, 128, 4, 2, 2>, 4>(s, p);
      case 55:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6>(s, p);
      case 56:
        return launch_f<X6Cfg<128, 128, 2, 4, 2>, 6>(s, p);
      case 57:
        return launch_f<X6Cfg<256, 128, 4, 2, 2>, 6>(s, p);
      case 59:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 7>(s, p);
      // weights in LDS, activations in registers
      case 170:
        return launch_w<X6WCfg<128, 256, 8>>(s, p);
      case 171:
        return launch_w<X6WCfg<128, 128, 8>>(s, p);
      case 172:
        return launch_w<X6WCfg<64, 256, 8>>(s, p);
      case 173:
        return launch_w<X6WCfg<128, 256, 8>, 1>(s, p);
      case 174:
        return launch_w<X6WCfg<128, 128, 8>, 1>(s, p);
      // weight planes by LDS-DMA, activations in registers
      case 180:
        return launch_v<X6WCfg<128, 256, 8>>(s, p);
      case 181:
        return launch_v<X6WCfg<128, 128, 8>>(s, p);
      // ablations of 55 (wrong results: timing only)
      case 91:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 1>(s, p);
      case 92:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 2>(s, p);
      case 94:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 4>(s, p);
      case 96:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 16>(s, p);
      case 98:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 8>(s, p);
      case 99:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 3>(s, p);
      case 100:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 27>(s, p);
      case 101:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 59>(s, p);
      case 102:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 32>(s, p);
      case 103:
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6, 43>(s, p);
      // 32x32x16 MFMA kernels; odd = weights from the load-time planes
      case 60:
        return launch_m<X6MCfg<128, 256, 2, 4>, false>(s, p);
      case 61:
        return launch_m<X6MCfg<128, 256, 2, 4>, true>(s, p);
      case 62:
        return launch_m<X6MCfg<256, 128, 4, 2>, false>(s, p);
      case 63:
        return launch_m<X6MCfg<256, 128, 4, 2>, true>(s, p);
      case 64:
        return launch_m<X6MCfg<128, 128, 2, 2>, false>(s, p);
      case 65:
        return launch_m<X6MCfg<128, 128, 2, 2>, true>(s, p);
      case 66:
        return launch_m<X6MCfg<128, 128, 2, 4>, false>(s, p);
      case 67:
        return launch_m<X6MCfg<128, 128, 2, 4>, true>(s, p);
      // chunked split/MFMA interleave
      case 70:
        return launch_c<X6CCfg<128, 256, 2, 4, 32>, false>(s, p);
      case 71:
        return launch_c<X6CCfg<128, 256, 2, 4, 32>, true>(s, p);
      case 72:
        return launch_c<X6CCfg<128, 256, 2, 4, 16>, false>(s, p);
      case 73:
        return launch_c<X6CCfg<128, 256, 2, 4, 16>, true>(s, p);
      case 74:
        return launch_c<X6CCfg<256, 128, 4, 2, 32>, true>(s, p);
      case 75:
        return launch_c<X6CCfg<256, 128, 4, 2, 16>, true>(s, p);
      // ablations of 70 (wrong results: timing only)
      case 81:
        return launch_c<X6CCfg<128, 256, 2, 4, 32>, false, 1>(s, p);
      case 82:
        return launch_c<X6CCfg<128, 256, 2, 4, 32>, false, 2>(s, p);
      case 83:
        return launch_c<X6CCfg<128, 256, 2, 4, 32>, false, 3>(s, p);
      case 42:  // round-1 default: split of tile kt+1, then the MFMAs of tile kt
        return launch_f<X6Cfg<128, 256, 2, 4, 2>>(s, p);
      default:  // = 160: region-scheduled loop
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 8>(s, p);
    }
  }
  switch (x6_variant()) {
    case 1:
      return launch_cfg<X6Cfg<128, 128, 2, 2, 3>>(s, p, out16);
    case 2:
      return launch_cfg<X6Cfg<64, 128, 2, 2, 2>>(s, p, out16);
    case 3:
      return launch_cfg<X6Cfg<128, 64, 2, 2, 2>>(s, p, out16);
    case 4:
      return launch_cfg<X6Cfg<64, 128, 2, 2, 3>>(s, p, out16);
    case 5:
      return launch_cfg<X6Cfg<128, 64, 2, 2, 3>>(s, p, out16);
    case 6:
      return launch_phased<X6Cfg<128, 128, 2, 2, 3>>(s, p, out16);
    case 7:
      return launch_phased<X6Cfg<128, 128, 2, 4, 3>>(s, p, out16);
    case 8:
      return launch_phased<X6Cfg<128, 128, 4, 2, 3>>(s, p, out16);
    case 9:
      return launch_cfg<X6Cfg<128, 128, 2, 4, 2>>(s, p, out16);
    case 10:
      return launch_phased<X6Cfg<128, 128, 2, 4, 3>, true>(s, p, out16);
    case 11:
      return launch_phased<X6Cfg<128, 128, 2, 2, 3>, true>(s, p, out16);
    case 12:
      return launch_phased<X6Cfg<64, 128, 2, 2, 3>>(s, p, out16);
    case 93:
      return launch_cfg<X6Cfg<128, 128, 2, 4, 3>>(s, p, out16);
    case 95:
      return launch_cfg<X6Cfg<256, 128, 4, 2, 2>>(s, p, out16);
    case 97:
      return launch_cfg<X6Cfg<128, 256, 2, 4, 2>>(s, p, out16);
    case 14:
      return launch_reg<X6Cfg<128, 128, 2, 4, 2>>(s, p, out16);
    case 15:
      return launch_reg<X6Cfg<128, 128, 2, 2, 2>>(s, p, out16);
    case 16:
      return launch_reg<X6Cfg<128, 256, 2, 4, 2>>(s, p, out16);
    case 17:
      return launch_reg<X6Cfg<256, 128, 4, 2, 2>>(s, p, out16);
    case 18:
      return launch_reg<X6Cfg<64, 128, 2, 2, 2>>(s, p, out16);
    case 20:
      return launch_q<X6Cfg<128, 128, 2, 4, 3>, 0>(s, p, out16);
    case 21:
      return launch_q<X6Cfg<128, 128, 2, 4, 3>, 1>(s, p, out16);
    case 22:
      return launch_q<X6Cfg<128, 128, 4, 2, 3>, 0>(s, p, out16);
    case 23:
      return launch_q<X6Cfg<128, 128, 2, 2, 3>, 0>(s, p, out16);
    case 24:
      return launch_q<X6Cfg<128, 128, 4, 4, 3>, 0>(s, p, out16);
    case 25:
      return launch_q<X6Cfg<128, 128, 8, 2, 3>, 0>(s, p, out16);
    case 26:
      return launch_q<X6Cfg<256, 128, 4, 2, 2>, 0>(s, p, out16);
    case 27:
      return launch_q<X6Cfg<128, 256, 2, 4, 2>, 0>(s, p, out16);
    case 28:
      return launch_q<X6Cfg<128, 128, 4, 2, 2>, 0>(s, p, out16);
    case 29:
      return launch_q<X6Cfg<64, 128, 2, 2, 2>, 0>(s, p, out16);
    case 30:
      return launch_q<X6Cfg<128, 64, 2, 2, 2>, 0>(s, p, out16);
    case 31:
      return launch_q<X6Cfg<64, 128, 1, 4, 2>, 0>(s, p, out16);
    case 32:
      return launch_z<X6Cfg<128, 128, 4, 2, 3>>(s, p, out16);
    case 33:
      return launch_z<X6Cfg<128, 128, 2, 4, 3>>(s, p, out16);
    case 13:
      return launch_cfg<X6Cfg<128, 128, 2, 2, 2>>(s, p, out16);
    default:  // = 22
      return launch_q<X6Cfg<128, 128, 4, 2, 3>, 0>(s, p, out16);
  }
}

int launch_splice_pad_split(hipStream_t s, const float *in, int ld_in, int rows, int din, int nseg, const int *off,
                            const int *row_map, uint16_t *out, int po) {
  if (nseg < 1 || nseg > 8 || nseg * din > po) return fail(CE_GPU_EINVAL, "splice_pad_split: bad geometry");
  SpliceIdx8 idx = {};
  for (int i = 0; i < nseg; ++i) idx.v[i] = off[i];
  if (rows > 0)
    hipLaunchKernelGGL(splice_pad_split_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, in, ld_in, rows, din, nseg,
                       idx, row_map, out, po);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
