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

#ifndef CATEARS_X6_NT
#define CATEARS_X6_NT 0
#endif

namespace catears {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2t __attribute__((ext_vector_type(2)));

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
  const uint16_t *wd;  // weights as MFMA A fragments (gemm_bf16x6d_kernel), see X6Gemm::wd
  int wd_kt;           // K-tiles per 16-unit block in that image
  // first layer read straight from the caller's rows (gemm_bf16x6d_kernel
  // FIRST): nseg segments of din (a multiple of 8) floats, segment s of
  // packed row r = xf row row_map[clamp(r + off[s])]; zeros past them
  const int *row_map;
  int nseg;
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
#if CATEARS_X6_NT
          // measurement build (X6FLAGS=-DCATEARS_X6_NT=1): non-temporal output stores
          __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(p.y32 + (int64_t)f * p.ldy + n));
#else
          *reinterpret_cast<f32x4 *>(p.y32 + (int64_t)f * p.ldy + n) = v;
#endif
        }
      }
    }
  });
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
// SCHED: 0 = split of tile kt+1 before the MFMAs of tile kt (round 1);
// 6 = MFMAs first; 8 = MFMAs first in explicit regions (the default).
// DIAG (ablation builds of the SCHED 6 loop, wrong results; timing only,
// DESIGN.md §8; compiled only with -DCATEARS_DIAG, `make EXPERIMENTS=1`): bit 1 = no split (raw fp32 bits as the three planes),
// 2 = no global loads after the prologue, 4 = no MFMAs, 8 = no fragment
// reads after the first tile, 16 = no K-tile barrier, 32 = no plane writes
// after the prologue.
template <class C, int SCHED, int DIAG = 0>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6f_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT, STAGE = C::STAGE;
#ifndef CATEARS_DIAG
  static_assert(DIAG == 0, "ablation builds (wrong results) only with -DCATEARS_DIAG");
#endif
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
  const int kbeg = 0, ktiles = p.kpad / 32;
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

  load(kbeg);
  store(kbeg);
  load(kbeg + 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (SCHED >= 6) {
    // SCHED 6: the MFMAs of tile kt first, then the split of tile kt+1
    // (which the compiler interleaves into the MFMA stream); SCHED 8: the
    // same order in explicit regions (below).  Same barrier count and LDS
    // protocol as the SCHED 0 loop:
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
    for (int kt = 0; kt < ktiles; ++kt) {
      mfma_tile(kt);
      store(kt + 1);
      load(kt + 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr ((DIAG & 16) == 0) __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x6_epilogue<TW, TF, false>(p, acc, n0 + wrow, f0 + frow, lane);
    return;
  }
  for (int kt = kbeg; kt < ktiles; ++kt) {
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  x6_epilogue<TW, TF, false>(p, acc, n0 + wrow, f0 + frow, lane);
}

// Direct-weight schedule (the default): the constant weights are split into
// their three bf16 planes once, at model load, and stored in the order the
// MFMA reads its A operand (X6Gemm::wd: per 16-unit block, K-tile and plane
// one contiguous 1 KB fragment, lane l's 16 bytes at 16 l).  Each wave loads
// its weight fragments straight from L2 into registers with one
// global_load_dwordx4 per fragment -- no split VALU, no LDS write and no LDS
// read for the weights -- so LDS carries only the activations, split once per
// block on their way in (as gemm_bf16x6f_kernel does).  Per K-tile and CU
// that removes 2/3 of the ds_write_b128 traffic, half the fragment reads and
// 2/3 of the split VALU of the fp32-operand kernel, whose ablations placed its
// overhead over the bare MFMA loop in exactly that LDS-write path (DESIGN.md
// §8).  Tile: BW = 256 units x BF = 128 frames, 8 waves of 64 x 64 (4 along
// the units, 2 along the frames: each weight fragment is loaded by two waves,
// the second from L1).  Products, their order per output element and the
// planes are those of gemm_bf16x6f_kernel, so results are bit-identical to
// it.  Per K-tile, in order (the weights of tile kt+1 are issued as soon as
// tile kt's registers are free: a0 one tile ahead in a second buffer, a1
// after its last product, a2 at the end of the tile):
//   read b0 b1 (planes 0, 1 of the activations) | load a0 of kt+1 |
//   16 MFMAs a0 b0 | split + write activation tile kt+1, load tile kt+2 |
//   48 MFMAs a0 b1, a1 b0, a1 b1 | read b2 | load a1 of kt+1 |
//   32 MFMAs a0 b2, a2 b0 | load a2 of kt+1 | lgkmcnt(0), barrier.
//   WAR: activation stage (kt+1) % 2 was last read in tile kt-1, before the
//        barrier that closed it; RAW: its writes precede the barrier that
//        closes tile kt.
// DIAG (ablation builds, wrong results, timing only; -DCATEARS_DIAG): bit 1 =
// no split (the fp32 bits written as the planes), 2 = no activation stage
// writes at all, 4 = no activation loads after the prologue, 8 = no weight
// loads after the prologue, 16 = no K-tile barrier, 32 = no MFMAs.
// KS: K-tiles per LDS stage.  KS = 2 holds two K-tiles per stage (96 KB for
// both stages), so the block barrier comes once per two K-tiles; tile t
// lives in sub-stage t & 1 of stage (t >> 1) & 1, tile t + 2 is split and
// written during tile t and loaded during tile t - 1 (one tile more of load
// slack).  Same products in the same order: bit-identical to KS = 1.
// PIN / OUT16 (the plane chain, x6_plane_chain in capi.cc): the activations
// arrive already split -- three bf16 planes per row, written once by the
// previous layer's OUT16 epilogue -- so the loader moves three 16-byte plane
// chunks per thread into LDS with no split VALU; OUT16 writes this layer's
// output the same way for the next.  The planes are split3's, the loader's
// split3_pair gives the same bits, so the chain is bit-identical to the fp32
// chain.  Each activation is split once instead of once per unit tile that
// reads it (4 per hidden layer, 14 for the output layer).
// PRIO (experiment builds; the product runs 0): 1 raises the wave's issue
// priority around its global load issues (s_setprio 1), 2 around its MFMA
// regions, 3 around the load issues and LDS writes, 4 around the load issues
// and fragment reads, 5 as 1 with the activation loads issued at the top of
// the K-tile.  None is faster than 0 once the run order is balanced
// (profiles/r05z8_x6_setprio.txt).  Same bits.
template <class C, bool FIRST = false, int DIAG = 0, int KS = 1, bool PIN = false, bool OUT16 = false, int PRIO = 0>
__global__ __launch_bounds__(C::NT, 512 / C::NT) void gemm_bf16x6d_kernel(X6Args p) {  // 8 waves per CU
#ifndef CATEARS_DIAG
  static_assert(DIAG == 0, "ablation builds (wrong results) only with -DCATEARS_DIAG");
#endif
  static_assert(KS == 1 || (KS == 2 && !FIRST), "two K-tiles per stage: hidden layers only (even K-tile count)");
  static_assert(!PIN || (!FIRST && KS == 1 && DIAG == 0), "plane input: hidden / output layers, one K-tile per stage");
  constexpr int BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT;
  constexpr int RPP = NT / 4;  // activation rows per pass (4 threads x 32 B per row)
  static_assert(BF == RPP, "one activation row chunk per thread");
  constexpr int ASTAGE = 3 * BF * 64;  // bytes: one K-tile of activation planes
  __shared__ __attribute__((aligned(1024))) char smem[2 * KS * ASTAGE];
  auto stage_of = [&](int t) -> char * {
    if constexpr (KS == 1) return smem + (t & 1) * ASTAGE;
    else return smem + ((((t >> 1) & 1) << 1) + (t & 1)) * ASTAGE;
  };
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4v gvec;
  typedef const __attribute__((address_space(1))) bf16x8 gfrag;
  typedef const __attribute__((address_space(1))) u32x4 gchunk;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * C::BW;
  const int prow = tid >> 2, pch = tid & 3;
  const int ktiles = p.kpad / 32;

  // weight fragment i of this wave: 16-unit block (n0 + 64 ww + 16 i) / 16
  gfrag *wb[TW];
#pragma unroll
  for (int i = 0; i < TW; ++i)
    wb[i] = (gfrag *)(p.wd + ((size_t)((n0 >> 4) + ww * TW + i) * p.wd_kt * 3 * 64 + lane) * 8);
  auto load_w = [&](int kt, int pl, bf16x8 *dst) {
    if constexpr ((DIAG & 8) != 0) {
      if (kt > 0) return;
    }
    kt = min(kt, ktiles - 1);
#pragma unroll
    for (int i = 0; i < TW; ++i) dst[i] = wb[i][(kt * 3 + pl) * 64];
  };
  f32x4v rx0[2], rx1[2];  // activation row chunks of tiles kt+1 / kt+2 (by parity)
  u32x4 rp[3][2];         // PIN: the three plane chunks of tiles kt+1 / kt+2
  // FIRST: every (segment, tile row)'s source row, gathered once into LDS
  // (a row_map load per K-tile would put a dependent global load in front of
  // every activation load; eight values in registers went to scratch)
  __shared__ int src_tab[FIRST ? 8 * BF : 1];
  if constexpr (FIRST) {
    for (int i = tid; i < 8 * BF; i += NT) {
      const int sg = i / BF, row = i % BF;
      const int shift = (int)(signed char)(p.off_packed >> (8 * min(sg, p.nseg - 1)));
      const int src = clampi(clampi(f0 + row, 0, p.m - 1) + shift, 0, p.m - 1);
      src_tab[i] = p.row_map ? p.row_map[src] : src;
    }
    __syncthreads();
  }
  auto load_x = [&](int kt, int r) {
    if constexpr ((DIAG & 4) != 0) {
      if (kt > 1) return;
    }
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    if constexpr (FIRST) {
      // the splice (5 x 40 for TDNN-S) and row_map gather of splice_pad,
      // per thread: its 8 k lie in one segment; past the segments, zeros
      // (read from column 0 of a valid row)
      const int k = k0 + 8 * pch, seg = k / p.din, segc = min(seg, p.nseg - 1);
      const int src = src_tab[segc * BF + prow];
      gvec *xb = (gvec *)(p.xf + (size_t)src * p.ldx + (seg < p.nseg ? k - segc * p.din : 0));
      rx0[r] = xb[0];
      rx1[r] = xb[1];
      if (seg >= p.nseg) rx0[r] = rx1[r] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    } else if constexpr (PIN) {
      // row src's 8 bf16 at k of each plane: element src * ldx + pl * px + k
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
      const int src = clampi(f0 + prow + shift, 0, p.m - 1);
      const uint32_t o = ((uint32_t)(src * p.ldx) + col0 + 8 * pch) / 8, ps = (uint32_t)p.px / 8;
      gchunk *xb = (gchunk *)p.x;
      rp[0][r] = xb[o];
      rp[1][r] = xb[o + ps];
      rp[2][r] = xb[o + 2 * ps];
    } else {
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
      gvec *xb = (gvec *)(p.xf + col0 + 8 * pch);
      const int src = clampi(f0 + prow + shift, 0, p.m - 1);
      const uint32_t o = (uint32_t)(src * p.ldx) / 4;
      rx0[r] = xb[o];
      rx1[r] = xb[o + 1];
    }
  };
  auto put = [&](char *st, int r) {
    if constexpr ((DIAG & 2) != 0) return;
    if constexpr (PIN) {
      const int off = prow * 64 + ((pch ^ swz(prow)) * 16);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4 *>(st + pl * BF * 64 + off) = rp[pl][r];
      return;
    }
    Planes2 q0, q1, q2, q3;
    if constexpr ((DIAG & 1) != 0) {
      auto raw = [](float a, float b) {
        const uint32_t u = __builtin_bit_cast(uint32_t, a) ^ __builtin_bit_cast(uint32_t, b);
        return Planes2{u, u >> 1, u >> 2};
      };
      q0 = raw(rx0[r].x, rx0[r].y), q1 = raw(rx0[r].z, rx0[r].w);
      q2 = raw(rx1[r].x, rx1[r].y), q3 = raw(rx1[r].z, rx1[r].w);
    } else {
      q0 = split3_pair(rx0[r].x, rx0[r].y), q1 = split3_pair(rx0[r].z, rx0[r].w);
      q2 = split3_pair(rx1[r].x, rx1[r].y), q3 = split3_pair(rx1[r].z, rx1[r].w);
    }
    const int off = prow * 64 + ((pch ^ swz(prow)) * 16);
    *reinterpret_cast<u32x4 *>(st + off) = u32x4{q0.h, q1.h, q2.h, q3.h};
    *reinterpret_cast<u32x4 *>(st + BF * 64 + off) = u32x4{q0.m, q1.m, q2.m, q3.m};
    *reinterpret_cast<u32x4 *>(st + 2 * BF * 64 + off) = u32x4{q0.l, q1.l, q2.l, q3.l};
  };
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int frow = wf * TF * 16;
  auto read_b = [&](const char *st, int pl, bf16x8 *b) {
#pragma unroll
    for (int j = 0; j < TF; ++j) b[j] = *reinterpret_cast<const bf16x8 *>(st + (pl * BF + frow + j * 16) * 64 + foff);
  };

  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  bf16x8 a0[2][TW], a1[TW], a2[TW], b0[TF], b1[TF], b2[TF];
  load_x(0, 0);
  load_w(0, 0, a0[0]);
  load_w(0, 1, a1);
  load_w(0, 2, a2);
  if constexpr (KS == 1) {
    put(smem, 0);
    load_x(1, 1);
  } else {
    load_x(1, 1);
    put(stage_of(0), 0);
    put(stage_of(1), 1);
    load_x(2, 0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  auto body = [&](int kt, auto cc) {
    constexpr int c = decltype(cc)::value;
    const char *st = stage_of(kt);
    char *sn = stage_of(kt + KS);
    // Regions (sched_barrier): the compiler would otherwise sink every load
    // to its registers' last use and then wait on it at the next tile's
    // head.  The loads sit in regions of their own at the top of the
    // phase after their registers' last use; the split VALU of the next
    // activation tile shares the 48-MFMA region so it interleaves.
    // Activation registers alternate by tile parity: tile kt+1's chunk
    // (loaded one tile ago) is written while tile kt+2's is loaded.
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(1);
    read_b(st, 0, b0);
    read_b(st, 1, b1);
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(0);
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(1);
    load_w(kt + 1, 0, a0[c ^ 1]);
    if constexpr (PRIO == 5) load_x(kt + KS + 1, KS == 1 ? c : c ^ 1);  // activations issued first thing
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    if constexpr ((DIAG & 32) == 0) {
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[c][i], b0[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // KS 1: load tile kt + 2 into rx[c], write tile kt + 1 from rx[c ^ 1];
    // KS 2: load tile kt + 3 into rx[c ^ 1], write tile kt + 2 from rx[c]
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(1);
    if constexpr (PRIO != 5) load_x(kt + KS + 1, KS == 1 ? c : c ^ 1);
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    if constexpr (PRIO == 3) __builtin_amdgcn_s_setprio(1);
    put(sn, KS == 1 ? c ^ 1 : c);
    if constexpr (PRIO == 3) __builtin_amdgcn_s_setprio(0);
    if constexpr ((DIAG & 32) == 0) {
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[c][i], b1[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b0[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
        }
    }
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(1);
    read_b(st, 2, b2);
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(1);
    load_w(kt + 1, 1, a1);
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    if constexpr ((DIAG & 32) == 0) {
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[c][i], b2[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[i], b0[j], acc[i][j], 0, 0, 0);
        }
    } else {
      // keep the fragment registers live
#pragma unroll
      for (int j = 0; j < TF; ++j) acc[0][j][0] += (float)b0[j][0] + (float)b1[j][0] + (float)b2[j][0] +
                                                   (float)a0[c][0][0] + (float)a1[0][0] + (float)a2[0][0];
    }
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(1);
    load_w(kt + 1, 2, a2);
    if constexpr (PRIO == 1 || PRIO == 3 || PRIO == 4 || PRIO == 5) __builtin_amdgcn_s_setprio(0);
    if constexpr (KS == 1 || c == 1) {  // KS 2: once per stage (after its odd tile)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr ((DIAG & 16) == 0) __builtin_amdgcn_s_barrier();
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  int kt = 0;
  for (; kt + 1 < ktiles; kt += 2) {
    body(kt, std::integral_constant<int, 0>());
    body(kt + 1, std::integral_constant<int, 1>());
  }
  if (KS == 1 && kt < ktiles) body(kt, std::integral_constant<int, 0>());
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail prefetches
  x6_epilogue<TW, TF, OUT16>(p, acc, n0 + ww * TW * 16, f0 + frow, lane);
}

// One wave per SIMD (gemm_bf16x6w_kernel): 4 waves per block, each with up
// to 512 registers (the 256 accumulators of a 128 x 128 wave tile live in
// AGPRs), so every operand fragment feeds twice the products of the 8-wave
// kernel.  Block BW units x BF frames as WGW x WGF waves of TW x TF 16 x 16
// fragments.  At 512 x 128 (4 x 1 waves of 128 units x 128 frames), per
// output element and K-tile this halves the weight fragments loaded (each is
// loaded by exactly one wave), the activation fragments read from LDS (read
// by 4 waves for 128 frames x 512 units instead of 4 for 128 x 256) and the
// activation loads + split + LDS writes (one block covers 512 units) -- the
// bytes and VALU that cost clock at the chip's power cap (DESIGN.md §8 r5,
// r05z5 ablations).
// Per K-tile the wave runs its TW unit blocks in order; unit block i takes
// the TF frame blocks with the six products in gemm_bf16x6d_kernel's order
// per accumulator (a0b0, a0b1, a1b0, a1b1, a0b2, a2b0; K-tiles in order), so
// the results are bit-identical to it.
//   * weights: a ring of 4 unit-block buffers (3 planes each), each loaded
//     3 unit blocks (3 x 6 TF MFMAs) ahead of its use, straight from the
//     fragment image to registers, across K-tile boundaries;
//   * activations: the TF x 3 plane fragments of the K-tile stay in registers
//     for all TW unit blocks; in the last unit block each frame block's
//     fragments are replaced by the next K-tile's as soon as its six
//     products are issued;
//   * unit block 0: the next K-tile's activation rows (loaded one K-tile
//     ago) are split into the free LDS stage and the one after is loaded;
//     after unit block TW/2 - 1: lgkmcnt(0) and the block barrier (RAW for
//     the next K-tile's stage; WAR: a stage is rewritten one K-tile after
//     the barrier that follows its last reads).
template <int BW_, int BF_, int WGW_, int WGF_>
struct W6Cfg {
  static constexpr int BW = BW_, BF = BF_, WGW = WGW_, WGF = WGF_;
  static constexpr int NW = WGW * WGF, NT = 64 * NW;
  static constexpr int TW = BW / WGW / 16, TF = BF / WGF / 16;  // 16 x 16 fragments per wave
  static_assert(TW * WGW * 16 == BW && TF * WGF * 16 == BF, "bad one-wave-per-SIMD tile");
};

// SG: pin the interleave with sched_group_barrier -- the split + LDS writes of
// unit block 0 between its MFMAs (1 MFMA : 2 VALU), and in the last unit
// block each frame block's three fragment reads right after its six MFMAs
// (the compiler otherwise issues the split as one VALU block ahead of the
// MFMAs and sinks the reads to the end of the K-tile).
// RING: unit-block weight buffers in flight (RING - 1 unit blocks ahead).
// NW = 8 (two waves per SIMD, 256 registers each) is the same schedule with
// the accumulators of a 128 x 64 wave tile in AGPRs.
template <class C, bool SG = false, int RING = 4>
__global__ __launch_bounds__(C::NT, C::NW / 4) void gemm_bf16x6w_kernel(X6Args p) {
  constexpr int BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT;
  static_assert(C::NW == 4 || C::NW == 8, "one or two waves per SIMD");
  static_assert(TW % RING == 0, "a ring of unit-block weight buffers that divides the unit blocks");
  constexpr int RQ = BF / (NT / 4);  // activation rows per thread per K-tile
  static_assert(RQ >= 1 && RQ * (NT / 4) == BF, "whole activation rows per thread");
  constexpr int ASTAGE = 3 * BF * 64;
  __shared__ __attribute__((aligned(1024))) char smem[2 * ASTAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4v gvec;
  typedef const __attribute__((address_space(1))) bf16x8 gfrag;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * C::BW;
  const int prow = tid >> 2, pch = tid & 3;
  const int ktiles = p.kpad / 32;

  // the wave's unit block i, K-tile kt, plane pl: fragment
  // ((ub0 + i) * wd_kt + kt) * 3 + pl of the image, lane's 16 bytes
  gfrag *wbase = (gfrag *)(p.wd + ((size_t)((n0 >> 4) + ww * TW) * p.wd_kt * 3 * 64 + lane) * 8);
  bf16x8 wa[RING][3];
  auto load_w = [&](int kt, int i, int buf) {
    kt = min(kt, ktiles - 1);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) wa[buf][pl] = wbase[((size_t)(i * p.wd_kt + kt) * 3 + pl) * 64];
  };
  f32x4v rx0[RQ], rx1[RQ];
  auto load_x = [&](int kt) {
    kt = min(kt, ktiles - 1);
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
    gvec *xb = (gvec *)(p.xf + col0 + 8 * pch);
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const int src = clampi(f0 + prow + q * (NT / 4) + shift, 0, p.m - 1);
      const uint32_t o = (uint32_t)(src * p.ldx) / 4;
      rx0[q] = xb[o];
      rx1[q] = xb[o + 1];
    }
  };
  auto put = [&](char *st) {
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
      const Planes2 q0 = split3_pair(rx0[q].x, rx0[q].y), q1 = split3_pair(rx0[q].z, rx0[q].w);
      const Planes2 q2 = split3_pair(rx1[q].x, rx1[q].y), q3 = split3_pair(rx1[q].z, rx1[q].w);
      const int row = prow + q * (NT / 4);
      const int off = row * 64 + ((pch ^ swz(row)) * 16);
      *reinterpret_cast<u32x4 *>(st + off) = u32x4{q0.h, q1.h, q2.h, q3.h};
      *reinterpret_cast<u32x4 *>(st + BF * 64 + off) = u32x4{q0.m, q1.m, q2.m, q3.m};
      *reinterpret_cast<u32x4 *>(st + 2 * BF * 64 + off) = u32x4{q0.l, q1.l, q2.l, q3.l};
    }
  };
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int frow = wf * TF * 16;
  auto frag = [&](const char *st, int pl, int j) {
    return *reinterpret_cast<const bf16x8 *>(st + (pl * BF + frow + j * 16) * 64 + foff);
  };

  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  bf16x8 b0[TF], b1[TF], b2[TF];

  load_x(0);
#pragma unroll
  for (int i = 0; i < RING - 1; ++i) load_w(0, i, i);
  put(smem);
  load_x(1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < TF; ++j) {
    b0[j] = frag(smem, 0, j);
    b1[j] = frag(smem, 1, j);
    b2[j] = frag(smem, 2, j);
  }

  for (int kt = 0; kt < ktiles; ++kt) {
    char *sn = smem + ((kt + 1) & 1) * ASTAGE;
#pragma unroll
    for (int i = 0; i < TW; ++i) {
      // the weights three unit blocks ahead (the next K-tile's first ones
      // from unit block TW - 3 on)
      load_w(kt + (i + RING - 1) / TW, (i + RING - 1) % TW, (i + RING - 1) % RING);
      if (i == 0) {
        if constexpr (!SG) {
          put(sn);
          load_x(kt + 2);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (SG) {
        if (i == 0) {
          put(sn);
          load_x(kt + 2);
#pragma unroll
          for (int g = 0; g < 6 * TF; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // 2 VALU
            if (g % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // an LDS write
          }
        }
      }
      constexpr int u = 0;  // (the ring slot is i % RING, a constant once unrolled)
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i % RING][u], b0[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i % RING][u], b1[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i % RING][u + 1], b0[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i % RING][u + 1], b1[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i % RING][u], b2[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i % RING][u + 2], b0[j], acc[i][j], 0, 0, 0);
        if (i == TW - 1) {  // frame block j is done for this K-tile: the next one's fragments
          b0[j] = frag(sn, 0, j);
          b1[j] = frag(sn, 1, j);
          b2[j] = frag(sn, 2, j);
        }
      }
      if constexpr (SG) {
        if (i == TW - 1) {
#pragma unroll
          for (int j = 0; j < TF; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);  // frame block j's six MFMAs
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // its next fragments
          }
        }
      }
      if (i == TW / 2 - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the clamped tail prefetches
  x6_epilogue<TW, TF, false>(p, acc, n0 + ww * TW * 16, f0 + frow, lane);
}

#ifdef CATEARS_EXPERIMENTS
// Register-direct schedule (variant 400): both operands go straight from
// L2 / L1 to registers -- the weights from the MFMA-fragment image as in
// gemm_bf16x6d_kernel, the activations as each lane's 8 consecutive floats of
// one row (the B-fragment layout of v_mfma_f32_16x16x32_bf16), split into
// their three bf16 planes in registers by the wave that multiplies them.  No
// LDS, no barrier: every wave runs its K loop at its own pace, with the next
// K-tile's loads in flight under this one's MFMAs.  The price is each
// activation fragment fetched by the WGW waves along the units (from L1 after
// the first) and split by each of them.  Products and their order per
// element are gemm_bf16x6d_kernel's (a0b0, a0b1, a1b0, a1b1, a0b2, a2b0 per
// K-tile, K-tiles in order): bit-identical results.
template <class C>
__global__ __launch_bounds__(C::NT, 1) void gemm_bf16x6r_kernel(X6Args p) {
  constexpr int TW = C::TW, TF = C::TF;
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4v gvec;
  typedef const __attribute__((address_space(1))) bf16x8 gfrag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * C::BF + wf * TF * 16, n0 = tn * C::BW;
  const int ktiles = p.kpad / 32;
  gfrag *wb[TW];
#pragma unroll
  for (int i = 0; i < TW; ++i)
    wb[i] = (gfrag *)(p.wd + ((size_t)((n0 >> 4) + ww * TW + i) * p.wd_kt * 3 * 64 + lane) * 8);
  // the lane's rows (frame f0 + 16 j + (lane & 15)) and k chunk (8 (lane >> 4))
  int xrow[TF];
#pragma unroll
  for (int j = 0; j < TF; ++j) xrow[j] = f0 + 16 * j + (lane & 15);
  bf16x8 a[2][3][TW];
  f32x4v x[2][TF][2];
  auto load = [&](int kt, int buf) {
    kt = min(kt, ktiles - 1);  // the tail's prefetch refetches the last tile (unused)
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int i = 0; i < TW; ++i) a[buf][pl][i] = wb[i][(kt * 3 + pl) * 64];
    const int k0 = kt * 32;
    const int seg = k0 / p.din, col = k0 - seg * p.din + 8 * (lane >> 4);
    const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const int src = clampi(xrow[j] + shift, 0, p.m - 1);
      gvec *xp = (gvec *)(p.xf + (size_t)src * p.ldx + col);
      x[buf][j][0] = xp[0];
      x[buf][j][1] = xp[1];
    }
  };
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  auto compute = [&](int buf) {
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const f32x4v v0 = x[buf][j][0], v1 = x[buf][j][1];
      const Planes2 q0 = split3_pair(v0.x, v0.y), q1 = split3_pair(v0.z, v0.w);
      const Planes2 q2 = split3_pair(v1.x, v1.y), q3 = split3_pair(v1.z, v1.w);
      const bf16x8 b0 = __builtin_bit_cast(bf16x8, u32x4{q0.h, q1.h, q2.h, q3.h});
      const bf16x8 b1 = __builtin_bit_cast(bf16x8, u32x4{q0.m, q1.m, q2.m, q3.m});
      const bf16x8 b2 = __builtin_bit_cast(bf16x8, u32x4{q0.l, q1.l, q2.l, q3.l});
      // each product over the TW accumulators before the next: TW
      // independent MFMAs between an accumulator's dependent ones
#pragma unroll
      for (int i = 0; i < TW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][0][i], b0, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][0][i], b1, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][1][i], b0, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][1][i], b1, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][0][i], b2, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[buf][2][i], b0, acc[i][j], 0, 0, 0);
    }
  };
  load(0, 0);
  int kt = 0;
  for (; kt + 1 < ktiles; kt += 2) {
    load(kt + 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(0);
    __builtin_amdgcn_sched_barrier(0);
    load(kt + 2, 0);
    __builtin_amdgcn_sched_barrier(0);
    compute(1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (kt < ktiles) compute(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail prefetch
  x6_epilogue<TW, TF, false>(p, acc, n0 + ww * TW * 16, f0, lane);
}

#endif  // CATEARS_EXPERIMENTS

// Warp-specialised fp32-in schedule: the block is C::NW MFMA waves plus
// NPV producer waves.  The producers do all the global loads, splits and
// plane writes of tile kt+1 while the MFMA waves read and multiply tile kt,
// so the split VALU issues in the cycles the matrix pipe leaves free on the
// same SIMD instead of between a wave's own MFMAs.  Same LDS stages, layout,
// product order and per-K-tile barrier as gemm_bf16x6f_kernel's SCHED 0 loop
// (bit-identical results):
//   WAR: stage (kt+1) % 2 was read in step kt-1, whose reads were drained
//        (lgkmcnt(0)) before the barrier closing it;
//   RAW: the producers' writes of tile kt+1 are drained before the barrier
//        closing step kt, and the MFMA waves read them after it.
// Both roles pass the same number of barriers (one prologue + one per K-tile;
// the role test is wave-uniform, readfirstlane).  Producer rows: the stage's
// BW weight rows then BF activation rows, 4 threads x 32 B per row, pass i
// covering rows i RPP .. i RPP + RPP - 1 (a pass may straddle the two kinds:
// per-thread selects).  Measured against the default: DESIGN.md §8.
template <class C, int NPV>
__global__ __launch_bounds__(C::NT + 64 * NPV, 1) void gemm_bf16x6ws_kernel(X6Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, NT = C::NT, STAGE = C::STAGE;
  constexpr int RPP = 16 * NPV;  // producer rows per pass
  static_assert((BW + BF) % RPP == 0, "rows per pass");
  constexpr int NP = (BW + BF) / RPP;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) f32x4v gvec;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;
  const int ktiles = p.kpad / 32;

  if (wave >= C::NW) {  // producer
    const int pt = tid - NT, prow = pt >> 2, pch = pt & 3;
    bool isw[NP];
    int trow[NP];         // row within its plane block
    uint32_t wsrc[NP];    // weight rows: float offset at k = 0
    int dst[NP];          // byte offset of the chunk in the stage
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int r = i * RPP + prow;
      isw[i] = BW % RPP == 0 ? i < BW / RPP : r < BW;  // compile-time when no pass straddles
      trow[i] = isw[i] ? r : r - BW;
      wsrc[i] = (uint32_t)(min(n0 + trow[i], p.n - 1) * p.ldw + 8 * pch);
      dst[i] = (isw[i] ? 0 : 3 * BW * 64) + trow[i] * 64 + ((pch ^ swz(trow[i])) * 16);
    }
    f32x4v r0[NP], r1[NP];
    auto load = [&](int kt) {
      kt = min(kt, ktiles - 1);
      const int k0 = kt * 32;
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        gvec *src;
        if (isw[i]) {
          src = (gvec *)(p.wf + k0 + wsrc[i]);
        } else {
          const int x = clampi(f0 + trow[i] + shift, 0, p.m - 1);
          src = (gvec *)(p.xf + (uint32_t)(x * p.ldx) + col0 + 8 * pch);
        }
        r0[i] = src[0];
        r1[i] = src[1];
      }
    };
    auto store = [&](int kt) {
      char *st = smem + (kt & 1) * STAGE;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const f32x4v v0 = r0[i], v1 = r1[i];
        const Planes2 q0 = split3_pair(v0.x, v0.y), q1 = split3_pair(v0.z, v0.w);
        const Planes2 q2 = split3_pair(v1.x, v1.y), q3 = split3_pair(v1.z, v1.w);
        const int ps = (isw[i] ? BW : BF) * 64;  // plane stride in the stage
        char *d = st + dst[i];
        *reinterpret_cast<u32x4 *>(d) = u32x4{q0.h, q1.h, q2.h, q3.h};
        *reinterpret_cast<u32x4 *>(d + ps) = u32x4{q0.m, q1.m, q2.m, q3.m};
        *reinterpret_cast<u32x4 *>(d + 2 * ps) = u32x4{q0.l, q1.l, q2.l, q3.l};
      }
    };
    load(0);
    store(0);
    load(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < ktiles; ++kt) {
      store(kt + 1);  // past the end: the clamped last tile into a stage no step reads
      load(kt + 2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // MFMA waves
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;
  f32x4 acc[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  __builtin_amdgcn_s_barrier();
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  x6_epilogue<TW, TF, false>(p, acc, n0 + wrow, f0 + frow, lane);
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

template <class C, int SCHED = 0, int DIAG = 0>
int launch_f(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6f_kernel<C, SCHED, DIAG>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

#ifdef CATEARS_EXPERIMENTS
template <class C>
int launch_r(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  hipLaunchKernelGGL((gemm_bf16x6r_kernel<C>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}
#endif

// CATEARS_X6_KS: K-tiles per LDS stage of the direct-weight kernel's hidden
// layers (1 or 2; same bits).  Measured (tools/experiments/gpu_r5e.sh, one
// box, alternating): two per stage is 2 % slower -- serial hidden layer 158.5
// vs 155.6 us, C3 at the driver's flags 6.36-6.38 vs 6.40-6.46 M frames/s --
// so one stays the default; the barrier is not what the loop waits on.
int x6_ks() {
  static int v = CE_KNOB("CATEARS_X6_KS", 1);
  return v;
}

template <class C, int DIAG = 0, int PRIO = 0>
int launch_d(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  const bool out16 = p.y16 != nullptr;
  if (p.row_map || p.din % 32 != 0) {  // the same rule as launch_gemm_bf16x6's `first`
    if (out16)
      hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, true, 0, 1, false, true>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, true>), grid, block, 0, s, p);
  } else if (!p.xf) {  // plane input (the plane chain)
    if (out16)
      hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, false, 0, 1, true, true>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, false, 0, 1, true, false>), grid, block, 0, s, p);
  } else if (out16) {  // fp32 input, planes out (a chain's whole-K-tile first layer)
    hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, false, 0, 1, false, true>), grid, block, 0, s, p);
  } else if (x6_ks() == 2 && (p.kpad / 32) % 2 == 0)
    hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, false, DIAG, 2>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_bf16x6d_kernel<C, false, DIAG, 1, false, false, PRIO>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

// 512 x 128 tiles (the default kernel) only for layers of at least this many
constexpr int kX6WideMinTiles = 48;

// the one-wave-per-SIMD kernel; false when the fragment image does not cover
// the last unit tile (the image pads units to a multiple of 256)
// The XCD tile groups of the 512-unit tiles (tile_order.h), by the layer's
// column tiles.  A 1024-unit layer (2 column tiles, 64 tiles): groups of 1
// put 8 row panels x 1 weight panel on each XCD (each row panel fetched into
// 2 XCDs' L2s, each weight panel into 4 -- the a . w = 8 minimum of DESIGN.md
// §8 r5): PMC 200 MB per hidden-layer launch against 223 MB with groups of 2
// (the whole width, a = 1, w = 8), C3 +1.1 % at the driver's flags
// (profiles/r06h_group_abc.txt).  The 3456-unit output layer (7 column
// tiles) keeps groups of 2: 214 MB against 243 MB.  CATEARS_X6W_GROUP
// (experiments library) forces one value.
int x6w_group(int tiles_n) {
  static int v = CE_KNOB("CATEARS_X6W_GROUP", 0);
  return v > 0 ? v : (tiles_n <= 2 ? 1 : 2);
}

template <class C, bool SG = false, int RING = 4>
bool launch_w(hipStream_t s, X6Args p, int min_tiles = 0) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  if ((p.n + 255) / 256 * 256 < p.tiles_n * C::BW) return false;
  if (p.tiles_n * p.tiles_m < min_tiles) return false;
  p.group = x6w_group(p.tiles_n);
  hipLaunchKernelGGL((gemm_bf16x6w_kernel<C, SG, RING>), dim3(p.tiles_m * p.tiles_n), dim3(C::NT), 0, s, p);
  return true;
}

template <class C, int NPV>
int launch_ws(hipStream_t s, X6Args p) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT + 64 * NPV);
  hipLaunchKernelGGL((gemm_bf16x6ws_kernel<C, NPV>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

// CATEARS_X6_VARIANT (experiments library only, CE_KNOB): the schedule of
// the fp32-activation bf16x6 GEMM.  The product build runs the default (0 =
// 300, direct weights: 256 x 128 tiles, weight fragments straight from L2 to
// registers) and, for a model without the fragment image, the round-2
// default 160 (region-scheduled 128 x 256 tiles, weights split in the
// kernel).  The bit-identical alternatives -- 40 (128 x 128 tiles), 200
// (warp-specialised 128 x 128), the measurement variants -- and the DIAG
// ablations, which give wrong results, exist only in `make EXPERIMENTS=1`
// builds (libcatears_hip_exp.so, tools/, tests/test_gpu_x6_variants.py);
// any other value there makes every bf16x6 launch fail with CE_GPU_EINVAL.
int x6_variant() {
  static int v = CE_KNOB("CATEARS_X6_VARIANT", 0);
  return v;
}

// CATEARS_X6_FIRST_TILE: unit width of the gathered first layer's tiles.
// 128 (default): 256 blocks for a 4072-row batch instead of 128, 26.5 ->
// 20.9 us per launch in a serial run (r4c); 256: the hidden layers' tiles.
// Same bits either way (tests/test_gpu_x6_variants.py).
int x6_first_tile() {
  static int v = CE_KNOB("CATEARS_X6_FIRST_TILE", 128);
  return v;
}

}  // namespace

int launch_gemm_bf16x6(hipStream_t s, const X6Gemm &a) {
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  // a first layer gathered in the loader (row_map, or segments that are not
  // whole K-tiles) needs the direct-weight kernel and din % 8 == 0
  const bool first = a.row_map != nullptr || a.din % 32 != 0;
  if (a.kpad % 32 != 0 || a.din % (first ? 8 : 32) != 0 || a.din <= 0 || a.nseg < 1 || a.nseg > 8 ||
      a.nseg * a.din > a.kpad)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6: bad K geometry");
  if (first && (!a.xf || !a.wd || (x6_variant() != 0 && x6_variant() != 300 && (x6_variant() < 310 || x6_variant() > 316))))
    return fail(CE_GPU_EINVAL, "gemm_bf16x6: a gathered first layer needs fp32 input and the direct-weight kernel");
  if (a.n % 4 != 0 || a.ldy % 4 != 0 || (a.y16 && a.py % 4 != 0))
    return fail(CE_GPU_EINVAL, "gemm_bf16x6: output width must be a multiple of 4");
  const bool f32in = a.xf != nullptr;
  // the plane chain (capi.cc x6_plane_chain): planes in and / or out of the
  // direct-weight kernel
  const bool direct = a.wd && (x6_variant() == 0 || x6_variant() == 300);
  const bool pin = !f32in && a.x && a.wd;
  if (pin) {
    if (!direct || first || a.ldx % 8 || a.px % 8 || (reinterpret_cast<uintptr_t>(a.x) & 15) ||
        (int64_t)a.m * a.ldx >= ((int64_t)1 << 31) || (int64_t)a.m * a.ldy >= ((int64_t)1 << 31))
      return fail(CE_GPU_EINVAL, "gemm_bf16x6: plane input needs the direct-weight kernel, din % 32 == 0, "
                                 "16-byte aligned planes and 2^31-element operands");
  }
  if (a.y16 && f32in && !direct)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6: fp32 input with split output needs the direct-weight kernel");
  if (f32in) {
    if (!a.wf || !(a.y32 || a.y16) || a.ldw % 4 || a.ldx % 4 || (reinterpret_cast<uintptr_t>(a.wf) & 15) ||
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
  p.nseg = a.nseg;
  p.row_map = a.row_map;
  p.off_packed = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (a.off[i] < -128 || a.off[i] > 127) return fail(CE_GPU_ENOTSUP, "gemm_bf16x6: splice offset beyond +-127");
    p.off_packed |= (uint64_t)(uint8_t)(int8_t)a.off[i] << (8 * i);
  }
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.post_mode = post_mode(a.post, a.npost);
// Column tiles per XCD tile group (tile_order.h).  A hidden layer's 128
// tiles (32 row x 4 unit) give each XCD 16: group 2 makes that 8 row x 2
// unit tiles -- 9.5 MB of weight fragments + 12.5 MB of activations into its
// L2, against 18.9 + 6.3 MB for the whole-width group 8 (C3 at the driver's
// step counts, alternating builds: 5.53-5.61 vs 5.45-5.52 M frames/s).
#ifndef CATEARS_X6_GROUP
#define CATEARS_X6_GROUP 2
#endif
  p.group = CATEARS_X6_GROUP;
  p.wd = a.wd;
  p.wd_kt = a.wd_kt;
  const bool out16 = a.y16 != nullptr;
  if (pin || (f32in && out16)) {
    if (a.wd_kt * 32 < a.kpad || (reinterpret_cast<uintptr_t>(a.wd) & 15))
      return fail(CE_GPU_EINVAL, "gemm_bf16x6: weight fragment image does not cover K");
    if (a.wide || (first && x6_first_tile() == 128)) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
    return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>>(s, p);
  }
  if (f32in) {
    switch (x6_variant()) {
      case 0:    // the default (round 6): direct weights, the layers after the first on 512 x 128
                 // tiles of 8 waves of 128 units x 64 frames (gemm_bf16x6w_kernel, variant 508)
      case 300:  // direct weights on 256 x 128 tiles (gemm_bf16x6d_kernel, the rounds 3-5 default)
        if (a.wd) {
          if (a.wd_kt * 32 < a.kpad || (reinterpret_cast<uintptr_t>(a.wd) & 15))
            return fail(CE_GPU_EINVAL, "gemm_bf16x6: weight fragment image does not cover K");
          // the gathered first layer (K of a few tiles: prologue and
          // epilogue bound) on 128 x 128 tiles -- twice the blocks; every
          // layer so with ce_gpu_ctx_set_wide_tiles (a batch scored while
          // no other is in flight then fills all CUs)
          if (a.wide || (first && x6_first_tile() == 128)) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
          // 512-unit tiles: each block splits and stages its activation
          // rows once for 512 units and each wave reads its B fragments once
          // for 128 units -- half the activation path and LDS reads per
          // product of 256 x 128; falls back when the
          // fragment image (units padded to 256) does not cover the last tile
          // -- when the layer has enough of them to spread over the chip
          // beside the other streams' batches (a 4096-row batch's hidden
          // layer: 64); a small block (a 70-row streaming chunk: 2 tiles)
          // keeps the 256 x 128 tiles
          if (x6_variant() == 0 && !first && launch_w<W6Cfg<512, 128, 4, 2>, true>(s, p, kX6WideMinTiles)) {
            CE_HIP(hipGetLastError());
            return CE_GPU_OK;
          }
          return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>>(s, p);
        }
        [[fallthrough]];
      case 160:  // region-scheduled fp32-operand loop (round-2 default; a model without the fragment image)
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 8>(s, p);
#ifdef CATEARS_EXPERIMENTS
      case 40:  // 128 x 128 tiles: fills all CUs on a 1024-wide layer (one batch at a time on an idle GPU)
        return launch_f<X6Cfg<128, 128, 4, 2, 2>>(s, p);
      case 200:  // warp-specialised: 4 MFMA waves (64 x 64 each) + 4 producer waves
        return launch_ws<X6Cfg<128, 128, 2, 2, 2>, 4>(s, p);
      // 400: register-direct, both operands straight to registers, no LDS
      // (bit-identical; C3 4.50-4.52 vs 5.67-5.69 M frames/s, serial layers
      // 0.183 vs 0.127 ms: the activation fragments fetched by all four waves
      // along the units and split by each make it L1-bound)
      case 400:
        if (!a.wd || a.wd_kt * 32 < a.kpad || (reinterpret_cast<uintptr_t>(a.wd) & 15))
          return fail(CE_GPU_EINVAL, "variant 400 needs the weight fragment image");
        return launch_r<X6Cfg<kX6DirUnits, 128, 4, 2, 2>>(s, p);
      case 302:  // direct weights, 128 x 128 tiles (twice the blocks of 300)
        if (!a.wd) return fail(CE_GPU_EINVAL, "variant 302 needs the weight fragment image");
        return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
      case 320:  // direct weights, 256 x 128 tiles as 8 waves of 32 units x 128 frames: no weight
                 // fragment loaded by two waves (300: two waves along the frames share each)
        if (!a.wd) return fail(CE_GPU_EINVAL, "variant 320 needs the weight fragment image");
        if (first) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
        return launch_d<X6Cfg<kX6DirUnits, 128, 8, 1, 2>>(s, p);
      case 340:  // direct weights, 256 x 64 tiles of 4 waves (64 x 64 each): two blocks per CU,
                 // barriers over four waves instead of eight
        if (!a.wd) return fail(CE_GPU_EINVAL, "variant 340 needs the weight fragment image");
        if (first) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
        return launch_d<X6Cfg<kX6DirUnits, 64, 4, 1, 2>>(s, p);
      case 331:  // 300 with s_setprio 1 around the load issues
      case 332:  // 300 with s_setprio 1 around the MFMA regions
      case 333:  // ... around the load issues and the LDS writes
      case 334:  // ... around the load issues and the fragment reads
      case 335:  // the default's priority, activation loads issued at the top of the K-tile
        if (!a.wd) return fail(CE_GPU_EINVAL, "variants 331-335 need the weight fragment image");
        if (first) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
        if (x6_variant() == 331) return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>, 0, 1>(s, p);
        if (x6_variant() == 333) return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>, 0, 3>(s, p);
        if (x6_variant() == 334) return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>, 0, 4>(s, p);
        if (x6_variant() == 335) return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>, 0, 5>(s, p);
        return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>, 0, 2>(s, p);
#endif
#if defined(CATEARS_EXPERIMENTS) || defined(CATEARS_X6W)
      case 500:  // one wave per SIMD: 512 x 128 tiles, 4 waves of 128 units x 128 frames
      case 501:  // 512 x 64, 4 waves of 128 x 64
      case 502:  // 256 x 128, 4 waves of 64 x 128
      case 503:    // 256 x 256, 2 x 2 waves of 128 x 128
      case 504:    // 500 with the interleave pinned (sched_group_barrier)
      case 505:    // 501 with the interleave pinned
      case 506:    // 505 with the weights 7 unit blocks ahead (a ring of 8)
      case 507:    // 502 (256 x 128) with the interleave pinned and a ring of 4
      case 508: {  // 512 x 128 as 8 waves (two per SIMD) of 128 units x 64 frames, pinned, ring of 4
        if (!a.wd || a.wd_kt * 32 < a.kpad) return fail(CE_GPU_EINVAL, "variants 500-503 need the weight fragment image");
        if (first || a.wide) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
        const int v = x6_variant();
        const bool ok = v == 500   ? launch_w<W6Cfg<512, 128, 4, 1>>(s, p)
                        : v == 504 ? launch_w<W6Cfg<512, 128, 4, 1>, true>(s, p)
                        : v == 505 ? launch_w<W6Cfg<512, 64, 4, 1>, true>(s, p)
                        : v == 506 ? launch_w<W6Cfg<512, 64, 4, 1>, true, 8>(s, p)
                        : v == 507 ? launch_w<W6Cfg<256, 128, 4, 1>, true>(s, p)
                        : v == 508 ? launch_w<W6Cfg<512, 128, 4, 2>, true>(s, p)
                        : v == 501 ? launch_w<W6Cfg<512, 64, 4, 1>>(s, p)
                        : v == 502 ? launch_w<W6Cfg<256, 128, 4, 1>>(s, p)
                                   : launch_w<W6Cfg<256, 256, 2, 2>>(s, p);
        if (!ok) return launch_d<X6Cfg<kX6DirUnits, 128, 4, 2, 2>>(s, p);
        CE_HIP(hipGetLastError());
        return CE_GPU_OK;
      }
#endif
#ifdef CATEARS_EXPERIMENTS
      case 42:  // round-1 default: split of tile kt+1, then the MFMAs of tile kt
        return launch_f<X6Cfg<128, 256, 2, 4, 2>>(s, p);
      case 55:  // MFMAs of tile kt first, the split interleaved by the compiler
        return launch_f<X6Cfg<128, 256, 2, 4, 2>, 6>(s, p);
      case 202:  // 128 x 256: 4 MFMA waves of 64 x 128 + 4 producers
        return launch_ws<X6Cfg<128, 256, 2, 2, 2>, 4>(s, p);
      case 204:  // 128 x 256: 8 MFMA waves of 64 x 64 + 4 producers (3 waves per SIMD)
        return launch_ws<X6Cfg<128, 256, 2, 4, 2>, 4>(s, p);
#endif
#ifdef CATEARS_DIAG
      // ablations of the direct-weight default 300 (layers 2-7; wrong results,
      // timing only): 310 no split, 311 no activation stage writes, 312 no
      // activation path, 313 no weight loads, 314 no barrier, 315 no MFMAs,
      // 316 MFMAs only
      case 310:
      case 311:
      case 312:
      case 313:
      case 314:
      case 315:
      case 316: {
        if (!a.wd) return fail(CE_GPU_EINVAL, "ablations of 300 need the weight fragment image");
        using D = X6Cfg<kX6DirUnits, 128, 4, 2, 2>;
        if (first) return launch_d<X6Cfg<128, 128, 2, 4, 2>>(s, p);
        switch (x6_variant()) {
          case 310: return launch_d<D, 1>(s, p);
          case 311: return launch_d<D, 2>(s, p);
          case 312: return launch_d<D, 6>(s, p);
          case 313: return launch_d<D, 8>(s, p);
          case 314: return launch_d<D, 16>(s, p);
          case 315: return launch_d<D, 32>(s, p);
          default: return launch_d<D, 2 | 4 | 8 | 16>(s, p);
        }
      }
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
#endif
      default:
        return fail(CE_GPU_EINVAL, "bf16x6 schedule " + std::to_string(x6_variant()) +
                                       " is not in this build (the experiments library: `make EXPERIMENTS=1`)");
    }
  }
  // plane operands (CATEARS_X6_F32IN=0 / CE_GPU_GEMM_BF16X6_PLANES)
  return launch_q<X6Cfg<128, 128, 4, 2, 3>, 0>(s, p, out16);
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
