// gemm_f16x3.hip -- the TDNN layers' fp32 GEMM on the fp16 matrix cores,
// operands as two scaled fp16 planes, three MFMA products.
//
// Same contraction as gemm_f32.hip / gemm_bf16x6.hip (Splice + Narrow +
// LinearLayer + bias / ReLU / BatchNorm, src/nnet.cc:22-43,50-75,106-117,
// 149-160,182-202; MatMat -> cblas_sgemm, src/matrix.cc:300-323).
//
// Representation.  An fp32 value x, pre-scaled by a power of two s (exact),
// is stored as two fp16 planes
//     u = x * 2^s,  x0 = f16(u),  x1 = f16((u - x0) * 2^11)
// so u = x0 + 2^-11 x1 to 22-23 significant bits (fp16 keeps 11; the
// subtraction is exact; u - x0 <= 2^-11 |u| keeps x1 in range).  Below fp16's
// normal range the absolute error stays under 2^-35 (in units of u).
// Activations use s = -8 (range |x| < 1.6e7, see the overflow flag below);
// each layer's weights a per-layer s chosen at load so max |w| 2^s < 2^15.
//
// Product.  w . x = w0 x0 + 2^-11 (w0 x1 + w1 x0) + 2^-22 w1 x1: the first
// two groups are accumulated in fp32 in two accumulator sets (acc0, acc1;
// fp16 x fp16 products are exact in the MFMA), the last term (< 2^-22 |w x|)
// is dropped, and the epilogue forms (acc0 + 2^-11 acc1) * 2^-(sw + sx).
// Measured on TDNN-S: log-likelihood error vs an fp64 evaluation equal to the
// fp32-MFMA path's (tests/test_gpu_parity.py).  Cost: 3 fp16 MFMAs per fp32
// multiply-add at 16x the fp32 MFMA rate (5.3x the fp32 ceiling), 4 bytes
// per operand element (as fp32).
//
// Overflow: a hidden layer's output beyond the activation range (or not
// finite) cannot be stored exactly; the epilogue then sets the context's
// overflow word (ce_gpu_ctx_overflow) and the caller reruns with
// CE_GPU_GEMM_FP32 or BF16X6.  Normalised TDNN activations are O(1-100).
//
// Layout (HBM), element = 16 bits:
//   weights  n x ldw, row j = [plane0 | plane1], plane stride pw (= kpad)
//   acts     rows x ldx, row r = [plane0 | plane1], plane stride px
//   output   split (hidden layer) or fp32 (the last layer; finalize reads it)
// MFMA A = weights (M = output units), B = activations (N = frames), so a
// lane's accumulator holds four consecutive units of one frame.
//
// Tiling: BW units x BF frames per block, K-tile BK (32 or 64) per LDS stage,
// WGW x WGF waves.  LDS-DMA (global_load_lds_dwordx4) moves one wave
// instruction = 1 KB = 1024 / (2 BK) rows of one plane; with BK = 64 that is
// 8 whole 128-B lines.  16-B chunk c of tile row r is stored at c ^ swz(r),
// applied on the source address, so every 16-lane group of a ds_read_b128
// fragment read ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) hits 16
// distinct bank slots (MI355X_MICROARCH.md, LDS).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "../internal.h"
#include "../lds_dma.h"
#include "../tile_order.h"

namespace catears {
namespace {

using dma::clampi;
using dma::glds16;
using dma::wait_vmcnt;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

constexpr float kLoScale = 2048.0f;          // x1 = residual * 2^11
constexpr float kLoUnscale = 1.0f / 2048.0f;
constexpr float kActScale = 1.0f / 256.0f;   // activations stored as x * 2^-8
constexpr float kActLimit = 16000000.0f;     // |x| 2^-8 stays below fp16's 65504

struct X3Args {
  const uint16_t *w;  // weights, n x ldw, plane stride pw
  const uint16_t *x;  // activations, rows x ldx, plane stride px
  const float *bias, *bn_scale, *bn_offset;
  float *y32;         // fp32 output (ldy floats per row), or
  uint16_t *y16;      // split output (ldy elements per row, plane stride py)
  int *overflow;      // set when a split output leaves the fp16 range
  int ldw, pw, ldx, px, ldy, py;
  int m, n, kpad, din;
  float unscale;      // 2^-(sw + sx): accumulator -> fp32 product
  uint64_t off_packed;  // splice offset of segment s in signed byte s
  int post[4];
  int npost, post_mode;
  int tiles_m, tiles_n, group;
};

__device__ __forceinline__ uint16_t h_bits(_Float16 h) { return __builtin_bit_cast(uint16_t, h); }

// u = x * 2^-8 -> (hi, lo) planes
__device__ __forceinline__ void split2(float v, uint16_t *h, uint16_t *l) {
  const float u = v * kActScale;
  const _Float16 x0 = (_Float16)u;
  *h = h_bits(x0);
  *l = h_bits((_Float16)((u - (float)x0) * kLoScale));
}

template <int BW_, int BF_, int WGW_, int WGF_, int STAGES_, int BK_>
struct X3Cfg {
  static constexpr int BW = BW_, BF = BF_, WGW = WGW_, WGF = WGF_, STAGES = STAGES_, BK = BK_;
  static constexpr int NW = WGW * WGF, NT = 64 * NW;
  static constexpr int TW = BW / WGW / 16, TF = BF / WGF / 16;  // 16 x 16 fragments per wave
  static constexpr int RB = 2 * BK;                              // bytes per tile row per plane
  static constexpr int CPR = RB / 16, RPI = 1024 / RB;           // 16-B chunks per row, rows per DMA
  static constexpr int QW = 2 * BW / RPI, QF = 2 * BF / RPI;     // DMA instructions per stage
  static constexpr int NQW = QW / NW, NQF = QF / NW;
  static constexpr int STAGE = 2 * (BW + BF) * RB;               // bytes per stage
  static constexpr int KS = BK / 32;                             // MFMA k-steps per K-tile
  static_assert(BK == 32 || BK == 64, "K-tile of 32 or 64");
  static_assert(TW >= 1 && TF >= 1 && QW % NW == 0 && QF % NW == 0, "bad f16x3 tile");
  static_assert(STAGES >= 2 && STAGES <= 4, "2..4 LDS stages");
  static_assert(STAGES * STAGE <= 160 * 1024, "LDS");
  // chunk c of tile row r is stored at chunk c ^ swz(r)
  __device__ static constexpr int swz(int r) { return BK == 32 ? ((r >> 3) & 1) << 1 : (r >> 1) & 7; }
};

template <class C, bool OUT16>
__global__ __launch_bounds__(C::NT, 1) void gemm_f16x3_kernel(X3Args p) {
  constexpr int BW = C::BW, BF = C::BF, TW = C::TW, TF = C::TF, RB = C::RB, CPR = C::CPR, RPI = C::RPI;
  constexpr int NQW = C::NQW, NQF = C::NQF, STAGES = C::STAGES, STAGE = C::STAGE, KS = C::KS, BK = C::BK;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ww = wave / C::WGF, wf = wave % C::WGF;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int f0 = tm * BF, n0 = tn * BW;

  // DMA lane geometry: lane -> (row lane / CPR of the instruction's RPI, chunk lane % CPR)
  const int lrow = lane / CPR, lch = lane % CPR;
  uint32_t woff[NQW];
#pragma unroll
  for (int i = 0; i < NQW; ++i) {
    const int q = wave * NQW + i, plane = q / (BW / RPI), row = (q % (BW / RPI)) * RPI + lrow;
    woff[i] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + plane * p.pw + 8 * (lch ^ C::swz(row))) * 2);
  }
  uint32_t xoff[NQF];
  int cur_seg = -1;
  auto issue = [&](int kt) {
    const int k0 = kt * BK;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
      for (int i = 0; i < NQF; ++i) {
        const int q = wave * NQF + i, plane = q / (BF / RPI), row = (q % (BF / RPI)) * RPI + lrow;
        const int src = clampi(f0 + row + shift, 0, p.m - 1);
        xoff[i] = (uint32_t)((src * p.ldx + plane * p.px + 8 * (lch ^ C::swz(row))) * 2);
      }
    }
    char *st = smem + (kt % STAGES) * STAGE;
    const char *wbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 2;
    const char *xbase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 2;
#pragma unroll
    for (int i = 0; i < NQW; ++i) glds16(wbase + woff[i], st + (wave * NQW + i) * 1024);
#pragma unroll
    for (int i = 0; i < NQF; ++i) glds16(xbase + xoff[i], st + 2 * BW * RB + (wave * NQF + i) * 1024);
  };

  // fragment read: lane reads row (lane & 15) of a 16-row fragment, logical
  // chunk 4 ks + (lane >> 4) (k = 32 ks + 8 (lane >> 4) .. +7)
  const int r16 = lane & 15;
  int foff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) foff[ks] = r16 * RB + (((4 * ks + (lane >> 4)) ^ C::swz(r16)) * 16);
  const int wrow = ww * TW * 16, frow = wf * TF * 16;

  f32x4 acc0[TW][TF], acc1[TW][TF];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < TF; ++j) acc0[i][j] = acc1[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  const int ktiles = p.kpad / BK;
  constexpr int NQ = NQW + NQF;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < ktiles) issue(s);
  for (int kt = 0; kt < ktiles; ++kt) {
    // this wave's DMAs for tile kt are done when at most the younger tiles'
    // (up to STAGES - 2 of them) are outstanding
    const int younger = min(ktiles - 1 - kt, STAGES - 2);
    if (STAGES >= 4 && younger >= 2)
      wait_vmcnt<(STAGES >= 4 ? 2 : 0) * NQ>();
    else if (STAGES >= 3 && younger >= 1)
      wait_vmcnt<NQ>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's tile kt landed; stage (kt-1) % STAGES is free
    if (kt + STAGES - 1 < ktiles) issue(kt + STAGES - 1);
    const char *st = smem + (kt % STAGES) * STAGE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f16x8 a[2][TW], b[2][TF];
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
#pragma unroll
        for (int i = 0; i < TW; ++i) a[pl][i] = *reinterpret_cast<const f16x8 *>(st + (pl * BW + wrow + i * 16) * RB + foff[ks]);
#pragma unroll
        for (int j = 0; j < TF; ++j)
          b[pl][j] = *reinterpret_cast<const f16x8 *>(st + 2 * BW * RB + (pl * BF + frow + j * 16) * RB + foff[ks]);
      }
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) acc0[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0][i], b[0][j], acc0[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TW; ++i)
#pragma unroll
        for (int j = 0; j < TF; ++j) {
          acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0][i], b[1][j], acc1[i][j], 0, 0, 0);
          acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1][i], b[0][j], acc1[i][j], 0, 0, 0);
        }
    }
  }

  // Epilogue: lane holds units n .. n+3 of frame f per fragment pair.  The
  // product, + bias, the post chain in model order with the reference's
  // roundings (an absent bias adds -0, the identity).  n % 4 == 0 (host).
  bool over = false;
  with_post_mode(p.post_mode, [&](auto M) {
#pragma unroll
    for (int i = 0; i < TW; ++i) {
      const int n = n0 + wrow + i * 16 + 4 * (lane >> 4);
      if (n >= p.n) continue;
      const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
      const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
      const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
#pragma unroll
      for (int j = 0; j < TF; ++j) {
        const int f = f0 + frow + j * 16 + r16;
        if (f >= p.m) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float prod = (acc0[i][j][e] + acc1[i][j][e] * kLoUnscale) * p.unscale;
          v[e] = apply_post<decltype(M)::value>(prod + bias[e], sc[e], of[e], p.post, p.npost);
        }
        if constexpr (OUT16) {
          uint16_t h[4], l[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            over |= !(__builtin_fabsf(v[e]) < kActLimit);
            split2(v[e], &h[e], &l[e]);
          }
          uint16_t *dst = p.y16 + (int64_t)f * p.ldy + n;
          *reinterpret_cast<u16x4 *>(dst) = u16x4{h[0], h[1], h[2], h[3]};
          *reinterpret_cast<u16x4 *>(dst + p.py) = u16x4{l[0], l[1], l[2], l[3]};
        } else {
          *reinterpret_cast<f32x4 *>(p.y32 + (int64_t)f * p.ldy + n) = v;
        }
      }
    }
  });
  if (OUT16 && __builtin_amdgcn_ballot_w64(over) != 0 && lane == 0) atomicOr(p.overflow, 1);
}

// First layer: splice_pad_kernel's block (rows x po, zero padded) written as
// the two activation planes.  Features beyond the range set the flag too.
struct SpliceIdx8 {
  int v[8];
};

__global__ __launch_bounds__(256) void splice_pad_f16_kernel(const float *__restrict__ in, int ld_in, int rows,
                                                             int din, int nseg, SpliceIdx8 idx,
                                                             const int *__restrict__ row_map,
                                                             uint16_t *__restrict__ out, int po, int *overflow) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  uint16_t *o = out + (int64_t)r * 2 * po;
  bool over = false;
  for (int c = lane; c < po; c += 64) {
    const int s = c / din;
    float v = 0.0f;
    if (s < nseg) {
      int src = clampi(r + idx.v[s], 0, rows - 1);
      if (row_map) src = row_map[src];
      v = in[(int64_t)src * ld_in + (c - s * din)];
    }
    over |= !(__builtin_fabsf(v) < kActLimit);
    uint16_t h, l;
    split2(v, &h, &l);
    o[c] = h;
    o[po + c] = l;
  }
  if (__builtin_amdgcn_ballot_w64(over) != 0 && lane == 0) atomicOr(overflow, 1);
}

template <class C>
int launch_cfg(hipStream_t s, X3Args p, bool out16) {
  p.tiles_n = (p.n + C::BW - 1) / C::BW;
  p.tiles_m = (p.m + C::BF - 1) / C::BF;
  if (p.kpad % C::BK != 0 || p.din % C::BK != 0)
    return fail(CE_GPU_EINVAL, "gemm_f16x3: K-tile must lie inside one splice segment");
  dim3 grid(p.tiles_m * p.tiles_n), block(C::NT);
  if (out16)
    hipLaunchKernelGGL((gemm_f16x3_kernel<C, true>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f16x3_kernel<C, false>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int x3_variant() {
  static int v = CE_KNOB("CATEARS_X3_VARIANT", 0);
  return v;
}

}  // namespace

int launch_gemm_f16x3(hipStream_t s, const X3Gemm &a) {
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  if (a.kpad % 32 != 0 || a.din % 32 != 0 || a.nseg < 1 || a.nseg > 8 || a.nseg * a.din > a.kpad)
    return fail(CE_GPU_EINVAL, "gemm_f16x3: bad K geometry");
  if (a.n % 4 != 0 || a.ldy % 4 != 0 || (a.y16 && (a.py % 4 != 0 || !a.overflow)))
    return fail(CE_GPU_EINVAL, "gemm_f16x3: output width must be a multiple of 4");
  if (a.ldw % 8 || a.pw % 8 || a.ldx % 8 || a.px % 8 || (reinterpret_cast<uintptr_t>(a.w) & 15) ||
      (reinterpret_cast<uintptr_t>(a.x) & 15))
    return fail(CE_GPU_EINVAL, "gemm_f16x3: operands must be 16-byte aligned");
  if ((int64_t)a.n * a.ldw * 2 >= ((int64_t)1 << 32) || (int64_t)a.m * a.ldx * 2 >= ((int64_t)1 << 32))
    return fail(CE_GPU_EINVAL, "gemm_f16x3: operand beyond 4 GiB");
  if (a.npost > 4) return fail(CE_GPU_EINVAL, "gemm_f16x3: too many post ops");
  X3Args p;
  p.w = a.w;
  p.x = a.x;
  p.bias = a.bias;
  p.bn_scale = a.bn_scale;
  p.bn_offset = a.bn_offset;
  p.y32 = a.y32;
  p.y16 = a.y16;
  p.overflow = a.overflow;
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
  p.unscale = a.unscale;
  p.off_packed = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (a.off[i] < -128 || a.off[i] > 127) return fail(CE_GPU_ENOTSUP, "gemm_f16x3: splice offset beyond +-127");
    p.off_packed |= (uint64_t)(uint8_t)(int8_t)a.off[i] << (8 * i);
  }
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.post_mode = post_mode(a.post, a.npost);
  p.group = 8;
  const bool out16 = a.y16 != nullptr;
  // K-tiles of 64 need every segment (and the padded K) a multiple of 64
  const bool k64 = a.din % 64 == 0 && a.kpad % 64 == 0;
  switch (x3_variant()) {
    case 0:
      return k64 ? launch_cfg<X3Cfg<128, 128, 2, 4, 2, 64>>(s, p, out16)
                 : launch_cfg<X3Cfg<128, 128, 2, 4, 3, 32>>(s, p, out16);
#ifdef CATEARS_EXPERIMENTS
    case 1:
      return launch_cfg<X3Cfg<128, 128, 2, 4, 3, 32>>(s, p, out16);
    case 2:
      return k64 ? launch_cfg<X3Cfg<128, 128, 2, 2, 2, 64>>(s, p, out16)
                 : launch_cfg<X3Cfg<128, 128, 2, 2, 3, 32>>(s, p, out16);
    case 3:
      return launch_cfg<X3Cfg<128, 256, 2, 4, 3, 32>>(s, p, out16);
    case 4:
      return launch_cfg<X3Cfg<256, 128, 4, 2, 3, 32>>(s, p, out16);
    case 5:
      return launch_cfg<X3Cfg<128, 128, 2, 4, 2, 32>>(s, p, out16);
    case 6:
      return launch_cfg<X3Cfg<128, 128, 2, 4, 4, 32>>(s, p, out16);
    case 7:
      return k64 ? launch_cfg<X3Cfg<64, 256, 1, 4, 2, 64>>(s, p, out16)
                 : launch_cfg<X3Cfg<128, 256, 2, 4, 3, 32>>(s, p, out16);
#endif
    default:
      return fail(CE_GPU_EINVAL, "f16x3 variant " + std::to_string(x3_variant()) +
                                     " is not in this build (the experiments library: `make EXPERIMENTS=1`)");
  }
}

int launch_splice_pad_f16(hipStream_t s, const float *in, int ld_in, int rows, int din, int nseg, const int *off,
                          const int *row_map, uint16_t *out, int po, int *overflow) {
  if (nseg < 1 || nseg > 8 || nseg * din > po || !overflow)
    return fail(CE_GPU_EINVAL, "splice_pad_f16: bad geometry");
  SpliceIdx8 idx = {};
  for (int i = 0; i < nseg; ++i) idx.v[i] = off[i];
  if (rows > 0)
    hipLaunchKernelGGL(splice_pad_f16_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, in, ld_in, rows, din, nseg,
                       idx, row_map, out, po, overflow);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
