// gemm_bf16x6_lat.hip -- latency mode of the TDNN GEMMs (ce_gpu_ctx_set_latency):
// the streaming AcousticModel chunk (src/am.cc:115-142: chunk_size + L + R
// rows, 70 for TDNN-S) or one utterance per call, where a row block is far
// too small to fill the chip with the throughput kernel's 256 x 128 tiles.
//
// Same contraction and products as gemm_bf16x6d_kernel (Splice + Narrow +
// LinearLayer + bias / ReLU / BatchNorm, src/nnet.cc:22-43,50-75,106-160;
// bf16x6: w0x0, w0x1, w1x0, w1x1, w0x2, w2x0 per K-tile, fp32 accumulate),
// as ONE launch per layer with no partial buffer in memory:
//
//   block = 16 units x 16 TF rows, kL2Waves waves.  Wave w takes the K-tiles
//   [w per, (w + 1) per) (per = ceil(K-tiles / kL2Waves): a function of K
//   only).  Both operands go straight to registers: the weights from the
//   MFMA-fragment image (X6Gemm::wd, one global_load_dwordx4 per lane and
//   plane), the activations as the lane's 8 consecutive floats of one row
//   (two 16-byte loads, through the splice offsets and, for the first layer,
//   the caller's row_map), split into the three bf16 planes in registers --
//   the B-fragment layout of v_mfma_f32_16x16x32_bf16 is one row's 8
//   consecutive k per lane, so no LDS transpose is needed.  The next K-tile's
//   loads are in flight during this one's MFMAs.  At the end the four waves'
//   fp32 partial tiles meet in LDS and are summed in wave order
//   (((p0 + p1) + p2) + p3), + bias, ReLU / BatchNorm in the reference's
//   rounding order, stored.
//
// Small row blocks get many blocks from the 16-unit tiles (70 rows of a
// 1024-unit layer: 64 x 5 = 320 blocks), so no K split across blocks -- and
// no reduce launch -- is needed to spread a chunk over the chip.  The sum
// order depends on K only, never on the row count or the tile shape (TF), so
// a row's result does not depend on the block it is scored in
// (AcousticModel's batching contract).
#include <hip/hip_runtime.h>

#include "../internal.h"

namespace catears {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kL2Waves = 4;  // K split among a block's waves (part of the summation order)

struct Lat2Args {
  const float *xf;
  const uint16_t *wd;
  const int *row_map;
  int ldx, wd_kt;
  int m, n, kpad, din, nseg;
  uint64_t off_packed;
  int per, tiles_n;
  const float *bias, *bn_scale, *bn_offset;
  int post[4];
  int npost;
  float *y;
  int ldy;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// v = h + m + l in bf16 for two values (the same conversions as
// gemm_bf16x6.hip split3_pair: bit-identical planes)
struct Planes2 {
  uint32_t h, m, l;
};
__device__ __forceinline__ Planes2 split3_pair(float a, float b) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  auto cvt = [](float x, float y) { return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){x, y}, bf16x2)); };
  auto lo = [](uint32_t u) { return __builtin_bit_cast(float, u << 16); };
  auto hi = [](uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); };
  const uint32_t p0 = cvt(a, b);
  const float ra = a - lo(p0), rb = b - hi(p0);
  const uint32_t p1 = cvt(ra, rb);
  const float sa = ra - lo(p1), sb = rb - hi(p1);
  return Planes2{p0, p1, cvt(sa, sb)};
}

// One K-tile's operands of a wave, in registers.
template <int TF>
struct Tile {
  bf16x8 w[3];
  f32x4 x[TF][2];
};

template <int TF>
__device__ __forceinline__ void load_tile(const Lat2Args &p, int kt, int f0, int lane,
                                          const __attribute__((address_space(1))) bf16x8 *wb, Tile<TF> &t) {
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) t.w[pl] = wb[(kt * 3 + pl) * 64];
  // this lane's 8 k of the K-tile lie in one segment (din % 8 == 0); k past
  // the segments is K's zero padding: column 0 of a valid row is read and the
  // value replaced by zeros (the address stays inside the row)
  const int k = kt * 32 + 8 * (lane >> 4);
  const int seg = k / p.din, segc = min(seg, p.nseg - 1);
  const int shift = (int)(signed char)(p.off_packed >> (8 * segc));
  const int col = seg < p.nseg ? k - segc * p.din : 0;
#pragma unroll
  for (int j = 0; j < TF; ++j) {
    int row = clampi(clampi(f0 + 16 * j + (lane & 15), 0, p.m - 1) + shift, 0, p.m - 1);
    if (p.row_map) row = p.row_map[row];
    const f32x4 *src = reinterpret_cast<const f32x4 *>(p.xf + (size_t)row * p.ldx + col);
    t.x[j][0] = src[0];
    t.x[j][1] = src[1];
  }
  if (seg >= p.nseg) {
#pragma unroll
    for (int j = 0; j < TF; ++j) t.x[j][0] = t.x[j][1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  }
}

// the six products of one K-tile, per element in the order of every bf16x6
// kernel: a0b0, a0b1, a1b0, a1b1, a0b2, a2b0
template <int TF>
__device__ __forceinline__ void mma_tile(const Tile<TF> &t, f32x4 (&acc)[TF]) {
  bf16x8 b0[TF], b1[TF], b2[TF];
#pragma unroll
  for (int j = 0; j < TF; ++j) {
    const f32x4 v0 = t.x[j][0], v1 = t.x[j][1];
    const Planes2 q0 = split3_pair(v0.x, v0.y), q1 = split3_pair(v0.z, v0.w);
    const Planes2 q2 = split3_pair(v1.x, v1.y), q3 = split3_pair(v1.z, v1.w);
    b0[j] = __builtin_bit_cast(bf16x8, u32x4{q0.h, q1.h, q2.h, q3.h});
    b1[j] = __builtin_bit_cast(bf16x8, u32x4{q0.m, q1.m, q2.m, q3.m});
    b2[j] = __builtin_bit_cast(bf16x8, u32x4{q0.l, q1.l, q2.l, q3.l});
  }
#pragma unroll
  for (int j = 0; j < TF; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t.w[0], b0[j], acc[j], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < TF; ++j) {
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t.w[0], b1[j], acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t.w[1], b0[j], acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t.w[1], b1[j], acc[j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < TF; ++j) {
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t.w[0], b2[j], acc[j], 0, 0, 0);
    acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(t.w[2], b0[j], acc[j], 0, 0, 0);
  }
}

template <int TF, int MODE>
__global__ __launch_bounds__(64 * kL2Waves) void lat2_kernel(Lat2Args p) {
  __shared__ f32x4 red[kL2Waves][TF][64];
  typedef const __attribute__((address_space(1))) bf16x8 gfrag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ct = blockIdx.x % p.tiles_n, rt = blockIdx.x / p.tiles_n;
  const int f0 = rt * 16 * TF;
  const int ktiles = p.kpad / 32, kt0 = wave * p.per, kt1 = min(kt0 + p.per, ktiles);
  gfrag *wb = (gfrag *)(p.wd + ((size_t)ct * p.wd_kt * 3 * 64 + lane) * 8);

  f32x4 acc[TF];
#pragma unroll
  for (int j = 0; j < TF; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  if (kt0 < kt1) {
    Tile<TF> cur, nxt;
    load_tile<TF>(p, kt0, f0, lane, wb, cur);
    int kt = kt0;
    for (; kt + 1 < kt1; kt += 2) {
      load_tile<TF>(p, kt + 1, f0, lane, wb, nxt);
      mma_tile<TF>(cur, acc);
      if (kt + 2 < kt1) load_tile<TF>(p, kt + 2, f0, lane, wb, cur);
      mma_tile<TF>(nxt, acc);
    }
    if (kt < kt1) mma_tile<TF>(cur, acc);
  }

  // the waves' partial tiles, summed in wave order; lane holds units
  // n .. n+3 of frame f of each fragment
#pragma unroll
  for (int j = 0; j < TF; ++j) red[wave][j][lane] = acc[j];
  __syncthreads();
  const int n = ct * 16 + 4 * (lane >> 4);
  if (n >= p.n) return;
  const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
  const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
  const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
  for (int j = wave; j < TF; j += kL2Waves) {
    const int f = f0 + 16 * j + (lane & 15);
    if (f >= p.m) continue;
    f32x4 s = red[0][j][lane];
#pragma unroll
    for (int w = 1; w < kL2Waves; ++w) s += red[w][j][lane];
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = apply_post<MODE>(s[e] + bias[e], sc[e], of[e], p.post, p.npost);
    *reinterpret_cast<f32x4 *>(p.y + (int64_t)f * p.ldy + n) = v;
  }
}

template <int TF>
void launch_lat2(hipStream_t s, const Lat2Args &p, int mode) {
  const int64_t blocks = (int64_t)p.tiles_n * ((p.m + 16 * TF - 1) / (16 * TF));
  const dim3 grid((unsigned)blocks), block(64 * kL2Waves);
  switch (mode) {
    case kPostModeNone: hipLaunchKernelGGL((lat2_kernel<TF, kPostModeNone>), grid, block, 0, s, p); break;
    case kPostModeRelu: hipLaunchKernelGGL((lat2_kernel<TF, kPostModeRelu>), grid, block, 0, s, p); break;
    case kPostModeBn: hipLaunchKernelGGL((lat2_kernel<TF, kPostModeBn>), grid, block, 0, s, p); break;
    case kPostModeReluBn: hipLaunchKernelGGL((lat2_kernel<TF, kPostModeReluBn>), grid, block, 0, s, p); break;
    case kPostModeBnRelu: hipLaunchKernelGGL((lat2_kernel<TF, kPostModeBnRelu>), grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL((lat2_kernel<TF, kPostModeGeneric>), grid, block, 0, s, p); break;
  }
}

}  // namespace

int launch_gemm_bf16x6_lat(hipStream_t s, const X6Gemm &a) {
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  if (!a.xf || !a.wd || !a.y32 || a.kpad % 32 != 0 || a.din % 8 != 0 || a.din <= 0 || a.nseg < 1 || a.nseg > 8 ||
      a.nseg * a.din > a.kpad || a.wd_kt * 32 < a.kpad)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6 latency: bad K geometry or missing weight fragments");
  if (a.n % 4 != 0 || a.ldy % 4 != 0 || a.ldx % 4 != 0 || (reinterpret_cast<uintptr_t>(a.xf) & 15) ||
      (reinterpret_cast<uintptr_t>(a.wd) & 15) || a.npost > 4)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6 latency: operands must be 16-byte aligned, widths multiples of 4");
  Lat2Args p;
  p.xf = a.xf;
  p.wd = a.wd;
  p.row_map = a.row_map;
  p.ldx = a.ldx;
  p.wd_kt = a.wd_kt;
  p.m = a.m;
  p.n = a.n;
  p.kpad = a.kpad;
  p.din = a.din;
  p.nseg = a.nseg;
  p.off_packed = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (a.off[i] < -128 || a.off[i] > 127) return fail(CE_GPU_ENOTSUP, "gemm_bf16x6: splice offset beyond +-127");
    p.off_packed |= (uint64_t)(uint8_t)(int8_t)a.off[i] << (8 * i);
  }
  p.per = (a.kpad / 32 + kL2Waves - 1) / kL2Waves;
  p.tiles_n = (a.n + 15) / 16;
  p.bias = a.bias;
  p.bn_scale = a.bn_scale;
  p.bn_offset = a.bn_offset;
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.y = a.y32;
  p.ldy = a.ldy;
  const int mode = post_mode(a.post, a.npost);
  // the row tile fitting the block count (results do not depend on it):
  // streaming chunks get 16-row tiles, whole utterances 64-row tiles that
  // reuse each weight fragment four times
  if (a.m <= 128)
    launch_lat2<1>(s, p, mode);
  else
    launch_lat2<4>(s, p, mode);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
