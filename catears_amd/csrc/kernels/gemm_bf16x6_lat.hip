// gemm_bf16x6_lat.hip -- latency mode of the TDNN GEMMs (ce_gpu_ctx_set_latency):
// the streaming AcousticModel chunk (src/am.cc:115-142: chunk_size + L + R
// rows, 70 for TDNN-S) or one utterance per call, where a row block is far
// too small to fill the chip with output tiles.
//
// Same contraction and products as gemm_bf16x6d_kernel (Splice + Narrow +
// LinearLayer + bias / ReLU / BatchNorm, src/nnet.cc:22-43,50-75,106-160;
// bf16x6: w0x0, w0x1, w1x0, w1x1, w0x2, w2x0 per K-tile, fp32 accumulate),
// with K split into S slices so a 70-row block still spreads over ~256 CUs:
//
//   lat_gemm_kernel    block (row tile, 64-unit column tile, slice s): every
//                      weight fragment of its <= 6 K-tiles is loaded at once,
//                      straight from the MFMA-fragment image into registers
//                      (X6Gemm::wd: the loads of the whole slice are in flight
//                      together -- a small block's K loop is latency bound
//                      otherwise), the activation tiles are split into bf16
//                      planes in LDS, and the slice's fp32 partial tile is
//                      stored to part[s][row][unit];
//   lat_reduce_kernel  sums the S partials of each output element in slice
//                      order, adds the bias and applies ReLU / BatchNorm in the
//                      reference's rounding order.
//
// The kernel boundary orders the partials for the reduction: no inter-block
// hand-off, no tickets, no fences.  S depends on K and N only
// (x6_lat_slices), never on the row count, so a row's result does not depend
// on the block it is scored in (AcousticModel batching contract).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "../internal.h"

namespace catears {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kLatNW = 4;              // waves per block, 16 units each
constexpr int kLatBW = 16 * kLatNW;    // units per block
constexpr int kLatMaxKt = 8;           // K-tiles (of 32) per slice: all its weights in registers
constexpr int kLatTarget = 256;        // blocks per row tile the slice rule aims at
constexpr int kLatTickets = kX6LatTickets;  // output tiles the fix-up can take

struct LatArgs {
  const float *xf;
  const uint16_t *wd;
  float *part;
  const int *row_map;
  int ldx, wd_kt;
  int m, n, kpad, din, nseg;
  uint64_t off_packed;
  int slices, per;  // S, K-tiles per slice
  int tiles_n, row0, rows;  // this window: rows row0 .. row0 + rows - 1
  int row_tiles, rtb;       // row tiles in the window, row tiles per block
  // FIX (lat_gemm_kernel): the tile's last slice block to finish does the
  // reduce + bias + post chain (lat_fix_tail) -- one ticket per output tile
  // (zeroed once at allocation, reset by that block)
  unsigned *tickets;
  const float *bias, *bn_scale, *bn_offset;
  float *y;
  int ldy;
  int post[4];
  int npost, post_mode;
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

// MULTI: the block loops over several row tiles (large windows); a single
// tile is straight-line code (a loop would make the compiler drain the weight
// loads before the activation loads are issued, at the loop header).
// KT: K-tiles per slice the block is sized for (>= the slice's per).
// The split-K fix-up (FIX, one row tile per block): the partial tiles are
// stored at agent scope (written through the XCD's L2 to the device's
// coherence point), each block waits for its stores to be acknowledged and
// takes its output tile's ticket, and the block that draws the last ticket
// reads the S partials back at agent scope, sums them in slice order
// (lat_slice_sum's order) and applies the bias and the post chain -- the
// reduce launch's arithmetic without its launch.  No block waits on another.
template <int TF>
__device__ __forceinline__ void lat_fix_tail(const LatArgs &p, int f0, int n0, int t, int *flag) {
  typedef unsigned long long u64;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned k = __hip_atomic_fetch_add(p.tickets + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = k == (unsigned)p.slices - 1;
  }
  __syncthreads();
  if (!flag[0]) return;
  constexpr int BF = 16 * TF, CH = BF * (kLatBW / 4);  // float4 chunks of the tile
  constexpr int NT = 64 * kLatNW, PER = (CH + NT - 1) / NT;
  const size_t stride = (size_t)p.rows * p.n;
  with_post_mode(p.post_mode, [&](auto M) {
    constexpr int MODE = decltype(M)::value;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int q = threadIdx.x + c * NT;
      const int f = f0 + q / (kLatBW / 4), n = n0 + 4 * (q % (kLatBW / 4));
      if (q >= CH || f >= p.row0 + p.rows || f >= p.m || n >= p.n) continue;
      const u64 *src = reinterpret_cast<const u64 *>(p.part + (size_t)(f - p.row0) * p.n + n);
      float4 sum = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      for (int s0 = 0; s0 < p.slices; s0 += 16) {
        u64 v[16][2];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (s0 + u < p.slices) {
            const u64 *a = src + (size_t)(s0 + u) * stride / 2;
            v[u][0] = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[u][1] = __hip_atomic_load(a + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (s0 + u < p.slices) {
            const float4 x = make_float4(__uint_as_float((uint32_t)v[u][0]), __uint_as_float((uint32_t)(v[u][0] >> 32)),
                                         __uint_as_float((uint32_t)v[u][1]), __uint_as_float((uint32_t)(v[u][1] >> 32)));
            sum = s0 + u == 0 ? x : make_float4(sum.x + x.x, sum.y + x.y, sum.z + x.z, sum.w + x.w);
          }
      }
      const f32x4 sm = f32x4{sum.x, sum.y, sum.z, sum.w};
      const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
      const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
      const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = apply_post<MODE>(sm[e] + bias[e], sc[e], of[e], p.post, p.npost);
      *reinterpret_cast<f32x4 *>(p.y + (int64_t)f * p.ldy + n) = y;
    }
  });
  if (threadIdx.x == 0) __hip_atomic_store(p.tickets + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int TF, int KT, bool MULTI, int DIAG = 0, bool FIX = false>
__global__ __launch_bounds__(64 * kLatNW, MULTI && TF == 4 && KT <= 6 ? 2 : 1) void lat_gemm_kernel(LatArgs p) {
  static_assert(!(FIX && MULTI), "the fix-up takes one row tile per block");
#ifndef CATEARS_DIAG
  static_assert(DIAG == 0, "diagnostic schedules are CATEARS_DIAG builds only");
#endif
  constexpr int BF = 16 * TF;
  constexpr int KSTAGE = 3 * BF * 64;  // bytes: the planes of one K-tile
  __shared__ __attribute__((aligned(1024))) char smem[KT * KSTAGE];
  typedef const __attribute__((address_space(1))) bf16x8 gfrag;
  typedef const __attribute__((address_space(1))) f32x4 gvec;
  auto swz = [](int row) { return ((row >> 3) & 1) << 1; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int s = blockIdx.x % p.slices, t = blockIdx.x / p.slices;
  const int ct = t % p.tiles_n, rg = t / p.tiles_n;
  const int n0 = ct * kLatBW;
  const int ktiles = p.kpad / 32, kt0 = s * p.per, nk = min(p.per, ktiles - kt0);

  // the activation rows of the slice: task q = (K-tile i, row, 8-float
  // chunk) spread evenly over the block's threads.  Every address first (the
  // row_map gather ahead of the weight loads: vector loads retire in order, so
  // a wait on it would otherwise wait on the weights too), then every load
  // (branch-free, so all of a thread's loads are in flight together), then the
  // splits and LDS stores.  A chunk's 8 k lie in one segment (din % 8 == 0);
  // k past the segments is K's zero padding, loaded from column 0 of the
  // clamped row; tasks past the slice load a clamped (valid) address.
  constexpr int NT = 64 * kLatNW, TASKS = KT * BF * 4, TPT = (TASKS + NT - 1) / NT;
  gvec *xptr[TPT];
  bool xlive[TPT];
  auto act_addr = [&](int rt) {
    const int f0 = p.row0 + rt * BF;
    int xrow[TPT], xcol[TPT];
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int q = min(tid + j * NT, TASKS - 1);
      const int i = q / (BF * 4), prow = (q >> 2) % BF, pch = q & 3;
      const int k = min(kt0 + i, ktiles - 1) * 32 + 8 * pch;
      const int seg = k / p.din, segc = min(seg, p.nseg - 1);
      const int shift = (int)(signed char)(p.off_packed >> (8 * segc));
      xrow[j] = clampi(clampi(f0 + prow, 0, p.m - 1) + shift, 0, p.m - 1);
      xlive[j] = tid + j * NT < TASKS && i < nk && seg < p.nseg && !(DIAG & 2);
      // a dead task (K padding past the segments, past the slice or the
      // task count) reads column 0 of its clamped row: never past the end
      // of the row, so never past the end of the caller's buffer
      xcol[j] = seg < p.nseg ? k - segc * p.din : 0;
    }
    if (p.row_map) {
#pragma unroll
      for (int j = 0; j < TPT; ++j) xrow[j] = p.row_map[xrow[j]];
    }
#pragma unroll
    for (int j = 0; j < TPT; ++j) xptr[j] = (gvec *)(p.xf + (size_t)xrow[j] * p.ldx + xcol[j]);
  };
  act_addr(rg * p.rtb);
  __builtin_amdgcn_sched_barrier(0);

  // 1. every weight fragment of the slice, at once (units n0 + 16 wave ..)
  bf16x8 wa[KT][3];
  {
    gfrag *wb = (gfrag *)(p.wd + ((size_t)((n0 >> 4) + wave) * p.wd_kt * 3 * 64 + lane) * 8);
    // branch-free: K-tiles past the slice load the last one (never used)
#pragma unroll
    for (int i = 0; i < KT; ++i)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        wa[i][pl] = wb[(min(kt0 + i, ktiles - 1) * 3 + pl) * 64];
        if (DIAG & 1) wa[i][pl] = bf16x8{};
      }
  }
  __builtin_amdgcn_sched_barrier(0);

  // the block's row tiles, one after another with the weights kept in
  // registers (a window of many row tiles reads each weight once per block)
  const int rt_end = min(p.row_tiles, (rg + 1) * p.rtb);
  const int foff = (lane & 15) * 64 + (((lane >> 4) ^ (((lane >> 3) & 1) << 1)) * 16);
  const int n = n0 + wave * 16 + 4 * (lane >> 4);
  for (int rt = rg * p.rtb; rt < rt_end; ++rt) {
  const int f0 = p.row0 + rt * BF;
  if (rt > rg * p.rtb) {
    __syncthreads();  // the previous tile's LDS reads are done
    act_addr(rt);
  }

  // 2. the activation rows (addresses computed above), split into planes
  f32x4 xv[TPT][2];
#pragma unroll
  for (int j = 0; j < TPT; ++j) {
    xv[j][0] = xptr[j][0];
    xv[j][1] = xptr[j][1];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < TPT; ++j) {
    const int q = tid + j * NT;
    const int i = q / (BF * 4), prow = (q >> 2) % BF, pch = q & 3;
    if (q >= TASKS || i >= nk) continue;
    const f32x4 zero = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const f32x4 v0 = xlive[j] ? xv[j][0] : zero, v1 = xlive[j] ? xv[j][1] : zero;
    const Planes2 q0 = split3_pair(v0.x, v0.y), q1 = split3_pair(v0.z, v0.w);
    const Planes2 q2 = split3_pair(v1.x, v1.y), q3 = split3_pair(v1.z, v1.w);
    char *st = smem + i * KSTAGE;
    const int off = prow * 64 + ((pch ^ swz(prow)) * 16);
    *reinterpret_cast<u32x4 *>(st + off) = u32x4{q0.h, q1.h, q2.h, q3.h};
    *reinterpret_cast<u32x4 *>(st + BF * 64 + off) = u32x4{q0.m, q1.m, q2.m, q3.m};
    *reinterpret_cast<u32x4 *>(st + 2 * BF * 64 + off) = u32x4{q0.l, q1.l, q2.l, q3.l};
  }
  __syncthreads();

  // 3. the slice's K-tiles in order, six products per tile in the order of
  //    every other bf16x6 kernel (per element: a0b0, a0b1, a1b0, a1b1, a0b2,
  //    a2b0)
  f32x4 acc[TF];
#pragma unroll
  for (int j = 0; j < TF; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    if (i >= nk) break;
    const char *st = smem + i * KSTAGE;
    const bf16x8 (&w)[3] = wa[i];
    bf16x8 b0[TF], b1[TF];
#pragma unroll
    for (int j = 0; j < TF; ++j) b0[j] = *reinterpret_cast<const bf16x8 *>(st + (j * 16) * 64 + foff);
#pragma unroll
    for (int j = 0; j < TF; ++j) b1[j] = *reinterpret_cast<const bf16x8 *>(st + (BF + j * 16) * 64 + foff);
    if constexpr ((DIAG & 4) != 0) {  // keep the operands live without the MFMAs
      const u32x4 a = __builtin_bit_cast(u32x4, w[0]) ^ __builtin_bit_cast(u32x4, w[1]) ^
                      __builtin_bit_cast(u32x4, w[2]) ^ __builtin_bit_cast(u32x4, b0[0]) ^
                      __builtin_bit_cast(u32x4, b1[TF - 1]);
      acc[0].x += __builtin_bit_cast(float, a.x ^ a.y ^ a.z ^ a.w);
      continue;
    }
#pragma unroll
    for (int j = 0; j < TF; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], b0[j], acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], b1[j], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], b0[j], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], b1[j], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(st + (2 * BF + j * 16) * 64 + foff);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], b2, acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], b0[j], acc[j], 0, 0, 0);
    }
  }

  // 4. the partial tile: lane holds units n .. n+3 of frame f per fragment
  if (n < p.n && !(DIAG & 8)) {
#pragma unroll
    for (int j = 0; j < TF; ++j) {
      const int f = f0 + j * 16 + (lane & 15);
      if (f >= p.row0 + p.rows || f >= p.m) continue;
      float *dst = p.part + ((size_t)s * p.rows + (f - p.row0)) * p.n + n;
      if constexpr (FIX) {
        typedef unsigned long long u64;
        const u64 lo = (u64)__float_as_uint(acc[j][0]) | (u64)__float_as_uint(acc[j][1]) << 32;
        const u64 hi = (u64)__float_as_uint(acc[j][2]) | (u64)__float_as_uint(acc[j][3]) << 32;
        __hip_atomic_store(reinterpret_cast<u64 *>(dst), lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(reinterpret_cast<u64 *>(dst) + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        *reinterpret_cast<f32x4 *>(dst) = acc[j];
      }
    }
  }
  if constexpr (FIX) lat_fix_tail<TF>(p, f0, n0, t, reinterpret_cast<int *>(smem));
  if constexpr (!MULTI) break;
  }  // row tiles
}

// The last layer's reduce fused into the finalize (LogSoftmax + log prior +
// row scatter): one 256-thread block per row, thread t holding float4 chunks
// t, t + 256, .. (rowops.hip finalize_vec_kernel's layout and order); each
// chunk summed over the slices exactly as lat_reduce_kernel does (+ bias,
// post chain), then the finalize's arithmetic in its order.
template <bool LOGSM, int MODE>
__global__ __launch_bounds__(256) void lat_finalize_kernel(LatTail t, int first, const float *prior,
                                                           const int *row_dst, float *out) {
  constexpr int kPer = 4;
  __shared__ float wsum[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int dst = row_dst ? row_dst[row] : row;
  if (dst < 0) return;  // block-uniform
  const int d4 = t.n >> 2;
  const float *src = t.part + (size_t)(first + row) * t.n;
  const size_t stride = (size_t)t.m * t.n;
  f32x4 v[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int c = min(tid + 256 * j, d4 - 1);  // clamped: used only when in range
    const float4 s4 = lat_slice_sum(src + 4 * c, stride, t.slices);
    const f32x4 bias = t.bias ? reinterpret_cast<const f32x4 *>(t.bias)[c] : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
    const f32x4 sc = t.bn_scale ? reinterpret_cast<const f32x4 *>(t.bn_scale)[c] : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
    const f32x4 of = t.bn_offset ? reinterpret_cast<const f32x4 *>(t.bn_offset)[c] : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
    const f32x4 sum = f32x4{s4.x, s4.y, s4.z, s4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) v[j][e] = apply_post<MODE>(sum[e] + bias[e], sc[e], of[e], t.post, t.npost);
  }
  float s = 0.0f;
  if (LOGSM) {
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (tid + 256 * j < d4) s += expf(v[j].x) + expf(v[j].y) + expf(v[j].z) + expf(v[j].w);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    if ((tid & 63) == 0) wsum[tid >> 6] = s;
    __syncthreads();
    s = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
  }
  const float ls = LOGSM ? logf(s) : 0.0f;
  f32x4 *o = reinterpret_cast<f32x4 *>(out + (int64_t)dst * t.n);
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int c = tid + 256 * j;
    if (c < d4) {
      f32x4 y = v[j];
      if (LOGSM) y = y - ls;
      if (prior) y = y - reinterpret_cast<const f32x4 *>(prior)[c];
      o[c] = y;
    }
  }
}

struct LatReduceArgs {
  const float *part;
  const float *bias, *bn_scale, *bn_offset;
  float *y;
  int slices, rows, n, row0, ldy;
  int post[4];
  int npost, post_mode;
};

// One thread per 4 consecutive units of one row: the slices' partials summed
// in slice order (the same value whatever row block the row was scored in),
// then + bias and the post chain (the GEMM epilogues' order and roundings).
template <int MODE>
__global__ __launch_bounds__(64) void lat_reduce_kernel(LatReduceArgs p) {
  const int n4 = p.n >> 2;
  const int64_t idx = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (idx >= (int64_t)p.rows * n4) return;
  const int r = (int)(idx / n4), n = (int)(idx - (int64_t)r * n4) * 4;
  const size_t stride = (size_t)p.rows * p.n;
  const float *src = p.part + (size_t)r * p.n + n;
  const float4 s4 = lat_slice_sum(src, stride, p.slices);
  const f32x4 sum = f32x4{s4.x, s4.y, s4.z, s4.w};
  const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4 *>(p.bias + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
  const f32x4 sc = p.bn_scale ? *reinterpret_cast<const f32x4 *>(p.bn_scale + n) : f32x4{1.0f, 1.0f, 1.0f, 1.0f};
  const f32x4 of = p.bn_offset ? *reinterpret_cast<const f32x4 *>(p.bn_offset + n) : f32x4{-0.0f, -0.0f, -0.0f, -0.0f};
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = apply_post<MODE>(sum[e] + bias[e], sc[e], of[e], p.post, p.npost);
  *reinterpret_cast<f32x4 *>(p.y + (int64_t)(p.row0 + r) * p.ldy + n) = v;
}

// Row tiles per block: enough blocks for two per CU (the many-tile kernel's
// occupancy), the rest looped with the weights kept in registers rather than
// re-read per tile.  The partition changes which block computes a tile, never
// the tile's sums.
int lat_rtb(int row_tiles, int blocks_per_tile) {
  static const int env = CE_KNOB("CATEARS_LAT_RTB", 0);
  const int rtb = env > 0 ? env : row_tiles * blocks_per_tile / (2 * kLatTarget);
  return std::max(1, std::min(rtb, row_tiles));
}

template <int TF, int KT>
void launch_lat_gemm_kt(hipStream_t s, const LatArgs &p, dim3 grid, dim3 block) {
#ifdef CATEARS_DIAG
  static const int diag = CE_KNOB("CATEARS_LAT_DIAG", 0);
  switch (diag) {
    case 0: break;
#define CE_LAT_DIAG(D) \
  case D: hipLaunchKernelGGL((lat_gemm_kernel<TF, KT, true, D>), grid, block, 0, s, p); return;
    CE_LAT_DIAG(1) CE_LAT_DIAG(2) CE_LAT_DIAG(3) CE_LAT_DIAG(4) CE_LAT_DIAG(8) CE_LAT_DIAG(12) CE_LAT_DIAG(15)
#undef CE_LAT_DIAG
    default: break;
  }
#endif
  if (p.rtb > 1)
    hipLaunchKernelGGL((lat_gemm_kernel<TF, KT, true>), grid, block, 0, s, p);
#ifdef CATEARS_EXPERIMENTS
  else if (p.tickets)
    hipLaunchKernelGGL((lat_gemm_kernel<TF, KT, false, 0, true>), grid, block, 0, s, p);
#endif
  else
    hipLaunchKernelGGL((lat_gemm_kernel<TF, KT, false>), grid, block, 0, s, p);
}

// Returns whether the GEMM also did the reduce (the fix-up: p.tickets set,
// one row tile per block, few enough output tiles for the ticket array).
template <int TF>
bool launch_lat_gemm(hipStream_t s, LatArgs p) {
  p.row_tiles = (p.rows + 16 * TF - 1) / (16 * TF);
  p.rtb = lat_rtb(p.row_tiles, p.tiles_n * p.slices);
  const int groups = (p.row_tiles + p.rtb - 1) / p.rtb;
  if (p.rtb > 1 || groups * p.tiles_n > kLatTickets) p.tickets = nullptr;
  const dim3 grid(groups * p.tiles_n * p.slices), block(64 * kLatNW);
  // the block sized for the slice (its weights all in registers)
  if (p.per <= 2)
    launch_lat_gemm_kt<TF, 2>(s, p, grid, block);
  else if (p.per <= 4)
    launch_lat_gemm_kt<TF, 4>(s, p, grid, block);
  else if (p.per <= 6)
    launch_lat_gemm_kt<TF, 6>(s, p, grid, block);
  else
    launch_lat_gemm_kt<TF, 8>(s, p, grid, block);
  return p.tickets != nullptr;
}

}  // namespace

// CATEARS_LAT_TARGET (experiments library only, tools/experiments/gpu_r5z16.sh):
// the blocks per row tile the slice rule aims at (default kLatTarget); other
// values change the fp32 summation order, so the product library ignores it.
static int lat_target() {
  static const int v = CE_KNOB("CATEARS_LAT_TARGET", 0);
  return v > 0 ? v : kLatTarget;
}

int x6_lat_slices(int kpad, int n) {
  const int ktiles = kpad / 32, cols = (n + kLatBW - 1) / kLatBW;
  // at most lat_target() blocks per row tile (one wave of blocks over the CUs)
  int slices = std::max(1, std::min(ktiles, lat_target() / cols));
  int per = (ktiles + slices - 1) / slices;
  per = std::min(per, kLatMaxKt);
  return (ktiles + per - 1) / per;  // no empty slice
}

size_t x6_lat_part_floats(int rows, int n, int slices) {
  return (size_t)std::min(rows, kX6LatWindow) * (size_t)n * (size_t)slices;
}

int launch_gemm_bf16x6_lat(hipStream_t s, const X6Gemm &a, float *part, size_t part_floats, unsigned *tickets) {
  if (a.tail) a.tail->active = false;
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  // the last layer's reduce inside the finalize when the rows are one window
  const bool reduce = !(a.tail && a.m <= kX6LatWindow && a.n % 4 == 0 && a.n <= 4096 && a.npost <= 4);
  if (!a.xf || !a.wd || (reduce && !a.y32) || a.kpad % 32 != 0 || a.din % 8 != 0 || a.din <= 0 || a.nseg < 1 ||
      a.nseg > 8 || a.nseg * a.din > a.kpad || a.wd_kt * 32 < a.kpad)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6 latency: bad K geometry or missing weight fragments");
  if (!reduce && a.m > kX6LatWindow)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6 latency: a deferred reduce needs rows <= kX6LatWindow");
  if (a.n % 4 != 0 || a.ldy % 4 != 0 || a.ldx % 4 != 0 || (reinterpret_cast<uintptr_t>(a.xf) & 15) ||
      (reinterpret_cast<uintptr_t>(a.wd) & 15) || a.npost > 4)
    return fail(CE_GPU_EINVAL, "gemm_bf16x6 latency: operands must be 16-byte aligned, widths multiples of 4");
  LatArgs p;
  p.xf = a.xf;
  p.wd = a.wd;
  p.part = part;
  p.ldx = a.ldx;
  p.wd_kt = a.wd_kt;
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
  p.slices = x6_lat_slices(a.kpad, a.n);
  p.per = (a.kpad / 32 + p.slices - 1) / p.slices;
  p.tiles_n = (a.n + kLatBW - 1) / kLatBW;
  LatReduceArgs r;
  r.part = part;
  r.bias = a.bias;
  r.bn_scale = a.bn_scale;
  r.bn_offset = a.bn_offset;
  r.y = a.y32;
  r.slices = p.slices;
  r.n = a.n;
  r.ldy = a.ldy;
  for (int i = 0; i < 4; ++i) r.post[i] = a.post[i];
  r.npost = a.npost;
  r.post_mode = post_mode(a.post, a.npost);
  // the fix-up (experiments library: CATEARS_LAT_FIXUP=1) for layers reduced
  // here; its tickets are zero between launches
#ifdef CATEARS_EXPERIMENTS
  static const int fixup = CE_KNOB("CATEARS_LAT_FIXUP", 0);
#else
  const int fixup = 0;
#endif
  p.tickets = fixup && reduce ? tickets : nullptr;
  p.bias = a.bias;
  p.bn_scale = a.bn_scale;
  p.bn_offset = a.bn_offset;
  p.y = a.y32;
  p.ldy = a.ldy;
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.post_mode = r.post_mode;
  for (int r0 = 0; r0 < a.m; r0 += kX6LatWindow) {
    p.row0 = r.row0 = r0;
    p.rows = r.rows = std::min(kX6LatWindow, a.m - r0);
    if ((size_t)p.rows * a.n * p.slices > part_floats || !part)
      return fail(CE_GPU_EINVAL, "gemm_bf16x6 latency: partial workspace too small");
    // the frame tile fitting the block (results do not depend on it)
    bool fixed;
    if (p.rows <= 32)
      fixed = launch_lat_gemm<2>(s, p);
    else if (p.rows <= 80)
      fixed = launch_lat_gemm<5>(s, p);
    else
      fixed = launch_lat_gemm<4>(s, p);  // many row tiles: 64-row tiles, two blocks per CU
    CE_HIP(hipGetLastError());
    if (fixed) continue;
    if (!reduce) {
      LatTail &t = *a.tail;
      t.active = true;
      t.part = part;
      t.slices = p.slices;
      t.m = a.m;
      t.n = a.n;
      t.bias = a.bias;
      t.bn_scale = a.bn_scale;
      t.bn_offset = a.bn_offset;
      for (int i = 0; i < 4; ++i) t.post[i] = a.post[i];
      t.npost = a.npost;
      break;
    }
    const int64_t threads = (int64_t)p.rows * (a.n / 4);
    const dim3 grid((unsigned)((threads + 63) / 64)), block(64);
    switch (r.post_mode) {
      case kPostModeNone: hipLaunchKernelGGL(lat_reduce_kernel<kPostModeNone>, grid, block, 0, s, r); break;
      case kPostModeRelu: hipLaunchKernelGGL(lat_reduce_kernel<kPostModeRelu>, grid, block, 0, s, r); break;
      case kPostModeBn: hipLaunchKernelGGL(lat_reduce_kernel<kPostModeBn>, grid, block, 0, s, r); break;
      case kPostModeReluBn: hipLaunchKernelGGL(lat_reduce_kernel<kPostModeReluBn>, grid, block, 0, s, r); break;
      case kPostModeBnRelu: hipLaunchKernelGGL(lat_reduce_kernel<kPostModeBnRelu>, grid, block, 0, s, r); break;
      default: hipLaunchKernelGGL(lat_reduce_kernel<kPostModeGeneric>, grid, block, 0, s, r); break;
    }
    CE_HIP(hipGetLastError());
  }
  return CE_GPU_OK;
}

int launch_lat_finalize(hipStream_t s, const LatTail &t, int first, int rows, bool log_softmax,
                        const float *log_prior, const int *row_dst, float *out) {
  if (rows <= 0) return CE_GPU_OK;
  if (!t.active || !t.part || !out || t.n % 4 != 0 || t.n > 4096 || first < 0 || first + rows > t.m ||
      t.npost > 4 ||
      ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(log_prior) |
        reinterpret_cast<uintptr_t>(t.bias) | reinterpret_cast<uintptr_t>(t.bn_scale) |
        reinterpret_cast<uintptr_t>(t.bn_offset)) & 15))
    return fail(CE_GPU_EINVAL, "lat_finalize: no deferred tail or bad geometry");
  const dim3 grid(rows), block(256);
  auto go = [&](auto ls) {
    constexpr bool LS = decltype(ls)::value;
    switch (post_mode(t.post, t.npost)) {
#define CE_LAT_FIN(M) \
  case M: hipLaunchKernelGGL((lat_finalize_kernel<LS, M>), grid, block, 0, s, t, first, log_prior, row_dst, out); break;
      CE_LAT_FIN(kPostModeNone) CE_LAT_FIN(kPostModeRelu) CE_LAT_FIN(kPostModeBn) CE_LAT_FIN(kPostModeReluBn)
      CE_LAT_FIN(kPostModeBnRelu)
#undef CE_LAT_FIN
      default:
        hipLaunchKernelGGL((lat_finalize_kernel<LS, kPostModeGeneric>), grid, block, 0, s, t, first, log_prior,
                           row_dst, out);
        break;
    }
  };
  if (log_softmax)
    go(std::true_type());
  else
    go(std::false_type());
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
