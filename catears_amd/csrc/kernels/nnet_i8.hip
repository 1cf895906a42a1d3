// nnet_i8.hip -- the int8 nnet path (BASELINE config C5): every LinearLayer
// as Quantize + MatMat_U8U8F32 + bias (src/matrix.cc:329-420, the pieces the
// reference ships but never wires into Nnet, src/nnet.cc:29).
//
// Per layer and per chunk of packed rows:
//   1. minmax_kernel     min / max over the layer input X (rows x width; the
//      params_kernel     first layer reads its rows through row_map): block
//                        partials, then one block folds them, both seeded
//                        with FLT_MAX and FLT_MIN exactly like FindMinMax
//                        (matrix.cc:331-345: max starts at FLT_MIN), and
//                        applies ComputeQuantizationParams (matrix.cc:348-362).
//                        Only rows the reference chain still holds count: the
//                        packed buffers keep full height, so the edge rows the
//                        earlier Narrows dropped (computed from clamped
//                        indices) are skipped by their distance to the
//                        segment edges.  Layers whose input is the previous
//                        GEMM's output skip minmax_kernel: that GEMM's
//                        epilogue leaves per-wave partials (I8Args::mm_part).
//   2. quantize_kernel   q = roundf(clamp(x / scale + zp, 0, 255)) stored as the
//                        signed byte q ^ 0x80 = q - 128, with the row sums of
//                        those bytes.  Layers whose segment width is not a
//                        multiple of the 64-byte K-tile (the 40-wide first layer)
//                        are written already spliced (rows x K, zero padded).
//   3. gemm_i8_nnet      v_mfma_i32_32x32x32_i8 on the shifted bytes with the
//                        splice folded into the A loader; int32 epilogue
//                        restores the zero points,
//                          sum (a-zA)(b-zB) = sum a'b' + cB*rowsum(a') + cA*colsum(b') + K*cA*cB
//                        (cA = 128 - zA), all modulo 2^32 like gemmlowp's
//                        accumulator, then float(acc) * (sA*sB) + bias, ReLU /
//                        BatchNorm in the reference's rounding order.
// Quantising the block entering the Splice is the same as quantising the
// spliced block: the tensor parameters depend only on min / max, and Splice +
// Narrow read every held row of the block.
#include <float.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "../internal.h"
#include "../tile_order.h"

namespace catears {
namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

// One wave per row (grid-stride over rows); rows outside what the reference
// chain holds at this layer (segment edges already narrowed away) are skipped.
// Each block leaves one (min, max) partial; params_kernel folds them.
constexpr int kMinmaxBlocks = 512;

__global__ __launch_bounds__(256) void minmax_kernel(const float *__restrict__ x, int ldx, int rows, int width,
                                                     const int *__restrict__ row_map,
                                                     const uint32_t *__restrict__ row_edge, int in_left,
                                                     int in_right, float2 *__restrict__ part) {
  float mn = FLT_MAX, mx = FLT_MIN;
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += gridDim.x * 4) {
    const int dl = row_edge ? (int)(row_edge[r] & 0xffff) : r;
    const int dr = row_edge ? (int)(row_edge[r] >> 16) : rows - 1 - r;
    if (dl < in_left || dr < in_right) continue;
    const int src = row_map ? row_map[r] : r;
    const float *xr = x + (int64_t)src * ldx;
    if ((width & 3) == 0 && (ldx & 3) == 0) {
      for (int c = 4 * lane; c < width; c += 256) {
        const float4 v = *reinterpret_cast<const float4 *>(xr + c);
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (e[t] > mx) mx = e[t];  // matrix.cc:337-342 (NaN never wins a comparison)
          if (e[t] < mn) mn = e[t];
        }
      }
    } else {
      for (int c = lane; c < width; c += 64) {
        const float v = xr[c];
        if (v > mx) mx = v;
        if (v < mn) mn = v;
      }
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const float omn = __shfl_xor(mn, d, 64), omx = __shfl_xor(mx, d, 64);
    mn = omn < mn ? omn : mn;
    mx = omx > mx ? omx : mx;
  }
  __shared__ float2 wv[4];
  if (lane == 0) wv[threadIdx.x >> 6] = make_float2(mn, mx);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      mn = wv[w].x < mn ? wv[w].x : mn;
      mx = wv[w].y > mx ? wv[w].y : mx;
    }
    part[blockIdx.x] = make_float2(mn, mx);
  }
}

struct QP {
  float scale;
  int32_t zp;
};

// ComputeQuantizationParams (matrix.cc:348-362) of a folded (min, max)
__device__ __forceinline__ QP qparams(float mn, float mx) {
  const double scale = (mx - mn) / 255.0;
  QP p;
  p.zp = (int32_t)round(-mn / scale);
  p.scale = (float)scale;
  return p;
}

// Folds the block partials and applies ComputeQuantizationParams
// (matrix.cc:348-362, double arithmetic) -- one block.
__global__ __launch_bounds__(256) void params_kernel(const float2 *__restrict__ part, int nparts,
                                                     QP *__restrict__ out) {
  float mn = FLT_MAX, mx = FLT_MIN;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    mn = part[i].x < mn ? part[i].x : mn;
    mx = part[i].y > mx ? part[i].y : mx;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const float omn = __shfl_xor(mn, d, 64), omx = __shfl_xor(mx, d, 64);
    mn = omn < mn ? omn : mn;
    mx = omx > mx ? omx : mx;
  }
  __shared__ float2 wv[4];
  if ((threadIdx.x & 63) == 0) wv[threadIdx.x >> 6] = make_float2(mn, mx);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      mn = wv[w].x < mn ? wv[w].x : mn;
      mx = wv[w].y > mx ? wv[w].y : mx;
    }
    *out = qparams(mn, mx);
  }
}

// The corrected reciprocal product below is the default: 0 differing
// quotients from IEEE division over 68.7e9 random pairs on the GPU
// (tools/probes/qdiv_probe.hip, denormal scales included), the int8 and
// parity tests bit-exact with it, the C5 checksum unchanged, C5 +1.2 %
// (profiles/r05z21_i8_qdiv.txt).  -DCATEARS_I8_QDIV=0 builds the division.
#ifndef CATEARS_I8_QDIV
#define CATEARS_I8_QDIV 1
#endif

// Quantize (matrix.cc:378-386) of one element -> shifted signed byte.
// CATEARS_I8_QDIV=1: x / scale as q0 = x * r, r = 1 / scale (correctly
// rounded), corrected once, q = fma(fma(-scale, q0, x), r, q0) (Markstein's
// correction: the correctly rounded quotient when r is the correctly rounded
// reciprocal and nothing overflows); rscale == 0 (1 / scale not finite: a
// denormal scale) and non-finite results fall back to the division.
__device__ __forceinline__ int qbyte(float x, float scale, float zp, float rscale = 0.0f) {
#if CATEARS_I8_QDIV
  float q;
  if (rscale != 0.0f) {
    const float q0 = x * rscale;
    q = __builtin_fmaf(__builtin_fmaf(-scale, q0, x), rscale, q0);
    if (__builtin_isinf(q) || __builtin_isnan(q)) q = x / scale;
  } else {
    q = x / scale;
  }
  float v = q + zp;
#else
  (void)rscale;
  float v = x / scale + zp;
#endif
  v = (255.0f < v) ? 255.0f : v;  // std::min(v, 255.0f)
  v = (0.0f < v) ? v : 0.0f;      // std::max(0.0f, v)
  return (int)(uint8_t)roundf(v) - 128;
}

// One wave per output row.  Plain mode: out row r = quantized X row
// (row_map[r] or r), width bytes, zero padded to ldq.  Spliced mode (nseg >
// 1 or width % 64): out row r = concat over segments s of quantized
// X[clamp(r + off[s])] (through row_map), zero padded to ldq.
struct SpliceOffsets {
  int off[8];
};

// Quantize row r of the layer input into q row r (one wave; lane = lane in
// the wave), and its row sum.
__device__ __forceinline__ void quantize_row(const float *__restrict__ x, int ldx, int rows, int width,
                                             const int *__restrict__ row_map, int nseg, const SpliceOffsets &so,
                                             float scale, float zp, int8_t *__restrict__ q, int ldq,
                                             int32_t *__restrict__ rowsum, int r, int lane) {
  int8_t *o = q + (int64_t)r * ldq;
  int32_t s = 0;
  float rs = CATEARS_I8_QDIV ? 1.0f / scale : 0.0f;
  if (__builtin_isinf(rs) || __builtin_isnan(rs)) rs = 0.0f;
  const bool vec = (width & 3) == 0 && (ldx & 3) == 0;
  for (int seg = 0; seg < nseg; ++seg) {
    int src = r + so.off[seg];
    src = src < 0 ? 0 : (src > rows - 1 ? rows - 1 : src);
    if (row_map) src = row_map[src];
    const float *xr = x + (int64_t)src * ldx;
    int8_t *os = o + seg * width;
    if (vec) {
      // 1024 floats of the row per pass, the lane's four float4 loads issued
      // together (clamped addresses, used only in range): one memory round
      // trip per pass instead of one per float4
      for (int c0 = 0; c0 < width; c0 += 1024) {
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = *reinterpret_cast<const float4 *>(xr + min(c0 + 4 * lane + 256 * j, width - 4));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = c0 + 4 * lane + 256 * j;
          if (c >= width) break;
          const int b0 = qbyte(v[j].x, scale, zp, rs), b1 = qbyte(v[j].y, scale, zp, rs);
          const int b2 = qbyte(v[j].z, scale, zp, rs), b3 = qbyte(v[j].w, scale, zp, rs);
          s += b0 + b1 + b2 + b3;
          const uint32_t packed = (uint32_t)(uint8_t)b0 | ((uint32_t)(uint8_t)b1 << 8) |
                                  ((uint32_t)(uint8_t)b2 << 16) | ((uint32_t)(uint8_t)b3 << 24);
          if ((((uintptr_t)(os + c)) & 3) == 0) {
            *reinterpret_cast<uint32_t *>(os + c) = packed;
          } else {
            os[c] = (int8_t)b0, os[c + 1] = (int8_t)b1, os[c + 2] = (int8_t)b2, os[c + 3] = (int8_t)b3;
          }
        }
      }
    } else {
      for (int c = lane; c < width; c += 64) {
        const int b = qbyte(xr[c], scale, zp, rs);
        os[c] = (int8_t)b;
        s += b;
      }
    }
  }
  for (int c = nseg * width + lane; c < ldq; c += 64) o[c] = 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (lane == 0) rowsum[r] = s;
}

// The vector path of quantize_row for RPW rows per wave (plain mode: one
// segment, width and ldx multiples of 4, no row map): every row's loads are
// issued before any is converted, and the reciprocal product's rare fallback
// (a non-finite quotient, qbyte) is one wave-level branch per row instead of
// one per element: the quotients are formed for the whole row, and only if
// some lane holds a non-finite one are those recomputed by division.  The
// same arithmetic per element as qbyte: the same bytes and row sums.
template <int RPW>
__device__ __forceinline__ void quantize_rows_fast(const float *__restrict__ x, int ldx, int rows, int width,
                                                   float scale, float zp, int8_t *__restrict__ q, int ldq,
                                                   int32_t *__restrict__ rowsum, int r0, int lane) {
  float rs = 1.0f / scale;
  const bool rs_ok = !(__builtin_isinf(rs) || __builtin_isnan(rs));
  int32_t rsum[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) rsum[i] = 0;
  for (int c0 = 0; c0 < width; c0 += 1024) {
    float4 v[RPW][4];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const float *xr = x + (int64_t)min(r0 + i, rows - 1) * ldx;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[i][j] = *reinterpret_cast<const float4 *>(xr + min(c0 + 4 * lane + 256 * j, width - 4));
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      if (r0 + i >= rows) break;
      float qv[16];
      bool bad = !rs_ok;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e[4] = {v[i][j].x, v[i][j].y, v[i][j].z, v[i][j].w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float q0 = e[t] * rs;
          const float qq = __builtin_fmaf(__builtin_fmaf(-scale, q0, e[t]), rs, q0);
          bad |= __builtin_isinf(qq) || __builtin_isnan(qq);
          qv[4 * j + t] = qq;
        }
      }
      if (__builtin_amdgcn_ballot_w64(bad)) {  // rare: the division, exactly as qbyte
        if (bad) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float e[4] = {v[i][j].x, v[i][j].y, v[i][j].z, v[i][j].w};
#pragma unroll
            for (int t = 0; t < 4; ++t)
              if (!rs_ok || __builtin_isinf(qv[4 * j + t]) || __builtin_isnan(qv[4 * j + t])) qv[4 * j + t] = e[t] / scale;
          }
        }
      }
      int8_t *os = q + (int64_t)(r0 + i) * ldq;
      int32_t &sum = rsum[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + 4 * lane + 256 * j;
        if (c >= width) break;
        int b[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float w = qv[4 * j + t] + zp;
          w = (255.0f < w) ? 255.0f : w;
          w = (0.0f < w) ? w : 0.0f;
          b[t] = (int)(uint8_t)roundf(w) - 128;
          sum += b[t];
        }
        const uint32_t packed = (uint32_t)(uint8_t)b[0] | ((uint32_t)(uint8_t)b[1] << 8) |
                                ((uint32_t)(uint8_t)b[2] << 16) | ((uint32_t)(uint8_t)b[3] << 24);
        *reinterpret_cast<uint32_t *>(os + c) = packed;
      }
    }
  }
  // the row sums (exact int32: any order)
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    int32_t sum = rsum[i];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if (lane == 0 && r0 + i < rows) rowsum[r0 + i] = sum;
  }
  // zero padding past the row (ldq > width)
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    if (r0 + i >= rows) break;
    int8_t *o = q + (int64_t)(r0 + i) * ldq;
    for (int c = width + lane; c < ldq; c += 64) o[c] = 0;
  }
}

template <int RPW>
__global__ __launch_bounds__(256) void quantize_fast_kernel(const float *__restrict__ x, int ldx, int rows, int width,
                                                            const QP *__restrict__ params, int8_t *__restrict__ q,
                                                            int ldq, int32_t *__restrict__ rowsum) {
  const QP p = *params;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW, lane = threadIdx.x & 63;
  if (r0 >= rows) return;
  quantize_rows_fast<RPW>(x, ldx, rows, width, p.scale, (float)p.zp, q, ldq, rowsum, r0, lane);
}

__global__ __launch_bounds__(256) void quantize_kernel(const float *__restrict__ x, int ldx, int rows, int width,
                                                       const int *__restrict__ row_map, int nseg,
                                                       SpliceOffsets so, const QP *__restrict__ params,
                                                       int8_t *__restrict__ q, int ldq, int32_t *__restrict__ rowsum) {
  const QP p = *params;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  quantize_row(x, ldx, rows, width, row_map, nseg, so, p.scale, (float)p.zp, q, ldq, rowsum, r, lane);
}

constexpr int IBM = 128, IBN = 128, IBK = 64, ILD = IBK + 16;  // bytes

struct I8Args {
  const int8_t *a;          // quantized layer input (rows x lda bytes)
  int lda, m;
  int din, nseg;            // segment width (bytes) and count; K = din * nseg
  int off[8];
  const int32_t *rowsum;    // per row of `a`
  const int8_t *w;          // shifted weights, n x kpad
  const int32_t *colsum;    // per column of w (shifted bytes)
  int n, k, kpad;
  const void *pa;           // device QP of the activations
  float w_scale;
  int32_t w_zp;
  const float *bias, *bn_scale, *bn_offset;
  int post[4];
  int npost, post_mode;
  float *y;
  int ldy;
  int tiles_n, tiles_m, group;
  int vec_epi;              // i8_epilogue_v (16-byte row stores)
  // Non-null: the epilogue also reduces the (min, max) of its outputs over the
  // rows the NEXT layer's Quantize reads (minmax_kernel's held-row rule with
  // that layer's in_left / in_right) into mm_part[blockIdx.x], so the next
  // layer's parameters fold these partials instead of re-reading the output.
  float2 *mm_part;
  const uint32_t *row_edge;
  int mm_left, mm_right;
};

// p.off[seg] through a select chain: a runtime index into the kernel
// argument's array can force the whole argument struct into scratch memory
// (the readfirstlane keeps the compiler from turning the chain back into a
// load from a selected address)
__device__ __forceinline__ int seg_off(const I8Args &p, int seg) {
  int v = __builtin_amdgcn_readfirstlane(p.off[0]);
#pragma unroll
  for (int i = 1; i < 8; ++i) v = seg >= i ? __builtin_amdgcn_readfirstlane(p.off[i]) : v;
  return v;
}

// minmax_kernel's row rule: does the next layer's Quantize count row `row`?
__device__ __forceinline__ uint32_t mm_held(const uint32_t *row_edge, int m, int left, int right, int row) {
  if (row >= m) return 0;
  const int dl = row_edge ? (int)(row_edge[row] & 0xffff) : row;
  const int dr = row_edge ? (int)(row_edge[row] >> 16) : m - 1 - row;
  return dl >= left && dr >= right;
}

// FindMinMax's comparisons (matrix.cc:337-342: NaN never wins one)
__device__ __forceinline__ void mm_take(float y, float &mn, float &mx) {
  if (y > mx) mx = y;
  if (y < mn) mn = y;
}

// Wave (min, max) of the epilogue's held outputs -> part[blockIdx.x * NW +
// wave] (no block barrier: a barrier under the epilogue's runtime `mm` test
// made the compiler copy the whole argument struct to scratch memory).
template <int NT>
__device__ __forceinline__ void mm_store(float2 *part, float mn, float mx) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const float omn = __shfl_xor(mn, d, 64), omx = __shfl_xor(mx, d, 64);
    mn = omn < mn ? omn : mn;
    mx = omx > mx ? omx : mx;
  }
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * (NT / 64) + (threadIdx.x >> 6)] = make_float2(mn, mx);
}

// Zero-point restore + bias + ReLU / BatchNorm + store of one wave's
// (TI x 32) x (TJ x 32) accumulator tile at (m0 + wrow, col0).  Column
// constants are read once into registers (the output stores could alias them
// as far as the compiler knows, so reads inside the store loop reload after
// every store) and the spliced row sums once per block row into LDS (`srs`,
// BM words; a per-lane loop over rows x segments is a chain of dependent L2
// round trips).  Every thread of the block must call it.
template <int TI, int TJ, int BM, int NT>
__device__ __forceinline__ void i8_epilogue(const I8Args &p, const i32x16 (&acc)[TI][TJ], int m0, int wrow, int col0,
                                            int r, int h, uint32_t *srs) {
  const QP pa = *static_cast<const QP *>(p.pa);
  const uint32_t ca = (uint32_t)(128 - pa.zp), cb = (uint32_t)(128 - p.w_zp);
  const uint32_t kterm = (uint32_t)p.k * ca * cb;
  const float cscale = pa.scale * p.w_scale;  // matrix.cc:404-405
  // cB * row sum of each spliced row of the block, one row per thread, into
  // LDS (the operand buffers are free once every wave is past the loop)
  __syncthreads();
  for (int t = threadIdx.x; t < BM; t += NT) {
    const int row = m0 + t;
    uint32_t sum = 0;
#pragma unroll
    for (int sg = 0; sg < 8; ++sg) {
      if (sg < p.nseg) {
        int src = row + p.off[sg];
        src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
        sum += (uint32_t)p.rowsum[src];
      }
    }
    srs[t] = cb * sum;
    if (p.mm_part) srs[BM + t] = mm_held(p.row_edge, p.m, p.mm_left, p.mm_right, row);
  }
  __syncthreads();
  const bool mm = p.mm_part != nullptr;
  const float2 mm2 = with_post_mode_r(p.post_mode, [&](auto M) {
    float mn = FLT_MAX, mx = FLT_MIN;  // matrix.cc:335-336
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = col0 + j * 32 + r;
      if (col >= p.n) continue;
      const uint32_t cterm = ca * (uint32_t)p.colsum[col] + kterm;
      const float bias = p.bias ? p.bias[col] : 0.0f;
      const float sc = p.bn_scale ? p.bn_scale[col] : 1.0f;
      const float of = p.bn_offset ? p.bn_offset[col] : 0.0f;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int lr = wrow + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          const uint32_t v = (uint32_t)acc[i][j][e] + srs[lr] + cterm;
          float y = (float)(int32_t)v * cscale;
          y = y + bias;  // +0 when absent: y is never -0 here (int * positive scale)
          y = apply_post<decltype(M)::value>(y, sc, of, p.post, p.npost);
          if (mm && srs[BM + lr]) mm_take(y, mn, mx);
          if (m0 + lr < p.m) p.y[(int64_t)(m0 + lr) * p.ldy + col] = y;
        }
      }
    }
    return make_float2(mn, mx);
  });
  if (mm) mm_store<NT>(p.mm_part, mm2.x, mm2.y);
}

// The same epilogue with the stores vectorised: each wave finishes its tile
// one 32-row slab at a time into a wave-private LDS slab (row stride padded
// by 32 B so the two row groups of a write land in different banks), then
// writes the slab back as 16-byte row chunks -- a quarter of the store
// instructions of i8_epilogue, whose 4-byte column stores made the epilogue
// store-issue bound.  Same values, same bits.  Needs n % 4 ==
// 0 and ldy % 4 == 0 (host-checked) and NW slabs of 32 x (TJ 32 + 8) floats
// plus BM words of row sums in `lds`.
template <int TI, int TJ, int BM, int NT>
__device__ __forceinline__ void i8_epilogue_v(const I8Args &p, const i32x16 (&acc)[TI][TJ], int m0, int wrow,
                                              int col0, int r, int h, char *lds) {
  constexpr int NW = NT / 64, SW = TJ * 32 + 8;  // slab row stride, floats
  const QP pa = *static_cast<const QP *>(p.pa);
  const uint32_t ca = (uint32_t)(128 - pa.zp), cb = (uint32_t)(128 - p.w_zp);
  const uint32_t kterm = (uint32_t)p.k * ca * cb;
  const float cscale = pa.scale * p.w_scale;  // matrix.cc:404-405
  uint32_t *srs = reinterpret_cast<uint32_t *>(lds + NW * 32 * SW * 4);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float *slab = reinterpret_cast<float *>(lds) + wave * 32 * SW;
  __syncthreads();
  for (int t = threadIdx.x; t < BM; t += NT) {
    const int row = m0 + t;
    uint32_t sum = 0;
#pragma unroll
    for (int sg = 0; sg < 8; ++sg) {
      if (sg < p.nseg) {
        int src = row + p.off[sg];
        src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
        sum += (uint32_t)p.rowsum[src];
      }
    }
    srs[t] = cb * sum;
  }
  __syncthreads();
  // the next layer's held rows among this wave's 64: bit t = row wrow + t
  static_assert(TI == 2, "one 64-row mask per wave");
  const bool mm = p.mm_part != nullptr;
  const uint64_t hmask =
      mm ? __builtin_amdgcn_ballot_w64(mm_held(p.row_edge, p.m, p.mm_left, p.mm_right, m0 + wrow + lane)) : 0;
  // column constants of this lane's TJ columns, loaded once (columns past n
  // take column n-1's, and so do their weight rows in the caller's B loader:
  // such lanes repeat a valid output, which cannot move a min or max)
  uint32_t cterm[TJ];
  float bias[TJ], sc[TJ], of[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = min(col0 + j * 32 + r, p.n - 1);
    cterm[j] = ca * (uint32_t)p.colsum[col] + kterm;
    bias[j] = p.bias ? p.bias[col] : 0.0f;
    sc[j] = p.bn_scale ? p.bn_scale[col] : 1.0f;
    of[j] = p.bn_offset ? p.bn_offset[col] : 0.0f;
  }
  constexpr int C4 = TJ * 8;  // float4 chunks per slab row
  const float2 mm2 = with_post_mode_r(p.post_mode, [&](auto M) {
    // FindMinMax (matrix.cc:331-345) as max / min: NaN never wins either way,
    // and a zero's sign cannot change the parameters
    float mn = FLT_MAX, mx = FLT_MIN;  // matrix.cc:335-336
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      float rmn[16], rmx[16];  // per row of the lane, over its TJ columns
#pragma unroll
      for (int e = 0; e < 16; ++e) rmn[e] = FLT_MAX, rmx[e] = FLT_MIN;
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;  // row within the slab
          const uint32_t v = (uint32_t)acc[i][j][e] + srs[wrow + i * 32 + rr] + cterm[j];
          float y = (float)(int32_t)v * cscale;
          y = y + bias[j];  // +0 when absent: y is never -0 here (int * positive scale)
          y = apply_post<decltype(M)::value>(y, sc[j], of[j], p.post, p.npost);
          rmx[e] = fmaxf(rmx[e], y);
          rmn[e] = fminf(rmn[e], y);
          slab[rr * SW + j * 32 + r] = y;
        }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;
        if ((hmask >> (i * 32 + rr)) & 1) {
          mx = fmaxf(mx, rmx[e]);
          mn = fminf(mn, rmn[e]);
        }
      }
      wave_lds_sync();
#pragma unroll
      for (int q = 0; q < 32 * C4 / 64; ++q) {
        const int idx = lane + 64 * q, rr = idx / C4, c4 = idx % C4;
        const int row = m0 + wrow + i * 32 + rr, col = col0 + 4 * c4;
        const float4 v = *reinterpret_cast<const float4 *>(slab + rr * SW + 4 * c4);
        // non-temporal: the next layer's Quantize reads it once, later
        // (serial hidden layer 36.8-37.0 -> 35.3-35.8 us, Quantize +0.4 us;
        // tools/experiments/i8_nt.sh)
        if (row < p.m && col < p.n) {
          typedef float nt4 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(nt4{v.x, v.y, v.z, v.w},
                                      reinterpret_cast<nt4 *>(p.y + (int64_t)row * p.ldy + col));
        }
      }
      wave_lds_sync();
    }
    return make_float2(mn, mx);
  });
  if (mm) mm_store<NT>(p.mm_part, mm2.x, mm2.y);
}

__global__ __launch_bounds__(256, 2) void gemm_i8_nnet_kernel(I8Args p) {
  __shared__ __attribute__((aligned(16))) int8_t As[IBM * ILD];
  __shared__ __attribute__((aligned(16))) int8_t Bs[IBN * ILD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, r = lane & 31, h = lane >> 5;
  const int tm = blockIdx.x / p.tiles_n, tn = blockIdx.x - tm * p.tiles_n;
  const int m0 = tm * IBM, n0 = tn * IBN;

  i32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  for (int k0 = 0; k0 < p.kpad; k0 += IBK) {
    // one K-tile never straddles a segment (din % 64 == 0 or nseg == 1)
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = seg_off(p, seg);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, row = idx >> 2, c16 = idx & 3;
      int src = m0 + row + shift;
      src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
      i32x4 v = (i32x4){0, 0, 0, 0};
      if (col0 + 16 * c16 < p.din && k0 < p.k)
        v = *reinterpret_cast<const i32x4 *>(p.a + (int64_t)src * p.lda + col0 + 16 * c16);
      *reinterpret_cast<i32x4 *>(As + row * ILD + 16 * c16) = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, row = idx >> 2, c16 = idx & 3;
      const int gn = min(n0 + row, p.n - 1);
      *reinterpret_cast<i32x4 *>(Bs + row * ILD + 16 * c16) =
          *reinterpret_cast<const i32x4 *>(p.w + (int64_t)gn * p.kpad + k0 + 16 * c16);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < IBK / 32; ++s) {
      i32x4 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const i32x4 *>(As + (wm * 64 + i * 32 + r) * ILD + 32 * s + 16 * h);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *reinterpret_cast<const i32x4 *>(Bs + (wn * 64 + j * 32 + r) * ILD + 32 * s + 16 * h);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  i8_epilogue<2, 2, IBM, 256>(p, acc, m0, wm * 64, n0 + wn * 64, r, h, reinterpret_cast<uint32_t *>(As));
}


// LDS-DMA form of the int8 GEMM (the fp32 kernel's structure, gemm_f32.hip):
// K-tiles of 128 bytes, global_load_lds_dwordx4 into two LDS stages with the
// XOR chunk swizzle applied on the source address, one barrier per K-tile.
// A 32x32x32 i8 MFMA operand is one ds_read_b128 per lane (row r, bytes
// 16h..16h+15 of its 32-byte k-step), so a tile row of 128 bytes holds the
// four k-steps of the tile.  BM x BN block tile, 2 x 2 waves.
// DIAG (CATEARS_DIAG builds only: timing breakdowns, wrong results): bit 1
// no DMA after the prologue, 2 no MFMAs (fragment reads kept live), 4 no
// fragment reads (MFMAs on constant operands).
template <int BM, int BN, int STAGES, int WGM = 2, int WGN = 2, int BKB = 128, int DIAG = 0>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_i8_glds_kernel(I8Args p) {
#ifndef CATEARS_DIAG
  static_assert(DIAG == 0, "diagnostic schedules are CATEARS_DIAG builds only");
#endif
  constexpr int NW = WGM * WGN;
  // BKB: bytes per K-tile row (128, or 64 so a 256 x 256 tile fits 4 stages)
  constexpr int CH = BKB / 16;              // 16-byte chunks per row
  constexpr int TI = BM / WGM / 32, TJ = BN / WGN / 32;
  constexpr int RPI = 1024 / BKB;           // rows per DMA instruction
  constexpr int NGA = BM * BKB / 1024 / NW, NGB = BN * BKB / 1024 / NW;
  constexpr int STAGE = (BM + BN) * BKB;    // bytes
  static_assert(NGA >= 1 && NGB >= 1 && TI >= 1 && TJ >= 1, "tile too small");
  static_assert(BKB == 128 || BKB == 64, "K-tile of 64 or 128 bytes");
  __shared__ __attribute__((aligned(1024))) int8_t smem[STAGES * STAGE];
  auto swz = [](int row) { return (row >> 1) & (CH - 1); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, r = lane & 31, h = lane >> 5;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int lrow = lane / CH, lchunk = lane & (CH - 1);
  uint32_t boff[NGB];
#pragma unroll
  for (int j = 0; j < NGB; ++j) {
    const int row = (wave * NGB + j) * RPI + lrow;
    boff[j] = (uint32_t)(min(n0 + row, p.n - 1) * p.kpad + 16 * (lchunk ^ swz(row)));
  }
  uint32_t aoff[NGA];
  int cur_seg = -1;
  auto issue = [&](int kt) {
    const int k0 = kt * BKB;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = seg_off(p, seg);
#pragma unroll
      for (int i = 0; i < NGA; ++i) {
        const int row = (wave * NGA + i) * RPI + lrow;
        int src = m0 + row + shift;
        src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
        aoff[i] = (uint32_t)(src * p.lda + 16 * (lchunk ^ swz(row)));
      }
    }
    int8_t *st = smem + (kt % STAGES) * STAGE;
    const char *abase = reinterpret_cast<const char *>(p.a) + col0;
    const char *bbase = reinterpret_cast<const char *>(p.w) + k0;
#pragma unroll
    for (int i = 0; i < NGA; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(abase + aoff[i]),
                                       (__attribute__((address_space(3))) void *)(st + (wave * NGA + i) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int j = 0; j < NGB; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(bbase + boff[j]),
                                       (__attribute__((address_space(3))) void *)(st + BM * BKB + (wave * NGB + j) * 1024),
                                       16, 0, 0);
  };

  i32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  const int xr = swz(r) ^ h;  // chunk 2s + h -> (2s) ^ xr
  const int a_row = (wm * TI * 32 + r) * BKB, b_row = BM * BKB + (wn * TJ * 32 + r) * BKB;
  const int ktiles = p.kpad / BKB;
  // STAGES-1 tiles in flight: tile kt has landed once at most STAGES-2 newer
  // tiles' DMAs are outstanding (counted vmcnt, raw barrier: the DMAs stay in
  // flight across it); the stage refilled at kt is the one read at kt-1.
  constexpr int NG = NGA + NGB;
  for (int t = 0; t < STAGES - 1 && t < ktiles; ++t) issue(t);
  for (int kt = 0; kt < ktiles; ++kt) {
    const int ahead = min(ktiles - 1 - kt, STAGES - 2);  // newer tiles already issued
    if (ahead >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NG) : "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (!(DIAG & 1) && kt + STAGES - 1 < ktiles) issue(kt + STAGES - 1);
    const int8_t *st = smem + (kt % STAGES) * STAGE;
#pragma unroll
    for (int s = 0; s < BKB / 32; ++s) {
      const int ch = ((2 * s) ^ xr) * 16;
      i32x4 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        af[i] = (DIAG & 4) ? i32x4{kt, s, i, 1} : *reinterpret_cast<const i32x4 *>(st + a_row + i * 32 * BKB + ch);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        bf[j] = (DIAG & 4) ? i32x4{s, kt, j, 2} : *reinterpret_cast<const i32x4 *>(st + b_row + j * 32 * BKB + ch);
      if constexpr ((DIAG & 2) != 0) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) acc[i][j][0] ^= af[i][0] ^ bf[j][1];
        continue;
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }

  if constexpr ((DIAG & 8) != 0) {  // no epilogue: one word per lane keeps the loop live
    int t = 0;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) t ^= acc[i][j][e];
    p.y[(int64_t)blockIdx.x * 64 * NW + tid] = (float)t;
    return;
  }
  // slabs + row sums in the stages; one 64-row held-row mask per wave
  constexpr bool kVecFits = TI == 2 && NW * 32 * (TJ * 32 + 8) * 4 + BM * 4 <= STAGES * STAGE;
  if constexpr (kVecFits) {
    if (p.vec_epi) {
      i8_epilogue_v<TI, TJ, BM, 64 * NW>(p, acc, m0, wm * TI * 32, n0 + wn * TJ * 32, r, h,
                                         reinterpret_cast<char *>(smem));
      return;
    }
  }
  i8_epilogue<TI, TJ, BM, 64 * NW>(p, acc, m0, wm * TI * 32, n0 + wn * TJ * 32, r, h,
                                   reinterpret_cast<uint32_t *>(smem));
}


// LDS-DMA through a buffer resource (buffer_load_dwordx4 ... lds): 16 bytes
// per lane from base + voff into LDS at the wave-uniform lds + 16 * lane.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, int8_t *lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds, 16, voff, 0, 0, 0);
}

// Software-pipelined form of gemm_i8_glds_kernel (the product default):
// the same tiles, LDS-DMA stages, source swizzle and epilogue, with the loop
// reordered so that the LDS fragment reads and the MFMAs overlap:
//   * fragments are double-buffered in registers: k-step s + 1's four
//     ds_read_b128 are issued before k-step s's four MFMAs, so a read's
//     latency hides under the MFMAs instead of a lgkmcnt(0) before each step;
//   * the K-tile hand-off (wait for tile kt + 1's DMA, barrier, refill of
//     the stage tile kt used, first reads of tile kt + 1) sits after tile
//     kt's last MFMAs are issued, so the barrier's wait overlaps them.
// int32 accumulation is exact, so any product order gives the same bits.
// STAG: waves NW/2 .. NW-1 (the second wave of every SIMD) run two k-steps
// behind the first half: their ks 0-1 of tile 0 before the loop, then per
// K-tile ks 2-3 of tile kt, the hand-off, ks 0-1 of tile kt+1.  The
// barriers, and so the stage protocol, are unchanged (a wave reaches tile
// kt's hand-off only after all its reads of tile kt); the two waves of a
// SIMD then read fragments while the other one multiplies
// (MI355X_MICROARCH.md, "try a stagger").  Exact int32: same bits.
template <int BM, int BN, int STAGES, int WGM, int WGN, bool STAG = false>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_i8_pipe_kernel(I8Args p) {
  static_assert(STAGES == 3, "tile kt + 3 refills tile kt's stage");
  constexpr int NW = WGM * WGN, BKB = 128, CH = BKB / 16;
  constexpr int TI = BM / WGM / 32, TJ = BN / WGN / 32;
  constexpr int RPI = 1024 / BKB;
  constexpr int NGA = BM * BKB / 1024 / NW, NGB = BN * BKB / 1024 / NW, NG = NGA + NGB;
  constexpr int STAGE = (BM + BN) * BKB;
  static_assert(NGA >= 1 && NGB >= 1 && TI >= 1 && TJ >= 1, "tile too small");
  __shared__ __attribute__((aligned(1024))) int8_t smem[STAGES * STAGE];
  auto swz = [](int row) { return (row >> 1) & (CH - 1); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, r = lane & 31, h = lane >> 5;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int lrow = lane / CH, lchunk = lane & (CH - 1);
  uint32_t boff[NGB];
#pragma unroll
  for (int j = 0; j < NGB; ++j) {
    const int row = (wave * NGB + j) * RPI + lrow;
    boff[j] = (uint32_t)(min(n0 + row, p.n - 1) * p.kpad + 16 * (lchunk ^ swz(row)));
  }
  uint32_t aoff[NGA];
  int cur_seg = -1;
  // the DMA as buffer_load ... lds (MUBUF): the compiler counts it in vmcnt
  // only, so the fragment reads keep exact lgkmcnt waits (a pending
  // global_load_lds, a FLAT access, makes every LDS wait lgkmcnt(0))
  const auto ra = buf_rsrc(p.a), rw = buf_rsrc(p.w);
  auto issue = [&](int kt) {
    const int k0 = kt * BKB;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = seg_off(p, seg);
#pragma unroll
      for (int i = 0; i < NGA; ++i) {
        const int row = (wave * NGA + i) * RPI + lrow;
        int src = m0 + row + shift;
        src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
        aoff[i] = (uint32_t)(src * p.lda + 16 * (lchunk ^ swz(row)));
      }
    }
    int8_t *st = smem + (kt % STAGES) * STAGE;
#pragma unroll
    for (int i = 0; i < NGA; ++i) buf_lds16(ra, st + (wave * NGA + i) * 1024, aoff[i] + col0);
#pragma unroll
    for (int j = 0; j < NGB; ++j) buf_lds16(rw, st + BM * BKB + (wave * NGB + j) * 1024, boff[j] + k0);
  };

  i32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  const int xr = swz(r) ^ h;  // chunk 2s + h -> (2s) ^ xr
  const int a_row = (wm * TI * 32 + r) * BKB, b_row = BM * BKB + (wn * TJ * 32 + r) * BKB;
  const int ktiles = p.kpad / BKB;
  i32x4 fa[2][TI], fb[2][TJ];
  auto read = [&](int kt, int s, int buf) {
    const int8_t *st = smem + (kt % STAGES) * STAGE;
    const int ch = ((2 * s) ^ xr) * 16;
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[buf][i] = *reinterpret_cast<const i32x4 *>(st + a_row + i * 32 * BKB + ch);
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[buf][j] = *reinterpret_cast<const i32x4 *>(st + b_row + j * 32 * BKB + ch);
  };
  auto mma = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[buf][i], fb[buf][j], acc[i][j], 0, 0, 0);
  };
  // tile kt has landed once at most the newer tiles' groups are outstanding
  auto wait_tile = [&](int newer) {
    if (newer >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NG) : "memory");
    else if (newer == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  for (int t = 0; t < STAGES - 1 && t < ktiles; ++t) issue(t);
  wait_tile(min(ktiles - 1, STAGES - 2));
  __builtin_amdgcn_s_barrier();
  if (STAGES - 1 < ktiles) issue(STAGES - 1);
  read(0, 0, 0);
  if (STAG && wave >= NW / 2) {
    // the late half: ks 0-1 of tile 0 now, then two k-steps behind
    read(0, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(0);
    __builtin_amdgcn_sched_barrier(0);
    read(0, 2, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma(1);
    __builtin_amdgcn_sched_barrier(0);
    for (int kt = 0; kt < ktiles; ++kt) {
      read(kt, 3, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(0);
      __builtin_amdgcn_sched_barrier(0);
      mma(1);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < ktiles) {
        wait_tile(kt + 2 < ktiles ? 1 : 0);
        __builtin_amdgcn_s_barrier();
        if (kt + STAGES < ktiles) issue(kt + STAGES);
        read(kt + 1, 0, 0);
        read(kt + 1, 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(0);
        __builtin_amdgcn_sched_barrier(0);
        read(kt + 1, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
        mma(1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else
  for (int kt = 0; kt < ktiles; ++kt) {
    // k-steps 0..2: the next step's reads, then this step's MFMAs
    read(kt, 1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(0);
    __builtin_amdgcn_sched_barrier(0);
    read(kt, 2, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma(1);
    __builtin_amdgcn_sched_barrier(0);
    read(kt, 3, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(0);
    __builtin_amdgcn_sched_barrier(0);
    // k-step 3's MFMAs first, then the hand-off to tile kt + 1 under them
    mma(1);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < ktiles) {
      // newer tiles than kt + 1 already issued: kt + 2 if it exists
      wait_tile(kt + 2 < ktiles ? 1 : 0);
      __builtin_amdgcn_s_barrier();  // every wave is past its reads of tile kt's stage
      if (kt + STAGES < ktiles) issue(kt + STAGES);
      read(kt + 1, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // slabs + row sums in the stages; one 64-row held-row mask per wave
  constexpr bool kVecFits = TI == 2 && NW * 32 * (TJ * 32 + 8) * 4 + BM * 4 <= STAGES * STAGE;
  if constexpr (kVecFits) {
    if (p.vec_epi) {
      i8_epilogue_v<TI, TJ, BM, 64 * NW>(p, acc, m0, wm * TI * 32, n0 + wn * TJ * 32, r, h,
                                         reinterpret_cast<char *>(smem));
      return;
    }
  }
  i8_epilogue<TI, TJ, BM, 64 * NW>(p, acc, m0, wm * TI * 32, n0 + wn * TJ * 32, r, h,
                                   reinterpret_cast<uint32_t *>(smem));
}

// Branch-free form of gemm_i8_glds_kernel with three stages and the DMA two
// K-tiles ahead (the structure of gemm_bf16x6q_kernel): step kt reads stage
// kt % 3 (four k-steps), drains its LDS reads (lgkmcnt(0)), retires its own
// pieces of tile kt+1 (vmcnt: all but tile kt+2's), passes one raw barrier
// and issues tile kt+3 into the stage it just freed.  Tail tiles are clamped
// to the last one (a refetch of identical bytes into the stage that holds
// it), so every step issues the same pieces and the body is one basic block.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_i8_q_kernel(I8Args p) {
  constexpr int NW = WGM * WGN;
  constexpr int BKB = 128;
  constexpr int TI = BM / WGM / 32, TJ = BN / WGN / 32;
  constexpr int RPI = 1024 / BKB;
  constexpr int NGA = BM * BKB / 1024 / NW, NGB = BN * BKB / 1024 / NW, NG = NGA + NGB;
  constexpr int STAGE = (BM + BN) * BKB;
  static_assert(NGA >= 1 && NGB >= 1 && TI >= 1 && TJ >= 1, "tile too small");
  static_assert(3 * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) int8_t smem[3 * STAGE];
  auto swz = [](int row) { return (row >> 1) & 7; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, r = lane & 31, h = lane >> 5;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;

  const int lrow = lane / 8, lchunk = lane & 7;
  uint32_t boff[NGB];
#pragma unroll
  for (int j = 0; j < NGB; ++j) {
    const int row = (wave * NGB + j) * RPI + lrow;
    boff[j] = (uint32_t)(min(n0 + row, p.n - 1) * p.kpad + 16 * (lchunk ^ swz(row)));
  }
  int arow[NGA];
  uint32_t achunk[NGA];
#pragma unroll
  for (int i = 0; i < NGA; ++i) {
    const int row = (wave * NGA + i) * RPI + lrow;
    arow[i] = m0 + row;
    achunk[i] = (uint32_t)(16 * (lchunk ^ swz(row)));
  }
  const int ktiles = p.kpad / BKB;
  auto issue = [&](int kt) {
    kt = min(kt, ktiles - 1);
    const int k0 = kt * BKB;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    const int shift = seg_off(p, seg);
    int8_t *st = smem + (kt % 3) * STAGE;
    const char *abase = reinterpret_cast<const char *>(p.a) + col0;
    const char *bbase = reinterpret_cast<const char *>(p.w) + k0;
#pragma unroll
    for (int i = 0; i < NGA; ++i) {
      int src = arow[i] + shift;
      src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void *)(abase + (uint32_t)(src * p.lda) + achunk[i]),
          (__attribute__((address_space(3))) void *)(st + (wave * NGA + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NGB; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(bbase + boff[j]),
                                       (__attribute__((address_space(3))) void *)(st + BM * BKB + (wave * NGB + j) * 1024),
                                       16, 0, 0);
  };

  i32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  const int xr = swz(r) ^ h;
  const int a_row = (wm * TI * 32 + r) * BKB, b_row = BM * BKB + (wn * TJ * 32 + r) * BKB;
  issue(0);
  issue(1);
  issue(2);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NG) : "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < ktiles; ++kt) {
    const int8_t *st = smem + (kt % 3) * STAGE;
#pragma unroll
    for (int s = 0; s < BKB / 32; ++s) {
      const int ch = ((2 * s) ^ xr) * 16;
      i32x4 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = *reinterpret_cast<const i32x4 *>(st + a_row + i * 32 * BKB + ch);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bf[j] = *reinterpret_cast<const i32x4 *>(st + b_row + j * 32 * BKB + ch);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NG) : "memory");
    __builtin_amdgcn_s_barrier();
    issue(kt + 3);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  i8_epilogue<TI, TJ, BM, 64 * NW>(p, acc, m0, wm * TI * 32, n0 + wn * TJ * 32, r, h, reinterpret_cast<uint32_t *>(smem));
}

// Register-staged form: the next K-tile is fetched with global_load_dwordx4
// into VGPRs while the current one is multiplied, then written to the other
// LDS buffer with ds_write_b128.  An LDS-DMA piece costs its wave ~60-180
// issue cycles per KiB (MI355X_MICROARCH.md, per-instruction constants), and
// an i8 MFMA consumes operands as fast as a bf16 one (1 KiB per 32 cycles),
// so at 128 x 128 the DMA issue alone matched the MFMA time; a plain
// 16-byte load + LDS write per KiB costs a few cycles.  One barrier per
// K-tile: the buffer written at kt was last read at kt-1, before that
// iteration's barrier.  BM x BN block tile, WGM x WGN waves, 128-byte
// K-tiles, the same XOR chunk swizzle and fragment reads as above.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_i8_reg_kernel(I8Args p) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int BKB = 128;
  constexpr int TI = BM / WGM / 32, TJ = BN / WGN / 32;
  constexpr int LA = BM * 8 / NT, LB = BN * 8 / NT;  // 16-byte chunks per thread
  constexpr int STAGE = (BM + BN) * BKB;
  static_assert(LA * NT == BM * 8 && LB * NT == BN * 8 && TI >= 1 && TJ >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * STAGE];
  auto swz = [](int row) { return (row >> 1) & 7; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, r = lane & 31, h = lane >> 5;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // thread -> (row, chunk) of the tile: chunk = tid & 7 for every piece
  const int chunk = tid & 7, row_base = tid >> 3;
  constexpr int RSTEP = NT / 8;
  uint32_t boff[LB], bdst[LB];
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int row = row_base + j * RSTEP;
    boff[j] = (uint32_t)(min(n0 + row, p.n - 1) * p.kpad + 16 * chunk);
    bdst[j] = (uint32_t)(BM * BKB + row * BKB + 16 * (chunk ^ swz(row)));
  }
  uint32_t aoff[LA], adst[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = row_base + i * RSTEP;
    adst[i] = (uint32_t)(row * BKB + 16 * (chunk ^ swz(row)));
  }
  int cur_seg = -1;
  i32x4 ra[LA], rb[LB];
  auto fetch = [&](int kt) {
    const int k0 = kt * BKB;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = seg_off(p, seg);
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        int src = m0 + row_base + i * RSTEP + shift;
        src = src < 0 ? 0 : (src > p.m - 1 ? p.m - 1 : src);
        aoff[i] = (uint32_t)(src * p.lda + 16 * chunk);
      }
    }
    const int8_t *abase = p.a + col0;
    const int8_t *bbase = p.w + k0;
#pragma unroll
    for (int i = 0; i < LA; ++i) ra[i] = *reinterpret_cast<const i32x4 *>(abase + aoff[i]);
#pragma unroll
    for (int j = 0; j < LB; ++j) rb[j] = *reinterpret_cast<const i32x4 *>(bbase + boff[j]);
  };
  auto stash = [&](int8_t *st) {
#pragma unroll
    for (int i = 0; i < LA; ++i) *reinterpret_cast<i32x4 *>(st + adst[i]) = ra[i];
#pragma unroll
    for (int j = 0; j < LB; ++j) *reinterpret_cast<i32x4 *>(st + bdst[j]) = rb[j];
  };

  i32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  const int xr = swz(r) ^ h;
  const int a_row = (wm * TI * 32 + r) * BKB, b_row = BM * BKB + (wn * TJ * 32 + r) * BKB;
  const int ktiles = p.kpad / BKB;
  fetch(0);
  stash(smem);
  __syncthreads();
  for (int kt = 0; kt < ktiles; ++kt) {
    const bool more = kt + 1 < ktiles;
    if (more) fetch(kt + 1);
    const int8_t *st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int s = 0; s < BKB / 32; ++s) {
      const int ch = ((2 * s) ^ xr) * 16;
      i32x4 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = *reinterpret_cast<const i32x4 *>(st + a_row + i * 32 * BKB + ch);
#pragma unroll
      for (int j = 0; j < TJ; ++j) bf[j] = *reinterpret_cast<const i32x4 *>(st + b_row + j * 32 * BKB + ch);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (more) stash(smem + ((kt + 1) & 1) * STAGE);
    __syncthreads();
  }
  i8_epilogue<TI, TJ, BM, NT>(p, acc, m0, wm * TI * 32, n0 + wn * TJ * 32, r, h, reinterpret_cast<uint32_t *>(smem));
}

}  // namespace

// Reduces the held rows of a layer input to QP params (minmax partials in
// `part`, kMinmaxBlocks float2).
int launch_i8_params(hipStream_t s, const float *x, int ldx, int rows, int width, const int *row_map,
                     const uint32_t *row_edge, int in_left, int in_right, void *part, void *params) {
  const int blocks = std::max(1, std::min(kMinmaxBlocks, (rows + 3) / 4));
  hipLaunchKernelGGL(minmax_kernel, dim3(blocks), dim3(256), 0, s, x, ldx, rows, width, row_map, row_edge, in_left,
                     in_right, static_cast<float2 *>(part));
  hipLaunchKernelGGL(params_kernel, dim3(1), dim3(256), 0, s, static_cast<const float2 *>(part), blocks,
                     static_cast<QP *>(params));
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

size_t i8_params_scratch_bytes() { return sizeof(float2) * kMinmaxBlocks + 256; }

int launch_i8_quantize(hipStream_t s, const float *x, int ldx, int rows, int width, const int *row_map, int nseg,
                       const int *offs, const void *params, int8_t *q, int ldq, int32_t *rowsum) {
  SpliceOffsets so = {};
  for (int i = 0; i < nseg; ++i) so.off[i] = offs[i];
  // Plain-mode layers (every layer after the first) go through
  // quantize_fast_kernel: one wave-level fallback branch per row instead of
  // one per element, same bytes and row sums; C5 +3.0 % (24.29 vs 23.58 M
  // frames/s, A B C C B A x2 on one box, same checksum,
  // profiles/r06k_c5_quantize.txt).  CATEARS_I8_QFAST (experiments
  // library): 0 = quantize_kernel, 2 = two rows per wave (+2.1 %).
  static const int qfast = CE_KNOB("CATEARS_I8_QFAST", 1);
  const bool plain = nseg == 1 && !row_map && so.off[0] == 0 && width % 4 == 0 && ldx % 4 == 0 && ldq % 4 == 0 &&
                     (reinterpret_cast<uintptr_t>(q) & 3) == 0;
  if (rows > 0 && plain && qfast == 1) {
    hipLaunchKernelGGL(quantize_fast_kernel<1>, dim3((rows + 3) / 4), dim3(256), 0, s, x, ldx, rows, width,
                       static_cast<const QP *>(params), q, ldq, rowsum);
  } else if (rows > 0 && plain && qfast == 2) {
    hipLaunchKernelGGL(quantize_fast_kernel<2>, dim3((rows + 7) / 8), dim3(256), 0, s, x, ldx, rows, width,
                       static_cast<const QP *>(params), q, ldq, rowsum);
  } else if (rows > 0)
    hipLaunchKernelGGL(quantize_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, ldx, rows, width, row_map, nseg,
                       so, static_cast<const QP *>(params), q, ldq, rowsum);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int launch_i8_params_fold(hipStream_t s, const void *part, int nparts, void *params) {
  hipLaunchKernelGGL(params_kernel, dim3(1), dim3(256), 0, s, static_cast<const float2 *>(part), nparts,
                     static_cast<QP *>(params));
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int launch_i8_gemm(hipStream_t s, const I8Layer &L, const int8_t *a, int lda, int m, const int32_t *rowsum,
                   const void *pa, float *y, int ldy, const I8NextMinMax *mm, int *nparts) {
  I8Args p = {};
  if (mm) {
    p.mm_part = static_cast<float2 *>(mm->part);
    p.row_edge = mm->row_edge;
    p.mm_left = mm->in_left;
    p.mm_right = mm->in_right;
  }
  p.a = a;
  p.lda = lda;
  p.m = m;
  p.din = L.a_din;
  p.nseg = L.a_nseg;
  for (int i = 0; i < 8; ++i) p.off[i] = L.a_off[i];
  p.rowsum = rowsum;
  p.w = L.wq.as<int8_t>();
  p.colsum = L.colsum.as<int32_t>();
  p.n = L.n;
  p.k = L.k;
  p.kpad = L.kpad;
  p.pa = pa;
  p.w_scale = L.w_scale;
  p.w_zp = L.w_zp;
  p.bias = L.bias;
  p.bn_scale = L.bn_scale;
  p.bn_offset = L.bn_offset;
  for (int i = 0; i < 4; ++i) p.post[i] = L.post[i];
  p.npost = L.npost;
  p.post_mode = post_mode(L.post, L.npost);
  p.y = y;
  p.ldy = ldy;
  static const int vec_epi = CE_KNOB("CATEARS_I8_EPI", 1);
  p.vec_epi = vec_epi && L.n % 4 == 0 && ldy % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;

  // 16: measured best on TDNN-S, frame batch 8192 (tools/i8_sweep.sh)
  static const int use_glds = CE_KNOB("CATEARS_I8_GEMM", 16);
  if (use_glds && p.kpad % 128 == 0 && p.din % 128 == 0 && lda % 16 == 0) {
    auto go = [&](auto kern, int bm, int bn, int threads = 256) {
      p.tiles_n = (L.n + bn - 1) / bn;
      p.tiles_m = (m + bm - 1) / bm;
      p.group = 8;  // an XCD's tiles: 8 column tiles x its row blocks
      if (nparts) *nparts = p.tiles_m * p.tiles_n * (threads / 64);  // one partial per wave
      hipLaunchKernelGGL(kern, dim3(p.tiles_m * p.tiles_n), dim3(threads), 0, s, p);
    };
    switch (use_glds) {
      // 15: 256 x 128, 3 stages (144 KiB), 8 waves of 64 x 64: one tile per
      // CU on the 1024-wide layers and two K-tiles in flight.  The serial
      // per-layer times of 1, 7, 10, 11 and 15 are within 5 % of each other
      // (the loop waits on L2 / MALL fetches, 43 % of wave cycles parked, MFMA
      // busy ~20 %); 9 (128 tiles) leaves half the CUs idle when alone.
      case 15: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2>, 256, 128, 512); break;
      // 16: 15's tiles with the loop software-pipelined (gemm_i8_pipe_kernel)
      case 16: go(gemm_i8_pipe_kernel<256, 128, 3, 4, 2>, 256, 128, 512); break;
#ifdef CATEARS_EXPERIMENTS  // tools/i8_sweep.sh
      // 17: 16 with waves 4-7 two k-steps behind waves 0-3 (stagger)
      case 17: go(gemm_i8_pipe_kernel<256, 128, 3, 4, 2, true>, 256, 128, 512); break;
      case 2: go(gemm_i8_glds_kernel<128, 128, 3>, 128, 128); break;
      case 3: go(gemm_i8_glds_kernel<128, 128, 4>, 128, 128); break;
      case 4: go(gemm_i8_glds_kernel<128, 64, 4>, 128, 64); break;
      case 5: go(gemm_i8_glds_kernel<64, 128, 4>, 64, 128); break;
      case 6: go(gemm_i8_glds_kernel<128, 64, 3>, 128, 64); break;
      case 7: go(gemm_i8_glds_kernel<256, 128, 2, 4, 2>, 256, 128, 512); break;
      // 9: 256 x 256 tiles, 8 waves of 64 x 128: twice the MFMA work per
      // K-tile iteration of the 128 x 128 form -- the loop is bound by the
      // DMA round trip per iteration, not by MFMA issue
      case 8: go(gemm_i8_glds_kernel<128, 256, 2, 2, 4>, 128, 256, 512); break;
      case 9: go(gemm_i8_glds_kernel<256, 256, 2, 4, 2>, 256, 256, 512); break;
      // 40-42: 256 x 256 tiles on 64-byte K-tiles (half the L2 bytes per
      // MFMA of 15), 3 / 4 stages; 16 waves of 64 x 64 (42)
      case 40: go(gemm_i8_glds_kernel<256, 256, 4, 4, 2, 64>, 256, 256, 512); break;
      case 41: go(gemm_i8_glds_kernel<256, 256, 3, 4, 2, 64>, 256, 256, 512); break;
      case 43: go(gemm_i8_glds_kernel<128, 256, 4, 2, 4, 64>, 128, 256, 512); break;
      case 44: go(gemm_i8_glds_kernel<256, 128, 4, 4, 2, 64>, 256, 128, 512); break;
      // 45-47: 256 x 256 tiles, 4 waves of 128 x 128 (accumulators in AGPRs):
      // one fragment read per two MFMAs instead of one per MFMA
      case 45: go(gemm_i8_glds_kernel<256, 256, 2, 2, 2, 128>, 256, 256, 256); break;
#ifdef CATEARS_DIAG
      // timing-only ablations of 15 (wrong results)
      case 61: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 1>, 256, 128, 512); break;
      case 62: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 2>, 256, 128, 512); break;
      case 64: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 4>, 256, 128, 512); break;
      case 65: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 5>, 256, 128, 512); break;
      case 63: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 3>, 256, 128, 512); break;
      case 68: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 8>, 256, 128, 512); break;
      case 71: go(gemm_i8_glds_kernel<256, 128, 3, 4, 2, 128, 11>, 256, 128, 512); break;
#endif
      case 46: go(gemm_i8_glds_kernel<256, 256, 4, 2, 2, 64>, 256, 256, 256); break;
      case 47: go(gemm_i8_glds_kernel<256, 256, 3, 2, 2, 64>, 256, 256, 256); break;
      // 48-49: 256 x 256, 8 waves of 128 x 64 (0.75 fragment reads per MFMA)
      case 48: go(gemm_i8_glds_kernel<256, 256, 3, 2, 4, 64>, 256, 256, 512); break;
      case 49: go(gemm_i8_glds_kernel<256, 256, 4, 2, 4, 64>, 256, 256, 512); break;
      case 50: go(gemm_i8_glds_kernel<256, 256, 2, 2, 4, 128>, 256, 256, 512); break;
      case 51: go(gemm_i8_glds_kernel<256, 128, 2, 2, 4, 128>, 256, 128, 512); break;
      case 10: go(gemm_i8_reg_kernel<128, 128, 2, 2>, 128, 128, 256); break;
      case 11: go(gemm_i8_reg_kernel<256, 128, 4, 2>, 256, 128, 512); break;
      // 20-22: branch-free, DMA two K-tiles ahead (gemm_i8_q_kernel)
      case 20: go(gemm_i8_q_kernel<256, 128, 4, 2>, 256, 128, 512); break;
      case 21: go(gemm_i8_q_kernel<128, 256, 2, 4>, 128, 256, 512); break;
      case 22: go(gemm_i8_q_kernel<128, 128, 2, 2>, 128, 128, 256); break;
      case 1: go(gemm_i8_glds_kernel<128, 128, 2>, 128, 128); break;
#endif
      default:
        return fail(CE_GPU_EINVAL, "int8 GEMM variant " + std::to_string(use_glds) +
                                       " is not in this build (the experiments library: `make EXPERIMENTS=1`)");
    }
    CE_HIP(hipGetLastError());
    return CE_GPU_OK;
  }
  p.tiles_n = (L.n + IBN - 1) / IBN;
  if (p.kpad % IBK != 0 || (p.nseg > 1 && p.din % IBK != 0) || lda % 16 != 0)
    return fail(CE_GPU_EINVAL, "gemm_i8_nnet: bad K geometry");
  const int tiles_m = (m + IBM - 1) / IBM;
  if (nparts) *nparts = tiles_m * p.tiles_n * 4;
  hipLaunchKernelGGL(gemm_i8_nnet_kernel, dim3(tiles_m * p.tiles_n), dim3(256), 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int i8_k_align() { return 128; }  // the LDS-DMA kernel's K-tile (bytes)

// one partial per wave; every int8 GEMM tile is at least 128 x 128 with at
// most 8 waves
size_t i8_gemm_parts(int m, int n) { return (size_t)((m + 127) / 128) * ((n + 127) / 128) * 8; }

}  // namespace catears
