// gemm_f32.hip -- fp32 MFMA GEMM for the TDNN layers, with the splice folded
// into the A-operand loader and bias / ReLU / BatchNorm fused in the epilogue.
//
// Replaces, per layer: SpliceLayer + NarrowLayer (src/nnet.cc:50-75, 182-202),
// LinearLayer::Propagate = MatMat -> cblas_sgemm + bias (nnet.cc:22-36,
// matrix.cc:300-323), ReLULayer (nnet.cc:149-160), BatchNormLayer
// (nnet.cc:106-117).
//
// A (rows x K): row r, column k reads source row r + off[k / din] (clamped into
// the chunk, optionally remapped through row_map for the first layer), column
// k % din.  So the spliced matrix is never materialised.
// B: the layer weights, uploaded once transposed (n x kpad, K contiguous), or
// for the generic MatMat entry a row-major k x n matrix.
//
// Tiling for CDNA4: 128 x 128 block tile, BK = 32, 256 threads = 4 waves in a
// 2 x 2 arrangement, each wave 64 x 64 = 2 x 2 tiles of
// v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 cycles per instruction per
// SIMD).  Operands are read from LDS with ds_read_b128: lane (r, h) of a
// 32 x 2 MFMA fragment fetches 4 consecutive k values, and the four MFMA
// k-steps of a group of 8 take k = 4h + s (s = 0..3) -- a permutation of k
// applied identically to A and B, so the sum is unchanged.  Rows of the LDS
// tiles are padded to 36 floats so every 16-lane ds_read_b128 group hits 16
// distinct 16-byte bank slots.  Two LDS stages; the next K-tile's global
// loads are issued before the current tile's MFMAs.
#include <hip/hip_runtime.h>

#include "../internal.h"

namespace catears {
namespace {

constexpr int BM = 128, BN = 128, BK = 32, LDT = BK + 4;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct KArgs {
  const float *x;
  const int *row_map;
  const float *w;
  const float *bias, *bn_scale, *bn_offset;
  float *y;
  int ldx, ldw, ldy;
  int m, n, k, kpad;
  int din, nseg;
  int off[8];
  int post[4];
  int npost;
  int tiles_n;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Global -> register staging of one K-tile.
template <bool A_FAST, bool B_NMAJOR>
struct Stage {
  f32x4 a[4];
  f32x4 b[4];
  float as[16];
  float bs[16];

  __device__ __forceinline__ void load(const KArgs &p, int m0, int n0, int k0, int tid) {
    if constexpr (A_FAST) {
      // whole K-tile inside one splice segment; 8 float4 per row
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      const int shift = p.off[seg];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + 256 * i, row = idx >> 3, c4 = idx & 7;
        int src = clampi(m0 + row + shift, 0, p.m - 1);
        if (p.row_map) src = p.row_map[src];
        a[i] = *reinterpret_cast<const f32x4 *>(p.x + (int64_t)src * p.ldx + col0 + 4 * c4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int idx = tid + 256 * i, row = idx >> 5, kk = idx & 31;
        const int kg = k0 + kk;
        float v = 0.0f;
        if (kg < p.k) {
          const int seg = kg / p.din, col = kg - seg * p.din;
          int src = clampi(m0 + row + p.off[seg], 0, p.m - 1);
          if (p.row_map) src = p.row_map[src];
          v = p.x[(int64_t)src * p.ldx + col];
        }
        as[i] = v;
      }
    }
    if constexpr (!B_NMAJOR) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + 256 * i, row = idx >> 3, c4 = idx & 7;
        const int nn = min(n0 + row, p.n - 1);
        b[i] = *reinterpret_cast<const f32x4 *>(p.w + (int64_t)nn * p.ldw + k0 + 4 * c4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int idx = tid + 256 * i, kk = idx >> 7, nn = idx & 127;
        const int kg = k0 + kk, ng = n0 + nn;
        bs[i] = (kg < p.k && ng < p.n) ? p.w[(int64_t)kg * p.ldw + ng] : 0.0f;
      }
    }
  }

  __device__ __forceinline__ void store(float *As, float *Bs, int tid) {
    if constexpr (A_FAST) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + 256 * i, row = idx >> 3, c4 = idx & 7;
        *reinterpret_cast<f32x4 *>(As + row * LDT + 4 * c4) = a[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int idx = tid + 256 * i, row = idx >> 5, kk = idx & 31;
        As[row * LDT + kk] = as[i];
      }
    }
    if constexpr (!B_NMAJOR) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + 256 * i, row = idx >> 3, c4 = idx & 7;
        *reinterpret_cast<f32x4 *>(Bs + row * LDT + 4 * c4) = b[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int idx = tid + 256 * i, kk = idx >> 7, nn = idx & 127;
        Bs[nn * LDT + kk] = bs[i];
      }
    }
  }
};

template <bool A_FAST, bool B_NMAJOR>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(KArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tm = blockIdx.x / p.tiles_n, tn = blockIdx.x - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int ktiles = p.kpad / BK;
  Stage<A_FAST, B_NMAJOR> st;
  st.load(p, m0, n0, 0, tid);
  st.store(smem, smem + BM * LDT, tid);
  __syncthreads();

  for (int kt = 0; kt < ktiles; ++kt) {
    const int cur = kt & 1;
    const float *As = smem + cur * (BM + BN) * LDT;
    const float *Bs = As + BM * LDT;
    if (kt + 1 < ktiles) st.load(p, m0, n0, (kt + 1) * BK, tid);
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      f32x4 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const f32x4 *>(As + (wm * 64 + i * 32 + r) * LDT + g * 8 + 4 * h);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *reinterpret_cast<const f32x4 *>(Bs + (wn * 64 + j * 32 + r) * LDT + g * 8 + 4 * h);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ktiles) {
      float *An = smem + (cur ^ 1) * (BM + BN) * LDT;
      st.store(An, An + BM * LDT, tid);
    }
    __syncthreads();
  }

  // Epilogue: + bias, then the fused post-ops in model order.
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + j * 32 + r;
    if (col >= p.n) continue;
    const float bias = p.bias ? p.bias[col] : 0.0f;
    const float sc = p.bn_scale ? p.bn_scale[col] : 1.0f;
    const float of = p.bn_offset ? p.bn_offset[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row >= p.m) continue;
        float v = acc[i][j][e];
        if (p.bias) v = v + bias;
        for (int q = 0; q < p.npost; ++q) {
          if (p.post[q] == kPostRelu) {
            v = v < 0.0f ? 0.0f : v;
          } else if (p.post[q] == kPostBatchNorm) {
            v = v * sc;
            v = v + of;
          }
        }
        p.y[(int64_t)row * p.ldy + col] = v;
      }
    }
  }
}

}  // namespace

int launch_gemm_f32(hipStream_t s, const GemmArgs &a) {
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  if (a.kpad % BK != 0 || a.k > a.kpad || a.nseg < 1 || a.nseg > 8 || a.din <= 0 ||
      a.nseg * a.din != a.k)
    return fail(CE_GPU_EINVAL, "gemm_f32: bad K geometry");
  if (a.npost > 4) return fail(CE_GPU_EINVAL, "gemm_f32: too many post ops");
  KArgs p;
  p.x = a.x;
  p.row_map = a.row_map;
  p.w = a.w;
  p.bias = a.bias;
  p.bn_scale = a.bn_scale;
  p.bn_offset = a.bn_offset;
  p.y = a.y;
  p.ldx = a.ldx;
  p.ldw = a.ldw;
  p.ldy = a.ldy;
  p.m = a.m;
  p.n = a.n;
  p.k = a.k;
  p.kpad = a.kpad;
  p.din = a.din;
  p.nseg = a.nseg;
  for (int i = 0; i < 8; ++i) p.off[i] = a.off[i];
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.tiles_n = (a.n + BN - 1) / BN;
  const int tiles_m = (a.m + BM - 1) / BM;
  // fast A path: every K-tile inside one segment, float4-aligned rows
  const bool a_fast = (a.din % BK == 0) && (a.ldx % 4 == 0) &&
                      ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0);
  if (!a.b_nmajor && (a.ldw % 4 != 0 || (reinterpret_cast<uintptr_t>(a.w) & 15) != 0))
    return fail(CE_GPU_EINVAL, "gemm_f32: K-major B must be 16-byte aligned");
  dim3 grid(tiles_m * p.tiles_n), block(256);
  if (a_fast && !a.b_nmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, block, 0, s, p);
  else if (!a_fast && !a.b_nmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, block, 0, s, p);
  else if (a_fast)
    hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
