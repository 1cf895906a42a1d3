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
// Tiling for CDNA4 (tile shape is a template; launch_gemm_f32 picks it):
// 256 threads = 4 waves, each wave a TI x TJ grid of v_mfma_f32_32x32x2_f32
// tiles (exact fp32 fma chain, 64 cycles per instruction per SIMD).  Operands are read from LDS with ds_read_b128: lane (r, h) of a
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
  int tiles_m, tiles_n;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Tile configuration: BM x BN block tile, BK deep, WGM x WGN waves.
template <int BM_, int BN_, int BK_, int WGM_, int WGN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WGM = WGM_, WGN = WGN_;
  static_assert(WGM * WGN == 4, "4 waves per block");
  static constexpr int LDT = BK + 4;                // padded LDS row (floats)
  static constexpr int TI = BM / WGM / 32, TJ = BN / WGN / 32;
  static constexpr int AV = BM * BK / 4 / 256;      // float4 of A per thread
  static constexpr int BV = BN * BK / 4 / 256;
  static constexpr int AS = BM * BK / 256;          // scalars of A per thread (gather path)
  static constexpr int BS = BN * BK / 256;
  static constexpr int SMEM = 2 * (BM + BN) * LDT;  // floats, two stages
  static_assert(TI >= 1 && TJ >= 1 && AV >= 1 && BV >= 1 && BK % 8 == 0, "bad tile");
};

// Global -> register staging of one K-tile.  ROWMAP (first layer only) is a
// template flag: a runtime `if (row_map)` around the index load makes hipcc
// wait vmcnt(0) on every staging load, serialising the prefetch.
template <class C, bool A_FAST, bool B_NMAJOR, bool ROWMAP>
struct Stage {
  static constexpr int NA = A_FAST ? C::AV : 1, NAS = A_FAST ? 1 : C::AS;
  static constexpr int NB = B_NMAJOR ? 1 : C::BV, NBS = B_NMAJOR ? C::BS : 1;
  f32x4 a[NA];
  float as[NAS];
  f32x4 b[NB];
  float bs[NBS];

  __device__ __forceinline__ void load(const KArgs &p, int m0, int n0, int k0, int tid) {
    constexpr int C4 = C::BK / 4;
    if constexpr (A_FAST) {
      // whole K-tile inside one splice segment
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      const int shift = p.off[seg];
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + 256 * i, row = idx / C4, c4 = idx % C4;
        int src = clampi(m0 + row + shift, 0, p.m - 1);
        if constexpr (ROWMAP) src = p.row_map[src];
        a[i] = *reinterpret_cast<const f32x4 *>(p.x + (int64_t)src * p.ldx + col0 + 4 * c4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NAS; ++i) {
        const int idx = tid + 256 * i, row = idx / C::BK, kk = idx % C::BK;
        const int kg = k0 + kk;
        float v = 0.0f;
        if (kg < p.k) {
          const int seg = kg / p.din, col = kg - seg * p.din;
          int src = clampi(m0 + row + p.off[seg], 0, p.m - 1);
          if constexpr (ROWMAP) src = p.row_map[src];
          v = p.x[(int64_t)src * p.ldx + col];
        }
        as[i] = v;
      }
    }
    if constexpr (!B_NMAJOR) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + 256 * i, row = idx / C4, c4 = idx % C4;
        const int nn = min(n0 + row, p.n - 1);
        b[i] = *reinterpret_cast<const f32x4 *>(p.w + (int64_t)nn * p.ldw + k0 + 4 * c4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NBS; ++i) {
        const int idx = tid + 256 * i, kk = idx / C::BN, nn = idx % C::BN;
        const int kg = k0 + kk, ng = n0 + nn;
        bs[i] = (kg < p.k && ng < p.n) ? p.w[(int64_t)kg * p.ldw + ng] : 0.0f;
      }
    }
  }

  __device__ __forceinline__ void store(float *As, float *Bs, int tid) {
    constexpr int C4 = C::BK / 4;
    if constexpr (A_FAST) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int idx = tid + 256 * i, row = idx / C4, c4 = idx % C4;
        *reinterpret_cast<f32x4 *>(As + row * C::LDT + 4 * c4) = a[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NAS; ++i) {
        const int idx = tid + 256 * i, row = idx / C::BK, kk = idx % C::BK;
        As[row * C::LDT + kk] = as[i];
      }
    }
    if constexpr (!B_NMAJOR) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + 256 * i, row = idx / C4, c4 = idx % C4;
        *reinterpret_cast<f32x4 *>(Bs + row * C::LDT + 4 * c4) = b[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NBS; ++i) {
        const int idx = tid + 256 * i, kk = idx / C::BN, nn = idx % C::BN;
        Bs[nn * C::LDT + kk] = bs[i];
      }
    }
  }
};

// XCD-aware tile order: blocks b and b+8 run on one XCD (round-robin
// dispatch), so give each XCD a contiguous run of tiles in column-major tile
// order -- the blocks of one XCD then share weight panels in its L2.  The
// remap is bijective for any grid size (a speed choice, never correctness).
__device__ __forceinline__ void tile_of(int b, int tiles_m, int tiles_n, int *tm, int *tn) {
  const int nwg = tiles_m * tiles_n, q = nwg / 8, r = nwg % 8, xcd = b % 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
  *tn = t / tiles_m;
  *tm = t - *tn * tiles_m;
}

template <class C, bool A_FAST, bool B_NMAJOR, bool ROWMAP>
__global__ __launch_bounds__(256, 1) void gemm_f32_kernel(KArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, LDT = C::LDT, TI = C::TI, TJ = C::TJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int ktiles = p.kpad / BK;
  Stage<C, A_FAST, B_NMAJOR, ROWMAP> st;
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
      f32x4 af[TI], bf[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i)
        af[i] = *reinterpret_cast<const f32x4 *>(As + (wm * TI * 32 + i * 32 + r) * LDT + g * 8 + 4 * h);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        bf[j] = *reinterpret_cast<const f32x4 *>(Bs + (wn * TJ * 32 + j * 32 + r) * LDT + g * 8 + 4 * h);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < ktiles) {
      float *An = smem + (cur ^ 1) * (BM + BN) * LDT;
      st.store(An, An + BM * LDT, tid);
    }
    __syncthreads();
  }

  // Epilogue: + bias, then the fused post-ops in model order (reference
  // roundings: add, then multiply and add separately -- built without FMA
  // contraction).
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int col = n0 + wn * TJ * 32 + j * 32 + r;
    if (col >= p.n) continue;
    const float bias = p.bias ? p.bias[col] : 0.0f;
    const float sc = p.bn_scale ? p.bn_scale[col] : 1.0f;
    const float of = p.bn_offset ? p.bn_offset[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * TI * 32 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
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

template <class C>
int launch_cfg(hipStream_t s, KArgs p, bool a_fast, bool b_nmajor, bool rm) {
  p.tiles_n = (p.n + C::BN - 1) / C::BN;
  p.tiles_m = (p.m + C::BM - 1) / C::BM;
  if (p.kpad % C::BK != 0) return fail(CE_GPU_EINVAL, "gemm_f32: kpad not a multiple of BK");
  if (a_fast && p.din % C::BK != 0) a_fast = false;
  dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if (a_fast && !b_nmajor && !rm)
    hipLaunchKernelGGL((gemm_f32_kernel<C, true, false, false>), grid, block, 0, s, p);
  else if (a_fast && !b_nmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<C, true, false, true>), grid, block, 0, s, p);
  else if (!b_nmajor && rm)
    hipLaunchKernelGGL((gemm_f32_kernel<C, false, false, true>), grid, block, 0, s, p);
  else if (!b_nmajor)
    hipLaunchKernelGGL((gemm_f32_kernel<C, false, false, false>), grid, block, 0, s, p);
  else if (a_fast)
    hipLaunchKernelGGL((gemm_f32_kernel<C, true, true, false>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<C, false, true, false>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

// Tile variants (CATEARS_GEMM_VARIANT selects one for tuning runs).
using V0 = Cfg<128, 128, 32, 2, 2>;
using V1 = Cfg<128, 128, 64, 2, 2>;
using V2 = Cfg<128, 64, 32, 2, 2>;
using V3 = Cfg<64, 128, 32, 2, 2>;
using V4 = Cfg<128, 64, 64, 2, 2>;

int variant() {
  static int v = [] {
    const char *e = getenv("CATEARS_GEMM_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

}  // namespace

// K is padded to a multiple of this for every variant (weights upload).
int gemm_k_align() { return 64; }

int launch_gemm_f32(hipStream_t s, const GemmArgs &a) {
  if (a.m <= 0 || a.n <= 0) return CE_GPU_OK;
  if (a.k > a.kpad || a.nseg < 1 || a.nseg > 8 || a.din <= 0 || a.nseg * a.din != a.k)
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
  // fast A path: every K-tile inside one segment, float4-aligned rows
  const bool a_fast = (a.ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0);
  if (!a.b_nmajor && (a.ldw % 4 != 0 || (reinterpret_cast<uintptr_t>(a.w) & 15) != 0))
    return fail(CE_GPU_EINVAL, "gemm_f32: K-major B must be 16-byte aligned");
  const bool rm = a.row_map != nullptr;
  if (a.b_nmajor && rm) return fail(CE_GPU_EINVAL, "gemm_f32: row_map needs K-major weights");
  // K-tiles deeper than 32 only where K allows it
  const bool deep = a.kpad % 64 == 0;
  switch (variant()) {
    case 1:
      return deep ? launch_cfg<V1>(s, p, a_fast, a.b_nmajor, rm) : launch_cfg<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 2:
      return launch_cfg<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 3:
      return launch_cfg<V3>(s, p, a_fast, a.b_nmajor, rm);
    case 4:
      return deep ? launch_cfg<V4>(s, p, a_fast, a.b_nmajor, rm) : launch_cfg<V2>(s, p, a_fast, a.b_nmajor, rm);
    default:
      return launch_cfg<V0>(s, p, a_fast, a.b_nmajor, rm);
  }
}

}  // namespace catears
