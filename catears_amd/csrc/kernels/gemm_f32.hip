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
#include <stdlib.h>

#include "../internal.h"
#include "../tile_order.h"

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
  uint64_t off_packed;  // splice offset of segment s in signed byte s
  int post[4];
  int npost, post_mode;
  int tiles_m, tiles_n;
  int group;  // column tiles per tile group (tile_of)
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Epilogue of one wave's (TI x 32) x (TJ x 32) tile at (row0, col0): + bias,
// then the fused post-ops in model order with the reference's roundings
// (add, then multiply and add separately -- built without FMA contraction).
// An absent bias adds -0, an exact identity for every float (-0 included), so
// the add is unconditional; the post chain is one uniform mode per launch.
template <int TI, int TJ>
__device__ __forceinline__ void f32_epilogue(const KArgs &p, const f32x16 (&acc)[TI][TJ], int row0, int col0, int r,
                                             int h) {
  with_post_mode(p.post_mode, [&](auto M) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = col0 + j * 32 + r;
      if (col >= p.n) continue;
      const float bias = p.bias ? p.bias[col] : -0.0f;
      const float sc = p.bn_scale ? p.bn_scale[col] : 1.0f;
      const float of = p.bn_offset ? p.bn_offset[col] : -0.0f;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = row0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          const float v = apply_post<decltype(M)::value>(acc[i][j][e] + bias, sc, of, p.post, p.npost);
          if (row < p.m) p.y[(int64_t)row * p.ldy + col] = v;
        }
      }
    }
  });
}

// Tile configuration: BM x BN block tile, BK deep, WGM x WGN waves.
template <int BM_, int BN_, int BK_, int WGM_, int WGN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WGM = WGM_, WGN = WGN_;
  static constexpr int NW = WGM * WGN, NT = 64 * NW;  // waves / threads per block
  static_assert(NW == 4 || NW == 8, "4 or 8 waves per block (8: LDS-DMA kernel only)");
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
  static_assert(C::NW == 4, "register staging assumes 256 threads");
  static constexpr int NA = A_FAST ? C::AV : 1, NAS = A_FAST ? 1 : C::AS;
  static constexpr int NB = B_NMAJOR ? 1 : C::BV, NBS = B_NMAJOR ? C::BS : 1;
  f32x4 a[NA];
  float as[NAS];
  f32x4 b[NB];
  float bs[NBS];

  // The splice offsets travel packed in one 64-bit kernel argument (8 signed
  // bytes) that stays in SGPRs: a dynamically indexed p.off[seg] in the K loop
  // is an s_load, and a pending scalar load makes hipcc wait lgkmcnt(0) --
  // behind every outstanding LDS read and write -- before the next use of any
  // LDS result.
  __device__ __forceinline__ static int shift_of(const KArgs &p, int seg) {
    return (int)(signed char)(p.off_packed >> (8 * seg));
  }

  // Per-thread byte offsets of the staged rows, recomputed only when the
  // splice segment changes (A) or never (B): a K-tile's loads are then a
  // wave-uniform base (SGPR) plus a fixed 32-bit VGPR offset, i.e. no vector
  // address arithmetic between the MFMAs.
  uint32_t aoff[A_FAST ? NA : 1];
  uint32_t boff[B_NMAJOR ? 1 : NB];
  int cur_seg = -1;

  __device__ __forceinline__ void init(const KArgs &p, int n0, int tid) {
    constexpr int C4 = C::BK / 4;
    if constexpr (!B_NMAJOR) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int idx = tid + 256 * i, row = idx / C4, c4 = idx % C4;
        boff[i] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + 4 * c4) * 4);
      }
    }
  }

  __device__ __forceinline__ void load(const KArgs &p, int m0, int n0, int k0, int tid) {
    constexpr int C4 = C::BK / 4;
    if constexpr (A_FAST) {
      // whole K-tile inside one splice segment
      const int seg = k0 / p.din, col0 = k0 - seg * p.din;
      if (seg != cur_seg) {
        cur_seg = seg;
        const int shift = shift_of(p, seg);
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int idx = tid + 256 * i, row = idx / C4, c4 = idx % C4;
          int src = clampi(m0 + row + shift, 0, p.m - 1);
          if constexpr (ROWMAP) src = p.row_map[src];
          aoff[i] = (uint32_t)(src * p.ldx + 4 * c4) * 4u;
        }
      }
      const char *base = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 4;
#pragma unroll
      for (int i = 0; i < NA; ++i) a[i] = *reinterpret_cast<const f32x4 *>(base + aoff[i]);
    } else {
#pragma unroll
      for (int i = 0; i < NAS; ++i) {
        const int idx = tid + 256 * i, row = idx / C::BK, kk = idx % C::BK;
        const int kg = k0 + kk;
        float v = 0.0f;
        if (kg < p.k) {
          const int seg = kg / p.din, col = kg - seg * p.din;
          int src = clampi(m0 + row + shift_of(p, seg), 0, p.m - 1);
          if constexpr (ROWMAP) src = p.row_map[src];
          v = p.x[(int64_t)src * p.ldx + col];
        }
        as[i] = v;
      }
    }
    if constexpr (!B_NMAJOR) {
      const char *base = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 4;
#pragma unroll
      for (int i = 0; i < NB; ++i) b[i] = *reinterpret_cast<const f32x4 *>(base + boff[i]);
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

template <class C, bool A_FAST, bool B_NMAJOR, bool ROWMAP>
__global__ __launch_bounds__(256, 1) void gemm_f32_kernel(KArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, LDT = C::LDT, TI = C::TI, TJ = C::TJ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
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
  st.init(p, n0, tid);
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

  f32_epilogue<TI, TJ>(p, acc, m0 + wm * TI * 32, n0 + wn * TJ * 32, r, h);
}

// Software-pipelined variant: fragments of k-group g+1 are read from LDS
// while the MFMAs of group g run, and the single barrier per K-tile sits
// before the tile's LAST group, so the MFMAs of that group cover the LDS
// latency of the next tile's first fragments.  The next-next tile's global
// loads are issued right after the staged registers are written to LDS, a
// full K-tile ahead of their use.
//   LDS WAR: buffer b is rewritten in tile kt only after the barrier of tile
//   kt-1, which every wave passes with lgkmcnt(0) -- i.e. after its last
//   read of b.  RAW: tile kt+1 is stored before tile kt's barrier and read
//   after it.
template <class C, bool A_FAST, bool B_NMAJOR, bool ROWMAP>
__global__ __launch_bounds__(256, 1) void gemm_f32_pipe_kernel(KArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, LDT = C::LDT, TI = C::TI, TJ = C::TJ;
  constexpr int G = BK / 8;
  static_assert(G >= 2, "pipeline needs >= 2 k-groups per tile");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int r = lane & 31, h = lane >> 5;
  const int a_off = (wm * TI * 32 + r) * LDT + 4 * h;
  const int b_off = (wn * TJ * 32 + r) * LDT + 4 * h;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  auto frag = [&](const float *As, int g, f32x4 *fa, f32x4 *fb) {
    const float *Bs = As + BM * LDT;
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = *reinterpret_cast<const f32x4 *>(As + a_off + i * 32 * LDT + g * 8);
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = *reinterpret_cast<const f32x4 *>(Bs + b_off + j * 32 * LDT + g * 8);
  };
  auto mma = [&](const f32x4 *fa, const f32x4 *fb) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  };

  const int ktiles = p.kpad / BK;
  Stage<C, A_FAST, B_NMAJOR, ROWMAP> st;
  st.init(p, n0, tid);
  st.load(p, m0, n0, 0, tid);
  st.store(smem, smem + BM * LDT, tid);
  if (ktiles > 1) st.load(p, m0, n0, BK, tid);
  __syncthreads();

  f32x4 fa0[TI], fb0[TJ], fa1[TI], fb1[TJ];
  frag(smem, 0, fa0, fb0);
  for (int kt = 0; kt < ktiles; ++kt) {
    const float *As = smem + (kt & 1) * (BM + BN) * LDT;
    float *An = smem + ((kt & 1) ^ 1) * (BM + BN) * LDT;
    const bool more = kt + 1 < ktiles;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      f32x4 *ca = (g & 1) ? fa1 : fa0, *cb = (g & 1) ? fb1 : fb0;
      f32x4 *na = (g & 1) ? fa0 : fa1, *nb = (g & 1) ? fb0 : fb1;
      if (g + 1 < G) {
        frag(As, g + 1, na, nb);
      } else if (more) {
        frag(An, 0, na, nb);  // next tile's first fragments, after the barrier
      }
      mma(ca, cb);
      if (g == G - 2 && more) {
        st.store(An, An + BM * LDT, tid);
        __syncthreads();
        if (kt + 2 < ktiles) st.load(p, m0, n0, (kt + 2) * BK, tid);
      }
    }
    // G is even, so the next tile's group 0 landed in fa0/fb0.
  }

  f32_epilogue<TI, TJ>(p, acc, m0 + wm * TI * 32, n0 + wn * TJ * 32, r, h);
}

// Pipeline v2 (write-after-barrier, the register-staging schedule of the
// CDNA guide's T14): staged registers of tile kt+1 are written to LDS right
// after the MFMAs of tile kt's second k-group are issued (so the ds_writes run
// under MFMAs), the loads of tile kt+2 are re-issued at once, and the one
// barrier per tile sits before the last k-group, whose MFMAs cover the LDS
// latency of tile kt+1's first fragments.
//   WAR: buffer (kt+1)&1 was last read by tile kt-1's group G-1, whose
//   fragments every wave fetched (lgkmcnt(0)) before the barrier of kt-1.
//   RAW: it is written at group 0 of kt and read after the barrier of kt.
template <class C, bool A_FAST, bool B_NMAJOR, bool ROWMAP>
__global__ __launch_bounds__(256, 1) void gemm_f32_pipe2_kernel(KArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, LDT = C::LDT, TI = C::TI, TJ = C::TJ;
  constexpr int G = BK / 8;
  static_assert(G >= 4 && G % 2 == 0, "pipeline needs an even number >= 4 of k-groups");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int r = lane & 31, h = lane >> 5;
  const int a_off = (wm * TI * 32 + r) * LDT + 4 * h;
  const int b_off = (wn * TJ * 32 + r) * LDT + 4 * h;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  auto frag = [&](const float *As, int g, f32x4 *fa, f32x4 *fb) {
    const float *Bs = As + BM * LDT;
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = *reinterpret_cast<const f32x4 *>(As + a_off + i * 32 * LDT + g * 8);
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = *reinterpret_cast<const f32x4 *>(Bs + b_off + j * 32 * LDT + g * 8);
  };
  auto mma = [&](const f32x4 *fa, const f32x4 *fb) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  };

  const int ktiles = p.kpad / BK;
  Stage<C, A_FAST, B_NMAJOR, ROWMAP> st;
  st.init(p, n0, tid);
  st.load(p, m0, n0, 0, tid);
  st.store(smem, smem + BM * LDT, tid);
  if (ktiles > 1) st.load(p, m0, n0, BK, tid);
  __syncthreads();

  f32x4 fa0[TI], fb0[TJ], fa1[TI], fb1[TJ];
  frag(smem, 0, fa0, fb0);
  for (int kt = 0; kt < ktiles; ++kt) {
    const float *As = smem + (kt & 1) * (BM + BN) * LDT;
    float *An = smem + ((kt & 1) ^ 1) * (BM + BN) * LDT;
    const bool more = kt + 1 < ktiles;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      f32x4 *ca = (g & 1) ? fa1 : fa0, *cb = (g & 1) ? fb1 : fb0;
      f32x4 *na = (g & 1) ? fa0 : fa1, *nb = (g & 1) ? fb0 : fb1;
      if (g + 1 < G) {
        frag(As, g + 1, na, nb);
      } else if (more) {
        frag(An, 0, na, nb);  // next tile's first fragments, after the barrier
      }
      mma(ca, cb);
      // store after group 1's MFMAs: the wait before group 1 then covers only
      // its fragment reads, and group 2's wait finds the writes long retired
      if (g == 1 && more) {
        st.store(An, An + BM * LDT, tid);
        if (kt + 2 < ktiles) st.load(p, m0, n0, (kt + 2) * BK, tid);
      }
      if (g == G - 2 && more) __syncthreads();
    }
  }

  f32_epilogue<TI, TJ>(p, acc, m0 + wm * TI * 32, n0 + wn * TJ * 32, r, h);
}

template <class C>
int launch_pipe2(hipStream_t s, KArgs p, bool a_fast, bool b_nmajor, bool rm) {
  p.tiles_n = (p.n + C::BN - 1) / C::BN;
  p.tiles_m = (p.m + C::BM - 1) / C::BM;
  if (p.kpad % C::BK != 0) return fail(CE_GPU_EINVAL, "gemm_f32: kpad not a multiple of BK");
  if (a_fast && p.din % C::BK != 0) a_fast = false;
  dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if (a_fast && !b_nmajor && !rm)
    hipLaunchKernelGGL((gemm_f32_pipe2_kernel<C, true, false, false>), grid, block, 0, s, p);
  else if (a_fast && !b_nmajor)
    hipLaunchKernelGGL((gemm_f32_pipe2_kernel<C, true, false, true>), grid, block, 0, s, p);
  else if (!b_nmajor && rm)
    hipLaunchKernelGGL((gemm_f32_pipe2_kernel<C, false, false, true>), grid, block, 0, s, p);
  else if (!b_nmajor)
    hipLaunchKernelGGL((gemm_f32_pipe2_kernel<C, false, false, false>), grid, block, 0, s, p);
  else if (a_fast)
    hipLaunchKernelGGL((gemm_f32_pipe2_kernel<C, true, true, false>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_pipe2_kernel<C, false, true, false>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

template <class C>
int launch_pipe(hipStream_t s, KArgs p, bool a_fast, bool b_nmajor, bool rm) {
  p.tiles_n = (p.n + C::BN - 1) / C::BN;
  p.tiles_m = (p.m + C::BM - 1) / C::BM;
  if (p.kpad % C::BK != 0) return fail(CE_GPU_EINVAL, "gemm_f32: kpad not a multiple of BK");
  if (a_fast && p.din % C::BK != 0) a_fast = false;
  dim3 grid(p.tiles_m * p.tiles_n), block(256);
  if (a_fast && !b_nmajor && !rm)
    hipLaunchKernelGGL((gemm_f32_pipe_kernel<C, true, false, false>), grid, block, 0, s, p);
  else if (a_fast && !b_nmajor)
    hipLaunchKernelGGL((gemm_f32_pipe_kernel<C, true, false, true>), grid, block, 0, s, p);
  else if (!b_nmajor && rm)
    hipLaunchKernelGGL((gemm_f32_pipe_kernel<C, false, false, true>), grid, block, 0, s, p);
  else if (!b_nmajor)
    hipLaunchKernelGGL((gemm_f32_pipe_kernel<C, false, false, false>), grid, block, 0, s, p);
  else if (a_fast)
    hipLaunchKernelGGL((gemm_f32_pipe_kernel<C, true, true, false>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_pipe_kernel<C, false, true, false>), grid, block, 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
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
using V8 = Cfg<64, 64, 32, 2, 2>;
using W0 = Cfg<128, 128, 32, 4, 2>;  // 8 waves, 32 x 64 each
using W1 = Cfg<128, 128, 32, 2, 4>;  // 8 waves, 64 x 32 each
using W2 = Cfg<64, 128, 64, 2, 2>;
using W3 = Cfg<128, 128, 64, 4, 2>;
using W4 = Cfg<64, 128, 32, 2, 4>;   // 8 waves, 32 x 32 each
using W5 = Cfg<128, 64, 32, 4, 2>;   // 8 waves, 32 x 32 each
using W6 = Cfg<64, 256, 32, 2, 4>;   // 8 waves, 32 x 64 each


// ---------------------------------------------------------------------------
// LDS-DMA pipeline (glds): operands go global -> LDS with
// global_load_lds_dwordx4 (no VGPR staging, no ds_write pass), three LDS
// stages, one raw s_barrier per K-tile and a counted vmcnt that keeps the
// next tile's DMAs in flight across it (CDNA guide: "Pipelining across
// barriers").  Requires the fast A path (every K-tile inside one splice
// segment) and K-major weights -- the TDNN layers after the first.
//
// An LDS-DMA writes 64 lanes x 16 B contiguously, so tiles are stored
// unpadded (BK = 32 floats = 128 B per row, 8 rows per instruction) and the
// bank spread comes from an XOR swizzle applied on the SOURCE address: chunk
// c of row r lands at chunk c ^ ((r >> 1) & 7).  The 16 lanes of a
// ds_read_b128 group (rows r..r+15 of one fragment, one chunk) then cover the
// 16 distinct 16-B slots of the 256-B bank row.
//
// Synchronisation per K-tile kt (stage kt % 3):
//   s_waitcnt vmcnt(this wave's DMAs for kt+1)  -> this wave's kt landed
//   s_barrier                                    -> every wave's kt landed, and
//                                                   every wave is past its reads
//                                                   of stage (kt-1) % 3
//   issue DMAs for kt+2 into stage (kt+2) % 3 == (kt-1) % 3   (WAR safe)
//   ds_read + MFMA on stage kt % 3
// All LDS is one __shared__ array and the loop holds no ordinary global
// loads, so hipcc adds no vmcnt(0) of its own.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void glds16(const char *src, float *lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                   (__attribute__((address_space(3))) void *)lds_dst, 16, 0, 0);
}

template <class C, int STAGES, bool PRIO = false>
__global__ __launch_bounds__(C::NT, 1) void gemm_f32_glds_kernel(KArgs p) {
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, TI = C::TI, TJ = C::TJ, NW = C::NW;
  static_assert(BK == 32 || BK == 64, "tile rows of 128 or 256 bytes");
  static_assert(STAGES == 2 || STAGES == 3, "2 or 3 LDS stages");
  constexpr int CPR = BK / 4;                          // 16-B chunks per tile row
  constexpr int RB = 256 / (BK * 4);                   // tile rows per 256-B bank row
  constexpr int RPI = 1024 / (BK * 4);                 // tile rows per DMA instruction
  constexpr int NGA = BM * BK * 4 / 1024 / NW;         // DMA instructions per wave, A
  constexpr int NGB = BN * BK * 4 / 1024 / NW;         // and B
  constexpr int NG = NGA + NGB;
  static_assert(NGA >= 1 && NGB >= 1, "tile too small for one DMA per wave");
  constexpr int STAGE = (BM + BN) * BK;                // floats per stage
  __shared__ __attribute__((aligned(1024))) float smem[STAGES * STAGE];
  // chunk c of tile row `row` is stored at chunk c ^ swz(row)
  auto swz = [](int row) { return (row / RB) & (CPR - 1); };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, p.group, &tm, &tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int r = lane & 31, h = lane >> 5;

  // per-lane DMA source offsets (bytes from the tile's uniform base)
  const int lrow = lane / CPR, lchunk = lane % CPR;
  uint32_t boff[NGB];
#pragma unroll
  for (int j = 0; j < NGB; ++j) {
    const int row = (wave * NGB + j) * RPI + lrow;
    const int c = lchunk ^ swz(row);
    boff[j] = (uint32_t)((min(n0 + row, p.n - 1) * p.ldw + 4 * c) * 4);
  }
  uint32_t aoff[NGA];
  int cur_seg = -1;

  auto issue = [&](int kt) {
    const int k0 = kt * BK;
    const int seg = k0 / p.din, col0 = k0 - seg * p.din;
    if (seg != cur_seg) {
      cur_seg = seg;
      const int shift = (int)(signed char)(p.off_packed >> (8 * seg));
#pragma unroll
      for (int i = 0; i < NGA; ++i) {
        const int row = (wave * NGA + i) * RPI + lrow;
        const int c = lchunk ^ swz(row);
        const int src = clampi(m0 + row + shift, 0, p.m - 1);
        aoff[i] = (uint32_t)(src * p.ldx + 4 * c) * 4u;
      }
    }
    float *st = smem + (kt % STAGES) * STAGE;
    const char *abase = reinterpret_cast<const char *>(p.x) + (size_t)col0 * 4;
    const char *bbase = reinterpret_cast<const char *>(p.w) + (size_t)k0 * 4;
#pragma unroll
    for (int i = 0; i < NGA; ++i) glds16(abase + aoff[i], st + (wave * NGA + i) * RPI * BK);
#pragma unroll
    for (int j = 0; j < NGB; ++j) glds16(bbase + boff[j], st + BM * BK + (wave * NGB + j) * RPI * BK);
  };

  // fragment addresses: row base + swizzled chunk of k-group g (fragment
  // rows start at multiples of 32, so swz(row) == swz(r))
  const int xr = swz(r) ^ h;  // chunk 2g + h  ->  (2g) ^ xr
  const int a_row = (wm * TI * 32 + r) * BK, b_row = BM * BK + (wn * TJ * 32 + r) * BK;

  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  auto frag = [&](const float *st, int g, f32x4 *fa, f32x4 *fb) {
    const int ch = ((2 * g) ^ xr) * 4;
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = *reinterpret_cast<const f32x4 *>(st + a_row + i * 32 * BK + ch);
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = *reinterpret_cast<const f32x4 *>(st + b_row + j * 32 * BK + ch);
  };
  auto mma = [&](const f32x4 *fa, const f32x4 *fb) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
  };

  const int ktiles = p.kpad / BK;
  issue(0);
  if (STAGES == 3 && ktiles > 1) issue(1);
  for (int kt = 0; kt < ktiles; ++kt) {
    if (STAGES == 3 && kt + 1 < ktiles)
      wait_vmcnt<NG>();  // leave tile kt+1's DMAs in flight
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < ktiles) issue(kt + STAGES - 1);
    const float *st = smem + (kt % STAGES) * STAGE;
    f32x4 fa0[TI], fb0[TJ], fa1[TI], fb1[TJ];
    frag(st, 0, fa0, fb0);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      if (g + 1 < BK / 8) frag(st, g + 1, (g & 1) ? fa0 : fa1, (g & 1) ? fb0 : fb1);
      mma((g & 1) ? fa1 : fa0, (g & 1) ? fb1 : fb0);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  f32_epilogue<TI, TJ>(p, acc, m0 + wm * TI * 32, n0 + wn * TJ * 32, r, h);
}

// glds for the layers it fits, pipe2 for the rest (first layer's gather,
// N-major MatMat operands).
template <class C, int STAGES = 3, bool PRIO = false>
int launch_glds(hipStream_t s, KArgs p, bool a_fast, bool b_nmajor, bool rm) {
  if (!(a_fast && !b_nmajor && !rm && p.din % C::BK == 0 && p.kpad % C::BK == 0))
    return launch_pipe2<V3>(s, p, a_fast, b_nmajor, rm);
  p.tiles_n = (p.n + C::BN - 1) / C::BN;
  p.tiles_m = (p.m + C::BM - 1) / C::BM;
  hipLaunchKernelGGL((gemm_f32_glds_kernel<C, STAGES, PRIO>), dim3(p.tiles_m * p.tiles_n), dim3(C::NT), 0, s, p);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

// Default: LDS-DMA kernel, 128 x 64 tiles (64 x 32 per wave), two stages
// (48 KB LDS -> three blocks per CU) -- measured best on TDNN-S with three
// nnet streams (tools/gemm_variants.sh: 115.5 TF vs 110.5 for the register-
// staged 64 x 128 pipeline).  Layers it cannot take (the first layer's
// gather, N-major MatMat operands) fall back to pipe2 64 x 128.
// CATEARS_GEMM_VARIANT selects another tiling in `make EXPERIMENTS=1` builds
// (tools/); a value this build does not carry fails with CE_GPU_EINVAL.
constexpr int kDefaultVariant = 29;

int variant() {
  static int v = CE_KNOB("CATEARS_GEMM_VARIANT", kDefaultVariant);
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
  p.off_packed = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (a.off[i] < -128 || a.off[i] > 127) return fail(CE_GPU_ENOTSUP, "gemm_f32: splice offset beyond +-127");
    p.off_packed |= (uint64_t)(uint8_t)(int8_t)a.off[i] << (8 * i);
  }
  for (int i = 0; i < 4; ++i) p.post[i] = a.post[i];
  p.npost = a.npost;
  p.post_mode = post_mode(a.post, a.npost);
  static const int group_env = CE_KNOB("CATEARS_GEMM_GROUP", 0);
  p.group = group_env > 0 ? group_env : 16;  // tools: group sweep (16 >= 8 > 4 by 0.3-0.6 %)
  // fast A path: every K-tile inside one segment, float4-aligned rows
  const bool a_fast = (a.ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(a.x) & 15) == 0);
  if (!a.b_nmajor && (a.ldw % 4 != 0 || (reinterpret_cast<uintptr_t>(a.w) & 15) != 0))
    return fail(CE_GPU_EINVAL, "gemm_f32: K-major B must be 16-byte aligned");
  const bool rm = a.row_map != nullptr;
  if (a.b_nmajor && rm) return fail(CE_GPU_EINVAL, "gemm_f32: row_map needs K-major weights");
  // staged loads use 32-bit byte offsets from a uniform base
  if (!a.b_nmajor && (int64_t)a.n * a.ldw * 4 >= (int64_t)1 << 32)
    return fail(CE_GPU_EINVAL, "gemm_f32: weight matrix beyond 4 GiB");
  if (a_fast && (int64_t)(a.row_map ? INT32_MAX / 4 : a.m) * a.ldx * 4 >= (int64_t)1 << 32 && !a.row_map)
    return fail(CE_GPU_EINVAL, "gemm_f32: activation block beyond 4 GiB");
  // K-tiles deeper than 32 only where K allows it
  [[maybe_unused]] const bool deep = a.kpad % 64 == 0;
  switch (variant()) {
    case kDefaultVariant:
      return launch_glds<V2, 2>(s, p, a_fast, a.b_nmajor, rm);
#ifdef CATEARS_EXPERIMENTS  // tools/gemm_variants.sh
    case 1:
      return deep ? launch_cfg<V1>(s, p, a_fast, a.b_nmajor, rm) : launch_cfg<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 2:
      return launch_cfg<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 3:
      return launch_cfg<V3>(s, p, a_fast, a.b_nmajor, rm);
    case 4:
      return deep ? launch_cfg<V4>(s, p, a_fast, a.b_nmajor, rm) : launch_cfg<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 5:
      return launch_pipe<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 6:
      return launch_pipe<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 7:
      return launch_pipe<V3>(s, p, a_fast, a.b_nmajor, rm);
    case 8:
      return launch_cfg<V8>(s, p, a_fast, a.b_nmajor, rm);
    case 9:
      return launch_pipe<V8>(s, p, a_fast, a.b_nmajor, rm);
    case 10:
      return deep ? launch_pipe<V1>(s, p, a_fast, a.b_nmajor, rm) : launch_pipe<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 11:
      return launch_pipe2<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 12:
      return launch_pipe2<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 13:
      return launch_pipe2<V3>(s, p, a_fast, a.b_nmajor, rm);
    case 14:
      return launch_pipe2<V8>(s, p, a_fast, a.b_nmajor, rm);
    case 15:
      return deep ? launch_pipe2<V1>(s, p, a_fast, a.b_nmajor, rm) : launch_pipe2<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 16:
      return deep ? launch_pipe2<V4>(s, p, a_fast, a.b_nmajor, rm) : launch_pipe2<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 20:
      return launch_glds<V3>(s, p, a_fast, a.b_nmajor, rm);
    case 21:
      return launch_glds<V0>(s, p, a_fast, a.b_nmajor, rm);
    case 22:
      return launch_glds<V2>(s, p, a_fast, a.b_nmajor, rm);
    case 23:
      return launch_glds<W0>(s, p, a_fast, a.b_nmajor, rm);
    case 24:
      return launch_glds<W1>(s, p, a_fast, a.b_nmajor, rm);
    case 25:
      return launch_glds<V3, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 26:
      return deep ? launch_glds<W2, 2>(s, p, a_fast, a.b_nmajor, rm) : launch_glds<V3>(s, p, a_fast, a.b_nmajor, rm);
    case 27:
      return deep ? launch_glds<W3, 2>(s, p, a_fast, a.b_nmajor, rm) : launch_glds<W0>(s, p, a_fast, a.b_nmajor, rm);
    case 28:
      return launch_glds<W0, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 30:
      return launch_glds<V8, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 31:
      return launch_glds<W4, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 32:
      return launch_glds<W5, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 33:
      return launch_glds<W6, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 34:
      return launch_glds<V0, 2>(s, p, a_fast, a.b_nmajor, rm);
    case 36:
      return launch_glds<V2, 2, true>(s, p, a_fast, a.b_nmajor, rm);
    case 37:
      return launch_glds<V2, 3, true>(s, p, a_fast, a.b_nmajor, rm);
    case 35:
      return deep ? launch_glds<V1, 2>(s, p, a_fast, a.b_nmajor, rm) : launch_glds<V0, 2>(s, p, a_fast, a.b_nmajor, rm);
#endif
    default:
      return fail(CE_GPU_EINVAL, "gemm_f32 variant " + std::to_string(variant()) +
                                     " is not in this build (the experiments library: `make EXPERIMENTS=1`)");
  }
}

}  // namespace catears
