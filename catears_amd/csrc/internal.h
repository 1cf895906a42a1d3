// internal.h -- private structures of libcatears_hip (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <type_traits>
#include <vector>

#include "catears_gpu.h"

namespace catears {

// ---------------------------------------------------------------- errors --

// Records `msg` as this thread's last error and returns `code`.
int fail(int code, const std::string &msg);
// HIP error -> CE_GPU_EHIP with context.
int hip_fail(hipError_t e, const char *what);

#define CE_HIP(expr)                                        \
  do {                                                      \
    hipError_t e_ = (expr);                                 \
    if (e_ != hipSuccess) return ::catears::hip_fail(e_, #expr); \
  } while (0)

#define CE_TRY(expr)                 \
  do {                               \
    int rc_ = (expr);                \
    if (rc_ != CE_GPU_OK) return rc_; \
  } while (0)

// -------------------------------------------------- measurement knobs --

// CE_KNOB("CATEARS_...", default): a tuning switch of the measurement tools
// (tools/).  Only the experiments library (make EXPERIMENTS=1,
// -DCATEARS_DIAG) reads it from the environment; the product library
// compiles the default in, so its behaviour never depends on the
// environment and no CATEARS_* name is in it (tests/test_abi.py).  Model and
// context choices go through the C-ABI (ce_gpu_model_set_gemm,
// ce_gpu_ctx_set_latency / _set_fbank / _set_wide_tiles).
#ifdef CATEARS_DIAG
int knob_env(const char *name, int dflt);  // getenv + atoi, read once per name by the caller
#define CE_KNOB(name, dflt) ::catears::knob_env(name, dflt)
#else
#define CE_KNOB(name, dflt) (dflt)
#endif

// ------------------------------------------------------- device buffers --

// Owning device allocation (hipMalloc); never copied.
struct DevBuf {
  void *ptr = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : ptr(o.ptr), bytes(o.bytes) { o.ptr = nullptr, o.bytes = 0; }
  DevBuf &operator=(DevBuf &&o) noexcept {
    if (this != &o) {
      release();
      ptr = o.ptr, bytes = o.bytes;
      o.ptr = nullptr, o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  int alloc(size_t n);
  int upload(const void *src, size_t n);  // alloc + synchronous H2D copy
  void release();
  template <typename T>
  T *as() const { return static_cast<T *>(ptr); }
};

// ------------------------------------------------------------ fbank tables --

// Fixed fbank geometry (src/fbank.h:7-13).
constexpr int kShift = 160;
constexpr int kWinLen = 400;
constexpr int kPadded = 512;
constexpr int kHalf = 256;   // complex FFT points
constexpr int kMel = 40;

// Tables shared by every frame; built on the host by the reference's formulas
// and uploaded once per context.  Layout is what kernels/fbank.hip indexes.
struct FbankTables {
  float window[kWinLen];            // Hamming, src/fbank.cc:248-255
  float twiddle[6 * 64 * 5];        // levels 4..8, 6 x (m/4 - 2) each
  int twiddle_base[9];              // start of level lg in `twiddle`
  float kn[2 * 129];                // real-FFT post twiddles kN_k, k = 1..128
  int mel_off[kMel];                // first FFT bin of each triangle
  int mel_len[kMel];
  int mel_wbase[kMel];              // start of its weights in mel_w
  float mel_w[512];                 // 492 nonzero weights in total
  int mel_total;
  // exact kernel (fbank8_ops.h): phase-A twiddle records [op][lane r][8],
  // the length-16 node's twiddles (n = 1, n = 3), mel slot windows: lane q
  // of slot c starts at bin fb8_mel_st[c * 8 + q], weights at
  // fb8_mel_w[q * kMelWTot + kMelWBase[c] ...]
  float fb8_twa[23 * 8 * 8];
  float fb8_tw16[12];
  int fb8_mel_st[5 * 8];
  float fb8_mel_w[92 * 8];
};

// Builds the tables (tables.cc).
void build_fbank_tables(FbankTables *t);

// -------------------------------------------------------------- nnet ops --

// Post-ops fused into a GEMM epilogue (applied in order, up to 4).
enum PostOp : int { kPostNone = 0, kPostRelu = 1, kPostBatchNorm = 2 };

// The chains nnet programs produce, as one uniform mode per launch so an
// epilogue is straight-line code (a runtime loop over the chain per element
// is a scalar branch ladder per stored value).  kPostModeGeneric keeps the
// loop for anything else.
enum PostMode : int {
  kPostModeNone = 0, kPostModeRelu = 1, kPostModeBn = 2, kPostModeReluBn = 3, kPostModeBnRelu = 4,
  kPostModeGeneric = 5
};
inline int post_mode(const int *post, int npost) {
  if (npost == 0) return kPostModeNone;
  if (npost == 1) return post[0] == kPostRelu ? kPostModeRelu : post[0] == kPostBatchNorm ? kPostModeBn : kPostModeGeneric;
  if (npost == 2 && post[0] == kPostRelu && post[1] == kPostBatchNorm) return kPostModeReluBn;
  if (npost == 2 && post[0] == kPostBatchNorm && post[1] == kPostRelu) return kPostModeBnRelu;
  return kPostModeGeneric;
}

// y after the post chain in the reference's rounding order (ReLU as
// y < 0 ? 0 : y, which keeps NaN; BatchNorm as a rounded product then a
// rounded sum, matrix.cc / nnet.cc).
template <int MODE>
__device__ __forceinline__ float apply_post(float y, float sc, float of, const int *post, int npost) {
  auto relu = [](float v) { return v < 0.0f ? 0.0f : v; };
  auto bn = [&](float v) {
    v = v * sc;
    return v + of;
  };
  if (MODE == kPostModeRelu) return relu(y);
  if (MODE == kPostModeBn) return bn(y);
  if (MODE == kPostModeReluBn) return bn(relu(y));
  if (MODE == kPostModeBnRelu) return relu(bn(y));
  if (MODE == kPostModeGeneric) {
    // static indices (unrolled to the 4-op maximum): a runtime index into the
    // kernel argument's array would force the whole argument struct into
    // scratch memory
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < npost) y = post[q] == kPostRelu ? relu(y) : post[q] == kPostBatchNorm ? bn(y) : y;
  }
  return y;
}

// Cross-lane hand-off through LDS inside one wave (the fbank transposes, the
// int8 epilogue's row slabs): lanes read what other lanes of the same wave
// wrote just before, or overwrite what they just read.  The wave waits for
// all of its LDS operations to complete (lgkmcnt(0)) before it issues the
// next one; the "memory" clobber keeps the compiler from moving LDS accesses
// across.  The rounds 1-4 form (a wavefront-scope fence plus wave_barrier)
// emits no wait and relies on a wave's LDS operations taking effect in issue
// order.  It was suspected for round 4's fast-fbank differences, but the
// stress test cleared it (the cause was packed-FP32 VALU);
// the explicit wait is kept because it costs nothing measurable (C2 exact
// 1.66 -> 1.68 G frames/s, tools/experiments/gpu_r5a.sh) and does not depend
// on that ordering.
__device__ __forceinline__ void wave_lds_sync() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#endif
}

// The latency GEMM's split-K reduce (kernels/gemm_bf16x6_lat.hip): the S
// slice partials of 4 consecutive outputs (slice s at src + s * stride) summed
// in slice order, 16 loads in flight at a time.
__device__ __forceinline__ float4 lat_slice_sum(const float *src, size_t stride, int slices) {
  float4 sum = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  for (int s0 = 0; s0 < slices; s0 += 16) {
    float4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (s0 + u < slices) v[u] = *reinterpret_cast<const float4 *>(src + (size_t)(s0 + u) * stride);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (s0 + u < slices)
        sum = s0 + u == 0 ? v[u] : make_float4(sum.x + v[u].x, sum.y + v[u].y, sum.z + v[u].z, sum.w + v[u].w);
  }
  return sum;
}

// Calls f(std::integral_constant<int, MODE>) for the runtime mode.
template <class F>
__device__ __forceinline__ void with_post_mode(int mode, F &&f) {
  switch (mode) {
    case kPostModeNone: f(std::integral_constant<int, kPostModeNone>()); break;
    case kPostModeRelu: f(std::integral_constant<int, kPostModeRelu>()); break;
    case kPostModeBn: f(std::integral_constant<int, kPostModeBn>()); break;
    case kPostModeReluBn: f(std::integral_constant<int, kPostModeReluBn>()); break;
    case kPostModeBnRelu: f(std::integral_constant<int, kPostModeBnRelu>()); break;
    default: f(std::integral_constant<int, kPostModeGeneric>()); break;
  }
}

// The same, returning f's result.
template <class F>
__device__ __forceinline__ auto with_post_mode_r(int mode, F &&f) {
  switch (mode) {
    case kPostModeNone: return f(std::integral_constant<int, kPostModeNone>());
    case kPostModeRelu: return f(std::integral_constant<int, kPostModeRelu>());
    case kPostModeBn: return f(std::integral_constant<int, kPostModeBn>());
    case kPostModeReluBn: return f(std::integral_constant<int, kPostModeReluBn>());
    case kPostModeBnRelu: return f(std::integral_constant<int, kPostModeBnRelu>());
    default: return f(std::integral_constant<int, kPostModeGeneric>());
  }
}

struct GemmLayer {
  int din = 0;            // input row width (one splice segment)
  int nseg = 1;           // splice indices (segments of the K dimension)
  int off[8] = {0};       // row offset of each segment
  int k = 0, kpad = 0, n = 0;
  DevBuf wt;              // n x kpad, K-contiguous (transposed MAT0)
  DevBuf wsplit;          // n x 3*kpad bf16: wt as three planes (bf16x6 GEMM)
  DevBuf wf16;            // n x 2*kpad fp16: wt * 2^w_shift as two planes (f16x3 GEMM)
  DevBuf wdir;            // wt's planes in MFMA A-fragment order (X6Gemm::wd), units padded to 256
  int w_shift = 0;
  DevBuf bias;            // n
  DevBuf bn_scale, bn_offset;  // n, when a BatchNorm is fused
  int post[4] = {0, 0, 0, 0};
  int npost = 0;
  // rows of the block entering this layer's Splice that the reference chain
  // still holds: the Narrows before it dropped in_left / in_right rows
  int in_left = 0, in_right = 0;
};

// Same numbering as the ABI's CE_GPU_ROW_* (checked in capi.cc).
// int8 form of one Linear layer (kernels/nnet_i8.hip), built by
// ce_gpu_model_quantize.  The A operand is the quantized layer input: either
// read through the splice offsets (segment width a_din a multiple of the
// 64-byte K-tile) or, when `spliced`, written already spliced by the
// quantize pass (a_nseg = 1, a_din = kpad).
struct I8Layer {
  DevBuf wq;                   // n x kpad, (u8 - 128), zero padded
  DevBuf colsum;               // n int32: sums of the shifted weight bytes
  int n = 0, k = 0, kpad = 0;
  float w_scale = 0.0f;
  int32_t w_zp = 0;
  bool spliced = false;
  int in_width = 0;            // width of the float layer input
  int a_din = 0, a_nseg = 1;
  int a_off[8] = {0};
  int in_left = 0, in_right = 0;  // see GemmLayer
  const float *bias = nullptr, *bn_scale = nullptr, *bn_offset = nullptr;
  int post[4] = {0, 0, 0, 0};
  int npost = 0;
};

enum RowOpKind : int { kRowRelu, kRowBatchNorm, kRowLogSoftmax, kRowSoftmax, kRowNormalize };

struct RowOp {
  int kind = 0;
  int dim = 0;
  DevBuf scale, offset;  // BatchNorm
};

// One executable step of the nnet program.
struct Step {
  bool is_gemm = true;
  GemmLayer gemm;
  I8Layer i8;  // filled by ce_gpu_model_quantize
  RowOp row;
};

// One bf16x6 GEMM launch (kernels/gemm_bf16x6*.hip).
struct X6Gemm {
  const uint16_t *x = nullptr;
  int ldx = 0, px = 0;
  const uint16_t *w = nullptr;
  int ldw = 0, pw = 0;
  // fp32 operands instead (xf rows x ldx floats, wf n x ldw floats, both
  // K-contiguous): split into the three planes on the way into LDS; the
  // output is then fp32 (y32) for every layer
  const float *xf = nullptr, *wf = nullptr;
  // the same weights as MFMA A fragments (gemm_bf16x6d_kernel, the default
  // with fp32 activations): for 16-unit block u, K-tile t (32 k) and plane p
  // the 1 KB at ((u * wd_kt + t) * 3 + p) * 512 elements holds lane l's 8
  // bf16 (unit 16 u + (l & 15), k = 32 t + 8 (l >> 4) ..+7) at 8 l; units
  // zero-padded to a multiple of kX6DirUnits
  const uint16_t *wd = nullptr;
  int wd_kt = 0;
  int m = 0, n = 0, kpad = 0, din = 0, nseg = 1;
  int off[8] = {0};
  // latency kernel only: input row r of segment s is xf row
  // row_map[clamp(r + off[s])] (the first layer reading the caller's rows)
  const int *row_map = nullptr;
  const float *bias = nullptr, *bn_scale = nullptr, *bn_offset = nullptr;
  int post[4] = {0, 0, 0, 0};
  int npost = 0;
  float *y32 = nullptr;
  uint16_t *y16 = nullptr;
  int ldy = 0, py = 0;
  // latency kernel: leave the last layer's slice reduce to
  // launch_lat_finalize (described in *tail) when it can run there
  struct LatTail *tail = nullptr;
  // ce_gpu_ctx_set_wide_tiles: the direct-weight kernel on 128 x 128 tiles
  // for every layer (twice the blocks of the 256 x 128 default)
  bool wide = false;
};

// The last layer's slice partials when its reduce runs inside the finalize
// (latency mode): out(f, c) = post(((p0 + p1) + ..) + bias), rows f of
// part[s * m + f][n].
struct LatTail {
  bool active = false;
  const float *part = nullptr;
  int slices = 0, m = 0, n = 0;
  const float *bias = nullptr, *bn_scale = nullptr, *bn_offset = nullptr;
  int post[4] = {0, 0, 0, 0};
  int npost = 0;
};

}  // namespace catears

// ------------------------------------------------------------ ABI objects --

struct ce_gpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  catears::FbankTables host_tables;
  catears::DevBuf d_tables;    // FbankTables image on device
  catears::DevBuf workspace;   // nnet activations (grown on demand)
  size_t workspace_floats = 0;
  catears::DevBuf scratch;     // reductions / int8 operand staging (grown on demand)
  catears::DevBuf blk_maps;    // ce_gpu_nnet_propagate_blocks: row_dst + row_edge
  catears::DevBuf overflow;    // int: an f16x3 split left the fp16 range (ce_gpu_ctx_overflow)
  catears::DevBuf lat_part;    // latency GEMM: slice partials (grown on demand)
  catears::DevBuf lat_tickets; // latency GEMM fix-up: kX6LatTickets words, zero between launches
  int latency = 0;             // ce_gpu_ctx_set_latency: split-K GEMMs for small batches
  int wide_tiles = 0;          // ce_gpu_ctx_set_wide_tiles: 128 x 128 bf16x6 tiles (all CUs per launch)
  int fbank_mode = 0;          // ce_gpu_ctx_set_fbank: CE_GPU_FBANK_EXACT / _FAST
  std::vector<int32_t> h_blk_maps;
  // optional per-class launch timing (ce_gpu_ctx_profile)
  bool profiling = false;
  unsigned prof_mask = ~0u;  // classes timed while profiling (ce_gpu_ctx_profile_classes)
  struct Timed {
    int cls;
    hipEvent_t a, b;
    bool own_a;  // false: a is the previous launch's b (chained, see ProfChain)
  };
  // consecutive launches of one class inside a ProfChain share the boundary
  // event: the previous launch's end is this launch's start
  bool chain_open = false;
  int chain_cls = -1;
  hipEvent_t chain_end = nullptr;
  std::vector<Timed> timed;
  std::vector<hipEvent_t> event_pool;
};

namespace catears {
// Brackets one launch with events when ctx->profiling is set (and the
// class is in ctx->prof_mask).
struct ProfScope {
  ce_gpu_ctx *ctx;
  int cls;
  hipEvent_t b = nullptr;
  ProfScope(ce_gpu_ctx *c, int k);
  ~ProfScope();
};
// Within its scope, back-to-back launches of one class on the context's
// stream (nothing else enqueued between them) are timed with one event per
// launch instead of two: fewer event records in the timed region.
struct ProfChain {
  ce_gpu_ctx *ctx;
  explicit ProfChain(ce_gpu_ctx *c) : ctx(c) {
    ctx->chain_open = true;
    ctx->chain_end = nullptr;
  }
  ~ProfChain() {
    ctx->chain_open = false;
    ctx->chain_end = nullptr;
  }
};
}  // namespace catears

struct ce_gpu_model {
  int left = 0, right = 0, chunk = 0;  // context the caller pads with (config)
  int net_left = 0, net_right = 0;     // rows the Narrow layers drop
  int input_dim = 0, num_pdfs = 0, num_linear = 0, max_width = 0;
  int64_t num_params = 0;
  bool final_log_softmax = false;
  bool int8 = false;                 // Linear layers run as Quantize + u8 GEMM
  int gemm = 0;                      // CE_GPU_GEMM_* for the fp32 program
  bool x6_ok = false;                // program shape the bf16x6 / f16x3 paths take
  bool x3_ok = false;                // ... and every weight fits the f16x3 planes
  std::vector<catears::Step> steps;  // all but the final log-softmax
  catears::DevBuf log_prior;         // num_pdfs
  std::vector<int32_t> tid2pdf;
};

struct ce_gpu_plan {
  int n_utt = 0;
  int64_t total_samples = 0, total_frames = 0;
  std::vector<int64_t> sample_off, frame_off;  // n_utt + 1 each (host)
  // fbank launch map: per block of kFramesPerBlock frames, first utterance
  catears::DevBuf d_sample_off, d_frame_off, d_block_utt;
  int fbank_blocks = 0;
  // nnet chunks
  struct Chunk {
    int rows = 0;          // packed rows (<= max_rows)
    int64_t map_base = 0;  // offset into d_row_src / d_row_dst
  };
  std::vector<Chunk> chunks;
  catears::DevBuf d_row_src;  // int32 per packed row: source feature row
  catears::DevBuf d_row_dst;  // int32 per packed row: output row or -1
  catears::DevBuf d_row_edge; // uint32 per packed row: rows to its segment's start | end << 16
  int max_chunk_rows = 0;
  int left = 0, right = 0;
  bool has_model = false;
};

namespace catears {

// Kernel launchers (kernels/*.hip).  All enqueue on `s` and return a status.
int launch_fbank(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const float *pcm,
                 float *feats, float *mel);
int launch_fbank_s16(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const int16_t *pcm,
                     float *feats, float *mel);
// fast mode (ce_gpu_ctx_set_fbank(ctx, CE_GPU_FBANK_FAST))
// the fast mode: fbank.hip's lane program with FMA contraction (fbank_fma.hip)
#ifdef CATEARS_EXPERIMENTS  // kernels/fbank_nocase.hip: timing only
int launch_fbank_nocase(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const float *pcm, float *feats,
                        float *mel);
int launch_fbank_nocase_s16(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const int16_t *pcm,
                            float *feats, float *mel);
#endif
int launch_fbank_fma(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const float *pcm, float *feats,
                     float *mel);
int launch_fbank_fma_s16(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const int16_t *pcm,
                         float *feats, float *mel);
int launch_cmvn(hipStream_t s, const ce_gpu_plan *p, const float *gstats, const float *in,
                float *out);

struct GemmArgs {
  const float *x = nullptr;   // A source rows
  int ldx = 0;
  const int *row_map = nullptr;  // optional: packed row -> source row of x
  int m = 0, n = 0, k = 0, kpad = 0;
  int din = 0, nseg = 1;
  int off[8] = {0};
  const float *w = nullptr;   // B: n x kpad (K-major) or k x ldw (N-major)
  int ldw = 0;
  bool b_nmajor = false;
  const float *bias = nullptr, *bn_scale = nullptr, *bn_offset = nullptr;
  int post[4] = {0, 0, 0, 0};
  int npost = 0;
  float *y = nullptr;
  int ldy = 0;
};
int launch_gemm_f32(hipStream_t s, const GemmArgs &a);
// Weights' K dimension is zero-padded to a multiple of this (every tile variant's BK).
int gemm_k_align();

// fp32-accurate GEMM on the bf16 matrix cores (kernels/gemm_bf16x6.hip):
// operands as three bf16 planes, six MFMA products.  x: rows x ldx, plane
// stride px, read through the splice offsets (K-tile of 32 inside one
// segment); w: n x ldw, plane stride pw (zero padded to kpad); output split
// (y16, plane stride py) or fp32 (y32).
int launch_gemm_bf16x6(hipStream_t s, const X6Gemm &a);
constexpr int kX6DirUnits = 256;  // gemm_bf16x6d_kernel's unit tile
// Latency mode (kernels/gemm_bf16x6_lat.hip): K split into
// x6_lat_slices(kpad, n) slices (a function of K and N only), every slice's
// fp32 partial stored, then summed in slice order by a reduce kernel that
// applies bias / ReLU / BatchNorm; needs the weight fragment image (a.wd) and
// fp32 activations (din a multiple of 8: a segment may end inside a K-tile).
// part: x6_lat_part_floats(rows, n, slices) floats.  With a.tail set and the
// rows within one window (rows <= kX6LatWindow, n % 4 == 0, n <= 4096) the
// reduce is left to launch_lat_finalize (a.tail->active).
constexpr int kX6LatWindow = 1024;
int x6_lat_slices(int kpad, int n);
size_t x6_lat_part_floats(int rows, int n, int slices);
// tickets: kX6LatTickets zeroed words for the split-K fix-up (may be null)
constexpr int kX6LatTickets = 1024;
int launch_gemm_bf16x6_lat(hipStream_t s, const X6Gemm &a, float *part, size_t part_floats,
                           unsigned *tickets = nullptr);
// The last layer's slice reduce fused with the finalize: rows first ..
// first + rows - 1 of a deferred tail summed, + bias, post chain, then
// (log-softmax) - prior into out (row_dst as launch_finalize) -- the bits of
// the reduce launch followed by launch_finalize.
int launch_lat_finalize(hipStream_t s, const LatTail &t, int first, int rows, bool log_softmax,
                        const float *log_prior, const int *row_dst, float *out);
// splice_pad (below) written as three bf16 planes of width po: out row r at
// out + r * 3 * po.
int launch_splice_pad_split(hipStream_t s, const float *in, int ld_in, int rows, int din, int nseg, const int *off,
                            const int *row_map, uint16_t *out, int po);

// fp32-accurate GEMM on the fp16 matrix cores (kernels/gemm_f16x3.hip):
// operands as two scaled fp16 planes, three MFMA products; same geometry as
// X6Gemm with two planes.  unscale = 2^-(weight shift + activation shift);
// overflow: device word set when a split output leaves the fp16 range.
struct X3Gemm {
  const uint16_t *x = nullptr;
  int ldx = 0, px = 0;
  const uint16_t *w = nullptr;
  int ldw = 0, pw = 0;
  int m = 0, n = 0, kpad = 0, din = 0, nseg = 1;
  int off[8] = {0};
  float unscale = 1.0f;
  const float *bias = nullptr, *bn_scale = nullptr, *bn_offset = nullptr;
  int post[4] = {0, 0, 0, 0};
  int npost = 0;
  float *y32 = nullptr;
  uint16_t *y16 = nullptr;
  int ldy = 0, py = 0;
  int *overflow = nullptr;
};
int launch_gemm_f16x3(hipStream_t s, const X3Gemm &a);
int launch_splice_pad_f16(hipStream_t s, const float *in, int ld_in, int rows, int din, int nseg, const int *off,
                          const int *row_map, uint16_t *out, int po, int *overflow);
// activations enter the f16x3 GEMM as x * 2^kF16ActShift
constexpr int kF16ActShift = -8;
// ce_gpu_nnet_propagate runs longer fp32 blocks as overlapping windows of
// this many input rows (bit-identical; bounds 32-bit offsets and workspace)
constexpr int kPropagateWindow = 1 << 16;

// Final step: optional log-softmax per row, minus log prior, scatter to the
// output rows named by row_dst (-1 = drop).
int launch_finalize(hipStream_t s, const float *x, int ldx, int rows, int dim, bool log_softmax,
                    const float *log_prior, const int *row_dst, float *out);
int launch_rowop(hipStream_t s, const RowOp &op, float *x, int ldx, int rows);
int launch_trace_mark(hipStream_t s, int tag);
int launch_loglik_gather(hipStream_t s, const float *ll, int rows, int ld, int dim, const int32_t *tpm, int n_tid,
                         const int32_t *row, const int32_t *trans, int n, float scale, float *out);
int launch_loglik_columns(hipStream_t s, const float *ll, int rows, int ld, int dim, const int32_t *cols,
                          int n_cols, float *out);
int launch_sum_f64(hipStream_t s, int count, const float *const *x, const int64_t *n, double *part, double *acc);
int launch_rowop_raw(hipStream_t s, int kind, int dim, const float *scale, const float *offset, float *x,
                     int ldx, int rows);
int launch_splice(hipStream_t s, int rows, int dim, const float *in, int ld_in, const int32_t *h_idx,
                  int n_idx, float *out);
// out[r][s*din + c] = in[row_map(clamp(r + off[s]))][c], zero for columns
// nseg*din .. ldo-1 (the fused program's first-layer block).
int launch_splice_pad(hipStream_t s, const float *in, int ld_in, int rows, int din, int nseg, const int *off,
                      const int *row_map, float *out, int ldo);

int launch_quantize(hipStream_t s, const float *x, int64_t count, uint8_t *q, void *params,
                    void *scratch);
size_t gemm_u8_scratch_bytes(int m, int n, int k);
// int8 nnet path (kernels/nnet_i8.hip)
// min / max over the rows the reference chain holds: row r counts when its
// distances to its segment's edges (row_edge, or r / rows-1-r for one
// segment) are >= in_left / in_right.
int launch_i8_params(hipStream_t s, const float *x, int ldx, int rows, int width, const int *row_map,
                     const uint32_t *row_edge, int in_left, int in_right, void *part, void *params);
size_t i8_params_scratch_bytes();
int launch_i8_quantize(hipStream_t s, const float *x, int ldx, int rows, int width, const int *row_map, int nseg,
                       const int *offs, const void *params, int8_t *q, int ldq, int32_t *rowsum);
// The next layer's min / max, fused into this GEMM's epilogue: one float2
// per wave into `part` (at least i8_gemm_parts(m, n)), over the rows the
// next layer holds (as launch_i8_params); launch_i8_params_fold then forms
// that layer's parameters from the *nparts partials.
struct I8NextMinMax {
  void *part;
  const uint32_t *row_edge;
  int in_left, in_right;
};
int launch_i8_gemm(hipStream_t s, const I8Layer &L, const int8_t *a, int lda, int m, const int32_t *rowsum,
                   const void *pa, float *y, int ldy, const I8NextMinMax *mm = nullptr, int *nparts = nullptr);
int launch_i8_params_fold(hipStream_t s, const void *part, int nparts, void *params);
size_t i8_gemm_parts(int m, int n);
int i8_k_align();
int launch_gemm_u8_ws(hipStream_t s, int m, int n, int k, const uint8_t *a, const void *pa,
                      const uint8_t *b, const void *pb, float *c_f32, int32_t *c_i32, void *ws);

}  // namespace catears
