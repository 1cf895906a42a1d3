// capi.cc -- extern "C" entry points of libcatears_hip (include/catears_gpu.h):
// errors, contexts, model loading (NN02 / MAT0 / VEC0 / key=value config),
// batch planning, and the host-side sequencing of the kernels.
#include <float.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cctype>
#include <fstream>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "internal.h"
#include "model_io.h"

namespace catears {

// ---------------------------------------------------------------- errors --

int hip_fail(hipError_t e, const char *what) {
  return fail(CE_GPU_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------- DevBuf --

int DevBuf::alloc(size_t n) {
  release();
  if (n == 0) return CE_GPU_OK;
  hipError_t e = hipMalloc(&ptr, n);
  if (e != hipSuccess) {
    ptr = nullptr;
    (void)hipGetLastError();
    return fail(CE_GPU_ENOMEM, fmt("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e)));
  }
  bytes = n;
  return CE_GPU_OK;
}

int DevBuf::upload(const void *src, size_t n) {
  CE_TRY(alloc(n));
  if (n) CE_HIP(hipMemcpy(ptr, src, n, hipMemcpyHostToDevice));
  return CE_GPU_OK;
}

void DevBuf::release() {
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  bytes = 0;
}

// Turns the layer list into fused device steps.  The reference's converter
// always emits Splice immediately followed by Narrow(-min(idx,0), max(idx,0))
// (tool/convert_am.py:272-285); under that shape the output of a chunk does
// not depend on where the chunk boundaries are, which is what lets the GPU run
// whole utterances.  Other shapes are rejected with CE_GPU_ENOTSUP.
// fp32 -> bf16, round to nearest even (v_cvt_pk_bf16_f32; NaN stays NaN).
static uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static float bf16_float(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// The bf16x6 GEMM's weight image: row j of the n x kpad matrix as three bf16
// planes [w0 | w1 | w2], w = w0 + w1 + w2 (kernels/gemm_bf16x6.hip).
static int upload_split(const std::vector<float> &wt, int n, int kpad, DevBuf *out) {
  std::vector<uint16_t> sp((size_t)n * 3 * kpad);
  for (int j = 0; j < n; ++j)
    for (int k = 0; k < kpad; ++k) {
      const float v = wt[(size_t)j * kpad + k];
      const uint16_t h = bf16_rne(v);
      const float r1 = v - bf16_float(h);
      const uint16_t m = bf16_rne(r1);
      const float r2 = r1 - bf16_float(m);
      uint16_t *row = sp.data() + (size_t)j * 3 * kpad;
      row[k] = h;
      row[kpad + k] = m;
      row[2 * kpad + k] = bf16_rne(r2);
    }
  return out->upload(sp.data(), sp.size() * 2);
}

// The direct-weight kernel's image (X6Gemm::wd): the same three planes in
// MFMA A-fragment order, units zero-padded to a multiple of kX6DirUnits.
static int upload_wdir(const std::vector<float> &wt, int n, int kpad, DevBuf *out) {
  const int npad = (n + kX6DirUnits - 1) / kX6DirUnits * kX6DirUnits, kt = kpad / 32;
  std::vector<uint16_t> img((size_t)npad * 3 * kpad, 0);
  for (int ub = 0; ub < npad / 16; ++ub)
    for (int t = 0; t < kt; ++t)
      for (int l = 0; l < 64; ++l) {
        const int j = ub * 16 + (l & 15), k0 = t * 32 + (l >> 4) * 8;
        if (j >= n) continue;
        for (int e = 0; e < 8; ++e) {
          const float v = wt[(size_t)j * kpad + k0 + e];
          const uint16_t h = bf16_rne(v);
          const float r1 = v - bf16_float(h);
          const uint16_t m = bf16_rne(r1);
          const uint16_t lo = bf16_rne(r1 - bf16_float(m));
          const size_t base = (((size_t)ub * kt + t) * 3) * 512 + (size_t)l * 8 + e;
          img[base] = h;
          img[base + 512] = m;
          img[base + 1024] = lo;
        }
      }
  return out->upload(img.data(), img.size() * 2);
}

// fp32 -> fp16 bits, round to nearest even (v_cvt_f16_f32), inf beyond 65504.
static uint16_t f16_rne(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
  const uint32_t a = x & 0x7fffffffu;
  if (a >= 0x7f800000u) return sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u);
  if (a >= 0x477ff000u) return sign | 0x7c00u;  // >= 65520 rounds to infinity
  if (a < 0x38800000u) {                          // below 2^-14: subnormal
    float v;
    memcpy(&v, &a, 4);
    return sign | (uint16_t)nearbyintf(v * 16777216.0f);  // units of 2^-24
  }
  const uint32_t r = a - 0x38000000u;  // rebias 127 -> 15
  return sign | (uint16_t)((r + 0xfffu + ((r >> 13) & 1u)) >> 13);
}
static float f16_float(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 31u, m = h & 0x3ffu;
  float v;
  if (e == 0) {
    v = ldexpf((float)m, -24);
  } else if (e == 31) {
    const uint32_t u = 0x7f800000u | (m << 13);
    memcpy(&v, &u, 4);
  } else {
    const uint32_t u = ((e + 112u) << 23) | (m << 13);
    memcpy(&v, &u, 4);
  }
  uint32_t u;
  memcpy(&u, &v, 4);
  u |= sign;
  memcpy(&v, &u, 4);
  return v;
}

// The f16x3 GEMM's weight image (kernels/gemm_f16x3.hip): u = w * 2^shift
// with max |u| in [2^14, 2^15), row j = [f16(u) | f16((u - f16(u)) * 2^11)].
// Returns false (image not built) when the weights are not all finite.
static int upload_f16(const std::vector<float> &wt, int n, int kpad, DevBuf *out, int *shift, bool *ok) {
  float mx = 0.0f;
  for (float v : wt) {
    if (!std::isfinite(v)) {
      *ok = false;
      return CE_GPU_OK;
    }
    mx = std::max(mx, std::fabs(v));
  }
  int e = 0;
  if (mx > 0.0f) frexpf(mx, &e);  // mx in [2^(e-1), 2^e)
  *shift = std::max(-100, std::min(100, 15 - e));
  std::vector<uint16_t> sp((size_t)n * 2 * kpad);
  for (int j = 0; j < n; ++j)
    for (int k = 0; k < kpad; ++k) {
      const float u = ldexpf(wt[(size_t)j * kpad + k], *shift);
      const uint16_t h = f16_rne(u);
      uint16_t *row = sp.data() + (size_t)j * 2 * kpad;
      row[k] = h;
      row[kpad + k] = f16_rne((u - f16_float(h)) * 2048.0f);
    }
  *ok = true;
  return out->upload(sp.data(), sp.size() * 2);
}

#ifdef CATEARS_DIAG
int knob_env(const char *name, int dflt) {
  const char *e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}
#endif

// Default matrix-core form of the fp32 program: bf16x6.  Another mode is a
// per-model choice through ce_gpu_model_set_gemm; the experiments library
// also takes CATEARS_NNET_GEMM (0 fp32, 1 bf16x6, 2 f16x3, 3 bf16x6p, the
// ce_gpu_model_set_gemm numbers) for the tools.
static int default_gemm() {
  static const int g = CE_KNOB("CATEARS_NNET_GEMM", (int)CE_GPU_GEMM_BF16X6);
  return g >= CE_GPU_GEMM_FP32 && g <= CE_GPU_GEMM_BF16X6_PLANES ? g : -1;
}

static int build_program(const std::vector<RawLayer> &layers, int left, int right, ce_gpu_model *m) {
  m->x3_ok = true;           // cleared by a weight matrix the f16 planes cannot hold
  std::vector<int> pending;  // splice offsets waiting for their Linear
  bool have_pending = false, gemm_open = false;
  int width = -1, sum_l = 0, sum_r = 0, pend_l = 0, pend_r = 0;
  for (size_t i = 0; i < layers.size(); ++i) {
    const RawLayer &L = layers[i];
    switch (L.id) {
      case kSplice: {
        if (have_pending) return fail(CE_GPU_ENOTSUP, "two Splice layers without a Linear between them");
        if (L.idx.empty() || L.idx.size() > 8) return fail(CE_GPU_ENOTSUP, "Splice needs 1..8 indices");
        int lo = 0, hi = 0;
        for (int v : L.idx) lo = std::min(lo, v), hi = std::max(hi, v);
        if (i + 1 >= layers.size() || layers[i + 1].id != kNarrow || layers[i + 1].left != -lo ||
            layers[i + 1].right != hi)
          return fail(CE_GPU_ENOTSUP, "Splice must be followed by Narrow(-min(idx,0), max(idx,0))");
        pending.assign(L.idx.begin(), L.idx.end());
        have_pending = true;
        pend_l = -lo;
        pend_r = hi;
        gemm_open = false;
        ++i;  // the Narrow
        sum_l += -lo;
        sum_r += hi;
        if (!(i + 1 < layers.size() && layers[i + 1].id == kLinear))
          return fail(CE_GPU_ENOTSUP, "Splice/Narrow must feed a Linear layer");
        break;
      }
      case kNarrow:
        if (L.left != 0 || L.right != 0) return fail(CE_GPU_ENOTSUP, "Narrow without a preceding Splice");
        break;
      case kLinear: {
        Step st;
        GemmLayer &g = st.gemm;
        const int in = L.rows, out = L.cols;
        if ((int)L.b.size() != out)
          return fail(CE_GPU_ECORRUPT, "Corruption: Linear bias size does not match W");
        g.nseg = have_pending ? (int)pending.size() : 1;
        g.in_left = sum_l - (have_pending ? pend_l : 0);
        g.in_right = sum_r - (have_pending ? pend_r : 0);
        if (in % g.nseg != 0) return fail(CE_GPU_ECORRUPT, "Corruption: Linear input does not match Splice");
        g.din = in / g.nseg;
        for (int s = 0; s < g.nseg; ++s) g.off[s] = have_pending ? pending[s] : 0;
        if (width >= 0 && g.din != width)
          return fail(CE_GPU_ECORRUPT, fmt("Corruption: layer %zu expects width %d, got %d", i, g.din, width));
        if (m->steps.empty()) m->input_dim = g.din;
        g.k = in;
        g.kpad = (in + gemm_k_align() - 1) / gemm_k_align() * gemm_k_align();
        g.n = out;
        std::vector<float> wt((size_t)out * g.kpad, 0.0f);  // transpose to n x kpad
        for (int k = 0; k < in; ++k)
          for (int j = 0; j < out; ++j) wt[(size_t)j * g.kpad + k] = L.w[(size_t)k * out + j];
        CE_TRY(g.wt.upload(wt.data(), wt.size() * 4));
        CE_TRY(upload_split(wt, out, g.kpad, &g.wsplit));
        if (g.kpad % 32 == 0) CE_TRY(upload_wdir(wt, out, g.kpad, &g.wdir));
        bool f16_ok = false;
        CE_TRY(upload_f16(wt, out, g.kpad, &g.wf16, &g.w_shift, &f16_ok));
        if (!f16_ok) m->x3_ok = false;
        CE_TRY(g.bias.upload(L.b.data(), L.b.size() * 4));
        m->num_params += (int64_t)in * out + out;
        m->max_width = std::max(m->max_width, out);
        ++m->num_linear;
        m->steps.push_back(std::move(st));
        have_pending = false;
        gemm_open = true;
        width = out;
        break;
      }
      case kReLU:
      case kBatchNorm: {
        if (width < 0) return fail(CE_GPU_ENOTSUP, "the first layer must be a (spliced) Linear");
        if (L.id == kBatchNorm && ((int)L.scale.size() != width || (int)L.offset.size() != width))
          return fail(CE_GPU_ECORRUPT, "Corruption: BatchNorm size does not match its input");
        GemmLayer &g = m->steps.back().gemm;
        const bool bn_free = L.id != kBatchNorm || !g.bn_scale.ptr;
        if (gemm_open && m->steps.back().is_gemm && g.npost < 4 && bn_free) {
          g.post[g.npost++] = L.id == kReLU ? kPostRelu : kPostBatchNorm;
          if (L.id == kBatchNorm) {
            CE_TRY(g.bn_scale.upload(L.scale.data(), width * 4));
            CE_TRY(g.bn_offset.upload(L.offset.data(), width * 4));
            m->num_params += 2 * width;
          }
        } else {
          Step st;
          st.is_gemm = false;
          st.row.kind = L.id == kReLU ? kRowRelu : kRowBatchNorm;
          st.row.dim = width;
          if (L.id == kBatchNorm) {
            CE_TRY(st.row.scale.upload(L.scale.data(), width * 4));
            CE_TRY(st.row.offset.upload(L.offset.data(), width * 4));
          }
          m->steps.push_back(std::move(st));
          gemm_open = false;
        }
        break;
      }
      case kLogSoftmax:
      case kSoftmax:
      case kNormalize: {
        if (width < 0) return fail(CE_GPU_ENOTSUP, "the first layer must be a (spliced) Linear");
        if (L.id == kLogSoftmax && i + 1 == layers.size()) {
          m->final_log_softmax = true;
        } else {
          Step st;
          st.is_gemm = false;
          st.row.kind = L.id == kLogSoftmax ? kRowLogSoftmax : (L.id == kSoftmax ? kRowSoftmax : kRowNormalize);
          st.row.dim = width;
          m->steps.push_back(std::move(st));
        }
        gemm_open = false;
        break;
      }
      default:
        return fail(CE_GPU_ECORRUPT, "Corruption: unexpected layer");
    }
  }
  if (m->steps.empty() || !m->steps.front().is_gemm)
    return fail(CE_GPU_ENOTSUP, "the nnet must start with a (spliced) Linear layer");
  m->net_left = sum_l;
  m->net_right = sum_r;
  if (left < 0 && right < 0) {
    m->left = sum_l;
    m->right = sum_r;
  } else if (sum_l != left || sum_r != right)
    return fail(CE_GPU_ECORRUPT, fmt("Corruption: config context (%d, %d) differs from the nnet's (%d, %d)",
                                     left, right, sum_l, sum_r));
  m->num_pdfs = width;
  // bf16x6 program: every step a Linear with its ReLU / BatchNorm fused, a
  // K-tile of 32 inside one splice segment after the first layer (whose
  // spliced block is written padded), output widths multiples of 4
  m->x6_ok = true;
  for (size_t i = 0; i < m->steps.size(); ++i) {
    const Step &st = m->steps[i];
    if (!st.is_gemm || st.gemm.n % 4 != 0 || (i > 0 && st.gemm.din % 32 != 0) || st.gemm.kpad % 32 != 0)
      m->x6_ok = false;
  }
  m->x3_ok = m->x3_ok && m->x6_ok;
  const int want = default_gemm();
  if (want < 0) return fail(CE_GPU_EINVAL, "default GEMM mode: not one of 0 fp32, 1 bf16x6, 2 f16x3, 3 bf16x6p");
  m->gemm = want == CE_GPU_GEMM_F16X3 && m->x3_ok   ? CE_GPU_GEMM_F16X3
            : want == CE_GPU_GEMM_BF16X6_PLANES && m->x6_ok ? CE_GPU_GEMM_BF16X6_PLANES
            : want != CE_GPU_GEMM_FP32 && m->x6_ok ? CE_GPU_GEMM_BF16X6
                                                    : CE_GPU_GEMM_FP32;
  return CE_GPU_OK;
}

// Nnet::Read into a device program; `rd` is positioned at the NN02 tag.
// left/right < 0: take the context from the network's Narrow layers.
static int read_program(ce_gpu_ctx *ctx, Reader &rd, int left, int right, ce_gpu_model *m) {
  CE_HIP(hipSetDevice(ctx->device));
  if ((left < 0) != (right < 0)) return fail(CE_GPU_EINVAL, "negative context");
  m->left = left;
  m->right = right;
  std::vector<RawLayer> layers;
  int hl = 0, hr = 0;
  CE_TRY(read_nnet(rd, &layers, &hl, &hr));
  return build_program(layers, left, right, m);
}

// Prior probabilities -> device log prior (ApplyLog, src/am.cc:40-44).
static int set_prior(ce_gpu_model *m, const float *prior, int dim) {
  if (dim != m->num_pdfs)
    return fail(CE_GPU_ECORRUPT, fmt("Corruption: prior has %d entries, nnet outputs %d", dim, m->num_pdfs));
  std::vector<float> lp(prior, prior + dim);
  for (float &v : lp) v = logf(v);
  return m->log_prior.upload(lp.data(), lp.size() * 4);
}

static int load_model(ce_gpu_ctx *ctx, const std::string &nnet, const std::string &prior, int left,
                      int right, const std::string &tid2pdf, ce_gpu_model **out) {
  std::unique_ptr<ce_gpu_model> m(new (std::nothrow) ce_gpu_model());
  if (!m) return fail(CE_GPU_ENOMEM, "out of host memory");
  if (left < 0 || right < 0) return fail(CE_GPU_EINVAL, "negative context");
  {
    Reader rd;
    CE_TRY(rd.open(nnet));
    CE_TRY(read_program(ctx, rd, left, right, m.get()));
  }
  Reader rp;
  CE_TRY(rp.open(prior));
  std::vector<float> pr;
  CE_TRY(rp.vec(&pr));
  CE_TRY(set_prior(m.get(), pr.data(), (int)pr.size()));
  if (!tid2pdf.empty()) {
    Reader rt;
    CE_TRY(rt.open(tid2pdf));
    CE_TRY(rt.vec(&m->tid2pdf));
  }
  *out = m.release();
  return CE_GPU_OK;
}

// ------------------------------------------------------------ workspace --

static int ensure_workspace(ce_gpu_ctx *ctx, size_t floats) {
  if (ctx->workspace_floats >= floats) return CE_GPU_OK;
  CE_HIP(hipStreamSynchronize(ctx->stream));  // old buffer may still be in use
  CE_TRY(ctx->workspace.alloc(floats * sizeof(float)));
  ctx->workspace_floats = floats;
  return CE_GPU_OK;
}

static int ensure_scratch(ce_gpu_ctx *ctx, size_t bytes) {
  if (ctx->scratch.bytes >= bytes) return CE_GPU_OK;
  CE_HIP(hipStreamSynchronize(ctx->stream));
  return ctx->scratch.alloc(bytes);
}

// the latency GEMM's slice partials (one window of rows)
static int ensure_lat_part(ce_gpu_ctx *ctx, size_t floats) {
#ifdef CATEARS_EXPERIMENTS
  // the split-K fix-up's tickets (CATEARS_LAT_FIXUP, measured slower:
  // DESIGN.md §8 round 6), zeroed once: every fix-up launch leaves them zero
  if (!ctx->lat_tickets.ptr) {
    CE_TRY(ctx->lat_tickets.upload(std::vector<unsigned>(kX6LatTickets, 0u).data(), kX6LatTickets * sizeof(unsigned)));
  }
#endif
  if (ctx->lat_part.bytes >= floats * sizeof(float)) return CE_GPU_OK;
  CE_HIP(hipStreamSynchronize(ctx->stream));
  return ctx->lat_part.alloc(floats * sizeof(float));
}

int fbank_frames_per_block();

static hipEvent_t pool_event(ce_gpu_ctx *ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

ProfScope::ProfScope(ce_gpu_ctx *c, int k) : ctx(c), cls(k) {
  if (!ctx->profiling || !(ctx->prof_mask & (1u << cls))) {
    ctx->chain_end = nullptr;  // an untimed launch breaks a chain
    return;
  }
  hipEvent_t a = nullptr;
  bool own_a = true;
  if (ctx->chain_open && ctx->chain_end && ctx->chain_cls == cls) {
    a = ctx->chain_end;
    own_a = false;
  } else {
    a = pool_event(ctx);
    if (!a) return;
  }
  b = pool_event(ctx);
  if (!b) {
    if (own_a) ctx->event_pool.push_back(a);
    ctx->chain_end = nullptr;
    return;
  }
  if (own_a) (void)hipEventRecord(a, ctx->stream);
  ctx->timed.push_back({cls, a, b, own_a});
}

ProfScope::~ProfScope() {
  if (!b) return;
  (void)hipEventRecord(b, ctx->stream);
  if (ctx->chain_open) {
    ctx->chain_end = b;
    ctx->chain_cls = cls;
  }
}

}  // namespace catears

using namespace catears;

// =================================================================== ABI ==

extern "C" {

const char *ce_gpu_last_error(void) { return last_error(); }

const char *ce_gpu_version(void) { return "catears-mi355x 0.5 (gfx950)"; }

int ce_gpu_ctx_create(int device, void *stream, ce_gpu_ctx **out) {
  if (!out) return fail(CE_GPU_EINVAL, "out is NULL");
  *out = nullptr;
  int n = 0;
  CE_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(CE_GPU_EINVAL, fmt("no HIP device %d (have %d)", device, n));
  CE_HIP(hipSetDevice(device));
  std::unique_ptr<ce_gpu_ctx> c(new (std::nothrow) ce_gpu_ctx());
  if (!c) return fail(CE_GPU_ENOMEM, "out of host memory");
  c->device = device;
  c->stream = static_cast<hipStream_t>(stream);
  build_fbank_tables(&c->host_tables);
  CE_TRY(c->d_tables.upload(&c->host_tables, sizeof(FbankTables)));
  *out = c.release();
  return CE_GPU_OK;
}

int ce_gpu_ctx_destroy(ce_gpu_ctx *ctx) {
  if (!ctx) return CE_GPU_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto &t : ctx->timed) {
    if (t.own_a) (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
  delete ctx;
  return CE_GPU_OK;
}

int ce_gpu_ctx_set_stream(ce_gpu_ctx *ctx, void *stream) {
  if (!ctx) return fail(CE_GPU_EINVAL, "ctx is NULL");
  hipStream_t next = static_cast<hipStream_t>(stream);
  if (next != ctx->stream) {
    // Work already queued on the old stream may still use the context's
    // workspaces; the new stream starts after it (no host wait).
    CE_HIP(hipSetDevice(ctx->device));
    hipEvent_t done;
    CE_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    hipError_t e = hipEventRecord(done, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(next, done, 0);
    (void)hipEventDestroy(done);
    CE_HIP(e);
    ctx->stream = next;
  }
  return CE_GPU_OK;
}

int ce_gpu_ctx_overflow(ce_gpu_ctx *ctx, int *overflow) {
  if (!ctx || !overflow) return fail(CE_GPU_EINVAL, "NULL argument");
  *overflow = 0;
  if (!ctx->overflow.ptr) return CE_GPU_OK;
  CE_HIP(hipSetDevice(ctx->device));
  CE_HIP(hipStreamSynchronize(ctx->stream));
  CE_HIP(hipMemcpy(overflow, ctx->overflow.ptr, sizeof(int), hipMemcpyDeviceToHost));
  CE_HIP(hipMemset(ctx->overflow.ptr, 0, sizeof(int)));
  return CE_GPU_OK;
}

int ce_gpu_ctx_set_latency(ce_gpu_ctx *ctx, int on) {
  if (!ctx) return fail(CE_GPU_EINVAL, "NULL argument");
  ctx->latency = on ? 1 : 0;
  return CE_GPU_OK;
}

int ce_gpu_ctx_set_wide_tiles(ce_gpu_ctx *ctx, int on) {
  if (!ctx) return fail(CE_GPU_EINVAL, "NULL argument");
  ctx->wide_tiles = on ? 1 : 0;
  return CE_GPU_OK;
}

int ce_gpu_ctx_set_fbank(ce_gpu_ctx *ctx, int mode) {
  if (!ctx) return fail(CE_GPU_EINVAL, "NULL argument");
  if (mode != CE_GPU_FBANK_EXACT && mode != CE_GPU_FBANK_FAST) return fail(CE_GPU_EINVAL, "unknown fbank mode");
  ctx->fbank_mode = mode;
  return CE_GPU_OK;
}

int ce_gpu_ctx_synchronize(ce_gpu_ctx *ctx) {
  if (!ctx) return fail(CE_GPU_EINVAL, "ctx is NULL");
  CE_HIP(hipStreamSynchronize(ctx->stream));
  return CE_GPU_OK;
}

int ce_gpu_ctx_profile(ce_gpu_ctx *ctx, int enable) {
  if (!ctx) return fail(CE_GPU_EINVAL, "ctx is NULL");
  ctx->profiling = enable != 0;
  return CE_GPU_OK;
}

int ce_gpu_ctx_profile_classes(ce_gpu_ctx *ctx, unsigned mask) {
  if (!ctx) return fail(CE_GPU_EINVAL, "ctx is NULL");
  ctx->prof_mask = mask;
  return CE_GPU_OK;
}

int ce_gpu_ctx_profile_read(ce_gpu_ctx *ctx, int kernel_class, double *total_ms, int64_t *launches) {
  if (!ctx || kernel_class < 0 || kernel_class >= CE_GPU_PROF_CLASSES) return fail(CE_GPU_EINVAL, "bad argument");
  CE_HIP(hipStreamSynchronize(ctx->stream));
  double ms = 0.0;
  int64_t n = 0;
  std::vector<ce_gpu_ctx::Timed> keep;
  for (const ce_gpu_ctx::Timed &t : ctx->timed) {
    if (t.cls != kernel_class) {
      keep.push_back(t);
      continue;
    }
    float e = 0.0f;
    CE_HIP(hipEventElapsedTime(&e, t.a, t.b));
    ms += e;
    ++n;
    if (t.own_a) ctx->event_pool.push_back(t.a);
    ctx->event_pool.push_back(t.b);
  }
  ctx->timed.swap(keep);
  if (total_ms) *total_ms = ms;
  if (launches) *launches = n;
  return CE_GPU_OK;
}

static hipEvent_t g_anchor[64];

int ce_gpu_profile_anchor(int device, void *stream) {
  if (device < 0 || device >= 64) return fail(CE_GPU_EINVAL, "bad device");
  CE_HIP(hipSetDevice(device));
  if (!g_anchor[device]) CE_HIP(hipEventCreate(&g_anchor[device]));
  CE_HIP(hipEventRecord(g_anchor[device], static_cast<hipStream_t>(stream)));
  return CE_GPU_OK;
}

int ce_gpu_trace_mark(int device, void *stream, int tag) {
  if (device < 0 || device >= 64 || tag < 1 || tag > 64) return fail(CE_GPU_EINVAL, "bad device or tag");
  CE_HIP(hipSetDevice(device));
  return launch_trace_mark(static_cast<hipStream_t>(stream), tag);
}

int ce_gpu_ctx_profile_intervals(ce_gpu_ctx *ctx, int kernel_class, double *h_start_ms, double *h_end_ms,
                                 int capacity, int *count) {
  if (!ctx || !count || kernel_class < 0 || kernel_class >= CE_GPU_PROF_CLASSES)
    return fail(CE_GPU_EINVAL, "bad argument");
  hipEvent_t anchor = ctx->device < 64 ? g_anchor[ctx->device] : nullptr;
  if (!anchor) return fail(CE_GPU_EINVAL, "no anchor recorded (ce_gpu_profile_anchor)");
  CE_HIP(hipStreamSynchronize(ctx->stream));
  CE_HIP(hipEventSynchronize(anchor));
  int n = 0;
  for (const ce_gpu_ctx::Timed &t : ctx->timed) n += t.cls == kernel_class;
  *count = n;
  if (n > capacity || (n > 0 && (!h_start_ms || !h_end_ms)))
    return fail(CE_GPU_EINVAL, fmt("capacity %d < %d launches", capacity, n));
  std::vector<ce_gpu_ctx::Timed> keep;
  int i = 0;
  for (const ce_gpu_ctx::Timed &t : ctx->timed) {
    if (t.cls != kernel_class) {
      keep.push_back(t);
      continue;
    }
    float a = 0.0f, b = 0.0f;
    CE_HIP(hipEventElapsedTime(&a, anchor, t.a));
    CE_HIP(hipEventElapsedTime(&b, anchor, t.b));
    h_start_ms[i] = a;
    h_end_ms[i] = b;
    ++i;
    if (t.own_a) ctx->event_pool.push_back(t.a);
    ctx->event_pool.push_back(t.b);
  }
  ctx->timed.swap(keep);
  return CE_GPU_OK;
}

int ce_gpu_model_load(ce_gpu_ctx *ctx, const char *nnet_path, const char *prior_path, int left_context,
                      int right_context, ce_gpu_model **out) {
  if (!ctx || !nnet_path || !prior_path || !out) return fail(CE_GPU_EINVAL, "NULL argument");
  *out = nullptr;
  return load_model(ctx, nnet_path, prior_path, left_context, right_context, "", out);
}

int ce_gpu_model_load_config(ce_gpu_ctx *ctx, const char *config_path, ce_gpu_model **out) {
  if (!ctx || !config_path || !out) return fail(CE_GPU_EINVAL, "NULL argument");
  *out = nullptr;
  Config cf;
  CE_TRY(cf.read(config_path));
  std::string nnet, prior, tid2pdf;
  int left = 0, right = 0, chunk = 0, num_pdfs = 0;
  CE_TRY(cf.path("nnet", &nnet));
  CE_TRY(cf.path("prior", &prior));
  CE_TRY(cf.integer("left_context", &left));
  CE_TRY(cf.integer("right_context", &right));
  CE_TRY(cf.integer("chunk_size", &chunk));
  CE_TRY(cf.integer("num_pdfs", &num_pdfs));
  CE_TRY(cf.path("tid2pdf", &tid2pdf));
  ce_gpu_model *m = nullptr;
  CE_TRY(load_model(ctx, nnet, prior, left, right, tid2pdf, &m));
  m->chunk = chunk;
  *out = m;
  return CE_GPU_OK;
}

int ce_gpu_model_info(const ce_gpu_model *m, int *left_context, int *right_context, int *input_dim,
                      int *num_pdfs, int *num_linear, int64_t *num_params) {
  if (!m) return fail(CE_GPU_EINVAL, "model is NULL");
  if (left_context) *left_context = m->left;
  if (right_context) *right_context = m->right;
  if (input_dim) *input_dim = m->input_dim;
  if (num_pdfs) *num_pdfs = m->num_pdfs;
  if (num_linear) *num_linear = m->num_linear;
  if (num_params) *num_params = m->num_params;
  return CE_GPU_OK;
}

int ce_gpu_model_set_gemm(ce_gpu_model *m, int mode) {
  if (!m) return fail(CE_GPU_EINVAL, "NULL model");
  if (mode != CE_GPU_GEMM_FP32 && mode != CE_GPU_GEMM_BF16X6 && mode != CE_GPU_GEMM_F16X3 &&
      mode != CE_GPU_GEMM_BF16X6_PLANES)
    return fail(CE_GPU_EINVAL, "unknown GEMM mode");
  if (mode != CE_GPU_GEMM_FP32 && !m->x6_ok)
    return fail(CE_GPU_ENOTSUP, "this nnet program cannot run on split planes (unfused row op or widths)");
  if (mode == CE_GPU_GEMM_F16X3 && !m->x3_ok)
    return fail(CE_GPU_ENOTSUP, "a weight matrix is not finite: no f16x3 image");
  m->gemm = mode;
  return CE_GPU_OK;
}

int ce_gpu_model_get_gemm(const ce_gpu_model *m, int *mode) {
  if (!m || !mode) return fail(CE_GPU_EINVAL, "NULL argument");
  *mode = m->gemm;
  return CE_GPU_OK;
}

int ce_gpu_model_tid2pdf(const ce_gpu_model *m, int32_t *h_out, int capacity, int *size) {
  if (!m) return fail(CE_GPU_EINVAL, "model is NULL");
  const int n = (int)m->tid2pdf.size();
  if (size) *size = n;
  if (h_out && capacity > 0) memcpy(h_out, m->tid2pdf.data(), sizeof(int32_t) * std::min(n, capacity));
  return CE_GPU_OK;
}

int ce_gpu_model_destroy(ce_gpu_model *m) {
  delete m;
  return CE_GPU_OK;
}

int64_t ce_gpu_fbank_num_frames(int64_t n) {
  return n < kWinLen ? 0 : 1 + (n - kWinLen) / kShift;
}

int ce_gpu_plan_create(ce_gpu_ctx *ctx, const ce_gpu_model *model, const int64_t *h_num_samples, int n_utt,
                       int max_rows, ce_gpu_plan **out) {
  if (!ctx || !out || n_utt < 0 || (n_utt > 0 && !h_num_samples)) return fail(CE_GPU_EINVAL, "bad argument");
  *out = nullptr;
  CE_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<ce_gpu_plan> p(new (std::nothrow) ce_gpu_plan());
  if (!p) return fail(CE_GPU_ENOMEM, "out of host memory");
  p->n_utt = n_utt;
  p->sample_off.assign(n_utt + 1, 0);
  p->frame_off.assign(n_utt + 1, 0);
  for (int u = 0; u < n_utt; ++u) {
    if (h_num_samples[u] < 0) return fail(CE_GPU_EINVAL, "negative sample count");
    p->sample_off[u + 1] = p->sample_off[u] + h_num_samples[u];
    p->frame_off[u + 1] = p->frame_off[u] + ce_gpu_fbank_num_frames(h_num_samples[u]);
  }
  p->total_samples = p->sample_off[n_utt];
  p->total_frames = p->frame_off[n_utt];
  if (p->total_frames >= (int64_t)INT32_MAX) return fail(CE_GPU_EINVAL, "too many frames in one plan");
  // fbank block -> first utterance
  const int fpb = fbank_frames_per_block();
  const int64_t blocks = (p->total_frames + fpb - 1) / fpb;
  std::vector<int32_t> block_utt(std::max<int64_t>(blocks, 1), 0);
  {
    int u = 0;
    for (int64_t b = 0; b < blocks; ++b) {
      while (p->frame_off[u + 1] <= b * fpb) ++u;
      block_utt[b] = u;
    }
  }
  p->fbank_blocks = (int)blocks;
  CE_TRY(p->d_sample_off.upload(p->sample_off.data(), p->sample_off.size() * 8));
  CE_TRY(p->d_frame_off.upload(p->frame_off.data(), p->frame_off.size() * 8));
  CE_TRY(p->d_block_utt.upload(block_utt.data(), block_utt.size() * 4));

  if (model) {
    const int L = model->left, R = model->right;
    if (max_rows <= 0) max_rows = 4096;
    if (max_rows < L + R + 1) return fail(CE_GPU_EINVAL, "max_rows smaller than the nnet context");
    p->has_model = true;
    p->left = L;
    p->right = R;
    std::vector<int32_t> src, dst;
    std::vector<uint32_t> edge;
    ce_gpu_plan::Chunk cur;
    auto close = [&]() {
      if (cur.rows > 0) {
        p->max_chunk_rows = std::max(p->max_chunk_rows, cur.rows);
        p->chunks.push_back(cur);
      }
      cur = ce_gpu_plan::Chunk();
      cur.map_base = (int64_t)src.size();
    };
    cur.map_base = 0;
    for (int u = 0; u < n_utt; ++u) {
      const int64_t T = p->frame_off[u + 1] - p->frame_off[u];
      int64_t t = 0;
      while (t < T) {
        int64_t room = max_rows - cur.rows - L - R;
        if (room < T - t && cur.rows > 0) {  // start the utterance in a fresh chunk
          close();
          room = max_rows - L - R;
        }
        const int64_t n = std::min(T - t, room);
        const int64_t seg_rows = n + L + R;
        for (int64_t j = 0; j < seg_rows; ++j) {
          const uint32_t dl = (uint32_t)std::min<int64_t>(j, 0xffff), dr = (uint32_t)std::min<int64_t>(seg_rows - 1 - j, 0xffff);
          edge.push_back(dl | (dr << 16));
          int64_t fr = t - L + j;
          fr = fr < 0 ? 0 : (fr > T - 1 ? T - 1 : fr);
          src.push_back((int32_t)(p->frame_off[u] + fr));
          dst.push_back(j >= L && j < L + n ? (int32_t)(p->frame_off[u] + t + j - L) : -1);
        }
        cur.rows += (int)(n + L + R);
        t += n;
      }
    }
    close();
    if (!src.empty()) {
      CE_TRY(p->d_row_src.upload(src.data(), src.size() * 4));
      CE_TRY(p->d_row_dst.upload(dst.data(), dst.size() * 4));
      CE_TRY(p->d_row_edge.upload(edge.data(), edge.size() * 4));
    }
  }
  *out = p.release();
  return CE_GPU_OK;
}

int ce_gpu_plan_info(const ce_gpu_plan *p, int *n_utt, int64_t *total_samples, int64_t *total_frames,
                     int *n_chunks, int *max_chunk_rows) {
  if (!p) return fail(CE_GPU_EINVAL, "plan is NULL");
  if (n_utt) *n_utt = p->n_utt;
  if (total_samples) *total_samples = p->total_samples;
  if (total_frames) *total_frames = p->total_frames;
  if (n_chunks) *n_chunks = (int)p->chunks.size();
  if (max_chunk_rows) *max_chunk_rows = p->max_chunk_rows;
  return CE_GPU_OK;
}

int ce_gpu_plan_frame_offsets(const ce_gpu_plan *p, int64_t *h_out) {
  if (!p || !h_out) return fail(CE_GPU_EINVAL, "NULL argument");
  memcpy(h_out, p->frame_off.data(), sizeof(int64_t) * p->frame_off.size());
  return CE_GPU_OK;
}

int ce_gpu_plan_destroy(ce_gpu_plan *p) {
  delete p;
  return CE_GPU_OK;
}

}  // extern "C"

// CATEARS_SKIP (measurement builds only, -DCATEARS_DIAG: wrong results, timing
// only): launches left out of every call, to price each stage of a pipeline
// by its absence -- 1 first GEMM layer, 2 finalize, 4 fbank, 8 CMVN, 16 last
// GEMM layer, 32 the hidden GEMM layers, 64 the int8 path's min / max and
// Quantize passes.  0 in the product library.
static int diag_skip() {
  static const int v = CE_KNOB("CATEARS_SKIP", 0);
  return v;
}

extern "C" {

int ce_gpu_fbank(ce_gpu_ctx *ctx, const ce_gpu_plan *p, const float *d_pcm, float *d_feats, float *d_mel) {
  if (!ctx || !p || (p->total_frames > 0 && (!d_pcm || !d_feats))) return fail(CE_GPU_EINVAL, "NULL argument");
  ProfScope prof(ctx, CE_GPU_PROF_FBANK);
  if (diag_skip() & 4) return CE_GPU_OK;
  const FbankTables *t = ctx->d_tables.as<FbankTables>();
#ifdef CATEARS_EXPERIMENTS
  // timing only: phase A without its lane-dependent twiddle cases
  static const int nocase = CE_KNOB("CATEARS_FB_NOCASE", 0);
  if (nocase && ctx->fbank_mode != CE_GPU_FBANK_FAST) return launch_fbank_nocase(ctx->stream, t, p, d_pcm, d_feats, d_mel);
#endif
  return ctx->fbank_mode == CE_GPU_FBANK_FAST ? launch_fbank_fma(ctx->stream, t, p, d_pcm, d_feats, d_mel)
                                              : launch_fbank(ctx->stream, t, p, d_pcm, d_feats, d_mel);
}

int ce_gpu_fbank_s16(ce_gpu_ctx *ctx, const ce_gpu_plan *p, const int16_t *d_pcm, float *d_feats, float *d_mel) {
  if (!ctx || !p || (p->total_frames > 0 && (!d_pcm || !d_feats))) return fail(CE_GPU_EINVAL, "NULL argument");
  ProfScope prof(ctx, CE_GPU_PROF_FBANK);
  const FbankTables *t = ctx->d_tables.as<FbankTables>();
  return ctx->fbank_mode == CE_GPU_FBANK_FAST ? launch_fbank_fma_s16(ctx->stream, t, p, d_pcm, d_feats, d_mel)
                                              : launch_fbank_s16(ctx->stream, t, p, d_pcm, d_feats, d_mel);
}

int ce_gpu_cmvn(ce_gpu_ctx *ctx, const ce_gpu_plan *p, const float *d_global_stats, const float *d_feats,
                float *d_out) {
  if (!ctx || !p || !d_global_stats || (p->total_frames > 0 && (!d_feats || !d_out)))
    return fail(CE_GPU_EINVAL, "NULL argument");
  const char *a = reinterpret_cast<const char *>(d_feats), *b = reinterpret_cast<const char *>(d_out);
  const size_t bytes = (size_t)p->total_frames * kMel * sizeof(float);
  if (bytes && a < b + bytes && b < a + bytes) return fail(CE_GPU_EINVAL, "cmvn: d_out overlaps d_feats");
  ProfScope prof(ctx, CE_GPU_PROF_CMVN);
  if (diag_skip() & 8) return CE_GPU_OK;
  return launch_cmvn(ctx->stream, p, d_global_stats, d_feats, d_out);
}

}  // extern "C"

namespace catears {
// CATEARS_SPLICE_FIRST=0 (experiments library) keeps the gather loader for
// narrow segments (A/B).
static bool splice_first_layer() {
  static const bool on = CE_KNOB("CATEARS_SPLICE_FIRST", 1) != 0;
  return on;
}

// Runs the program's steps on `rows` packed rows starting at x (row_map: the
// first layer's packed row -> source row, or NULL for identity).  Returns the
// last activation via *y / *ldy.
static int run_steps_f32(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *x, int ldx, int rows,
                         const int *row_map, const float **y, int *ldy) {
  const size_t per = (size_t)rows * m->max_width;
  CE_TRY(ensure_workspace(ctx, 2 * per));
  float *buf[2] = {ctx->workspace.as<float>(), ctx->workspace.as<float>() + per};
  int cur = 0;
  bool first = true;
  for (const Step &st : m->steps) {
    if (st.is_gemm) {
      const GemmLayer &g = st.gemm;
      GemmArgs a;
      a.x = x;
      a.ldx = ldx;
      a.row_map = first ? row_map : nullptr;
      a.m = rows;
      a.n = g.n;
      a.k = g.k;
      a.kpad = g.kpad;
      a.din = g.din;
      a.nseg = g.nseg;
      for (int i = 0; i < 8; ++i) a.off[i] = g.off[i];
      a.w = g.wt.as<float>();
      a.ldw = g.kpad;
      a.bias = g.bias.as<float>();
      a.bn_scale = g.bn_scale.as<float>();
      a.bn_offset = g.bn_offset.as<float>();
      for (int i = 0; i < 4; ++i) a.post[i] = g.post[i];
      a.npost = g.npost;
      a.y = buf[cur];
      a.ldy = g.n;
      {
        ProfScope prof(ctx, g.din % 32 == 0 ? CE_GPU_PROF_GEMM : CE_GPU_PROF_GEMM_GATHER);
        if (g.din % 32 != 0 && splice_first_layer()) {
          // Segments narrower than a K-tile (the 40-wide first layer):
          // write the spliced block once (rows x kpad, zero padded) and run
          // the fast kernel on it -- cheaper than a per-element gather loader.
          CE_TRY(ensure_scratch(ctx, (size_t)rows * g.kpad * sizeof(float)));
          float *xs = static_cast<float *>(ctx->scratch.ptr);
          CE_TRY(launch_splice_pad(ctx->stream, x, ldx, rows, g.din, g.nseg, g.off, a.row_map, xs, g.kpad));
          a.x = xs;
          a.ldx = g.kpad;
          a.row_map = nullptr;
          a.k = g.kpad;  // the padding columns are zero on both sides
          a.din = g.kpad;
          a.nseg = 1;
          for (int i = 0; i < 8; ++i) a.off[i] = 0;
        }
        CE_TRY(launch_gemm_f32(ctx->stream, a));
      }
      x = buf[cur];
      ldx = g.n;
      cur ^= 1;
      first = false;
    } else {
      CE_TRY(launch_rowop(ctx->stream, st.row, const_cast<float *>(x), ldx, rows));
    }
  }
  *y = x;
  *ldy = ldx;
  return CE_GPU_OK;
}
// The bf16x6 program (kernels/gemm_bf16x6.hip): the first layer's spliced
// block is written as three bf16 planes, every hidden layer's epilogue
// writes its output split for the next, the last layer writes fp32.
// bf16x6 with fp32 operands in HBM (gemm_bf16x6f_kernel: the split into
// planes happens on the way into LDS): the layers chain fp32 activations as
// the fp32 program does, the weights are the fp32 `wt` matrices.  4 B per
// operand element through L2 instead of the planes' 6; measured +3 % over
// the plane kernels (tools/ab.sh).
// Default; CATEARS_X6_F32IN=0 selects the plane-operand kernels
// (run_steps_x6: planes written by each epilogue, bit-identical results).
static int x6_variant_env() {
  static const int v = CE_KNOB("CATEARS_X6_VARIANT", 0);
  return v;
}

static bool x6_f32in() {
  static const bool v = CE_KNOB("CATEARS_X6_F32IN", 1) != 0;
  return v;
}

// CATEARS_X6_FIRST=0 keeps the round-3 splice_pad launch before the first
// layer's throughput GEMM (bit-identical; the default gathers in its loader)
static bool x6_first_direct() {
  static const bool v = CE_KNOB("CATEARS_X6_FIRST", 1) != 0;
  return v && (x6_variant_env() == 0 || x6_variant_env() == 300);
}

// CATEARS_X6_CHAIN: the layers hand each other their outputs as bf16 planes
// (the direct-weight kernel's OUT16 epilogue, read by its PIN loader), so
// each activation is split once, in the epilogue that produces it, instead of
// by every unit tile of the next layer that reads it.  Bit-identical to the
// fp32 chain (tests/test_gpu_x6_variants.py).
// 2: only the output layer reads planes (its 14 unit tiles would each split
// the same activations), written by the layer before it.
static int x6_plane_chain_env() {
  static const int v = CE_KNOB("CATEARS_X6_CHAIN", 0);
  return v;
}

// CATEARS_LAT_FUSED_FINAL=0 keeps the last layer's split-K reduce as its own
// launch before the finalize (bit-identical; the default fuses the two)
static bool lat_fused_final() {
  static const bool v = CE_KNOB("CATEARS_LAT_FUSED_FINAL", 1) != 0;
  return v;
}

static int run_steps_x6f(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *x, int ldx, int rows,
                         const int *row_map, const float **y, int *ldy, LatTail *tail) {
  int max_in = 0;
  for (const Step &st : m->steps) max_in = std::max(max_in, st.gemm.kpad);
  for (const Step &st : m->steps) max_in = std::max(max_in, (st.gemm.n + 31) / 32 * 32);
  // the plane chain: the first layer gathers the caller's fp32 rows in its
  // loader, every layer has the fragment image, the later layers' segments
  // are whole K-tiles
  const int chain_mode = x6_plane_chain_env();
  bool planes = chain_mode != 0 && !ctx->latency && x6_first_direct() && m->steps[0].gemm.din % 8 == 0 &&
               ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  for (size_t i = 0; planes && i < m->steps.size(); ++i)
    planes = m->steps[i].gemm.wdir.ptr && (i == 0 || m->steps[i].gemm.din % 32 == 0);
  // a block of planes is rows x 3 x width bf16: 1.5 floats per element
  const size_t blk = ((size_t)rows * max_in * (planes ? 3 : 2) / 2 + 63) / 64 * 64;
  CE_TRY(ensure_workspace(ctx, 2 * blk + (size_t)rows * m->num_pdfs));
  float *buf[2] = {ctx->workspace.as<float>(), ctx->workspace.as<float>() + blk};
  float *out = ctx->workspace.as<float>() + 2 * blk;
  const float *xs = nullptr;
  int px = 0, cur = 0;
  ProfChain chain(ctx);  // every step below is one launch; GEMMs back to back
  for (size_t i = 0; i < m->steps.size(); ++i) {
    const GemmLayer &g = m->steps[i].gemm;
    const bool last = i + 1 == m->steps.size();
    X6Gemm a;
    // the latency kernel and the default direct-weight kernel splice the
    // caller's rows themselves (din % 8 == 0): no splice_pad launch
    const bool lat_direct = i == 0 && g.din % 8 == 0 && ldx % 4 == 0 &&
                            (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                            (ctx->latency || (g.wdir.ptr && x6_first_direct()));
    if (lat_direct) {
      xs = x;
      px = ldx;
      a.din = g.din;
      a.nseg = g.nseg;
      for (int s = 0; s < 8; ++s) a.off[s] = g.off[s];
      a.row_map = row_map;
    } else if (i == 0) {
      ProfScope prof(ctx, CE_GPU_PROF_GEMM_GATHER);
      CE_TRY(launch_splice_pad(ctx->stream, x, ldx, rows, g.din, g.nseg, g.off, row_map, buf[cur], g.kpad));
      xs = buf[cur];
      px = g.kpad;
      cur ^= 1;
      a.din = g.kpad;
      a.nseg = 1;
    } else {
      a.din = g.din;
      a.nseg = g.nseg;
      for (int s = 0; s < 8; ++s) a.off[s] = g.off[s];
    }
    // planes into layer i / out of it: every layer after the first (mode 1),
    // or the output layer only (mode 2)
    const size_t nst = m->steps.size();
    const bool pin = planes && i > 0 && (chain_mode != 2 || i + 1 == nst);
    const bool pout = planes && !last && (chain_mode != 2 || i + 2 == nst);
    if (pin) {
      a.x = reinterpret_cast<const uint16_t *>(xs);
      a.ldx = 3 * px;
      a.px = px;
    } else {
      a.xf = xs;
      a.ldx = px;
    }
    a.wf = g.wt.as<float>();
    a.ldw = g.kpad;
    a.w = g.wsplit.as<uint16_t>();  // the same weights as planes (kernels that read them)
    a.pw = g.kpad;
    a.wd = g.wdir.as<uint16_t>();   // and as MFMA fragments (the default kernel)
    a.wd_kt = g.kpad / 32;
    a.wide = ctx->wide_tiles != 0;
    a.m = rows;
    a.n = g.n;
    a.kpad = i == 0 ? g.kpad : g.nseg * g.din;
    a.bias = g.bias.as<float>();
    a.bn_scale = g.bn_scale.as<float>();
    a.bn_offset = g.bn_offset.as<float>();
    for (int q = 0; q < 4; ++q) a.post[q] = g.post[q];
    a.npost = g.npost;
    const int pn = (g.n + 31) / 32 * 32;
    if (pout) {
      a.y16 = reinterpret_cast<uint16_t *>(buf[cur]);
      a.ldy = 3 * pn;
      a.py = pn;
    } else {
      a.y32 = last ? out : buf[cur];
      a.ldy = last ? g.n : pn;
    }
    {
      ProfScope prof(ctx, CE_GPU_PROF_GEMM);
      if (ctx->latency) {
        const size_t pf = x6_lat_part_floats(a.m, a.n, x6_lat_slices(a.kpad, a.n));
        CE_TRY(ensure_lat_part(ctx, pf));
        if (last && lat_fused_final()) a.tail = tail;  // the reduce may run inside the finalize
        CE_TRY(launch_gemm_bf16x6_lat(ctx->stream, a, ctx->lat_part.as<float>(), pf, ctx->lat_tickets.as<unsigned>()));
      } else if (!(diag_skip() & (i == 0 ? 1 : last ? 16 : 32))) {
        CE_TRY(launch_gemm_bf16x6(ctx->stream, a));
      }
    }
    xs = buf[cur];
    px = pn;
    cur ^= 1;
  }
  *y = out;
  *ldy = m->steps.back().gemm.n;
  return CE_GPU_OK;
}

static int run_steps_x6(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *x, int ldx, int rows,
                        const int *row_map, const float **y, int *ldy) {
  int max_in = 0;
  for (const Step &st : m->steps) max_in = std::max(max_in, st.gemm.kpad);
  for (const Step &st : m->steps) max_in = std::max(max_in, (st.gemm.n + 31) / 32 * 32);
  // two split ping-pong blocks (rows x 3 x max_in bf16) + the fp32 output
  const size_t split_floats = ((size_t)rows * 3 * max_in + 1) / 2;
  const size_t split_stride = (split_floats + 63) / 64 * 64;
  CE_TRY(ensure_workspace(ctx, 2 * split_stride + (size_t)rows * m->num_pdfs));
  uint16_t *sbuf[2] = {reinterpret_cast<uint16_t *>(ctx->workspace.as<float>()),
                       reinterpret_cast<uint16_t *>(ctx->workspace.as<float>() + split_stride)};
  float *out = ctx->workspace.as<float>() + 2 * split_stride;
  const uint16_t *xs = nullptr;
  int px = 0;
  int cur = 0;
  for (size_t i = 0; i < m->steps.size(); ++i) {
    const GemmLayer &g = m->steps[i].gemm;
    const bool last = i + 1 == m->steps.size();
    X6Gemm a;
    if (i == 0) {
      ProfScope prof(ctx, CE_GPU_PROF_GEMM_GATHER);
      CE_TRY(launch_splice_pad_split(ctx->stream, x, ldx, rows, g.din, g.nseg, g.off, row_map, sbuf[cur], g.kpad));
      xs = sbuf[cur];
      px = g.kpad;
      cur ^= 1;
      a.din = g.kpad;
      a.nseg = 1;
    } else {
      a.din = g.din;
      a.nseg = g.nseg;
      for (int s = 0; s < 8; ++s) a.off[s] = g.off[s];
    }
    a.x = xs;
    a.ldx = 3 * px;
    a.px = px;
    a.w = g.wsplit.as<uint16_t>();
    a.ldw = 3 * g.kpad;
    a.pw = g.kpad;
    a.m = rows;
    a.n = g.n;
    a.kpad = i == 0 ? g.kpad : g.nseg * g.din;
    a.bias = g.bias.as<float>();
    a.bn_scale = g.bn_scale.as<float>();
    a.bn_offset = g.bn_offset.as<float>();
    for (int q = 0; q < 4; ++q) a.post[q] = g.post[q];
    a.npost = g.npost;
    const int pn = (g.n + 31) / 32 * 32;
    if (last) {
      a.y32 = out;
      a.ldy = g.n;
    } else {
      a.y16 = sbuf[cur];
      a.ldy = 3 * pn;
      a.py = pn;
    }
    {
      ProfScope prof(ctx, CE_GPU_PROF_GEMM);
      CE_TRY(launch_gemm_bf16x6(ctx->stream, a));
    }
    xs = sbuf[cur];
    px = pn;
    cur ^= 1;
  }
  *y = out;
  *ldy = m->steps.back().gemm.n;
  return CE_GPU_OK;
}

static int ensure_overflow_word(ce_gpu_ctx *ctx) {
  if (ctx->overflow.ptr) return CE_GPU_OK;
  CE_TRY(ctx->overflow.alloc(256));
  CE_HIP(hipMemsetAsync(ctx->overflow.ptr, 0, 256, ctx->stream));
  return CE_GPU_OK;
}

// The f16x3 program (kernels/gemm_f16x3.hip): as run_steps_x6 with two fp16
// planes per operand; splits beyond the fp16 range set ctx->overflow.
static int run_steps_x3(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *x, int ldx, int rows,
                        const int *row_map, const float **y, int *ldy) {
  CE_TRY(ensure_overflow_word(ctx));
  int *overflow = ctx->overflow.as<int>();
  int max_in = 0;
  for (const Step &st : m->steps) max_in = std::max(max_in, st.gemm.kpad);
  for (const Step &st : m->steps) max_in = std::max(max_in, (st.gemm.n + 63) / 64 * 64);
  // two split ping-pong blocks (rows x 2 x max_in fp16) + the fp32 output
  const size_t split_floats = (size_t)rows * max_in;
  const size_t split_stride = (split_floats + 63) / 64 * 64;
  CE_TRY(ensure_workspace(ctx, 2 * split_stride + (size_t)rows * m->num_pdfs));
  uint16_t *sbuf[2] = {reinterpret_cast<uint16_t *>(ctx->workspace.as<float>()),
                       reinterpret_cast<uint16_t *>(ctx->workspace.as<float>() + split_stride)};
  float *out = ctx->workspace.as<float>() + 2 * split_stride;
  const uint16_t *xs = nullptr;
  int px = 0, cur = 0;
  for (size_t i = 0; i < m->steps.size(); ++i) {
    const GemmLayer &g = m->steps[i].gemm;
    const bool last = i + 1 == m->steps.size();
    X3Gemm a;
    if (i == 0) {
      ProfScope prof(ctx, CE_GPU_PROF_GEMM_GATHER);
      CE_TRY(launch_splice_pad_f16(ctx->stream, x, ldx, rows, g.din, g.nseg, g.off, row_map, sbuf[cur], g.kpad,
                                   overflow));
      xs = sbuf[cur];
      px = g.kpad;
      cur ^= 1;
      a.din = g.kpad;
      a.nseg = 1;
    } else {
      a.din = g.din;
      a.nseg = g.nseg;
      for (int s = 0; s < 8; ++s) a.off[s] = g.off[s];
    }
    a.x = xs;
    a.ldx = 2 * px;
    a.px = px;
    a.w = g.wf16.as<uint16_t>();
    a.ldw = 2 * g.kpad;
    a.pw = g.kpad;
    a.m = rows;
    a.n = g.n;
    a.kpad = i == 0 ? g.kpad : g.nseg * g.din;
    a.unscale = ldexpf(1.0f, -(g.w_shift + kF16ActShift));
    a.bias = g.bias.as<float>();
    a.bn_scale = g.bn_scale.as<float>();
    a.bn_offset = g.bn_offset.as<float>();
    for (int q = 0; q < 4; ++q) a.post[q] = g.post[q];
    a.npost = g.npost;
    a.overflow = overflow;
    const int pn = (g.n + 63) / 64 * 64;
    if (last) {
      a.y32 = out;
      a.ldy = g.n;
    } else {
      a.y16 = sbuf[cur];
      a.ldy = 2 * pn;
      a.py = pn;
    }
    {
      ProfScope prof(ctx, CE_GPU_PROF_GEMM);
      CE_TRY(launch_gemm_f16x3(ctx->stream, a));
    }
    xs = sbuf[cur];
    px = pn;
    cur ^= 1;
  }
  *y = out;
  *ldy = m->steps.back().gemm.n;
  return CE_GPU_OK;
}

// The int8 program (kernels/nnet_i8.hip): per Linear layer min/max ->
// quantize (+ row sums) -> u8 GEMM with float epilogue.
static int run_steps_i8(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *x, int ldx, int rows,
                        const int *row_map, const uint32_t *row_edge, const float **y, int *ldy) {
  const size_t per = (size_t)rows * m->max_width;
  CE_TRY(ensure_workspace(ctx, 2 * per));
  float *buf[2] = {ctx->workspace.as<float>(), ctx->workspace.as<float>() + per};
  int max_ldq = 16;
  for (const Step &st : m->steps)
    if (st.is_gemm) max_ldq = std::max(max_ldq, st.i8.spliced ? st.i8.kpad : st.i8.in_width);
  int max_n = 1;
  for (const Step &st : m->steps)
    if (st.is_gemm) max_n = std::max(max_n, st.i8.n);
  const size_t q_bytes = ((size_t)rows * max_ldq + 255) / 256 * 256;
  const size_t rs_bytes = ((size_t)rows * 4 + 255) / 256 * 256;
  const size_t part_bytes = std::max(i8_params_scratch_bytes(), sizeof(float) * 2 * i8_gemm_parts(rows, max_n));
  CE_TRY(ensure_scratch(ctx, q_bytes + rs_bytes + 256 + part_bytes));
  char *base = static_cast<char *>(ctx->scratch.ptr);
  int8_t *xq = reinterpret_cast<int8_t *>(base);
  int32_t *rowsum = reinterpret_cast<int32_t *>(base + q_bytes);
  void *params = base + q_bytes + rs_bytes;
  void *part = base + q_bytes + rs_bytes + 256;
  int cur = 0;
  bool first = true;
  int fused_parts = 0;  // > 0: the previous GEMM left this layer's min / max partials in `part`
  for (size_t si = 0; si < m->steps.size(); ++si) {
    const Step &st = m->steps[si];
    if (st.is_gemm) {
      const I8Layer &L = st.i8;
      const int *rm = first ? row_map : nullptr;
      const int ldq = L.spliced ? L.kpad : L.in_width;
      {
        ProfScope prof(ctx, CE_GPU_PROF_QUANT);
        const int zero[1] = {0};
        const int nseg = L.spliced ? st.gemm.nseg : 1;
        const int *offs = L.spliced ? st.gemm.off : zero;
        if (!(diag_skip() & 64)) {  // measurement library: 64 leaves the int8 quantize passes out
          if (fused_parts > 0)
            CE_TRY(launch_i8_params_fold(ctx->stream, part, fused_parts, params));
          else
            CE_TRY(launch_i8_params(ctx->stream, x, ldx, rows, L.in_width, rm, row_edge, L.in_left, L.in_right,
                                    part, params));
          CE_TRY(launch_i8_quantize(ctx->stream, x, ldx, rows, L.in_width, rm, nseg, offs, params, xq, ldq, rowsum));
        }
      }
      // the next step reads this GEMM's output directly: its min / max is
      // reduced in this GEMM's epilogue (the partials are read by the next
      // layer's fold before the next GEMM overwrites them: stream order)
      const bool fuse = si + 1 < m->steps.size() && m->steps[si + 1].is_gemm && m->steps[si + 1].i8.in_width == L.n;
      I8NextMinMax mm = {};
      if (fuse) {
        const I8Layer &N = m->steps[si + 1].i8;
        mm = I8NextMinMax{part, row_edge, N.in_left, N.in_right};
      }
      fused_parts = 0;
      ProfScope prof(ctx, CE_GPU_PROF_GEMM);
      CE_TRY(launch_i8_gemm(ctx->stream, L, xq, ldq, rows, rowsum, params, buf[cur], L.n, fuse ? &mm : nullptr,
                            fuse ? &fused_parts : nullptr));
      x = buf[cur];
      ldx = L.n;
      cur ^= 1;
      first = false;
    } else {
      fused_parts = 0;
      CE_TRY(launch_rowop(ctx->stream, st.row, const_cast<float *>(x), ldx, rows));
    }
  }
  *y = x;
  *ldy = ldx;
  return CE_GPU_OK;
}

static int run_steps(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *x, int ldx, int rows,
                     const int *row_map, const uint32_t *row_edge, const float **y, int *ldy,
                     LatTail *tail = nullptr) {
  if (tail) tail->active = false;
  if (m->int8) return run_steps_i8(ctx, m, x, ldx, rows, row_map, row_edge, y, ldy);
  if (m->gemm == CE_GPU_GEMM_F16X3) return run_steps_x3(ctx, m, x, ldx, rows, row_map, y, ldy);
  if (m->gemm == CE_GPU_GEMM_BF16X6_PLANES) return run_steps_x6(ctx, m, x, ldx, rows, row_map, y, ldy);
  if (m->gemm == CE_GPU_GEMM_BF16X6)
    return x6_f32in() ? run_steps_x6f(ctx, m, x, ldx, rows, row_map, y, ldy, tail)
                      : run_steps_x6(ctx, m, x, ldx, rows, row_map, y, ldy);
  return run_steps_f32(ctx, m, x, ldx, rows, row_map, y, ldy);
}

// The latency GEMM may defer its last layer's reduce into the finalize only
// when the fused finalize can write the caller's output: it stores 16-byte
// row chunks (launch_lat_finalize), so out and the log prior must be 16-byte
// aligned.  Otherwise the layer keeps its own reduce launch and the ordinary
// finalize (scalar path for unaligned rows) runs -- decided before any GEMM
// is launched.
static bool lat_tail_ok(const float *out, const float *log_prior) {
  return ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(log_prior)) & 15) == 0;
}

// launch_finalize on rows first .. first + rows - 1 of run_steps' output
// (or of its deferred latency tail: the last layer's reduce in the same
// launch)
static int finalize_output(ce_gpu_ctx *ctx, const float *y, int ldy, int first, int rows, int dim,
                           bool log_softmax, const float *log_prior, const int *row_dst, float *out,
                           const LatTail &tail = LatTail()) {
  if (diag_skip() & 2) return CE_GPU_OK;
  if (tail.active) return launch_lat_finalize(ctx->stream, tail, first, rows, log_softmax, log_prior, row_dst, out);
  return launch_finalize(ctx->stream, y + (size_t)first * ldy, ldy, rows, dim, log_softmax, log_prior, row_dst,
                         out);
}

// Quantize (src/matrix.cc:329-387) of one weight matrix on the host at load
// time: per-tensor parameters over the in x out MAT0 matrix, then the bytes
// stored shifted (q - 128) and transposed (n x kpad, zero padded) for the
// GEMM, with their column sums.
static int quantize_weights(ce_gpu_ctx *ctx, Step &st) {
  GemmLayer &g = st.gemm;
  I8Layer &L = st.i8;
  std::vector<float> wt((size_t)g.n * g.kpad);
  CE_HIP(hipMemcpy(wt.data(), g.wt.ptr, wt.size() * 4, hipMemcpyDeviceToHost));
  float mn = FLT_MAX, mx = FLT_MIN;  // FindMinMax (matrix.cc:329-345)
  for (int j = 0; j < g.n; ++j)
    for (int k = 0; k < g.k; ++k) {
      const float v = wt[(size_t)j * g.kpad + k];
      if (v > mx) mx = v;
      if (v < mn) mn = v;
    }
  const double scale = (mx - mn) / 255.0;  // ComputeQuantizationParams (matrix.cc:348-362)
  L.w_zp = (int32_t)round(-mn / scale);
  L.w_scale = (float)scale;
  const int ka = i8_k_align();
  L.n = g.n;
  L.k = g.k;
  L.kpad = (g.k + ka - 1) / ka * ka;
  std::vector<int8_t> q((size_t)g.n * L.kpad, 0);
  std::vector<int32_t> colsum(g.n, 0);
  for (int j = 0; j < g.n; ++j)
    for (int k = 0; k < g.k; ++k) {
      float v = wt[(size_t)j * g.kpad + k] / L.w_scale + L.w_zp;  // matrix.cc:378-386
      v = std::max(0.0f, std::min(v, 255.0f));
      const int b = (int)(uint8_t)roundf(v) - 128;
      q[(size_t)j * L.kpad + k] = (int8_t)b;
      colsum[j] += b;
    }
  CE_TRY(L.wq.upload(q.data(), q.size()));
  CE_TRY(L.colsum.upload(colsum.data(), colsum.size() * 4));
  L.in_width = g.din;
  L.in_left = g.in_left;
  L.in_right = g.in_right;
  L.spliced = g.din % ka != 0;
  if (L.spliced) {
    L.a_din = L.kpad;
    L.a_nseg = 1;
    for (int i = 0; i < 8; ++i) L.a_off[i] = 0;
  } else {
    L.a_din = g.din;
    L.a_nseg = g.nseg;
    for (int i = 0; i < 8; ++i) L.a_off[i] = g.off[i];
  }
  L.bias = g.bias.as<float>();
  L.bn_scale = g.bn_scale.as<float>();
  L.bn_offset = g.bn_offset.as<float>();
  for (int i = 0; i < 4; ++i) L.post[i] = g.post[i];
  L.npost = g.npost;
  (void)ctx;
  return CE_GPU_OK;
}
}  // namespace catears

extern "C" {

int ce_gpu_am_forward(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p, const float *d_feats,
                      float *d_loglik) {
  if (!ctx || !m || !p) return fail(CE_GPU_EINVAL, "NULL argument");
  if (!p->has_model || p->left != m->left || p->right != m->right)
    return fail(CE_GPU_EINVAL, "plan was not built for this model's context");
  if (p->chunks.empty()) return CE_GPU_OK;
  if (!d_feats || !d_loglik) return fail(CE_GPU_EINVAL, "NULL argument");
  if (!m->log_prior.ptr) return fail(CE_GPU_EINVAL, "am_forward needs a model loaded with a prior");
  if (m->left != m->net_left || m->right != m->net_right)
    return fail(CE_GPU_EINVAL, "model context differs from its network's");
  for (const ce_gpu_plan::Chunk &c : p->chunks) {
    const int *row_src = p->d_row_src.as<int>() + c.map_base;
    const int *row_dst = p->d_row_dst.as<int>() + c.map_base;
    const float *y = nullptr;
    int ldy = 0;
    const uint32_t *row_edge = p->d_row_edge.as<uint32_t>() + c.map_base;
    LatTail tail;
    CE_TRY(run_steps(ctx, m, d_feats, m->input_dim, c.rows, row_src, row_edge, &y, &ldy,
                     lat_tail_ok(d_loglik, m->log_prior.as<float>()) ? &tail : nullptr));
    ProfScope prof(ctx, CE_GPU_PROF_FINALIZE);
    CE_TRY(finalize_output(ctx, y, ldy, 0, c.rows, m->num_pdfs, m->final_log_softmax, m->log_prior.as<float>(),
                           row_dst, d_loglik, tail));
  }
  return CE_GPU_OK;
}

int ce_gpu_model_load_mem(ce_gpu_ctx *ctx, const void *nnet, int64_t nbytes, const float *h_prior,
                          int prior_dim, int left_context, int right_context, ce_gpu_model **out) {
  if (!ctx || !out || !nnet || nbytes <= 0 || (prior_dim > 0 && !h_prior))
    return fail(CE_GPU_EINVAL, "bad argument");
  *out = nullptr;
  std::unique_ptr<ce_gpu_model> m(new (std::nothrow) ce_gpu_model());
  if (!m) return fail(CE_GPU_ENOMEM, "out of host memory");
  Reader rd;
  CE_TRY(rd.open_mem(nnet, (size_t)nbytes, "<nnet image>"));
  CE_TRY(read_program(ctx, rd, left_context, right_context, m.get()));
  if (h_prior) CE_TRY(set_prior(m.get(), h_prior, prior_dim));
  *out = m.release();
  return CE_GPU_OK;
}

int ce_gpu_nnet_check_mem(const void *nnet, int64_t nbytes, int *num_layers, int *left, int *right) {
  if (!nnet || nbytes <= 0) return fail(CE_GPU_EINVAL, "bad argument");
  Reader rd;
  CE_TRY(rd.open_mem(nnet, (size_t)nbytes, "<nnet image>"));
  std::vector<RawLayer> layers;
  int hl = 0, hr = 0;
  CE_TRY(read_nnet(rd, &layers, &hl, &hr));
  if (num_layers) *num_layers = (int)layers.size();
  if (left) *left = hl;
  if (right) *right = hr;
  return CE_GPU_OK;
}

int ce_gpu_nnet_propagate(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *d_in, int rows, int ld_in,
                          int subtract_prior, float *d_out) {
  if (!ctx || !m || !d_in || !d_out) return fail(CE_GPU_EINVAL, "NULL argument");
  if (ld_in < m->input_dim) return fail(CE_GPU_EINVAL, "ld_in smaller than the nnet input");
  const int out_rows = rows - m->net_left - m->net_right;
  if (out_rows <= 0)
    return fail(CE_GPU_EINVAL, fmt("nnet_propagate: %d rows do not cover the network context (%d, %d)", rows,
                                   m->net_left, m->net_right));
  if (subtract_prior && !m->log_prior.ptr) return fail(CE_GPU_EINVAL, "model has no prior");
  const int ctx_rows = m->net_left + m->net_right;
  if (!m->int8 && rows > kPropagateWindow) {
    // A very long block (hours of audio in one call) runs as overlapping
    // windows: output row t needs input rows t .. t + L + R only, so the
    // windows give the same bits as one pass, keep every GEMM operand well
    // inside the kernels' 32-bit row offsets and bound the workspace.  (An
    // int8 model quantizes per call, so it keeps the single pass.)
    const int step = kPropagateWindow - ctx_rows;
    for (int o = 0; o < out_rows; o += step) {
      const int n = std::min(step, out_rows - o);
      CE_TRY(ce_gpu_nnet_propagate(ctx, m, d_in + (size_t)o * ld_in, n + ctx_rows, ld_in, subtract_prior,
                                   d_out + (size_t)o * m->num_pdfs));
    }
    return CE_GPU_OK;
  }
  const float *y = nullptr;
  int ldy = 0;
  LatTail tail;
  CE_TRY(run_steps(ctx, m, d_in, ld_in, rows, nullptr, nullptr, &y, &ldy,
                   lat_tail_ok(d_out, m->log_prior.as<float>()) ? &tail : nullptr));
  ProfScope prof(ctx, CE_GPU_PROF_FINALIZE);
  return finalize_output(ctx, y, ldy, m->net_left, out_rows, m->num_pdfs, m->final_log_softmax,
                         subtract_prior ? m->log_prior.as<float>() : nullptr, nullptr, d_out, tail);
}

int ce_gpu_nnet_propagate_blocks(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *d_in, int ld_in,
                                 const int32_t *h_rows, int n_blocks, int subtract_prior, float *d_out) {
  if (!ctx || !m || !d_in || !d_out || !h_rows || n_blocks < 1) return fail(CE_GPU_EINVAL, "bad argument");
  if (ld_in < m->input_dim) return fail(CE_GPU_EINVAL, "ld_in smaller than the nnet input");
  if (subtract_prior && !m->log_prior.ptr) return fail(CE_GPU_EINVAL, "model has no prior");
  const int L = m->net_left, R = m->net_right;
  int64_t total = 0;
  for (int b = 0; b < n_blocks; ++b) {
    if (h_rows[b] <= L + R)
      return fail(CE_GPU_EINVAL, fmt("nnet_propagate_blocks: block %d has %d rows, context is (%d, %d)", b,
                                     h_rows[b], L, R));
    total += h_rows[b];
  }
  if (total >= INT32_MAX / 2) return fail(CE_GPU_EINVAL, "too many rows");
  if (m->int8) {
    // per-tensor activation parameters are reduced over the block being
    // scored: one block per call keeps each block's rows its own
    const float *in = d_in;
    float *o = d_out;
    for (int b = 0; b < n_blocks; ++b) {
      CE_TRY(ce_gpu_nnet_propagate(ctx, m, in, h_rows[b], ld_in, subtract_prior, o));
      in += (size_t)h_rows[b] * ld_in;
      o += (size_t)(h_rows[b] - L - R) * m->num_pdfs;
    }
    return CE_GPU_OK;
  }
  const int rows = (int)total;
  // per packed row: output row (or -1) and distances to its block's edges;
  // written only after the previous call's kernels are done with them
  CE_HIP(hipStreamSynchronize(ctx->stream));
  ctx->h_blk_maps.resize(2 * (size_t)rows);
  int32_t *dst = ctx->h_blk_maps.data();
  uint32_t *edge = reinterpret_cast<uint32_t *>(dst + rows);
  int r = 0, out = 0;
  for (int b = 0; b < n_blocks; ++b) {
    const int n = h_rows[b];
    for (int j = 0; j < n; ++j, ++r) {
      dst[r] = (j >= L && j < n - R) ? out++ : -1;
      const uint32_t dl = (uint32_t)std::min(j, 0xffff), dr = (uint32_t)std::min(n - 1 - j, 0xffff);
      edge[r] = dl | (dr << 16);
    }
  }
  const size_t bytes = ctx->h_blk_maps.size() * 4;
  if (ctx->blk_maps.bytes < bytes) CE_TRY(ctx->blk_maps.alloc(bytes));
  CE_HIP(hipMemcpyAsync(ctx->blk_maps.ptr, ctx->h_blk_maps.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
  const int32_t *d_dst = ctx->blk_maps.as<int32_t>();
  const uint32_t *d_edge = reinterpret_cast<const uint32_t *>(d_dst + rows);
  const float *y = nullptr;
  int ldy = 0;
  // blocks are independent: the rows a Splice reads across a block boundary
  // only feed rows that block's Narrow drops
  LatTail tail;
  CE_TRY(run_steps(ctx, m, d_in, ld_in, rows, nullptr, d_edge, &y, &ldy,
                   lat_tail_ok(d_out, m->log_prior.as<float>()) ? &tail : nullptr));
  ProfScope prof(ctx, CE_GPU_PROF_FINALIZE);
  return finalize_output(ctx, y, ldy, 0, rows, m->num_pdfs, m->final_log_softmax,
                         subtract_prior ? m->log_prior.as<float>() : nullptr, d_dst, d_out, tail);
}

static int score_feats(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p, const float *d_global_stats,
                       float *d_feats_ws, float *d_loglik) {
  const float *feats = d_feats_ws;
  if (d_global_stats) {
    float *norm = d_feats_ws + (size_t)p->total_frames * kMel;
    CE_TRY(ce_gpu_cmvn(ctx, p, d_global_stats, d_feats_ws, norm));
    feats = norm;
  }
  return ce_gpu_am_forward(ctx, m, p, feats, d_loglik);
}

int ce_gpu_score(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p, const float *d_pcm,
                 const float *d_global_stats, float *d_feats_ws, float *d_loglik) {
  if (!ctx || !m || !p) return fail(CE_GPU_EINVAL, "NULL argument");
  if (m->input_dim != kMel) return fail(CE_GPU_EINVAL, "nnet input is not 40-dim fbank");
  CE_TRY(ce_gpu_fbank(ctx, p, d_pcm, d_feats_ws, nullptr));
  return score_feats(ctx, m, p, d_global_stats, d_feats_ws, d_loglik);
}

int ce_gpu_score_s16(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p, const int16_t *d_pcm,
                     const float *d_global_stats, float *d_feats_ws, float *d_loglik) {
  if (!ctx || !m || !p) return fail(CE_GPU_EINVAL, "NULL argument");
  if (m->input_dim != kMel) return fail(CE_GPU_EINVAL, "nnet input is not 40-dim fbank");
  CE_TRY(ce_gpu_fbank_s16(ctx, p, d_pcm, d_feats_ws, nullptr));
  return score_feats(ctx, m, p, d_global_stats, d_feats_ws, d_loglik);
}

int ce_gpu_sgemm(ce_gpu_ctx *ctx, int m, int n, int k, const float *d_a, int lda, const float *d_b, int ldb,
                 float *d_c, int ldc) {
  if (!ctx || m < 0 || n < 0 || k < 0) return fail(CE_GPU_EINVAL, "bad argument");
  if (m == 0 || n == 0) return CE_GPU_OK;
  if (k == 0) {
    for (int i = 0; i < m; ++i) CE_HIP(hipMemsetAsync(d_c + (size_t)i * ldc, 0, sizeof(float) * n, ctx->stream));
    return CE_GPU_OK;
  }
  if (lda < k || ldb < n || ldc < n) return fail(CE_GPU_EINVAL, "leading dimension too small");
  GemmArgs a;
  a.x = d_a;
  a.ldx = lda;
  a.m = m;
  a.n = n;
  a.k = k;
  a.kpad = (k + gemm_k_align() - 1) / gemm_k_align() * gemm_k_align();
  a.din = k;
  a.nseg = 1;
  a.w = d_b;
  a.ldw = ldb;
  a.b_nmajor = true;
  a.y = d_c;
  a.ldy = ldc;
  return launch_gemm_f32(ctx->stream, a);
}

int ce_gpu_quantize(ce_gpu_ctx *ctx, const float *d_x, int64_t count, uint8_t *d_q, void *d_params) {
  if (!ctx || !d_x || !d_q || !d_params) return fail(CE_GPU_EINVAL, "NULL argument");
  CE_TRY(ensure_scratch(ctx, 1024 * 8));
  return launch_quantize(ctx->stream, d_x, count, d_q, d_params, ctx->scratch.ptr);
}

static int gemm_u8(ce_gpu_ctx *ctx, int m, int n, int k, const uint8_t *d_a, const void *d_pa,
                   const uint8_t *d_b, const void *d_pb, float *d_cf, int32_t *d_ci) {
  if (!ctx || !d_a || !d_pa || !d_b || !d_pb || (!d_cf && !d_ci)) return fail(CE_GPU_EINVAL, "NULL argument");
  if (m <= 0 || n <= 0 || k <= 0) return fail(CE_GPU_EINVAL, "gemm_u8: empty operand (reference asserts)");
  CE_TRY(ensure_scratch(ctx, gemm_u8_scratch_bytes(m, n, k)));
  return launch_gemm_u8_ws(ctx->stream, m, n, k, d_a, d_pa, d_b, d_pb, d_cf, d_ci, ctx->scratch.ptr);
}

int ce_gpu_gemm_u8u8f32(ce_gpu_ctx *ctx, int m, int n, int k, const uint8_t *d_a, const void *d_params_a,
                        const uint8_t *d_b, const void *d_params_b, float *d_c) {
  return gemm_u8(ctx, m, n, k, d_a, d_params_a, d_b, d_params_b, d_c, nullptr);
}

int ce_gpu_gemm_u8u8i32(ce_gpu_ctx *ctx, int m, int n, int k, const uint8_t *d_a, const void *d_params_a,
                        const uint8_t *d_b, const void *d_params_b, int32_t *d_c) {
  return gemm_u8(ctx, m, n, k, d_a, d_params_a, d_b, d_params_b, nullptr, d_c);
}

static_assert(kRowRelu == CE_GPU_ROW_RELU && kRowBatchNorm == CE_GPU_ROW_BATCHNORM &&
                  kRowLogSoftmax == CE_GPU_ROW_LOGSOFTMAX && kRowSoftmax == CE_GPU_ROW_SOFTMAX &&
                  kRowNormalize == CE_GPU_ROW_NORMALIZE,
              "row-op numbering");

int ce_gpu_linear(ce_gpu_ctx *ctx, int rows, int in_dim, int out_dim, const float *d_in, int ld_in,
                  const float *d_w, int ld_w, const float *d_b, float *d_out, int ld_out) {
  if (!ctx || rows < 0 || in_dim < 0 || out_dim < 0) return fail(CE_GPU_EINVAL, "bad argument");
  if (rows == 0 || out_dim == 0) return CE_GPU_OK;
  if (!d_in || !d_w || !d_out) return fail(CE_GPU_EINVAL, "NULL argument");
  if (in_dim == 0) return fail(CE_GPU_EINVAL, "linear: empty input");
  if (ld_in < in_dim || ld_w < out_dim || ld_out < out_dim) return fail(CE_GPU_EINVAL, "leading dimension too small");
  GemmArgs a;
  a.x = d_in;
  a.ldx = ld_in;
  a.m = rows;
  a.n = out_dim;
  a.k = in_dim;
  a.kpad = (in_dim + gemm_k_align() - 1) / gemm_k_align() * gemm_k_align();
  a.din = in_dim;
  a.nseg = 1;
  a.w = d_w;
  a.ldw = ld_w;
  a.b_nmajor = true;
  a.bias = d_b;
  a.y = d_out;
  a.ldy = ld_out;
  ProfScope prof(ctx, CE_GPU_PROF_GEMM_GATHER);
  return launch_gemm_f32(ctx->stream, a);
}

int ce_gpu_splice(ce_gpu_ctx *ctx, int rows, int dim, const float *d_in, int ld_in, const int32_t *h_idx,
                  int n_idx, float *d_out) {
  if (!ctx || rows < 0 || dim < 0 || n_idx < 1 || n_idx > CE_GPU_MAX_SPLICE || !h_idx)
    return fail(CE_GPU_EINVAL, "bad argument");
  if (rows == 0 || dim == 0) return CE_GPU_OK;
  if (!d_in || !d_out || ld_in < dim) return fail(CE_GPU_EINVAL, "bad operand");
  return launch_splice(ctx->stream, rows, dim, d_in, ld_in, h_idx, n_idx, d_out);
}

int ce_gpu_rowwise(ce_gpu_ctx *ctx, int op, int rows, int dim, float *d_x, int ld, const float *d_scale,
                   const float *d_offset) {
  if (!ctx || rows < 0 || dim < 0 || ld < dim) return fail(CE_GPU_EINVAL, "bad argument");
  if (op < CE_GPU_ROW_RELU || op > CE_GPU_ROW_NORMALIZE) return fail(CE_GPU_EINVAL, "unknown row op");
  if (op == CE_GPU_ROW_BATCHNORM && (!d_scale || !d_offset)) return fail(CE_GPU_EINVAL, "BatchNorm needs scale/offset");
  if (rows == 0 || dim == 0) return CE_GPU_OK;
  if (!d_x) return fail(CE_GPU_EINVAL, "NULL argument");
  return launch_rowop_raw(ctx->stream, op, dim, d_scale, d_offset, d_x, ld, rows);
}

int ce_gpu_loglik_gather(ce_gpu_ctx *ctx, const float *d_loglik, int rows, int ld, int dim,
                         const int32_t *d_tid2pdf, int n_tid, const int32_t *d_row, const int32_t *d_trans, int n,
                         float am_scale, float *d_out) {
  if (!ctx || rows < 0 || dim < 0 || ld < dim || n_tid < 0 || n < 0) return fail(CE_GPU_EINVAL, "bad argument");
  if (n == 0) return CE_GPU_OK;
  if (!d_loglik || !d_tid2pdf || !d_row || !d_trans || !d_out) return fail(CE_GPU_EINVAL, "NULL argument");
  CE_HIP(hipSetDevice(ctx->device));
  return launch_loglik_gather(ctx->stream, d_loglik, rows, ld, dim, d_tid2pdf, n_tid, d_row, d_trans, n, am_scale, d_out);
}

int ce_gpu_loglik_columns(ce_gpu_ctx *ctx, const float *d_loglik, int rows, int ld, int dim,
                          const int32_t *d_cols, int n_cols, float *d_out) {
  if (!ctx || rows < 0 || dim < 0 || ld < dim || n_cols < 0) return fail(CE_GPU_EINVAL, "bad argument");
  if (rows == 0 || n_cols == 0) return CE_GPU_OK;
  if (!d_loglik || !d_cols || !d_out) return fail(CE_GPU_EINVAL, "NULL argument");
  CE_HIP(hipSetDevice(ctx->device));
  return launch_loglik_columns(ctx->stream, d_loglik, rows, ld, dim, d_cols, n_cols, d_out);
}

int ce_gpu_sum_f64(void *stream, const float *d_x, int64_t n, double *d_part, double *d_acc) {
  return ce_gpu_sum_f64_many(stream, 1, &d_x, &n, d_part, d_acc);
}

int ce_gpu_sum_f64_many(void *stream, int count, const float *const *d_x, const int64_t *n, double *d_part,
                        double *d_acc) {
  if (count < 0 || count > CE_GPU_SUM_MAX_BUFS || (count > 0 && (!d_x || !n)))
    return fail(CE_GPU_EINVAL, "sum_f64: bad buffer list");
  bool any = false;
  for (int k = 0; k < count; ++k) {
    if (n[k] < 0) return fail(CE_GPU_EINVAL, "bad argument");
    if (n[k] > 0 && !d_x[k]) return fail(CE_GPU_EINVAL, "NULL argument");
    any = any || n[k] > 0;
  }
  if (!any) return CE_GPU_OK;
  if (!d_part || !d_acc) return fail(CE_GPU_EINVAL, "NULL argument");
  return launch_sum_f64(reinterpret_cast<hipStream_t>(stream), count, d_x, n, d_part, d_acc);
}

int ce_gpu_model_quantize(ce_gpu_ctx *ctx, ce_gpu_model *m) {
  if (!ctx || !m) return fail(CE_GPU_EINVAL, "NULL argument");
  if (m->int8) return CE_GPU_OK;
  CE_HIP(hipSetDevice(ctx->device));
  for (Step &st : m->steps)
    if (st.is_gemm) CE_TRY(quantize_weights(ctx, st));
  m->int8 = true;
  return CE_GPU_OK;
}

}  // extern "C"
