// rowops.hip -- per-row kernels of the nnet path.
//
// finalize: LogSoftmaxLayer (src/nnet.cc:137-146 -> ApplyLogSoftMax,
//   src/vector.cc:109-122: x - log(sum exp x), no max shift) fused with the
//   log-prior subtraction of AcousticModel::ComputeBatch (src/am.cc:108-112)
//   and the scatter of valid packed rows to their utterance's output rows.
//   One block (vector form) or one wave per row; the row is read once into
//   registers.
// rowop: stand-alone ReLU / BatchNorm / Softmax / LogSoftmax / Normalize for
//   layers that do not directly follow a LinearLayer (never emitted by the
//   reference's converter, but legal NN02).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "../internal.h"

namespace catears {
namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

constexpr int kMaxPerLane = 64;  // rows up to 4096 wide stay in registers

template <bool LOGSM>
__global__ __launch_bounds__(256) void finalize_kernel(const float *__restrict__ x, int ldx, int rows,
                                                       int dim, const float *__restrict__ prior,
                                                       const int *__restrict__ row_dst,
                                                       float *__restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int dst = row_dst ? row_dst[row] : row;
  if (dst < 0) return;
  const float *xr = x + (int64_t)row * ldx;
  float *o = out + (int64_t)dst * dim;
  if (dim <= 64 * kMaxPerLane) {
    float v[kMaxPerLane];
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kMaxPerLane; ++j) {
      const int c = lane + 64 * j;
      v[j] = c < dim ? xr[c] : 0.0f;
      if (LOGSM && c < dim) s += expf(v[j]);
    }
    const float ls = LOGSM ? logf(wave_sum(s)) : 0.0f;
#pragma unroll
    for (int j = 0; j < kMaxPerLane; ++j) {
      const int c = lane + 64 * j;
      if (c < dim) {
        float y = v[j];
        if (LOGSM) y = y - ls;
        o[c] = prior ? y - prior[c] : y;
      }
    }
  } else {
    float s = 0.0f;
    if (LOGSM)
      for (int c = lane; c < dim; c += 64) s += expf(xr[c]);
    const float ls = LOGSM ? logf(wave_sum(s)) : 0.0f;
    for (int c = lane; c < dim; c += 64) {
      float y = xr[c];
      if (LOGSM) y = y - ls;
      o[c] = prior ? y - prior[c] : y;
    }
  }
}

// The same with 16-byte accesses (dim, ldx multiples of 4, aligned rows),
// one 256-thread block per row: thread t holds float4 chunks t, t + 256, ...
// of its row (up to 4096 wide), everything loaded up front; the exp sum is
// per thread in chunk order, then per wave (xor tree), then the four waves'
// sums in wave order.  A function of the row alone, not of the row count.
constexpr int kMaxVecPerThread = 4;

template <bool LOGSM>
__global__ __launch_bounds__(256) void finalize_vec_kernel(const float *__restrict__ x, int ldx, int rows, int dim,
                                                           const float *__restrict__ prior,
                                                           const int *__restrict__ row_dst,
                                                           float *__restrict__ out) {
  __shared__ float wsum[4];
  const int row = blockIdx.x, t = threadIdx.x;
  const int dst = row_dst ? row_dst[row] : row;
  if (dst < 0) return;
  const float4 *xr = reinterpret_cast<const float4 *>(x + (int64_t)row * ldx);
  const float4 *pr = reinterpret_cast<const float4 *>(prior);
  float4 *o = reinterpret_cast<float4 *>(out + (int64_t)dst * dim);
  const int d4 = dim >> 2;
  float4 v[kMaxVecPerThread], pv[kMaxVecPerThread];
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < kMaxVecPerThread; ++j) {
    const int c = min(t + 256 * j, d4 - 1);  // clamped: loads branch-free, used only when in range
    v[j] = xr[c];
    if (prior) pv[j] = pr[c];
  }
  if (LOGSM) {
#pragma unroll
    for (int j = 0; j < kMaxVecPerThread; ++j)
      if (t + 256 * j < d4) s += expf(v[j].x) + expf(v[j].y) + expf(v[j].z) + expf(v[j].w);
    s = wave_sum(s);
    if ((t & 63) == 0) wsum[t >> 6] = s;
    __syncthreads();
    s = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
  }
  const float ls = LOGSM ? logf(s) : 0.0f;
#pragma unroll
  for (int j = 0; j < kMaxVecPerThread; ++j) {
    const int c = t + 256 * j;
    if (c < d4) {
      float4 y = v[j];
      if (LOGSM) y = make_float4(y.x - ls, y.y - ls, y.z - ls, y.w - ls);
      if (prior) y = make_float4(y.x - pv[j].x, y.y - pv[j].y, y.z - pv[j].z, y.w - pv[j].w);
      o[c] = y;
    }
  }
}

__global__ __launch_bounds__(256) void rowop_kernel(int kind, float *__restrict__ x, int ldx, int rows,
                                                    int dim, const float *__restrict__ scale,
                                                    const float *__restrict__ offset) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  float *xr = x + (int64_t)row * ldx;
  switch (kind) {
    case kRowRelu:  // nnet.cc:149-160
      for (int c = lane; c < dim; c += 64) xr[c] = xr[c] < 0.0f ? 0.0f : xr[c];
      break;
    case kRowBatchNorm:  // nnet.cc:106-117: MulElements then AddVec(1.0)
      for (int c = lane; c < dim; c += 64) {
        float v = xr[c] * scale[c];
        xr[c] = v + offset[c];
      }
      break;
    case kRowLogSoftmax: {  // vector.cc:109-122
      float s = 0.0f;
      for (int c = lane; c < dim; c += 64) s += expf(xr[c]);
      const float ls = logf(wave_sum(s));
      for (int c = lane; c < dim; c += 64) xr[c] = xr[c] - ls;
      break;
    }
    case kRowSoftmax: {  // vector.cc:94-107
      float s = 0.0f;
      for (int c = lane; c < dim; c += 64) s += expf(xr[c]);
      s = wave_sum(s);
      for (int c = lane; c < dim; c += 64) xr[c] = expf(xr[c]) / s;
      break;
    }
    case kRowNormalize: {  // nnet.cc:163-178
      float s = 0.0f;
      for (int c = lane; c < dim; c += 64) s += xr[c] * xr[c];
      s = wave_sum(s);
      const float sc = (float)sqrt((double)(float)dim / (double)s);
      for (int c = lane; c < dim; c += 64) xr[c] = xr[c] * sc;
      break;
    }
    default:
      break;
  }
}

// SpliceLayer::Propagate (src/nnet.cc:50-95): out[t] = concat over s of
// in[clamp(t + idx[s], 0, rows - 1)].  One block per output row; a pure copy.
struct SpliceIdx {
  int v[CE_GPU_MAX_SPLICE];
};

__global__ __launch_bounds__(256) void splice_kernel(int rows, int dim, const float *__restrict__ in, int ld_in,
                                                     SpliceIdx idx, int n_idx, float *__restrict__ out) {
  const int t = blockIdx.x;
  const int width = dim * n_idx;
  float *o = out + (int64_t)t * width;
  for (int c = threadIdx.x; c < width; c += blockDim.x) {
    const int s = c / dim, j = c - s * dim;
    int src = t + idx.v[s];
    src = src < 0 ? 0 : (src > rows - 1 ? rows - 1 : src);
    o[c] = in[(int64_t)src * ld_in + j];
  }
}

__global__ __launch_bounds__(256) void splice_pad_kernel(const float *__restrict__ in, int ld_in, int rows, int din,
                                                         int nseg, SpliceIdx idx, const int *__restrict__ row_map,
                                                         float *__restrict__ out, int ldo) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  float *o = out + (int64_t)r * ldo;
  for (int c = lane; c < ldo; c += 64) {
    const int s = c / din;
    float v = 0.0f;
    if (s < nseg) {
      int src = r + idx.v[s];
      src = src < 0 ? 0 : (src > rows - 1 ? rows - 1 : src);
      if (row_map) src = row_map[src];
      v = in[(int64_t)src * ld_in + (c - s * din)];
    }
    o[c] = v;
  }
}

}  // namespace

int launch_splice_pad(hipStream_t s, const float *in, int ld_in, int rows, int din, int nseg, const int *off,
                      const int *row_map, float *out, int ldo) {
  SpliceIdx idx = {};
  for (int i = 0; i < nseg && i < CE_GPU_MAX_SPLICE; ++i) idx.v[i] = off[i];
  if (rows > 0)
    hipLaunchKernelGGL(splice_pad_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, in, ld_in, rows, din, nseg, idx,
                       row_map, out, ldo);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int launch_splice(hipStream_t s, int rows, int dim, const float *in, int ld_in, const int32_t *h_idx,
                  int n_idx, float *out) {
  SpliceIdx idx = {};
  for (int i = 0; i < n_idx; ++i) idx.v[i] = h_idx[i];
  hipLaunchKernelGGL(splice_kernel, dim3(rows), dim3(256), 0, s, rows, dim, in, ld_in, idx, n_idx, out);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}


int launch_finalize(hipStream_t s, const float *x, int ldx, int rows, int dim, bool log_softmax,
                    const float *log_prior, const int *row_dst, float *out) {
  if (rows <= 0) return CE_GPU_OK;
  dim3 grid((rows + 3) / 4), block(256);
  const bool vec = dim % 4 == 0 && ldx % 4 == 0 && dim <= 4 * 256 * kMaxVecPerThread &&
                   ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                     reinterpret_cast<uintptr_t>(log_prior)) & 15) == 0;
  if (vec) {
    if (log_softmax)
      hipLaunchKernelGGL(finalize_vec_kernel<true>, dim3(rows), block, 0, s, x, ldx, rows, dim, log_prior, row_dst,
                         out);
    else
      hipLaunchKernelGGL(finalize_vec_kernel<false>, dim3(rows), block, 0, s, x, ldx, rows, dim, log_prior, row_dst,
                         out);
    CE_HIP(hipGetLastError());
    return CE_GPU_OK;
  }
  if (log_softmax)
    hipLaunchKernelGGL(finalize_kernel<true>, grid, block, 0, s, x, ldx, rows, dim, log_prior,
                       row_dst, out);
  else
    hipLaunchKernelGGL(finalize_kernel<false>, grid, block, 0, s, x, ldx, rows, dim, log_prior,
                       row_dst, out);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int launch_rowop_raw(hipStream_t s, int kind, int dim, const float *scale, const float *offset, float *x,
                     int ldx, int rows) {
  if (rows <= 0) return CE_GPU_OK;
  hipLaunchKernelGGL(rowop_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, kind, x, ldx, rows, dim, scale,
                     offset);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

namespace {

// One (frame, transition id) pair per thread: two dependent 4-byte reads
// (the map, then the loglik element) -- latency, not bandwidth, so a wide
// grid of small blocks.
__global__ __launch_bounds__(256) void loglik_gather_kernel(const float *__restrict__ ll, int rows, int ld, int dim,
                                                            const int32_t *__restrict__ tpm, int n_tid,
                                                            const int32_t *__restrict__ row,
                                                            const int32_t *__restrict__ trans, int n, float scale,
                                                            float *__restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int r = row[i], t = trans[i];
  float v = __builtin_nanf("");
  if (r >= 0 && r < rows && t >= 0 && t < n_tid) {
    const int p = tpm[t];
    if (p >= 0 && p < dim) v = scale * ll[(int64_t)r * ld + p];
  }
  out[i] = v;
}

// out row r = the selected columns of ll row r; a block per row, the column
// list read once per block into registers.
__global__ __launch_bounds__(256) void loglik_columns_kernel(const float *__restrict__ ll, int ld, int dim,
                                                             const int32_t *__restrict__ cols, int n_cols,
                                                             float *__restrict__ out) {
  const int r = blockIdx.x;
  const float *src = ll + (int64_t)r * ld;
  float *dst = out + (int64_t)r * n_cols;
  for (int j = threadIdx.x; j < n_cols; j += 256) {
    const int c = cols[j];
    dst[j] = (c >= 0 && c < dim) ? src[c] : __builtin_nanf("");
  }
}

}  // namespace

int launch_loglik_gather(hipStream_t s, const float *ll, int rows, int ld, int dim, const int32_t *tpm, int n_tid,
                         const int32_t *row, const int32_t *trans, int n, float scale, float *out) {
  if (n > 0)
    hipLaunchKernelGGL(loglik_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ll, rows, ld, dim, tpm, n_tid, row,
                       trans, n, scale, out);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int launch_loglik_columns(hipStream_t s, const float *ll, int rows, int ld, int dim, const int32_t *cols,
                          int n_cols, float *out) {
  if (rows > 0 && n_cols > 0)
    hipLaunchKernelGGL(loglik_columns_kernel, dim3(rows), dim3(256), 0, s, ll, ld, dim, cols, n_cols, out);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

namespace {

// Float64 sum of up to kSumMaxBufs float buffers (ce_gpu_sum_f64 /
// ce_gpu_sum_f64_many): each thread adds its strided float4s of every
// buffer in double -- four accumulators, one per load slot, so four loads are
// in flight per thread -- then a fixed wave / block tree, one partial per
// block, and one wave folds the partials in block order.  The order depends
// on the buffer sizes, on each buffer's 16-byte alignment (float4 or scalar
// path) and on the list of buffers folded together (shared accumulators, a
// grid sized by the largest): the same buffers at the same alignments give
// the same double (include/catears_gpu.h).  Several buffers share one launch
// pair (rank 0 folds every peer's rows of a step at once).
constexpr int kSumThreads = 256;
constexpr int kSumMaxBufs = 16;

struct SumBufs {
  const float *x[kSumMaxBufs];
  int64_t n[kSumMaxBufs];
  int count;
};

__global__ __launch_bounds__(kSumThreads) void sum_f64_kernel(SumBufs bufs, double *__restrict__ part) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kSumThreads, t = (int64_t)blockIdx.x * kSumThreads + threadIdx.x;
  for (int k = 0; k < bufs.count; ++k) {
    const float *x = bufs.x[k];
    const int64_t n = bufs.n[k];
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {  // uniform per buffer
      const float4 *x4 = reinterpret_cast<const float4 *>(x);
      const int64_t n4 = n >> 2;
      int64_t i = t;
      for (; i + 3 * stride < n4; i += 4 * stride) {
        const float4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
        s0 += (((double)a.x + (double)a.y) + (double)a.z) + (double)a.w;
        s1 += (((double)b.x + (double)b.y) + (double)b.z) + (double)b.w;
        s2 += (((double)c.x + (double)c.y) + (double)c.z) + (double)c.w;
        s3 += (((double)d.x + (double)d.y) + (double)d.z) + (double)d.w;
      }
      for (; i < n4; i += stride) {
        const float4 a = x4[i];
        s0 += (((double)a.x + (double)a.y) + (double)a.z) + (double)a.w;
      }
      if (t < (n & 3)) s1 += (double)x[(n4 << 2) + t];
    } else {
      for (int64_t i = t; i < n; i += stride) s0 += (double)x[i];
    }
  }
  double s = (s0 + s1) + (s2 + s3);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  __shared__ double ws[kSumThreads / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

__global__ __launch_bounds__(64) void sum_parts_kernel(const double *__restrict__ part, int nparts,
                                                       double *__restrict__ acc) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (threadIdx.x == 0) *acc += s;
}

}  // namespace

int launch_sum_f64(hipStream_t s, int count, const float *const *x, const int64_t *n, double *part, double *acc) {
  if (count < 0 || count > kSumMaxBufs) return fail(CE_GPU_EINVAL, "sum_f64: 0..16 buffers per call");
  SumBufs b{};
  int64_t units = 0;
  for (int k = 0; k < count; ++k) {
    if (n[k] <= 0) continue;
    b.x[b.count] = x[k];
    b.n[b.count] = n[k];
    ++b.count;
    units = std::max<int64_t>(units, n[k] >> 2);
  }
  if (b.count == 0) return CE_GPU_OK;
  // (128 or 32 blocks measured no better beside the GEMMs, profiles/r05t_rank0_rehearsal.txt)
  const int64_t want = (std::max<int64_t>(units, 1) + 4 * kSumThreads - 1) / (4 * kSumThreads);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(want, CE_GPU_SUM_PARTS));
  hipLaunchKernelGGL(sum_f64_kernel, dim3(blocks), dim3(kSumThreads), 0, s, b, part);
  CE_HIP(hipGetLastError());
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(64), 0, s, part, blocks, acc);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

int launch_rowop(hipStream_t s, const RowOp &op, float *x, int ldx, int rows) {
  return launch_rowop_raw(s, op.kind, op.dim, op.scale.as<float>(), op.offset.as<float>(), x, ldx, rows);
}

namespace {
// ce_gpu_trace_mark: a kernel that does nothing, seen by a kernel trace under
// its name with `tag` workgroups (the window markers of bench.py's timed steps)
__global__ __launch_bounds__(64) void trace_mark_kernel() {}
}  // namespace

int launch_trace_mark(hipStream_t s, int tag) {
  hipLaunchKernelGGL(trace_mark_kernel, dim3(tag), dim3(64), 0, s);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
