// quant.hip -- the int8 path: Quantize (src/matrix.cc:329-387) and
// MatMat_U8U8F32 (src/matrix.cc:389-420 -> gemmlowp EightBitIntGemm,
// src/gemmlowp/eight_bit_int_gemm/eight_bit_int_gemm.cc:338-400).
//
// Quantize = min/max reduction (order-independent, so exact) -> parameters in
// double exactly as ComputeQuantizationParams -> elementwise
// roundf(clamp(x / scale + zp, 0, 255)).  Bit-identical to the reference.
//
// The u8 x u8 GEMM runs on CDNA4's signed v_mfma_i32_32x32x32_i8: operands are
// shifted to s8 (a - 128, a byte XOR) and the zero points are restored in the
// int32 epilogue:
//   sum_k (a - zpA)(b - zpB) = sum a'b' + cB*rowsum(a') + cA*colsum(b') + K*cA*cB
// with a' = a - 128, cA = 128 - zpA (likewise B).  Every term is int32 modulo
// 2^32 -- the same ring gemmlowp's int32 accumulator lives in -- so the int32
// result is bit-exact for any K.  B is transposed once per call into the
// context scratch (K-contiguous columns) so both operands load as 16-byte
// vectors; tiles are 128 x 128 x 64 bytes, 4 waves of 2 x 2 MFMA 32x32x32.
#include <float.h>
#include <hip/hip_runtime.h>

#include "../internal.h"

namespace catears {
namespace {

struct QParams {
  float scale;
  int32_t zp;
};

constexpr int kRedBlocks = 1024;

__global__ __launch_bounds__(256) void minmax_kernel(const float *__restrict__ x, int64_t n,
                                                     float2 *__restrict__ part) {
  float mn = FLT_MAX, mx = FLT_MIN;  // matrix.cc:331-332: max starts at FLT_MIN
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i];
    mx = v > mx ? v : mx;
    mn = v < mn ? v : mn;
  }
  __shared__ float smn[256], smx[256];
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smn[threadIdx.x] = fminf(smn[threadIdx.x], smn[threadIdx.x + s]);
      smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = make_float2(smn[0], smx[0]);
}

__global__ __launch_bounds__(256) void qparams_kernel(const float2 *__restrict__ part, int nparts,
                                                      QParams *__restrict__ out) {
  __shared__ float smn[256], smx[256];
  float mn = FLT_MAX, mx = FLT_MIN;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    mn = fminf(mn, part[i].x);
    mx = fmaxf(mx, part[i].y);
  }
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smn[threadIdx.x] = fminf(smn[threadIdx.x], smn[threadIdx.x + s]);
      smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // ComputeQuantizationParams (matrix.cc:348-362)
    const float lo = smn[0], hi = smx[0];
    const double scale = (hi - lo) / 255.0;
    const double fzp = -lo / scale;
    out->zp = (int32_t)round(fzp);
    out->scale = (float)scale;
  }
}

__global__ __launch_bounds__(256) void quantize_kernel(const float *__restrict__ x, int64_t n,
                                                       const QParams *__restrict__ prm,
                                                       uint8_t *__restrict__ q) {
  const float scale = prm->scale;
  const float zp = (float)prm->zp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float v = x[i] / scale + zp;
    v = (255.0f < v) ? 255.0f : v;  // std::min(v, 255.0f)  (NaN stays NaN)
    v = (0.0f < v) ? v : 0.0f;      // std::max(0.0f, v)     (NaN -> 0)
    q[i] = (uint8_t)roundf(v);
  }
}

// B (k x n, row-major u8) -> Bt (n x kpad, s8 = b - 128, zero padded) and
// colsum(b') per column.
__global__ __launch_bounds__(256) void transpose_b_kernel(const uint8_t *__restrict__ b, int k, int n,
                                                          int kpad, int8_t *__restrict__ bt,
                                                          int32_t *__restrict__ colsum) {
  __shared__ uint8_t tile[64][65];
  const int n0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int kk = k0 + r, nn = n0 + tx;
    tile[r][tx] = (kk < k && nn < n) ? b[(int64_t)kk * n + nn] : (uint8_t)128;  // pad -> s8 0
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int nn = n0 + r, kk = k0 + tx;
    if (nn < n && kk < kpad) bt[(int64_t)nn * kpad + kk] = (int8_t)(tile[tx][r] ^ 0x80);
  }
  if (threadIdx.x < 64) {
    const int nn = n0 + threadIdx.x;
    int32_t s = 0;
    for (int r = 0; r < 64; ++r) s += (int32_t)tile[r][threadIdx.x] - 128;
    if (nn < n) atomicAdd(colsum + nn, s);
  }
}

// A (m x k u8) -> rowsum(a') per row.
__global__ __launch_bounds__(256) void rowsum_a_kernel(const uint8_t *__restrict__ a, int m, int k,
                                                       int32_t *__restrict__ rowsum) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= m) return;
  int32_t s = 0;
  for (int c = lane; c < k; c += 64) s += (int32_t)a[(int64_t)row * k + c] - 128;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (lane == 0) rowsum[row] = s;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int QBM = 128, QBN = 128, QBK = 64, QLD = QBK + 16;  // bytes

__global__ __launch_bounds__(256, 2) void gemm_i8_kernel(const uint8_t *__restrict__ a, int m, int k,
                                                         const int8_t *__restrict__ bt, int n, int kpad,
                                                         const int32_t *__restrict__ rowsum,
                                                         const int32_t *__restrict__ colsum,
                                                         const QParams *__restrict__ pa,
                                                         const QParams *__restrict__ pb, int tiles_n,
                                                         float *__restrict__ cf, int32_t *__restrict__ ci) {
  __shared__ __attribute__((aligned(16))) int8_t As[QBM * QLD];
  __shared__ __attribute__((aligned(16))) int8_t Bs[QBN * QLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, r = lane & 31, h = lane >> 5;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int m0 = tm * QBM, n0 = tn * QBN;
  const bool a_vec = (k % 16) == 0 && ((reinterpret_cast<uintptr_t>(a) & 15) == 0);

  i32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  for (int k0 = 0; k0 < kpad; k0 += QBK) {
    // A tile: 128 rows x 64 bytes = 512 x 16 B -> 2 per thread
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, row = idx >> 2, c16 = idx & 3;
      const int gr = min(m0 + row, m - 1), gk = k0 + 16 * c16;
      i32x4 v;
      if (a_vec && gk + 16 <= k) {
        v = *reinterpret_cast<const i32x4 *>(a + (int64_t)gr * k + gk);
        v ^= (i32x4){(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
      } else {
        uint8_t tmp[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) tmp[e] = gk + e < k ? (uint8_t)(a[(int64_t)gr * k + gk + e] ^ 0x80) : 0;
        v = *reinterpret_cast<const i32x4 *>(tmp);
      }
      *reinterpret_cast<i32x4 *>(As + row * QLD + 16 * c16) = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, row = idx >> 2, c16 = idx & 3;
      const int gn = min(n0 + row, n - 1);
      *reinterpret_cast<i32x4 *>(Bs + row * QLD + 16 * c16) =
          *reinterpret_cast<const i32x4 *>(bt + (int64_t)gn * kpad + k0 + 16 * c16);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < QBK / 32; ++s) {
      i32x4 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const i32x4 *>(As + (wm * 64 + i * 32 + r) * QLD + 32 * s + 16 * h);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *reinterpret_cast<const i32x4 *>(Bs + (wn * 64 + j * 32 + r) * QLD + 32 * s + 16 * h);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  const uint32_t ca = (uint32_t)(128 - pa->zp), cb = (uint32_t)(128 - pb->zp);
  const uint32_t kterm = (uint32_t)k * ca * cb;
  const float cscale = pa->scale * pb->scale;  // matrix.cc:405
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + j * 32 + r;
    if (col >= n) continue;
    const uint32_t csum = (uint32_t)colsum[col];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row >= m) continue;
        const uint32_t v = (uint32_t)acc[i][j][e] + cb * (uint32_t)rowsum[row] + ca * csum + kterm;
        if (ci) ci[(int64_t)row * n + col] = (int32_t)v;
        if (cf) cf[(int64_t)row * n + col] = (float)(int32_t)v * cscale;
      }
  }
}

}  // namespace

int launch_quantize(hipStream_t s, const float *x, int64_t count, uint8_t *q, void *params, void *scratch) {
  if (count <= 0) return fail(CE_GPU_EINVAL, "quantize: empty input (reference asserts)");
  const int blocks = (int)std::min<int64_t>(kRedBlocks, (count + 255) / 256);
  float2 *part = static_cast<float2 *>(scratch);
  hipLaunchKernelGGL(minmax_kernel, dim3(blocks), dim3(256), 0, s, x, count, part);
  hipLaunchKernelGGL(qparams_kernel, dim3(1), dim3(256), 0, s, part, blocks, static_cast<QParams *>(params));
  const int qb = (int)std::min<int64_t>(4096, (count + 255) / 256);
  hipLaunchKernelGGL(quantize_kernel, dim3(qb), dim3(256), 0, s, x, count,
                     static_cast<const QParams *>(params), q);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

size_t gemm_u8_scratch_bytes(int m, int n, int k) {
  const size_t kpad = (size_t)(k + QBK - 1) / QBK * QBK;
  return (size_t)n * kpad + 4 * ((size_t)m + n) + 256;
}

int launch_gemm_u8_ws(hipStream_t s, int m, int n, int k, const uint8_t *a, const void *pa, const uint8_t *b,
                      const void *pb, float *c_f32, int32_t *c_i32, void *ws) {
  if (m <= 0 || n <= 0 || k <= 0) return fail(CE_GPU_EINVAL, "gemm_u8: empty operand");
  const int kpad = (k + QBK - 1) / QBK * QBK;
  int8_t *bt = static_cast<int8_t *>(ws);
  const size_t bt_bytes = ((size_t)n * kpad + 255) / 256 * 256;
  int32_t *colsum = reinterpret_cast<int32_t *>(static_cast<char *>(ws) + bt_bytes);
  int32_t *rowsum = colsum + n;
  CE_HIP(hipMemsetAsync(colsum, 0, sizeof(int32_t) * n, s));
  hipLaunchKernelGGL(transpose_b_kernel, dim3((n + 63) / 64, kpad / 64), dim3(256), 0, s, b, k, n, kpad, bt,
                     colsum);
  hipLaunchKernelGGL(rowsum_a_kernel, dim3((m + 3) / 4), dim3(256), 0, s, a, m, k, rowsum);
  const int tiles_n = (n + QBN - 1) / QBN, tiles_m = (m + QBM - 1) / QBM;
  hipLaunchKernelGGL(gemm_i8_kernel, dim3(tiles_m * tiles_n), dim3(256), 0, s, a, m, k, bt, n, kpad, rowsum,
                     colsum, static_cast<const QParams *>(pa), static_cast<const QParams *>(pb), tiles_n,
                     c_f32, c_i32);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
