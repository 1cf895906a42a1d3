// mfma_rate_probe.hip -- MFMA throughput per instruction kind on gfx950:
// every CU runs 4 waves (one per SIMD), each a back-to-back chain over 4
// independent accumulators in registers (no memory in the loop); reports
// TOP/s and cycles per MFMA at the measured clock (s_memtime ticks).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_rate_probe.hip -o /tmp/mrp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void rate(int seed, int *out, long long *ticks) {
  const int lane = threadIdx.x & 63;
  long long t0 = __builtin_readcyclecounter();
  if constexpr (KIND == 0) {  // v_mfma_i32_32x32x32_i8
    i32x4 a = {seed + lane, lane, 3, 4}, b = {lane, seed, 5, 6};
    i32x16 acc[4] = {};
    for (int it = 0; it < kIters; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[q], 0, 0, 0);
    int s = 0;
    for (int q = 0; q < 4; ++q)
      for (int e = 0; e < 16; ++e) s += acc[q][e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if constexpr (KIND == 1) {  // v_mfma_i32_16x16x64_i8
    i32x4 a = {seed + lane, lane, 3, 4}, b = {lane, seed, 5, 6};
    i32x4 acc[4] = {};
    for (int it = 0; it < kIters; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[q], 0, 0, 0);
    int s = 0;
    for (int q = 0; q < 4; ++q)
      for (int e = 0; e < 4; ++e) s += acc[q][e];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else if constexpr (KIND == 2) {  // v_mfma_f32_16x16x32_bf16
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
      a[e] = (__bf16)(float)(lane + e + seed);
      b[e] = (__bf16)(float)(e - lane);
    }
    f32x4 acc[4] = {};
    for (int it = 0; it < kIters; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[q], 0, 0, 0);
    float s = 0;
    for (int q = 0; q < 4; ++q)
      for (int e = 0; e < 4; ++e) s += acc[q][e];
    out[blockIdx.x * 256 + threadIdx.x] = (int)s;
  }
  long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char *name, double ops_per_mfma, int cus) {
  int *out;
  long long *ticks;
  CK(hipMalloc(&out, cus * 256 * sizeof(int)));
  CK(hipMalloc(&ticks, cus * sizeof(long long)));
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  hipLaunchKernelGGL(rate<KIND>, dim3(cus), dim3(256), 0, 0, 1, out, ticks);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(rate<KIND>, dim3(cus), dim3(256), 0, 0, 2, out, ticks);
  CK(hipEventRecord(z, 0));
  CK(hipEventSynchronize(z));
  float ms;
  CK(hipEventElapsedTime(&ms, a, z));
  long long t = 0;
  CK(hipMemcpy(&t, ticks, sizeof(t), hipMemcpyDeviceToHost));
  const double n = (double)cus * 4 * kIters * 4;  // MFMAs
  printf("%-28s %8.1f TOP/s   %6.1f cycles/MFMA per SIMD (counter ticks)   %.3f ms\n", name,
         n * ops_per_mfma / (ms * 1e-3) / 1e12, (double)t / (kIters * 4), ms);
  CK(hipFree(out));
  CK(hipFree(ticks));
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  run<0>("mfma_i32_32x32x32_i8", 2.0 * 32 * 32 * 32, cus);
  run<1>("mfma_i32_16x16x64_i8", 2.0 * 16 * 16 * 64, cus);
  run<2>("mfma_f32_16x16x32_bf16", 2.0 * 16 * 16 * 32, cus);
  printf("ok\n");
  return 0;
}
