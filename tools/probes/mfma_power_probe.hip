// mfma_power_probe.hip -- sustained bf16 MFMA rate on the whole chip, with
// operands that change from one MFMA to the next (four random operand sets
// per wave, cycled), for the two bf16 shapes gfx950 offers:
//   v_mfma_f32_16x16x32_bf16 (the bf16x6 GEMM's) and v_mfma_f32_32x32x16_bf16
//   (twice the products per operand register read).
// Every CU runs 8 waves (two per SIMD, as the GEMM does), a chain over four
// independent accumulators.  Each kind first runs ~0.6 s to reach the power-
// capped clock, then ~0.4 s is timed.  The question it answers: under the
// socket power cap, does the larger shape sustain a higher rate?
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_power_probe.hip -o /tmp/mpp
#include <hip/hip_runtime.h>

#include <chrono>
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

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 2048;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

template <int KIND>
__global__ __launch_bounds__(512) void rate(int seed, float *out) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[4];
  for (int q = 0; q < 4; ++q)
    for (int e = 0; e < 8; ++e) {
      const uint32_t h = mix(seed * 7919u + blockIdx.x * 4099u + threadIdx.x * 131u + q * 17u + e);
      a[q][e] = (__bf16)((float)(h & 0xffff) * (1.0f / 65536.0f) - 0.5f);
      b[q][e] = (__bf16)((float)(h >> 16) * (1.0f / 65536.0f) - 0.5f);
    }
  float s = 0;
  if constexpr (KIND == 0) {  // v_mfma_f32_16x16x32_bf16
    f32x4 acc[4] = {};
    for (int it = 0; it < kIters; it += 4)  // operand indices compile-time (no scratch)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[q], b[(q + j) & 3], acc[q], 0, 0, 0);
    for (int q = 0; q < 4; ++q)
      for (int e = 0; e < 4; ++e) s += acc[q][e];
  } else {  // v_mfma_f32_32x32x16_bf16
    f32x16 acc[4] = {};
    for (int it = 0; it < kIters; it += 4)  // operand indices compile-time (no scratch)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q], b[(q + j) & 3], acc[q], 0, 0, 0);
    for (int q = 0; q < 4; ++q)
      for (int e = 0; e < 16; ++e) s += acc[q][e];
  }
  out[blockIdx.x * 512 + threadIdx.x] = s;
  (void)lane;
}

template <int KIND>
void run(const char *name, double flops_per_mfma, int cus) {
  float *out;
  CK(hipMalloc(&out, (size_t)cus * 512 * sizeof(float)));
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  // warm: ~0.6 s of launches
  auto t0 = std::chrono::steady_clock::now();
  int launches = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.6) {
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(rate<KIND>, dim3(cus), dim3(512), 0, 0, i, out);
    CK(hipDeviceSynchronize());
    launches += 20;
  }
  // timed: the launch count that took ~0.4 s of the warm phase
  const int n = launches * 2 / 3 + 1;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(rate<KIND>, dim3(cus), dim3(512), 0, 0, i, out);
  CK(hipEventRecord(z, 0));
  CK(hipEventSynchronize(z));
  float ms;
  CK(hipEventElapsedTime(&ms, a, z));
  const double mfmas = (double)n * cus * 8 * kIters * 4;
  printf("%-26s %8.1f TFLOP/s sustained over %.0f ms (%d launches)\n", name,
         mfmas * flops_per_mfma / (ms * 1e-3) / 1e12, ms, n);
  CK(hipFree(out));
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  for (int r = 0; r < 2; ++r) {
    run<0>("mfma_f32_16x16x32_bf16", 2.0 * 16 * 16 * 32, cus);
    run<1>("mfma_f32_32x32x16_bf16", 2.0 * 32 * 32 * 16, cus);
  }
  printf("ok\n");
  return 0;
}
