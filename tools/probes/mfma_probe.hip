// mfma_probe.hip -- ablation microbenchmark for the fp32 MFMA GEMM loop
// (development tool, not part of the product).  Each mode adds one piece of
// the real kernel: registers only -> LDS fragment reads -> barrier per tile
// -> global loads + LDS stores.  256 blocks x 256 threads, 96 K-tiles of 64
// MFMAs per wave (the K=3072, N=1024 layer on 128x128 tiles).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// MODE 4: as MODE 0 but the register operands are random data (MFMA power --
// and therefore clock -- depends on operand bits).  Block 0 records its
// s_memtime span so the effective shader clock can be derived.
__device__ unsigned long long g_cycles;

template <int MODE>
__global__ __launch_bounds__(256) void probe(const float *__restrict__ g, float *out, int ktiles) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  __shared__ __attribute__((aligned(16))) float smem[2 * 256 * 36];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  for (int i = tid; i < 2 * 256 * 36; i += 256) smem[i] = g[(i * 2654435761u + blockIdx.x) % (65536 * 32)];
  __syncthreads();
  f32x16 acc[2][2] = {};
  f32x4 st[8];
  f32x4 fa[2], fb[2];
  fa[0] = fa[1] = fb[0] = fb[1] = (f32x4){1.0f, 2.0f, 3.0f, 4.0f};
  if (MODE == 4) {
    fa[0] = *reinterpret_cast<const f32x4 *>(g + (tid * 16 + blockIdx.x * 4096) % (65536 * 32));
    fa[1] = *reinterpret_cast<const f32x4 *>(g + (tid * 16 + 4 + blockIdx.x * 4096) % (65536 * 32));
    fb[0] = *reinterpret_cast<const f32x4 *>(g + (tid * 16 + 8 + blockIdx.x * 4096) % (65536 * 32));
    fb[1] = *reinterpret_cast<const f32x4 *>(g + (tid * 16 + 12 + blockIdx.x * 4096) % (65536 * 32));
  }
  for (int kt = 0; kt < ktiles; ++kt) {
    const float *As = smem + (kt & 1) * 256 * 36, *Bs = As + 128 * 36;
    if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = tid + 256 * i;
        st[i] = *reinterpret_cast<const f32x4 *>(g + ((size_t)(blockIdx.x * 131 + kt * 7 + (idx >> 3)) % 65536) * 32 + 4 * (idx & 7));
      }
    }
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      if (MODE >= 1 && MODE <= 3) {
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const f32x4 *>(As + (wm * 64 + i * 32 + r) * 36 + gg * 8 + 4 * h);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const f32x4 *>(Bs + (wn * 64 + j * 32 + r) * 36 + gg * 8 + 4 * h);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
    }
    if (MODE == 3) {
      float *An = smem + ((kt & 1) ^ 1) * 256 * 36;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = tid + 256 * i;
        *reinterpret_cast<f32x4 *>(An + (idx >> 3) * 36 + 4 * (idx & 7)) = st[i];
      }
    }
    if (MODE >= 2 && MODE <= 3) __syncthreads();
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[i][j][e];
  out[blockIdx.x * 256 + tid] = s;
  if (blockIdx.x == 0 && tid == 0) g_cycles = __builtin_amdgcn_s_memtime() - t0;
}

template <int MODE>
void run(const float *g, float *o, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int kt = 96;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, g, o, kt);
  hipEventRecord(a);
  const int iters = 20;
  for (int it = 0; it < iters; ++it) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, g, o, kt);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= iters;
  const double flops = (double)blocks * 4 * kt * 64 * 2.0 * 32 * 32 * 2;
  unsigned long long cyc = 0;
  hipMemcpyFromSymbol(&cyc, HIP_SYMBOL(g_cycles), sizeof(cyc));
  printf("mode %d blocks %d: %.1f us  %.1f TFLOP/s  block0 %.0f cycles (%.0f MHz if block0 spans the launch)\n", MODE,
         blocks, ms * 1e3, flops / (ms * 1e-3) / 1e12, (double)cyc, cyc / (ms * 1e3));
}

int main() {
  float *g, *o;
  hipMalloc(&g, 65536 * 32 * 4 + 4096);
  hipMalloc(&o, 4096 * 256 * 4);
  hipMemset(g, 0, 65536 * 32 * 4);
  for (int rnd = 0; rnd < 2; ++rnd) {
  if (rnd) {
    float *hbuf = (float *)malloc(65536 * 32 * 4);
    unsigned x = 12345;
    for (int i = 0; i < 65536 * 32; ++i) { x = x * 1664525u + 1013904223u; hbuf[i] = (float)((int)(x >> 8) - (1 << 23)) / (1 << 23); }
    hipMemcpy(g, hbuf, 65536 * 32 * 4, hipMemcpyHostToDevice);
    free(hbuf);
    printf("random operands:\n");
  } else printf("zero operands:\n");
  for (int blocks : {256, 512}) {
    run<0>(g, o, blocks);
    run<1>(g, o, blocks);
    run<2>(g, o, blocks);
    run<3>(g, o, blocks);
    run<4>(g, o, blocks);
  }
  }
  return 0;
}
