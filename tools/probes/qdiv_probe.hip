// qdiv_probe.hip -- x / s (IEEE division) against the int8 Quantize's
// corrected reciprocal product (kernels/nnet_i8.hip qbyte, CATEARS_I8_QDIV):
// q0 = x * r, r = RN(1 / s), q = fma(fma(-s, q0, x), r, q0), falling back to
// x / s when r or q is not finite.  Counts differing quotients over random
// fp32 pairs: x over [-2^20, 2^20] with random exponents, s over scales the
// quantize sees (2^-40 .. 2^10, denormal ones included).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/qdiv_probe.hip -o tools/probes/qdp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

__global__ void probe(uint32_t seed, unsigned long long *bad, float *ex) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t local = 0;
  for (int i = 0; i < 64; ++i) {
    const uint32_t h1 = mix(seed ^ (t * 64u + i) * 2654435761u), h2 = mix(h1 + 0x9e3779b9u);
    // x: random sign / significand, exponent in [-40, 20]
    const float x = __builtin_bit_cast(float, (h1 & 0x807fffffu) | ((uint32_t)(127 - 40 + (h1 >> 23) % 61) << 23));
    // s: significand random, exponent in [-40, 10] (some denormal by the bit pattern below)
    uint32_t sb = (h2 & 0x007fffffu) | ((uint32_t)(127 - 40 + (h2 >> 23) % 51) << 23);
    if ((h2 & 0xff) == 0) sb = h2 & 0x007fffffu;  // a denormal scale now and then
    const float s = __builtin_bit_cast(float, sb);
    if (s == 0.0f) continue;
    const float ref = x / s;
    float r = 1.0f / s;
    if (__builtin_isinf(r) || __builtin_isnan(r)) r = 0.0f;
    float q;
    if (r != 0.0f) {
      const float q0 = x * r;
      q = __builtin_fmaf(__builtin_fmaf(-s, q0, x), r, q0);
      if (__builtin_isinf(q) || __builtin_isnan(q)) q = x / s;
    } else {
      q = x / s;
    }
    if (__builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, ref)) {
      ++local;
      ex[0] = x, ex[1] = s, ex[2] = q, ex[3] = ref;
    }
  }
  if (local) atomicAdd(bad, (unsigned long long)local);
}

int main() {
  unsigned long long *bad;
  float *ex;
  hipMalloc(&bad, 8);
  hipMalloc(&ex, 16);
  hipMemset(bad, 0, 8);
  hipMemset(ex, 0, 16);
  const int blocks = 65536, threads = 256, launches = 64;
  for (int l = 0; l < launches; ++l) hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, 1234u + l, bad, ex);
  unsigned long long h = 0;
  float e[4];
  hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(e, ex, 16, hipMemcpyDeviceToHost);
  printf("pairs %llu, differing quotients %llu", (unsigned long long)blocks * threads * 64ull * launches, h);
  if (h) printf(" (e.g. x=%a s=%a q=%a ref=%a)", e[0], e[1], e[2], e[3]);
  printf("\n");
  return 0;
}
