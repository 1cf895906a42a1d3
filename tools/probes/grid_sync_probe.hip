// Probe: cost of a cooperative-groups grid barrier (hipLaunchCooperativeKernel
// + this_grid().sync()) against a kernel boundary, at the latency path's grid
// (256 blocks x 256 threads, one per CU).  Each phase writes a 1 KB slab per
// block and the next phase reads another block's slab (the cross-XCD hand-off
// the latency GEMM's split-K reduce needs).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/grid_sync_probe.hip -o /tmp/gsp
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

namespace cg = cooperative_groups;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ __launch_bounds__(256) void phases_coop(float *buf, int phases) {
  cg::grid_group g = cg::this_grid();
  const int nb = gridDim.x, b = blockIdx.x, t = threadIdx.x;
  float v = 1.0f;
  for (int p = 0; p < phases; ++p) {
    float *cur = buf + (size_t)(p & 1) * nb * 256;
    const float *prev = buf + (size_t)((p + 1) & 1) * nb * 256;
    if (p > 0) v += prev[(size_t)((b + 37) % nb) * 256 + t];
    cur[(size_t)b * 256 + t] = v;
    g.sync();
  }
}

__global__ __launch_bounds__(256) void phase_kernel(float *buf, int p) {
  const int nb = gridDim.x, b = blockIdx.x, t = threadIdx.x;
  float *cur = buf + (size_t)(p & 1) * nb * 256;
  const float *prev = buf + (size_t)((p + 1) & 1) * nb * 256;
  float v = 1.0f;
  if (p > 0) v += prev[(size_t)((b + 37) % nb) * 256 + t];
  cur[(size_t)b * 256 + t] = v;
}

int main() {
  int dev = 0, coop = 0;
  CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, phases_coop, 256, 0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  printf("cooperative launch %d, CUs %d, blocks/CU %d\n", coop, prop.multiProcessorCount, per_cu);
  float *buf;
  const int nb = prop.multiProcessorCount;
  CK(hipMalloc(&buf, (size_t)2 * nb * 256 * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  for (int phases : {1, 16, 64}) {
    void *args[] = {&buf, &phases};
    for (int w = 0; w < 5; ++w)
      CK(hipLaunchCooperativeKernel((void *)phases_coop, dim3(nb), dim3(256), args, 0, s));
    CK(hipStreamSynchronize(s));
    const int reps = 50;
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r)
      CK(hipLaunchCooperativeKernel((void *)phases_coop, dim3(nb), dim3(256), args, 0, s));
    CK(hipEventRecord(z, s));
    CK(hipEventSynchronize(z));
    float ms;
    CK(hipEventElapsedTime(&ms, a, z));
    printf("cooperative: %3d phases per launch  %8.2f us/launch  %6.2f us/phase\n", phases, ms * 1e3 / reps,
           ms * 1e3 / reps / phases);
  }
  for (int phases : {1, 16, 64}) {
    for (int w = 0; w < 5; ++w)
      for (int p = 0; p < phases; ++p) hipLaunchKernelGGL(phase_kernel, dim3(nb), dim3(256), 0, s, buf, p);
    CK(hipStreamSynchronize(s));
    const int reps = 50;
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r)
      for (int p = 0; p < phases; ++p) hipLaunchKernelGGL(phase_kernel, dim3(nb), dim3(256), 0, s, buf, p);
    CK(hipEventRecord(z, s));
    CK(hipEventSynchronize(z));
    float ms;
    CK(hipEventElapsedTime(&ms, a, z));
    printf("kernels:     %3d phases per group   %8.2f us/group   %6.2f us/phase\n", phases, ms * 1e3 / reps,
           ms * 1e3 / reps / phases);
  }
  CK(hipGetLastError());
  printf("ok\n");
  return 0;
}
