// lds_dma.h -- device helpers shared by the LDS-DMA GEMM kernels
// (gemm_bf16x6.hip, gemm_f16x3.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace catears {
namespace dma {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// s_waitcnt vmcnt(N): all but this wave's N youngest vector-memory operations
// (LDS-DMAs included) are done.  A compiler barrier too.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// global_load_lds_dwordx4: 16 bytes per lane from a per-lane global address
// into LDS at the wave-uniform base lds_dst + 16 * lane.
__device__ __forceinline__ void glds16(const char *src, char *lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                   (__attribute__((address_space(3))) void *)lds_dst, 16, 0, 0);
}

}  // namespace dma
}  // namespace catears
