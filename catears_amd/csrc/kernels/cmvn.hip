// cmvn.hip -- online (sliding-window) CMVN for every utterance of a batch.
//
// Replaces CMVN::GetFrame called for frames 0, 1, 2, ... (src/cmvn.cc:35-110).
// The reference carries the 41 running sums between frames as float with a
// double temporary per step (cmvn.cc:42-67), so the running sum of dimension d
// is an inherently sequential rounding chain.  The kernel therefore gives one
// lane to each (utterance, dimension) chain -- 40 lanes of one wave per
// utterance, reading one 160-byte feature row per step -- and replays the
// chain exactly: same float/double promotions, same order, no FMA (built with
// -ffp-contract=off).  The frame count is an exact small integer, so every
// lane recomputes it instead of carrying lane 40.  Output is bit-identical to
// the reference for any input.
#include <hip/hip_runtime.h>

#include "../internal.h"

namespace catears {
namespace {

constexpr int kWindow = 600;  // PK_ONLINECMVN_WINDOW, src/cmvn.h:10
constexpr int kGlobal = 200;  // PK_ONLINECMVN_GLOBALFRAMES, src/cmvn.h:11

__global__ __launch_bounds__(64) void cmvn_kernel(const int64_t *__restrict__ frame_off,
                                                  const float *__restrict__ gstats,
                                                  const float *__restrict__ in,
                                                  float *__restrict__ out) {
  const int u = blockIdx.x, d = threadIdx.x;
  if (d >= kMel) return;
  const int64_t r0 = frame_off[u];
  const int t_frames = (int)(frame_off[u + 1] - r0);
  const float g = gstats[d];
  const float g_count = gstats[kMel];
  const float *x = in + r0 * kMel + d;
  float *y = out + r0 * kMel + d;
  float carry = 0.0f;
#pragma unroll 4
  for (int t = 0; t < t_frames; ++t) {
    const float xt = x[(int64_t)t * kMel];
    // ComputeStats: double temp seeded from the float carry
    double acc = t > 0 ? (double)carry : 0.0;
    acc += (double)xt;
    float count = (float)(t + 1 < kWindow ? t + 1 : kWindow);
    if (t >= kWindow) acc += -1.0 * (double)x[(int64_t)(t - kWindow) * kMel];
    carry = (float)acc;
    // SmoothStats: add min(600 - n, 200) / N_g of the global stats
    float s = carry;
    if ((double)count < kWindow) {
      double from_global = kWindow - (double)count;
      if (from_global > kGlobal) from_global = kGlobal;
      const float alpha = (float)(from_global / (double)g_count);
      if (alpha != 1.0f) {
        s = s + alpha * g;
        count = count + alpha * g_count;
      } else {
        s = s + g;
        count = count + g_count;
      }
    }
    // Apply: scale = 1 / count in double, stored float; feats += -scale * s
    const float neg = -(float)(1 / (double)count);
    y[(int64_t)t * kMel] = neg != 1.0f ? xt + neg * s : xt + s;
  }
}

}  // namespace

int launch_cmvn(hipStream_t s, const ce_gpu_plan *p, const float *gstats, const float *in,
                float *out) {
  if (p->n_utt == 0 || p->total_frames == 0) return CE_GPU_OK;
  hipLaunchKernelGGL(cmvn_kernel, dim3(p->n_utt), dim3(64), 0, s, p->d_frame_off.as<int64_t>(),
                     gstats, in, out);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace catears
