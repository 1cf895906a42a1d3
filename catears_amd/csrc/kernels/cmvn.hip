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

constexpr int kTile = 32;  // frames prefetched into registers per step of the chain

// Everything in SmoothStats/Apply except the per-dimension sums depends only
// on the frame index t (count = min(t+1, 600)) and on N_g, so it is computed
// once per block into LDS: alpha_t (the float scalar of AddVec, cmvn.cc:80-88)
// and neg_t = -(float)(1 / smoothed count) (cmvn.cc:93-97).  For t >= 600 no
// smoothing happens and the count is exactly 600.
__global__ __launch_bounds__(64) void cmvn_kernel(const int64_t *__restrict__ frame_off,
                                                  const float *__restrict__ gstats,
                                                  const float *__restrict__ in,
                                                  float *__restrict__ out) {
  __shared__ float s_alpha[kWindow], s_neg[kWindow + 1];
  const int u = blockIdx.x, d = threadIdx.x;
  const float g_count = gstats[kMel];
  for (int t = d; t <= kWindow; t += 64) {
    float count = (float)(t + 1 < kWindow ? t + 1 : kWindow);
    float alpha = 0.0f;
    if ((double)count < kWindow) {  // SmoothStats (cmvn.cc:70-89)
      double from_global = kWindow - (double)count;
      if (from_global > kGlobal) from_global = kGlobal;
      alpha = (float)(from_global / (double)g_count);
      count = alpha != 1.0f ? count + alpha * g_count : count + g_count;
    }
    if (t < kWindow) s_alpha[t] = alpha;
    s_neg[t] = -(float)(1 / (double)count);  // Apply (cmvn.cc:91-98)
  }
  __syncthreads();
  if (d >= kMel) return;
  const int64_t r0 = frame_off[u];
  const int t_frames = (int)(frame_off[u + 1] - r0);
  const float g = gstats[d];
  const float *x = in + r0 * kMel + d;
  float *y = out + r0 * kMel + d;
  float cur[kTile], old[kTile], ncur[kTile], nold[kTile];
  // Unconditional loads at clamped (always valid) frames: a per-element
  // "load or zero" select makes hipcc branch around every load and wait
  // vmcnt(0) each time.  Frames past the end are never used.
  if (t_frames == 0) return;
  auto fetch = [&](int t0, float *c, float *o) {
#pragma unroll
    for (int i = 0; i < kTile; ++i) {
      const int t = min(t0 + i, t_frames - 1);
      c[i] = x[(int64_t)t * kMel];
      o[i] = x[(int64_t)max(t - kWindow, 0) * kMel];
    }
  };
  // per-frame scalars of a tile, read from LDS before the chain runs (a read
  // per step would put an LDS round trip on the critical path)
  float al[kTile], ng[kTile];
  auto scalars = [&](int t0) {
#pragma unroll
    for (int i = 0; i < kTile; ++i) {
      const int t = t0 + i;
      al[i] = s_alpha[min(t, kWindow - 1)];
      ng[i] = s_neg[min(t, kWindow)];
    }
  };
  fetch(0, cur, old);
  float carry = 0.0f;
  for (int t0 = 0; t0 < t_frames; t0 += kTile) {
    fetch(t0 + kTile, ncur, nold);
    scalars(t0);
#pragma unroll
    for (int i = 0; i < kTile; ++i) {
      const int t = t0 + i;
      if (t < t_frames) {
        // ComputeStats (cmvn.cc:35-68): double temp seeded from the float carry
        double acc = t > 0 ? (double)carry : 0.0;
        acc += (double)cur[i];
        if (t >= kWindow) acc += -1.0 * (double)old[i];
        carry = (float)acc;
        float s = carry;
        if (t < kWindow) s = al[i] != 1.0f ? s + al[i] * g : s + g;
        y[(int64_t)t * kMel] = ng[i] != 1.0f ? cur[i] + ng[i] * s : cur[i] + s;
      }
    }
#pragma unroll
    for (int i = 0; i < kTile; ++i) cur[i] = ncur[i], old[i] = nold[i];
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
