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

#ifndef CMVN_TILE
#define CMVN_TILE 48
#endif
// frames prefetched into registers per tile of the chain: 48 took the C4
// batch's CMVN from 0.098 to 0.092 ms (tools/experiments/gpu_r5j.sh)
constexpr int kTile = CMVN_TILE;

// The chain of one (utterance, dimension) runs in three regimes of t:
//   t <  599: SmoothStats adds alpha_t * [g, N_g] (count = t + 1 < 600);
//   t == 599: count = 600, neither smoothing nor window subtraction;
//   t >= 600: frame t - 600 leaves the window (no smoothing).
// Each regime is its own loop, so no step carries a select, and the per-step
// work is the reference's arithmetic only (the kernel is issue-bound: one
// wave per utterance, a latency chain per lane).
enum CmvnMode { kSmooth, kPlain, kWindowed };

template <int M>
__device__ __forceinline__ float cmvn_step(float &carry, float c, float o, float al, float ng, float g) {
  // ComputeStats (cmvn.cc:35-68): double temp seeded from the float carry
  double acc = (double)carry;
  acc += (double)c;
  if (M == kWindowed) acc += -1.0 * (double)o;
  carry = (float)acc;
  // SmoothStats / Apply (cmvn.cc:80-88, 91-98) are AddVec calls, whose
  // alpha == 1 branch (vector.cc:249-256) adds v instead of 1 * v: the same
  // float, so no select here
  float s = carry;
  if (M == kSmooth) s = s + al * g;
  return c + ng * s;
}

// Everything in SmoothStats/Apply except the per-dimension sums depends only
// on the frame index t (count = min(t+1, 600)) and on N_g, so it is computed
// once per block into LDS: alpha_t (the float scalar of AddVec, cmvn.cc:80-88)
// and neg_t = -(float)(1 / smoothed count) (cmvn.cc:93-97).  For t >= 599 no
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
  const int T = (int)(frame_off[u + 1] - r0);
  if (T == 0) return;
  const float g = gstats[d];
  const float *x = in + r0 * kMel + d;
  float *y = out + r0 * kMel + d;
  const float ng600 = s_neg[kWindow];
  float carry = 0.0f;

  // Frames [t0, t1) in regime M.  Whole tiles: the next tile's rows are
  // prefetched from a base clamped into [0, t1 - kTile] (all valid rows, one
  // base + immediate offsets per tile); the last, partial tile reloads with
  // per-row clamps.
  auto phase = [&](auto MC, int t0, int t1) {
    constexpr int M = decltype(MC)::value;
    if (t0 >= t1) return;
    float c[kTile], o[kTile];
    auto load_tile = [&](int b, float *cc, float *oo) {
      const float *xc = x + (int64_t)b * kMel;
#pragma unroll
      for (int i = 0; i < kTile; ++i) cc[i] = xc[i * kMel];
      if (M == kWindowed) {
        const float *xo = x + (int64_t)max(b - kWindow, 0) * kMel;
#pragma unroll
        for (int i = 0; i < kTile; ++i) oo[i] = xo[i * kMel];
      }
    };
    int t = t0;
    if (t + kTile <= t1) load_tile(t, c, o);
    for (; t + kTile <= t1; t += kTile) {
      float cn[kTile], on[kTile];
      load_tile(max(0, min(t + kTile, t1 - kTile)), cn, on);
      float al[kTile], ng[kTile];
#pragma unroll
      for (int i = 0; i < kTile; ++i) {
        al[i] = M == kSmooth ? s_alpha[t + i] : 0.0f;
        ng[i] = M == kSmooth ? s_neg[t + i] : ng600;
      }
      float *yt = y + (int64_t)t * kMel;
#pragma unroll
      for (int i = 0; i < kTile; ++i) yt[i * kMel] = cmvn_step<M>(carry, c[i], o[i], al[i], ng[i], g);
#pragma unroll
      for (int i = 0; i < kTile; ++i) c[i] = cn[i], o[i] = on[i];
    }
    if (t < t1) {  // partial tile
#pragma unroll
      for (int i = 0; i < kTile; ++i) {
        const int tt = min(t + i, t1 - 1);
        c[i] = x[(int64_t)tt * kMel];
        o[i] = M == kWindowed ? x[(int64_t)(tt - kWindow) * kMel] : 0.0f;
      }
#pragma unroll
      for (int i = 0; i < kTile; ++i) {
        if (t + i < t1) {
          const float al = M == kSmooth ? s_alpha[t + i] : 0.0f;
          const float ng = M == kSmooth ? s_neg[t + i] : ng600;
          y[(int64_t)(t + i) * kMel] = cmvn_step<M>(carry, c[i], o[i], al, ng, g);
        }
      }
    }
  };
  phase(std::integral_constant<int, kSmooth>(), 0, min(T, kWindow - 1));
  phase(std::integral_constant<int, kPlain>(), kWindow - 1, min(T, kWindow));
  phase(std::integral_constant<int, kWindowed>(), kWindow, T);
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
