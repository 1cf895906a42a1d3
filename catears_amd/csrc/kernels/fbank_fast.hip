// fbank_fast.hip -- the fast fbank mode (ce_gpu_ctx_set_fbank(ctx,
// CE_GPU_FBANK_FAST)): the same log-mel features as fbank.hip within 3e-5 on
// the log, but not the reference's operation order, so every lane does useful
// arithmetic.
//
// The default kernel (fbank.hip) keeps the reference's split-radix schedule
// (src/srfft.cc:124-265) for bit-exact pre-log energies: one wave per frame,
// seven generations of divergent lane ops and 40 lanes forming sequential mel
// dots -- bound by its instruction stream at about a quarter of useful lane
// slots.  Here a frame is 16 lanes (one DPP row), four frames
// per wave, and the 256-point complex FFT of the packed real frame
// (srfft.cc:318-324 packing, then the real-FFT post-pass of :370-459) is the
// four-step 16 x 16 decomposition, every lane running the same straight-line
// code:
//   1. lane j loads samples 32 n1 + 2 j, +1 (n1 = 0..12; 128 contiguous bytes
//      per n1 across the row), the DC mean is a row all-reduce (DPP rotates),
//      pre-emphasis takes the previous sample from the neighbour lane (DPP
//      row_ror:1) -- src/fbank.cc:44-100 -- and the Hamming window is applied;
//   2. a 16-point DFT (radix-4 x 4, in registers) over n1, times W256^(j k1);
//   3. a transpose through LDS (conflict-free swizzle), a second 16-point DFT
//      over n2: lane j now holds Z[j + 16 k2];
//   4. the real-FFT post-pass pairs Z[k] with Z[256 - k] (read back through
//      LDS) and forms the power spectrum (src/fbank.cc:193-211);
//   5. mel: each lane forms up to three triangles, one per slot (the 16
//      longest bands, the next 16, the last 8), as float dots over fixed
//      zero-padded windows of the power spectrum in LDS (src/fbank.cc:165-184),
//      floor at FLT_EPSILON, logf (:243-244).
// Twiddles are tabled on the host in double, rounded once.  Error against the
// oracle: the FFT's own fp32 rounding, measured <= 3e-5 on log-mel (tests).
#include <float.h>
#include <hip/hip_runtime.h>

#include "../internal.h"

namespace catears {
namespace {

constexpr int kWaves = 4;                  // per block
constexpr int kFramesPerWave = 4;          // 16 lanes (one DPP row) per frame
constexpr int kFramesPerBlk = kWaves * kFramesPerWave;
constexpr int kRegion = 272;               // complex slots per frame: 256 + 16 (odd rows' bank offset)
constexpr int kFastBlocksPerCU = 3;        // 43 KB of LDS per block, <= 168 VGPRs
constexpr int kFastMaxBlocks = 256 * kFastBlocksPerCU;

struct FastSmem {
  float2 frame[kWaves][kFramesPerWave * kRegion];
  float2 tw[256];       // [k1][n2]
  float2 post[kHalf];
  float window[kWinLen];
  float mel_w[16 * kFfSlotW];  // FbankTables::ff_slot_w
};

__device__ __forceinline__ void wave_sync() { wave_lds_sync(); }

// FF_DIAG (experiment builds only, tools/experiments/lds_race_stress.py):
// 1 = the four frames' LDS regions in reverse order, 2 = lane group g
// computes frame 3 - g, 3 = the row rotates by ds_bpermute instead of DPP
#ifndef FF_DIAG
#define FF_DIAG 0
#endif

// lane j of a 16-lane row receives lane (j - N) mod 16's value (DPP row_ror)
template <int N>
__device__ __forceinline__ float row_ror(float v) {
#if FF_DIAG == 3
  const int l = __lane_id();
  return __shfl(v, (l & ~15) | ((l - N) & 15));
#else
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + N, 0xf, 0xf,
                                                               false));
#endif
}

struct Cplx {
  float r, i;
};

__device__ __forceinline__ void dft4(Cplx &a, Cplx &b, Cplx &c, Cplx &d) {
  const Cplx y0 = {a.r + c.r, a.i + c.i}, y1 = {a.r - c.r, a.i - c.i};
  const Cplx y2 = {b.r + d.r, b.i + d.i}, y3 = {b.r - d.r, b.i - d.i};
  a = {y0.r + y2.r, y0.i + y2.i};
  c = {y0.r - y2.r, y0.i - y2.i};
  b = {y1.r + y3.i, y1.i - y3.r};  // y1 - i y3
  d = {y1.r - y3.i, y1.i + y3.r};  // y1 + i y3
}

// x *= W16^m = exp(-2 pi i m / 16), m a compile-time constant
template <int M>
__device__ __forceinline__ void tw16(Cplx &x) {
  constexpr int m = M & 15;
  if constexpr (m == 0) {
  } else if constexpr (m == 4) {
    x = {x.i, -x.r};
  } else if constexpr (m == 8) {
    x = {-x.r, -x.i};
  } else if constexpr (m == 12) {
    x = {-x.i, x.r};
  } else {
    // cos / sin(2 pi m / 16), m = 0..15
    constexpr double kC[16] = {1.0, 0.92387953251128674, 0.70710678118654752, 0.38268343236508977,
                               0.0, -0.38268343236508977, -0.70710678118654752, -0.92387953251128674,
                               -1.0, -0.92387953251128674, -0.70710678118654752, -0.38268343236508977,
                               0.0, 0.38268343236508977, 0.70710678118654752, 0.92387953251128674};
    constexpr float c = (float)kC[m], s = (float)kC[(m + 12) & 15];  // sin(a) = cos(a - pi/2)
    x = {x.r * c + x.i * s, x.i * c - x.r * s};  // (r + i im)(c - i s)
  }
}

// 16-point DFT X[k] = sum_n x[n] W16^(nk), in place; on return X[k] sits at
// x[4 (k & 3) + (k >> 2)] (n = 4 na + nb, k = ka + 4 kb: DFT-4 over na,
// twiddle W16^(nb ka), DFT-4 over nb).
__device__ __forceinline__ void dft16(Cplx (&x)[16]) {
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) dft4(x[nb], x[4 + nb], x[8 + nb], x[12 + nb]);  // -> T[nb][ka] at x[4 ka + nb]
  tw16<1>(x[5]);
  tw16<2>(x[6]);
  tw16<3>(x[7]);
  tw16<2>(x[9]);
  tw16<4>(x[10]);
  tw16<6>(x[11]);
  tw16<3>(x[13]);
  tw16<6>(x[14]);
  tw16<9>(x[15]);
#pragma unroll
  for (int ka = 0; ka < 4; ++ka) dft4(x[4 * ka], x[4 * ka + 1], x[4 * ka + 2], x[4 * ka + 3]);
}

__device__ __forceinline__ int dpos(int k) { return 4 * (k & 3) + (k >> 2); }

template <typename Sample>
__global__ __launch_bounds__(kWaves * 64, 3) void fbank_fast_kernel(const FbankTables *__restrict__ tab,
                                                                  const Sample *__restrict__ pcm,
                                                                  const int64_t *__restrict__ sample_off,
                                                                  const int64_t *__restrict__ frame_off,
                                                                  const int *__restrict__ block_utt,
                                                                  int64_t total_frames, float *__restrict__ feats,
                                                                  float *__restrict__ mel_out) {
  __shared__ FastSmem sm;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) sm.tw[i] = make_float2(tab->ff_tw[2 * i], tab->ff_tw[2 * i + 1]);
  for (int i = threadIdx.x; i < kHalf; i += blockDim.x)
    sm.post[i] = make_float2(tab->ff_post[2 * i], tab->ff_post[2 * i + 1]);
  for (int i = threadIdx.x; i < kWinLen; i += blockDim.x) sm.window[i] = tab->window[i];
  for (int i = threadIdx.x; i < 16 * kFfSlotW; i += blockDim.x) sm.mel_w[i] = tab->ff_slot_w[i];
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 4, j = lane & 15;
  int band[3], start[3];  // this lane's mel slots (tables.cc build_fast)
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    band[q] = tab->ff_slot_band[q * 16 + j];
    start[q] = tab->ff_slot_start[q * 16 + j];
  }
#if FF_DIAG == 1
  float2 *R = sm.frame[wave] + (3 - g) * kRegion;
#else
  float2 *R = sm.frame[wave] + g * kRegion;  // this frame's LDS region
#endif
  // the power spectrum reuses the region, 16 dwords in for odd frames: the
  // regions are 544 dwords apart (= 0 mod 32), so frames 2i and 2i+1 -- one
  // 32-lane group of a ds_read_b32 / ds_write_b32 -- would otherwise read and
  // write every bin on the same bank
  float *P = reinterpret_cast<float *>(R) + 16 * (g & 1);
  const int64_t stride = (int64_t)gridDim.x * kFramesPerBlk;
  for (int64_t fb = ((int64_t)blockIdx.x * kWaves + wave) * kFramesPerWave; fb < total_frames; fb += stride) {
#if FF_DIAG == 2
    const int64_t fr = fb + (3 - g);
#else
    const int64_t fr = fb + g;
#endif
    const bool active = fr < total_frames;
    const int64_t f = active ? fr : total_frames - 1;  // idle rows recompute the last frame, store nothing
    int u = block_utt[f / 4];  // the exact kernel's 4-frame blocks (ce_gpu_plan_create)
    while (f >= frame_off[u + 1]) ++u;
    const Sample *src = pcm + sample_off[u] + (f - frame_off[u]) * kShift;

    // 1. samples (n = 2 (16 n1 + j) and n + 1), DC mean, pre-emphasis, window
    float xe[13], xo[13];
    float part = 0.0f;
#pragma unroll
    for (int n1 = 0; n1 < 13; ++n1) {
      const int idx = 32 * n1 + 2 * j;
      const bool ok = n1 < 12 || j < 8;  // idx < 400
      xe[n1] = ok ? (float)src[idx] : 0.0f;
      xo[n1] = ok ? (float)src[idx + 1] : 0.0f;
      part += xe[n1] + xo[n1];
    }
    part += row_ror<8>(part);
    part += row_ror<4>(part);
    part += row_ror<2>(part);
    part += row_ror<1>(part);
    const float mean = part / (float)kWinLen;
    // x[idx - 1]: lane j-1's odd sample, or (j = 0) lane 15's of n1 - 1;
    // the first sample is its own predecessor (src/fbank.cc:57-61).  The
    // rotates run on every lane of the row (no divergence around a DPP).
    float rot[13];
#pragma unroll
    for (int n1 = 0; n1 < 13; ++n1) rot[n1] = row_ror<1>(xo[n1]);
    Cplx x[16];
#pragma unroll
    for (int n1 = 0; n1 < 13; ++n1) {
      const int idx = 32 * n1 + 2 * j;
      const bool ok = n1 < 12 || j < 8;
      const float prev = j != 0 ? rot[n1] : (n1 == 0 ? xe[0] : rot[n1 - 1]);
      const float de = xe[n1] - mean, dp = prev - mean, dodd = xo[n1] - mean;
      const float2 w = *reinterpret_cast<const float2 *>(sm.window + (ok ? idx : 0));
      x[n1] = ok ? Cplx{(de - 0.97f * dp) * w.x, (dodd - 0.97f * de) * w.y} : Cplx{0.0f, 0.0f};
    }
    x[13] = x[14] = x[15] = Cplx{0.0f, 0.0f};

    // 2. DFT over n1, twiddle W256^(j k1), into LDS at [k1][n2 = j], swizzled
    dft16(x);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) {
      Cplx t = x[dpos(k1)];
      if (k1 > 0) {
        const float2 w = sm.tw[k1 * 16 + j];
        t = {t.r * w.x - t.i * w.y, t.r * w.y + t.i * w.x};
      }
      R[k1 * 16 + (j ^ k1)] = make_float2(t.r, t.i);
    }
    wave_sync();
    // 3. lane j as column k1 = j: the 16 values of n2, DFT over n2
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
      const float2 v = R[j * 16 + (n2 ^ j)];
      x[n2] = {v.x, v.y};
    }
    wave_sync();
    dft16(x);  // Z[j + 16 k2] at x[dpos(k2)]
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) R[j + 16 * k2] = make_float2(x[dpos(k2)].r, x[dpos(k2)].i);
    wave_sync();
    // 4. real-FFT post-pass with Z[256 - k] and the power spectrum
    float pw[16];
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      const int k = j + 16 * k2;
      const float2 b = R[(256 - k) & 255];
      const Cplx a = x[dpos(k2)];
      const float e2r = a.r + b.x, e2i = a.i - b.y;  // 2 E[k]
      const float o2r = a.i + b.y, o2i = b.x - a.r;  // 2 O[k]
      const float2 w = sm.post[k];                   // W512^k
      const float xr = e2r + (w.x * o2r - w.y * o2i);
      const float xi = e2i + (w.x * o2i + w.y * o2r);
      pw[k2] = 0.25f * (xr * xr + xi * xi);
    }
    wave_sync();
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) P[j + 16 * k2] = pw[k2];
    wave_sync();
    // 5. this lane's mel triangles (one per slot), floor, log.  Fixed
    // windows: every LDS read of a slot issues before its first product (a
    // loop over the band's own length waited on each read); the zero weights
    // around the band add exact zeros, so each dot is the band's own
    // in-order sum.
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float *w = sm.mel_w + j * kFfSlotW + kFfSlotBase[q];
      const float *pq = P + start[q];
      float e = 0.0f;
#pragma unroll
      for (int i = 0; i < kFfSlot[q]; i += 4) {
        const float4 w4 = *reinterpret_cast<const float4 *>(w + i);
        e += w4.x * pq[i];
        e += w4.y * pq[i + 1];
        e += w4.z * pq[i + 2];
        e += w4.w * pq[i + 3];
      }
      const int b = band[q];
      if (active && b >= 0) {
        if (mel_out) mel_out[f * kMel + b] = e;
        feats[f * kMel + b] = logf(e < FLT_EPSILON ? FLT_EPSILON : e);
      }
    }
    wave_sync();  // the region is rewritten by the next frame
  }
}

template <typename Sample>
int launch_fast(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const Sample *pcm, float *feats,
                float *mel) {
  if (p->total_frames == 0) return CE_GPU_OK;
  const int64_t blocks = (p->total_frames + kFramesPerBlk - 1) / kFramesPerBlk;
  const unsigned grid = (unsigned)(blocks < kFastMaxBlocks ? blocks : kFastMaxBlocks);
  hipLaunchKernelGGL(fbank_fast_kernel<Sample>, dim3(grid), dim3(kWaves * 64), 0, s, d_tab, pcm,
                     p->d_sample_off.as<int64_t>(), p->d_frame_off.as<int64_t>(), p->d_block_utt.as<int>(),
                     p->total_frames, feats, mel);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace

int launch_fbank_fast(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const float *pcm, float *feats,
                      float *mel) {
  return launch_fast(s, d_tab, p, pcm, feats, mel);
}

int launch_fbank_fast_s16(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const int16_t *pcm,
                          float *feats, float *mel) {
  return launch_fast(s, d_tab, p, pcm, feats, mel);
}

}  // namespace catears
