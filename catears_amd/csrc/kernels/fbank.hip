// fbank.hip -- batched log-mel filterbank on gfx950.
//
// Replaces the per-frame loop of Fbank::Process (src/fbank.cc:297-303):
// ExtractWindow + ProcessWindow (fbank.cc:44-100), SRFFT::Compute
// (srfft.cc:370-459), ComputePowerSpectrum (fbank.cc:193-211),
// Melbanks::Compute (fbank.cc:165-184), floor + log (fbank.cc:243-244).
//
// Mapping: one wave (64 lanes) per frame, four frames per 256-thread block,
// frames of every utterance of the batch flattened into one grid.
//   1. the frame's 400 samples are read once from HBM (7 coalesced loads per
//      lane), the DC mean is a wave reduction;
//   2. pre-emphasis (double, as the reference) and the Hamming window are
//      applied while scattering even/odd samples into the wave's complex
//      re/im arrays in LDS (the real->complex packing of srfft.cc:318-324);
//   3. the 256-point split-radix complex FFT runs as 7 generations of lane
//      ops (tables.cc), each lane op touching 4 points in registers;
//   4. real-FFT post-pass + power spectrum for two k per lane, reading the
//      FFT output at bit-reversed positions instead of permuting it;
//   5. lanes 0..39 each form one mel energy (sequential dot, as the
//      reference), floor at FLT_EPSILON, logf, and store one row of 40 floats.
// Everything up to the final logf is the reference's float arithmetic in the
// reference's order (the DC sum is exact for integer-valued PCM, whose partial
// sums are integers below 2^24), so pre-log mel energies match bit for bit.
#include <float.h>
#include <hip/hip_runtime.h>

#include "../fbank_ops.h"
#include "../internal.h"

namespace catears {
namespace {

constexpr int kFramesPerBlock = 4;  // one wave per frame, 4 waves per block
#ifndef FBANK_GENS
#define FBANK_GENS kFftGens  // (timing experiments only may lower it)
#endif
constexpr int kBlocksPerCU = 5;     // residency of fbank_kernel (27 KB LDS, 96 VGPRs)
constexpr int kMaxBlocks = 256 * kBlocksPerCU;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

struct WaveSmem {
  float x[kWinLen];   // mean-removed samples, later the power spectrum
  float re[kHalf];
  float im[kHalf];
};

// Tables staged once per block in LDS (indexed by generation / band at run
// time): each lane op's twiddles and the mel weights (the op's slots and
// kind live in the lane's registers).
struct BlockTables {
  float tw[kFftGens * 64 * 6];  // each lane op's six twiddles
  float mel_w[512];
};

// Persistent blocks: each block stages the frame-independent tables once --
// into LDS what is indexed at run time (twiddles, generation ops, mel
// weights), into registers what depends only on the lane (window taps,
// post-pass twiddles and LDS slots, the lane's mel band) -- then its four
// waves walk frames f = 4 * block + wave, f += 4 * gridDim.x.  Per frame the
// only global traffic is the 1.6 kB PCM read and the 160 B feature write.
// 5 waves per SIMD (the LDS bound; unrolled, the compiler would otherwise
// take 117 VGPRs and 4 waves)
// Sample: float (raw int16 scale, the Vector<float> WaveReader::Process
// produces) or int16_t (the WAV payload itself, converted here exactly as
// src/pcm_reader.cc:174 does on the host -- int16 -> float is exact, so both
// inputs give the same bits; 2 B per sample read instead of 4).
template <typename Sample>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 5))) void fbank_kernel(const FbankTables *__restrict__ tab,
                                                    const Sample *__restrict__ pcm,
                                                    const int64_t *__restrict__ sample_off,
                                                    const int64_t *__restrict__ frame_off,
                                                    const int *__restrict__ block_utt,
                                                    int64_t total_frames, float *__restrict__ feats,
                                                    float *__restrict__ mel_out) {
  __shared__ WaveSmem smem[kFramesPerBlock];
  __shared__ BlockTables bt;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < kFftGens * 64 * 6; i += 256) bt.tw[i] = tab->fft_tw[i];
  for (int i = threadIdx.x; i < 512; i += 256) bt.mel_w[i] = tab->mel_w[i];
  float win[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int i = lane + 64 * j;
    win[j] = i < kWinLen ? tab->window[i] : 0.0f;
  }
  const int k0 = lane + 1, k1 = lane + 65;
  const float kn0r = tab->kn[2 * k0], kn0i = tab->kn[2 * k0 + 1];
  const float kn1r = tab->kn[2 * k1], kn1i = tab->kn[2 * k1 + 1];
  const int a0 = fb::sw(fb::bitrev8(k0)), b0 = fb::sw(fb::bitrev8(256 - k0));
  const int a1 = fb::sw(fb::bitrev8(k1)), b1 = fb::sw(fb::bitrev8((256 - k1) & 255));
  // this lane's FFT op slots and kinds for every generation, in registers
  // (the frame loop then needs no descriptor load before its LDS accesses)
  uint32_t gaddr[kFftGens];
  uint32_t gmeta = 0;
#pragma unroll
  for (int g = 0; g < kFftGens; ++g) {
    gaddr[g] = tab->fft_addr[g * 64 + lane];
    gmeta |= (tab->fft_meta[g * 64 + lane] & 15u) << (4 * g);
  }
  const int band = lane < kMel ? lane : 0;
  const int mel_off = tab->mel_off[band], mel_len = lane < kMel ? tab->mel_len[band] : 0;
  const int mel_wbase = tab->mel_wbase[band];
  __syncthreads();

  WaveSmem &S = smem[wave];
  const int64_t stride = (int64_t)gridDim.x * kFramesPerBlock;
  for (int64_t f = (int64_t)blockIdx.x * kFramesPerBlock + wave; f < total_frames; f += stride) {
    int u = block_utt[f / kFramesPerBlock];
    while (f >= frame_off[u + 1]) ++u;
    const Sample *src = pcm + sample_off[u] + (f - frame_off[u]) * kShift;

    // 1. samples + DC offset (sum exact for integer-valued PCM: any order)
    float v[7];
    float part = 0.0f;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int i = lane + 64 * j;
      v[j] = i < kWinLen ? (float)src[i] : 0.0f;
      part += v[j];
    }
    const float mean = wave_sum(part) / (float)kWinLen;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int i = lane + 64 * j;
      if (i < kWinLen) S.x[i] = v[j] - mean;
    }
    wave_sync();

    // 2. pre-emphasis, window, pack even/odd samples as re/im, zero pad
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int i = lane + 64 * j;
      if (i < kWinLen) {
        const float cur = S.x[i];
        const float prev = i > 0 ? S.x[i - 1] : cur;
        const float y = fb::preemph(cur, prev) * win[j];
        if (i & 1)
          S.im[fb::sw(i >> 1)] = y;
        else
          S.re[fb::sw(i >> 1)] = y;
      }
    }
    if (lane < kHalf - kWinLen / 2) {
      S.re[fb::sw(kWinLen / 2 + lane)] = 0.0f;
      S.im[fb::sw(kWinLen / 2 + lane)] = 0.0f;
    }
    wave_sync();

    // 3. split-radix generations, unrolled: each generation reads its own
    // descriptor register (a rolled loop rotated the seven descriptors
    // through the registers, 7 moves per generation: 2 % slower)
#pragma unroll
    for (int g = 0; g < FBANK_GENS; ++g) {
      const int o = g * 64 + lane;
      fb::fft_lane_op(gaddr[g], (gmeta >> (4 * g)) & 15u, bt.tw + 6 * o, S.re, S.im);
      wave_sync();
    }

    // 4. real-FFT post-pass + power spectrum into S.x[0..256]
    fb::post_power_ab(k0, a0, b0, S.re, S.im, kn0r, kn0i, S.x);
    fb::post_power_ab(k1, a1, b1, S.re, S.im, kn1r, kn1i, S.x);
    if (lane == 0) fb::edge_power(S.re, S.im, S.x);
    wave_sync();

    // 5. mel energies, floor, log
    if (lane < kMel) {
      const float e = fb::mel_dot(bt.mel_w + mel_wbase, S.x + mel_off, mel_len);
      if (mel_out) mel_out[f * kMel + lane] = e;
      feats[f * kMel + lane] = logf(e < FLT_EPSILON ? FLT_EPSILON : e);
    }
    wave_sync();  // S.x is rewritten by the next frame
  }
}

template <typename Sample>
int launch_fbank_t(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const Sample *pcm, float *feats,
                   float *mel) {
  if (p->total_frames == 0) return CE_GPU_OK;
  const int64_t blocks = (p->total_frames + kFramesPerBlock - 1) / kFramesPerBlock;
  const unsigned grid = (unsigned)(blocks < kMaxBlocks ? blocks : kMaxBlocks);
  hipLaunchKernelGGL(fbank_kernel<Sample>, dim3(grid), dim3(256), 0, s, d_tab, pcm,
                     p->d_sample_off.as<int64_t>(), p->d_frame_off.as<int64_t>(),
                     p->d_block_utt.as<int>(), p->total_frames, feats, mel);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace

int launch_fbank(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const float *pcm,
                 float *feats, float *mel) {
  return launch_fbank_t(s, d_tab, p, pcm, feats, mel);
}

int launch_fbank_s16(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const int16_t *pcm,
                     float *feats, float *mel) {
  return launch_fbank_t(s, d_tab, p, pcm, feats, mel);
}

int fbank_frames_per_block() { return kFramesPerBlock; }

}  // namespace catears
