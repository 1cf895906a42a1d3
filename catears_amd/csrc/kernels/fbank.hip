// fbank.hip -- batched log-mel filterbank on gfx950, the reference's
// operation order (exact mode, the default).
//
// Replaces the per-frame loop of Fbank::Process (src/fbank.cc:297-303):
// ExtractWindow + ProcessWindow (fbank.cc:44-100), SRFFT::Compute
// (srfft.cc:370-459), ComputePowerSpectrum (fbank.cc:193-211),
// Melbanks::Compute (fbank.cc:165-184), floor + log (fbank.cc:243-244).
//
// Mapping (fbank8_ops.h): eight lanes per frame, eight frames per wave.
//   1. lane r reads the frame's samples 16j + 2r, +1 (and the sample before
//      each pair); the DC sum is an exact butterfly over the frame's lanes;
//   2. DC removal, pre-emphasis (double, as the reference) and the Hamming
//      window give the lane's complex points r + 8j in registers;
//   3. phase A: the 23 node ops of the length-256/128/64/32 nodes that touch
//      the lane's residue class mod 8, in registers;
//   4. one transpose through the wave's LDS (re, then im), then phase B: the
//      length-16/8/4/2 nodes of the lane's two 16-point blocks, in registers;
//   5. the real-FFT post-pass + power spectrum for the lane's 16 pairs (k,
//      256 - k), both operands in its own registers (its blocks are the
//      residue classes r and 16 - r), power into LDS;
//   6. five mel bands per lane over zero-padded 4-aligned windows (16-byte
//      LDS reads), floor at FLT_EPSILON, logf, store.
// Every float operation up to the final logf is the reference's, in the
// reference's order, so pre-log mel energies match bit for bit (the CPU
// emulator of the same lane program, tests/native/emu_fbank.cc, and the GPU
// parity tests check it).  The kernel keeps every value in registers or LDS
// (no scratch: tests/test_abi.py).
#include <float.h>
#include <hip/hip_runtime.h>

#include "../fbank8_ops.h"
#include "../internal.h"

// FB8_FMA (kernels/fbank_fma.hip): the same lane program built with FMA
// contraction and a single-precision pre-emphasis -- the fast mode
#ifdef FB8_FMA
#define FB8_KERNEL fbank_fma_kernel
#define FB8_LAUNCH launch_fbank_fma
#define FB8_LAUNCH_S16 launch_fbank_fma_s16
#elif defined(FB8_NOCASE)
#define FB8_KERNEL fbank_nocase_kernel
#define FB8_LAUNCH launch_fbank_nocase
#define FB8_LAUNCH_S16 launch_fbank_nocase_s16
#else
#define FB8_KERNEL fbank_kernel
#define FB8_LAUNCH launch_fbank
#define FB8_LAUNCH_S16 launch_fbank_s16
#endif

namespace catears {
namespace {

using namespace fb8;

constexpr int kFramesPerBlock = 4;  // granularity of the plan's block_utt table
#ifndef FBANK_WAVES
#define FBANK_WAVES 8
#endif
constexpr int kWaves = FBANK_WAVES;  // waves per block (8 frames each)
constexpr int kBlocksPerCU = kWaves == 8 ? 2 : 3;  // LDS: kWaves x 8 frames x kStride x 4 B (1056 B at 264) + the tables

__device__ __forceinline__ void wave_sync() { wave_lds_sync(); }

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// frame-independent tables, staged once per (persistent) block
struct Fb8Lds {
  float twa[kOpsA * kLanes * kTwA];
  float win[kWinLen];
  float kn[2 * 129];
  alignas(16) float melw[kMelWTot * kLanes];  // read as 16-byte quads (mel_window)
  int mel_st[kMelSlots * kLanes];
};

// MEL: also store the pre-log mel energies (a template argument: a branch on
// the pointer inside the frame loop cost ~57 registers)
template <typename Sample, bool MEL>
__global__ __launch_bounds__(kWaves * 64, 4) void FB8_KERNEL(const FbankTables *__restrict__ tab,
                                                            const Sample *__restrict__ pcm,
                                                            const int64_t *__restrict__ sample_off,
                                                            const int64_t *__restrict__ frame_off,
                                                            const int *__restrict__ block_utt, int64_t total_frames,
                                                            float *__restrict__ feats, float *__restrict__ mel_out) {
  // the tables first: their addresses (a per-lane base plus constants) stay
  // below 64 KB, inside the ds_read immediate offset; behind the 66 KB of
  // frames each table access needed its own address VALU
  struct Smem {
    Fb8Lds T;
    float frames[kWaves * kLanes * kStride];
  };
  __shared__ __attribute__((aligned(16))) Smem sm;
  // kBlocksPerCU blocks must fit the CU's 160 KB of LDS, or occupancy drops
  // silently (the launch bound would still allow them)
  static_assert(kBlocksPerCU * sizeof(Smem) <= 160 * 1024, "fbank_kernel: LDS for kBlocksPerCU blocks exceeds 160 KB");
  static_assert(sizeof(Fb8Lds) % 16 == 0 && sizeof(Fb8Lds) < 64 * 1024, "tables: 16-byte frames, immediate offsets");
  Fb8Lds &T = sm.T;
  float *lds = sm.frames;
  for (int i = threadIdx.x; i < kOpsA * kLanes * kTwA; i += kWaves * 64) T.twa[i] = tab->fb8_twa[i];
  for (int i = threadIdx.x; i < kWinLen; i += kWaves * 64) T.win[i] = tab->window[i];
  for (int i = threadIdx.x; i < 2 * 129; i += kWaves * 64) T.kn[i] = tab->kn[i];
  for (int i = threadIdx.x; i < kMelWTot * kLanes; i += kWaves * 64) T.melw[i] = tab->fb8_mel_w[i];
  for (int i = threadIdx.x; i < kMelSlots * kLanes; i += kWaves * 64) T.mel_st[i] = tab->fb8_mel_st[i];
  const int lane0 = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float tw16[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) tw16[i] = tab->fb8_tw16[i];  // uniform: scalar loads
  __syncthreads();

  const int64_t stride = (int64_t)gridDim.x * kWaves;
  for (int64_t g = (int64_t)blockIdx.x * kWaves + wave; g * kLanes < total_frames; g += stride) {
    // the lane index, opaque per group of frames: the lane's LDS / table
    // addresses are re-derived here (a few adds) instead of being hoisted out
    // of the loop, where dozens of them would stay live in registers
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int r = lane & 7, fs = lane >> 3;
    float *fbuf = lds + (wave * kLanes + fs) * kStride;
    // lanes past the last frame take the last frame: the clamp as a
    // wave-uniform bound on fs (a 64-bit select against a uniform value kept
    // that value in a VGPR, which went to scratch)
    const int64_t left = total_frames - 1 - g * kLanes;  // >= 0 inside the loop
    const int last_fs = (int)(left < kLanes - 1 ? left : kLanes - 1);
    const int64_t fc = g * kLanes + (fs < last_fs ? fs : last_fs);
    int u = block_utt[fc / kFramesPerBlock];
    while (fc >= frame_off[u + 1]) ++u;
    const Sample *src = pcm + sample_off[u] + (fc - frame_off[u]) * kShift;

    // 1-2. samples, DC offset, pre-emphasis, window
    float re[kPts], im[kPts];
    {
      float part = lane_sum(src, r);
      // the frame's eight lanes: quad butterflies, then the other quad of
      // the eight (row_half_mirror); exact integer sums, any order
      part += dpp_f<0xB1>(part);   // quad_perm [1,0,3,2]
      part += dpp_f<0x4E>(part);   // quad_perm [2,3,0,1]
      part += dpp_f<0x141>(part);  // row_half_mirror
      // (the compiler may not reuse the first pass's loads here: that
      // would keep all 75 samples live at once)
      asm volatile("" ::: "memory");
      lane_window(src, part / (float)kWinLen, r, T.win, re, im);
    }
    // 3. phase A in registers
    phase_a(re, im, r, [&](int t) { return T.twa + (t * kLanes + r) * kTwA; });
    // 4. transpose, phase B in registers
    store_a(re, r, fbuf);
    wave_sync();
    load_b(r, fbuf, re);
    wave_sync();
    store_a(im, r, fbuf);
    wave_sync();
    load_b(r, fbuf, im);
    phase_b(re, im, r, tw16);
    wave_sync();  // every lane's load_b reads are done: the region takes the power spectrum
    // 5. real-FFT post-pass + power spectrum, operands from the lane's own
    // registers (fbank8_ops.h post_regs)
    __builtin_amdgcn_sched_barrier(0);
    post_regs(r, re, im, T.kn, fbuf);
    if (r == 0) {  // DC and Nyquist bins from B_0 (srfft.cc:446-451, fbank.cc:203-204)
      const float z = re[0] + im[0], nyq = re[0] - im[0];
      fbuf[0] = z * z;
      fbuf[256] = nyq * nyq;
    }
    wave_sync();
    // 6. mel energies, floor, log
    int st[kMelSlots];
#pragma unroll
    for (int c = 0; c < kMelSlots; ++c) st[c] = T.mel_st[c * kLanes + r];
    float e[kMelSlots];
    e[0] = mel_window<8>(T.melw + r * kMelWTot + kMelWBase[0], fbuf + st[0]);
    e[1] = mel_window<12>(T.melw + r * kMelWTot + kMelWBase[1], fbuf + st[1]);
    e[2] = mel_window<16>(T.melw + r * kMelWTot + kMelWBase[2], fbuf + st[2]);
    e[3] = mel_window<24>(T.melw + r * kMelWTot + kMelWBase[3], fbuf + st[3]);
    e[4] = mel_window<32>(T.melw + r * kMelWTot + kMelWBase[4], fbuf + st[4]);
    wave_sync();  // the frame region is rewritten by the next group of frames
    // lanes past the last frame computed that frame (fc) bit for bit, so
    // they store the same values to the same row: no divergent branch (one
    // costs ~70 registers here, the compiler's choice)
#pragma unroll
    for (int c = 0; c < kMelSlots; ++c) {
      const int b = mel_band(c, r);
      if (MEL) mel_out[fc * kMel + b] = e[c];
      feats[fc * kMel + b] = logf(e[c] < FLT_EPSILON ? FLT_EPSILON : e[c]);
    }
  }
}

template <typename Sample>
int launch_fbank_t(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const Sample *pcm, float *feats,
                   float *mel) {
  if (p->total_frames == 0) return CE_GPU_OK;
  const int64_t per_block = kWaves * kLanes, blocks = (p->total_frames + per_block - 1) / per_block;
  const int64_t max_blocks = 256 * kBlocksPerCU;
  const unsigned grid = (unsigned)(blocks < max_blocks ? blocks : max_blocks);
  if (mel)
    hipLaunchKernelGGL((FB8_KERNEL<Sample, true>), dim3(grid), dim3(kWaves * 64), 0, s, d_tab, pcm,
                     p->d_sample_off.as<int64_t>(), p->d_frame_off.as<int64_t>(),
                     p->d_block_utt.as<int>(), p->total_frames, feats, mel);
    else
    hipLaunchKernelGGL((FB8_KERNEL<Sample, false>), dim3(grid), dim3(kWaves * 64), 0, s, d_tab, pcm,
                     p->d_sample_off.as<int64_t>(), p->d_frame_off.as<int64_t>(),
                     p->d_block_utt.as<int>(), p->total_frames, feats, mel);
  CE_HIP(hipGetLastError());
  return CE_GPU_OK;
}

}  // namespace

int FB8_LAUNCH(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const float *pcm, float *feats,
               float *mel) {
  return launch_fbank_t(s, d_tab, p, pcm, feats, mel);
}

int FB8_LAUNCH_S16(hipStream_t s, const FbankTables *d_tab, const ce_gpu_plan *p, const int16_t *pcm,
                   float *feats, float *mel) {
  return launch_fbank_t(s, d_tab, p, pcm, feats, mel);
}

#if !defined(FB8_FMA) && !defined(FB8_NOCASE)
int fbank_frames_per_block() { return kFramesPerBlock; }
#endif

}  // namespace catears
