// emu_fbank.cc -- TEST HARNESS.  Runs the fbank kernel's lane schedule on the
// CPU: the same table builder (csrc/tables.cc) and the same per-lane
// arithmetic (csrc/fbank_ops.h) as kernels/fbank.hip, executing each wave
// generation's 64 lane ops one after another (they are independent by
// construction).  tests/test_emulation.py compares its pre-log mel energies
// bit for bit with the oracle, which proves the decomposition on a CPU.
// Never linked into the product.
#include <float.h>
#include <math.h>
#include <string.h>

#include "fbank_ops.h"
#include "internal.h"

using namespace catears;

extern "C" int emu_fbank(const float *wave, long n, float *mel, float *feats) {
  static FbankTables tab;
  static bool ready = false;
  if (!ready) {
    build_fbank_tables(&tab);
    ready = true;
  }
  const int frames = n < kWinLen ? 0 : (int)(1 + (n - kWinLen) / kShift);
  for (int f = 0; f < frames; ++f) {
    const float *src = wave + (long)f * kShift;
    float x[kWinLen], re[kHalf], im[kHalf], pw[kHalf + 1];
    // wave-reduction order of the kernel: per-lane partial over j, then
    // butterfly over lanes (xor 32, 16, ..., 1)
    float part[64];
    for (int l = 0; l < 64; ++l) {
      part[l] = 0.0f;
      for (int j = 0; j < 7; ++j) {
        int i = l + 64 * j;
        part[l] += i < kWinLen ? src[i] : 0.0f;
      }
    }
    for (int d = 32; d >= 1; d >>= 1) {
      float nxt[64];
      for (int l = 0; l < 64; ++l) nxt[l] = part[l] + part[l ^ d];
      memcpy(part, nxt, sizeof(part));
    }
    const float mean = part[0] / (float)kWinLen;
    for (int i = 0; i < kWinLen; ++i) x[i] = src[i] - mean;
    for (int i = 0; i < kWinLen; ++i) {
      float y = fb::preemph(x[i], i > 0 ? x[i - 1] : x[i]) * tab.window[i];
      if (i & 1) im[fb::sw(i >> 1)] = y; else re[fb::sw(i >> 1)] = y;
    }
    for (int i = kWinLen / 2; i < kHalf; ++i) re[fb::sw(i)] = im[fb::sw(i)] = 0.0f;
    for (int g = 0; g < kFftGens; ++g)
      for (int l = 0; l < 64; ++l) {
        const int o = g * 64 + l;
        fb::fft_lane_op(tab.fft_addr[o], tab.fft_meta[o], tab.fft_tw + 6 * o, re, im);
      }
    for (int l = 0; l < 64; ++l) {
      fb::post_power(l + 1, re, im, tab.kn, pw);
      fb::post_power(l + 65, re, im, tab.kn, pw);
    }
    fb::edge_power(re, im, pw);
    for (int b = 0; b < kMel; ++b) {
      float e = fb::mel_dot(tab.mel_w + tab.mel_wbase[b], pw + tab.mel_off[b], tab.mel_len[b]);
      mel[(long)f * kMel + b] = e;
      feats[(long)f * kMel + b] = logf(e < FLT_EPSILON ? FLT_EPSILON : e);
    }
  }
  return frames;
}
