// emu_fbank.cc -- TEST HARNESS.  Runs the exact fbank kernel's lane program
// on the CPU: the same table builder (csrc/tables.cc) and the same per-lane
// code (csrc/fbank8_ops.h) as kernels/fbank.hip, the eight lanes of a frame
// one after another between the kernel's synchronisation points, with a
// frame-sized array standing in for the wave's LDS region (each lane writes
// only its own points before a sync and reads any after it, so this order is
// the kernel's).  tests/test_emulation.py compares the pre-log mel energies
// bit for bit with the oracle, which proves the decomposition on a CPU.
// Never linked into the product.
#include <float.h>
#include <math.h>
#include <string.h>

#include "fbank8_ops.h"
#include "internal.h"

using namespace catears;
using namespace catears::fb8;

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
    float re[kLanes][kPts], im[kLanes][kPts];
    float part[kLanes];
    float lds[kStride];
    for (int r = 0; r < kLanes; ++r) part[r] = lane_sum(src, r);
    // the kernel's butterfly over the frame's eight lanes (xor 1, 2, 4)
    for (int d = 1; d < kLanes; d <<= 1) {
      float nxt[kLanes];
      for (int r = 0; r < kLanes; ++r) nxt[r] = part[r] + part[r ^ d];
      memcpy(part, nxt, sizeof(part));
    }
    for (int r = 0; r < kLanes; ++r) {
      lane_window(src, part[r] / (float)kWinLen, r, tab.window, re[r], im[r]);
      phase_a(re[r], im[r], r, [&](int t) { return tab.fb8_twa + (t * kLanes + r) * kTwA; });
    }
    // transpose (re, then im) through the frame's LDS region
    for (int r = 0; r < kLanes; ++r) store_a(re[r], r, lds);
    for (int q = 0; q < kLanes; ++q) load_b(q, lds, re[q]);
    for (int r = 0; r < kLanes; ++r) store_a(im[r], r, lds);
    for (int q = 0; q < kLanes; ++q) load_b(q, lds, im[q]);
    for (int q = 0; q < kLanes; ++q) phase_b(re[q], im[q], q, tab.fb8_tw16);
    // post-pass + power spectrum from each lane's registers into the LDS
    // region, DC / Nyquist by lane 0
    for (int q = 0; q < kLanes; ++q) post_regs(q, re[q], im[q], tab.kn, lds);
    {
      const float z = re[0][0] + im[0][0], nyq = re[0][0] - im[0][0];
      lds[0] = z * z;
      lds[256] = nyq * nyq;
    }
    for (int q = 0; q < kLanes; ++q) {
      float e[kMelSlots];
      const float *w = tab.fb8_mel_w;
      const int *st = tab.fb8_mel_st + q;
      e[0] = mel_window<8>(w + q * kMelWTot + kMelWBase[0], lds + st[0 * kLanes]);
      e[1] = mel_window<12>(w + q * kMelWTot + kMelWBase[1], lds + st[1 * kLanes]);
      e[2] = mel_window<16>(w + q * kMelWTot + kMelWBase[2], lds + st[2 * kLanes]);
      e[3] = mel_window<24>(w + q * kMelWTot + kMelWBase[3], lds + st[3 * kLanes]);
      e[4] = mel_window<32>(w + q * kMelWTot + kMelWBase[4], lds + st[4 * kLanes]);
      for (int c = 0; c < kMelSlots; ++c) {
        const int b = mel_band(c, q);
        mel[(long)f * kMel + b] = e[c];
        feats[(long)f * kMel + b] = logf(e[c] < FLT_EPSILON ? FLT_EPSILON : e[c]);
      }
    }
  }
  return frames;
}
