// tables.cc -- host-built constant tables of the fbank kernel.
//
// Every value is produced with the reference's own formula and precision on
// the host (glibc libm), then uploaded once, so the device never evaluates a
// transcendental for a table entry and the window / twiddles / mel weights are
// bit-identical to the reference's:
//   Hamming window        src/fbank.cc:248-255 (2*pi truncated to 6.28318530718,
//                         src/fbank.cc:18-20; cos(float) -> cosf)
//   mel triangles         src/fbank.cc:103-163 (all float; MelScale uses logf)
//   split-radix twiddles  src/srfft.cc:74-122 (float angle, cosf/sinf)
//   real-FFT post twiddle src/srfft.cc:382-392: kN_k = kN_{k-1} * rootN by a
//                         float complex multiply (srfft.cc:52-56), tabled so
//                         that the device can process every k in parallel.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "fbank8_ops.h"
#include "fbank_ops.h"
#include "internal.h"

namespace catears {
namespace {

constexpr double kTwoPiSrfft = 6.283185307179586476925286766559005;  // srfft.cc:37
constexpr double kTwoPiFbank = 6.28318530718;                          // fbank.cc:19

float mel_of(float hz) { return 1127.0f * logf(1.0f + hz / 700.0f); }

void build_window(FbankTables *t) {
  const float step = (float)(kTwoPiFbank / (kWinLen - 1));
  for (int i = 0; i < kWinLen; ++i) {
    float c = cosf(step * (float)i);
    t->window[i] = (float)(0.54 - 0.46 * (double)c);
  }
}

void build_mel(FbankTables *t) {
  const float bin_hz = 16000.0f / kPadded;
  const float mlo = mel_of(20.0f), mhi = mel_of(8000.0f);
  const float step = (mhi - mlo) / (kMel + 1);
  int cursor = 0;
  for (int b = 0; b < kMel; ++b) {
    const float left = mlo + b * step, centre = mlo + (b + 1) * step, right = mlo + (b + 2) * step;
    int first = -1;
    std::vector<float> w;
    for (int k = 0; k < kHalf; ++k) {
      float m = mel_of(bin_hz * k);
      if (!(m > left && m < right)) continue;
      if (first < 0) first = k;
      // zero entries inside the span keep their slot (contiguous weights)
      w.resize(k - first + 1, 0.0f);
      w[k - first] = m <= centre ? (m - left) / (centre - left) : (right - m) / (right - centre);
    }
    t->mel_off[b] = first;
    t->mel_len[b] = (int)w.size();
    t->mel_wbase[b] = cursor;
    for (float v : w) t->mel_w[cursor++] = v;
  }
  t->mel_total = cursor;
}

void build_twiddles(FbankTables *t) {
  int cursor = 0;
  for (int lg = 0; lg < 9; ++lg) t->twiddle_base[lg] = 0;
  for (int lg = 4; lg <= 8; ++lg) {
    const int m = 1 << lg, q = m / 4, e = m / 8, nel = q - 2;
    t->twiddle_base[lg] = cursor;
    float *dst = t->twiddle + cursor;
    int w = 0;
    for (int n = 1; n < q; ++n) {
      if (n == e) continue;
      float a = (float)(n * kTwoPiSrfft / m);
      float c = cosf(a), s = sinf(a);
      dst[w] = c;
      dst[nel + w] = -(s + c);
      dst[2 * nel + w] = s - c;
      a = (float)(3 * n * kTwoPiSrfft / m);
      c = cosf(a);
      s = sinf(a);
      dst[3 * nel + w] = c;
      dst[4 * nel + w] = -(s + c);
      dst[5 * nel + w] = s - c;
      ++w;
    }
    cursor += 6 * nel;
  }
}

void build_post_twiddles(FbankTables *t) {
  const float ang = (float)(kTwoPiSrfft / kPadded * -1);
  const float rr = cosf(ang), ri = sinf(ang);
  float kr = 1.0f, ki = 0.0f;
  t->kn[0] = kr;
  t->kn[1] = ki;
  for (int k = 1; k <= kHalf / 2; ++k) {
    float nr = (kr * rr) - (ki * ri);
    ki = kr * ri + ki * rr;
    kr = nr;
    t->kn[2 * k] = kr;
    t->kn[2 * k + 1] = ki;
  }
}

// Exact-kernel tables (fbank8_ops.h): each lane's phase-A twiddle records,
// the length-16 node's, and the mel slot windows.
void build_fb8(FbankTables *t) {
  auto twid = [&](int lg, int n, float *dst) {
    const int q = 1 << (lg - 2), e = q / 2, nel = q - 2;
    if (n == 0 || n == e) return;  // no table twiddles (srfft.cc:230-239)
    const int w = n - 1 - (n > e ? 1 : 0);
    for (int j = 0; j < 6; ++j) dst[j] = t->twiddle[t->twiddle_base[lg] + j * nel + w];
  };
  for (int op = 0; op < fb8::kOpsA; ++op)
    for (int r = 0; r < fb8::kLanes; ++r) {
      int lg, n;
      fb8::phase_a_op(op, r, &lg, &n);
      twid(lg, n, t->fb8_twa + (op * fb8::kLanes + r) * fb8::kTwA);
    }
  twid(4, 1, t->fb8_tw16);
  twid(4, 3, t->fb8_tw16 + 6);
  for (int c = 0; c < fb8::kMelSlots; ++c)
    for (int q = 0; q < fb8::kLanes; ++q) {
      const int b = fb8::mel_band(c, q), W = fb8::kMelW[c];
      const int st = std::min(t->mel_off[b] & ~3, kHalf - W);
      if (t->mel_off[b] < st || t->mel_off[b] + t->mel_len[b] > st + W) abort();  // fixed geometry (src/fbank.h)
      t->fb8_mel_st[c * fb8::kLanes + q] = st;
      float *w = t->fb8_mel_w + q * fb8::kMelWTot + fb8::kMelWBase[c];
      for (int i = 0; i < t->mel_len[b]; ++i) w[t->mel_off[b] - st + i] = t->mel_w[t->mel_wbase[b] + i];
    }
}

}  // namespace

void build_fbank_tables(FbankTables *t) {
  memset(t, 0, sizeof(*t));
  build_window(t);
  build_mel(t);
  build_twiddles(t);
  build_post_twiddles(t);
  build_fb8(t);
}

}  // namespace catears
