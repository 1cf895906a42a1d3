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

// The split-radix recursion (srfft.cc:124-265) as a DAG of node ops.  A node
// of length m = 2^lg (lg >= 3) becomes m/4 lane ops: lane n owns points n,
// n+m/4, n+m/2, n+3m/4 and performs the node's step-1 butterflies, step-2
// rotation and step-3/4 twiddles on them, in the reference's operation order.
// Nodes of length 4 and 2 are one lane op each.  Independent ops are packed
// into generations of <= 64 lanes (one wave); a node's children go to a later
// generation than the node itself.
struct Pending {
  int lg, base, ready;
};

void build_fft_schedule(FbankTables *t) {
  std::vector<std::vector<uint32_t>> gens(4 * kFftGens);
  std::vector<Pending> pending = {{8, 0, 0}};
  while (!pending.empty()) {
    // earliest-ready first; among equals the longest node (deepest subtree),
    // so leaves, which have no successors, absorb any generation overflow
    size_t pick = 0;
    for (size_t i = 1; i < pending.size(); ++i) {
      const Pending &a = pending[i], &b = pending[pick];
      if (a.ready < b.ready || (a.ready == b.ready && a.lg > b.lg)) pick = i;
    }
    Pending p = pending[pick];
    pending.erase(pending.begin() + pick);
    if (p.lg == 0) continue;
    const int width = p.lg >= 3 ? (1 << p.lg) / 4 : 1;
    int g = p.ready;
    while ((int)gens[g].size() + width > 64) ++g;  // list scheduling
    if (p.lg >= 3) {
      for (int n = 0; n < width; ++n) gens[g].push_back(fft_op(kOpNode, p.lg, n, p.base));
      const int m = 1 << p.lg;
      pending.push_back({p.lg - 1, p.base, g + 1});
      pending.push_back({p.lg - 2, p.base + m / 2, g + 1});
      pending.push_back({p.lg - 2, p.base + 3 * (m / 4), g + 1});
    } else {
      gens[g].push_back(fft_op(p.lg == 2 ? kOpLeaf4 : kOpLeaf2, p.lg, 0, p.base));
    }
  }
  for (size_t g = kFftGens; g < gens.size(); ++g)
    if (!gens[g].empty()) abort();  // schedule must fit kFftGens generations
  for (int g = 0; g < kFftGens; ++g)
    for (int l = 0; l < 64; ++l)
      t->fft_ops[g * 64 + l] = l < (int)gens[g].size() ? gens[g][l] : fft_op(kOpNone, 0, 0, 0);
}

// Lane descriptors of the scheduled ops (fbank_ops.h fft_lane_op): the LDS
// slots and twiddle values each op touches, resolved on the host so the
// kernel's lanes do no index arithmetic.
void build_fft_lanes(FbankTables *t) {
  for (int i = 0; i < kFftGens * 64; ++i) {
    const uint32_t op = t->fft_ops[i];
    const uint32_t kind = op & 3u;
    const int lg = (int)((op >> 2) & 15u), n = (int)((op >> 6) & 255u), base = (int)(op >> 14);
    int pts[4] = {0, 0, 0, 0};
    uint32_t twc = 0;
    if (kind == kOpLeaf2) {
      pts[0] = base, pts[1] = base + 1, pts[2] = base, pts[3] = base + 1;
    } else if (kind == kOpLeaf4) {
      for (int j = 0; j < 4; ++j) pts[j] = base + j;
    } else if (kind == kOpNode) {
      const int q = 1 << (lg - 2), h = 2 * q, e = q / 2;
      pts[0] = base + n, pts[1] = base + n + q, pts[2] = base + n + h, pts[3] = base + n + h + q;
      if (n == e) {
        twc = 1;
      } else if (n > 0) {
        twc = 2;
        const int nel = q - 2, w = n - 1 - (n > e ? 1 : 0);
        for (int j = 0; j < 6; ++j) t->fft_tw[i * 6 + j] = t->twiddle[t->twiddle_base[lg] + j * nel + w];
      }
    }
    uint32_t addr = 0;
    for (int j = 0; j < 4; ++j) addr |= (uint32_t)fb::sw(pts[j]) << (8 * j);
    t->fft_addr[i] = addr;
    t->fft_meta[i] = kind | (twc << 2);
  }
}

// Fast-mode tables: the four-step FFT's inter-pass twiddles, the real-FFT
// post twiddles (both in double, rounded once) and the 40 mel bands in three
// fixed-size slots of a frame's 16 lanes (zero-padded weight windows).
void build_fast(FbankTables *t) {
  const double tau = 6.283185307179586476925286766559005;
  for (int k1 = 0; k1 < 16; ++k1)
    for (int n2 = 0; n2 < 16; ++n2) {
      const double a = tau * n2 * k1 / 256.0;
      t->ff_tw[2 * (k1 * 16 + n2)] = (float)cos(a);
      t->ff_tw[2 * (k1 * 16 + n2) + 1] = (float)-sin(a);
    }
  for (int k = 0; k < kHalf; ++k) {
    const double a = tau * k / 512.0;
    t->ff_post[2 * k] = (float)cos(a);
    t->ff_post[2 * k + 1] = (float)-sin(a);
  }
  // bands by length, longest first: ranks 0-15 fill slot 0, 16-31 slot 1,
  // 32-39 slot 2 (lane = rank mod 16)
  std::vector<int> order(kMel);
  for (int b = 0; b < kMel; ++b) order[b] = b;
  std::sort(order.begin(), order.end(), [&](int a, int b) {
    return t->mel_len[a] != t->mel_len[b] ? t->mel_len[a] > t->mel_len[b] : a < b;
  });
  for (int i = 0; i < 3 * 16; ++i) t->ff_slot_band[i] = -1, t->ff_slot_start[i] = 0;
  for (int r = 0; r < kMel; ++r) {
    const int q = r / 16, j = r % 16, b = order[r], bound = kFfSlot[q];
    if (t->mel_len[b] > bound || t->mel_off[b] < 0) abort();  // the geometry is fixed (src/fbank.h)
    const int start = std::min(t->mel_off[b], kHalf - bound);
    t->ff_slot_band[q * 16 + j] = b;
    t->ff_slot_start[q * 16 + j] = start;
    float *w = t->ff_slot_w + j * kFfSlotW + kFfSlotBase[q] + (t->mel_off[b] - start);
    for (int i = 0; i < t->mel_len[b]; ++i) w[i] = t->mel_w[t->mel_wbase[b] + i];
  }
}

}  // namespace

void build_fbank_tables(FbankTables *t) {
  memset(t, 0, sizeof(*t));
  build_window(t);
  build_mel(t);
  build_twiddles(t);
  build_post_twiddles(t);
  build_fft_schedule(t);
  build_fft_lanes(t);
  build_fast(t);
}

}  // namespace catears
