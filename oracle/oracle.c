/*
 * oracle.c -- CPU restatement of CatEars' (pocketkaldi) fbank -> CMVN -> nnet
 * acoustic-scoring path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the MI355X product in catears_amd/.  It
 * is never linked into, loaded by, or called from the product path: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * Every function restates one reference routine with the same floating-point
 * operation order and the same float/double promotions, so that results can
 * be compared bit-for-bit where the reference is pure IEEE arithmetic.  The
 * reference file:line each function follows is cited above it.  Compile with
 * -ffp-contract=off (see oracle/Makefile): the reference is built for x86-64
 * without FMA, so no multiply-add is ever contracted there.
 *
 * Pinning: srfft is checked bit-for-bit against the reference's own srfft.cc
 * compiled from /root/reference (oracle/_ref), fbank / CMVN against the Kaldi
 * dumps the reference's tests hold (test/data/*.txt), nnet layers against the
 * known answers of test/nnet_test.cc, the int8 GEMM bit-for-bit against the
 * vendored gemmlowp compiled from /root/reference (oracle/_ref).  The fp32
 * GEMM inside LinearLayer is OpenBLAS in the reference (not vendored); here it
 * is the k-sequential fp32 sum of SimpleMatMat (src/matrix.cc:275-292).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

/* src/fbank.h:7-13 and src/fbank.cc:15-16 */
enum { ORC_SHIFT = 160, ORC_WINLEN = 400, ORC_PADDED = 512, ORC_NMEL = 40 };
/* src/cmvn.h:10-11 */
enum { ORC_CMVN_WINDOW = 600, ORC_CMVN_GLOBAL = 200 };

/* ------------------------------------------------------------------------ */
/* Split-radix FFT, restating src/srfft.cc.                                  */
/* ------------------------------------------------------------------------ */

typedef struct {
  int n_complex;     /* N_ in the reference: half the real length */
  int logn;
  int *seed;         /* Evans digit-reversal seed table (srfft.cc:80-89) */
  float *tw[32];     /* per level i>=4: 6 arrays of (2^i/4 - 2) coefficients */
} orc_srfft;

/* src/srfft.cc:74-122 -- tables.  Angles are float, cos/sin are the float
 * overloads (C++ <math.h> resolves cos(float) to cosf). */
static void orc_srfft_tables(orc_srfft *f) {
  int half = f->logn / 2 + (f->logn & 1);
  f->seed = (int *)calloc((size_t)1 << half, sizeof(int));
  f->seed[0] = 0;
  f->seed[1] = 1;
  for (int j = 2; j <= half; ++j) {
    int top = 1 << (j - 1);
    for (int i = 0; i < top; ++i) {
      f->seed[i] <<= 1;
      f->seed[i + top] = f->seed[i] + 1;
    }
  }
  for (int lv = f->logn; lv >= 4; --lv) {
    int m = 1 << lv, q = m / 4, e = m / 8, nel = q - 2;
    float *t = (float *)malloc(sizeof(float) * 6 * (size_t)nel);
    f->tw[lv] = t;
    int w = 0;
    for (int n = 1; n < q; ++n) {
      if (n == e) continue;
      float a1 = (float)(n * 6.283185307179586476925286766559005 / m);
      float c = cosf(a1), s = sinf(a1);
      t[0 * nel + w] = c;
      t[1 * nel + w] = -(s + c);
      t[2 * nel + w] = s - c;
      float a3 = (float)(3 * n * 6.283185307179586476925286766559005 / m);
      c = cosf(a3);
      s = sinf(a3);
      t[3 * nel + w] = c;
      t[4 * nel + w] = -(s + c);
      t[5 * nel + w] = s - c;
      ++w;
    }
  }
}

ORC_EXPORT orc_srfft *orc_srfft_new(int real_len) {
  orc_srfft *f = (orc_srfft *)calloc(1, sizeof(orc_srfft));
  f->n_complex = real_len / 2;
  int n = f->n_complex;
  while (n > 1) { n >>= 1; ++f->logn; }
  orc_srfft_tables(f);
  return f;
}

ORC_EXPORT void orc_srfft_free(orc_srfft *f) {
  if (!f) return;
  free(f->seed);
  for (int i = 0; i < 32; ++i) free(f->tw[i]);
  free(f);
}

/* src/srfft.cc:124-265 -- one split-radix pass on (re, im) of length 2^lg. */
static void orc_sr_pass(const orc_srfft *f, float *re, float *im, int lg) {
  float a, b;
  if (lg == 0) return;
  if (lg == 1) {
    a = re[0] + re[1]; re[1] = re[0] - re[1]; re[0] = a;
    a = im[0] + im[1]; im[1] = im[0] - im[1]; im[0] = a;
    return;
  }
  if (lg == 2) {
    a = re[0] + re[2]; re[2] = re[0] - re[2]; re[0] = a;
    a = im[0] + im[2]; im[2] = im[0] - im[2]; im[0] = a;
    a = re[1] + re[3]; re[3] = re[1] - re[3]; re[1] = a;
    a = im[1] + im[3]; im[3] = im[1] - im[3]; im[1] = a;
    a = re[0] + re[1]; re[1] = re[0] - re[1]; re[0] = a;
    a = im[0] + im[1]; im[1] = im[0] - im[1]; im[0] = a;
    a = re[2] + im[3];
    b = im[2] + re[3];
    im[2] = im[2] - re[3];
    re[3] = re[2] - im[3];
    re[2] = a;
    im[3] = b;
    return;
  }
  int m = 1 << lg, h = m / 2, q = m / 4, e = m / 8;
  /* step 1: half-length butterflies */
  for (int n = 0; n < h; ++n) {
    a = re[n] + re[n + h]; re[n + h] = re[n] - re[n + h]; re[n] = a;
    b = im[n] + im[n + h]; im[n + h] = im[n] - im[n + h]; im[n] = b;
  }
  /* step 2: the two odd quarters, multiplied by -j */
  for (int n = h; n < h + q; ++n) {
    int p = n + q;
    a = re[n] + im[p];
    b = im[n] + re[p];
    im[n] = im[n] - re[p];
    re[p] = re[n] - im[p];
    re[n] = a;
    im[p] = b;
  }
  /* steps 3 & 4: twiddles (three-multiply form from the tables) */
  const float sq = (float)0.70710678118654752440;
  int nel = q - 2, w = 0;
  const float *t = lg >= 4 ? f->tw[lg] : NULL;
  for (int n = 1; n < q; ++n) {
    int i1 = h + n, i2 = h + q + n;
    if (n == e) {
      a = sq * (re[i1] + im[i1]);
      im[i1] = sq * (im[i1] - re[i1]);
      re[i1] = a;
      b = sq * (im[i2] - re[i2]);
      im[i2] = -sq * (re[i2] + im[i2]);
      re[i2] = b;
    } else {
      b = t[0 * nel + w] * (re[i1] + im[i1]);
      a = t[1 * nel + w] * re[i1] + b;
      re[i1] = t[2 * nel + w] * im[i1] + b;
      im[i1] = a;
      b = t[3 * nel + w] * (re[i2] + im[i2]);
      a = t[4 * nel + w] * re[i2] + b;
      re[i2] = t[5 * nel + w] * im[i2] + b;
      im[i2] = a;
      ++w;
    }
  }
  orc_sr_pass(f, re, im, lg - 1);
  orc_sr_pass(f, re + h, im + h, lg - 2);
  orc_sr_pass(f, re + 3 * (m / 4), im + 3 * (m / 4), lg - 2);
}

/* src/srfft.cc:267-291 -- Evans' in-place digit-reversal permutation. */
static void orc_bitrev(const orc_srfft *f, float *x) {
  int lg = f->logn, half = lg >> 1, n = 1 << half;
  for (int off = 1; off < n; ++off) {
    int base = n * f->seed[off];
    float t = x[off]; x[off] = x[base]; x[base] = t;
    for (int g = 1; g < f->seed[off]; ++g) {
      int i = off + g * n, j = base + f->seed[g];
      t = x[i]; x[i] = x[j]; x[j] = t;
    }
  }
}

/* src/srfft.cc:310-340 + 293-308 -- forward complex FFT on interleaved data. */
static void orc_cfft_forward(const orc_srfft *f, float *x, float *tmp) {
  int n = f->n_complex;
  for (int i = 0; i < n; ++i) { x[i] = x[2 * i]; tmp[i] = x[2 * i + 1]; }
  memcpy(x + n, tmp, sizeof(float) * (size_t)n);
  orc_sr_pass(f, x, x + n, f->logn);
  if (f->logn > 1) { orc_bitrev(f, x); orc_bitrev(f, x + n); }
  memcpy(tmp, x + n, sizeof(float) * (size_t)n);
  for (int i = n - 1; i > 0; --i) { x[2 * i] = x[i]; x[2 * i + 1] = tmp[i]; }
  x[1] = tmp[0];
}

/* src/srfft.cc:370-459 -- forward real FFT of length 2n.  Output layout:
 * [Re0, Re_n, Re1, Im1, ..., Re_{n-1}, Im_{n-1}]. */
ORC_EXPORT void orc_srfft_forward(const orc_srfft *f, float *data, float *tmp) {
  int len = f->n_complex * 2, half = f->n_complex;
  orc_cfft_forward(f, data, tmp);
  float ang = (float)(6.283185307179586476925286766559005 / len * -1);
  float root_re = cosf(ang), root_im = sinf(ang);
  float k_re = 1.0f, k_im = 0.0f;
  for (int k = 1; 2 * k <= half; ++k) {
    /* kN *= rootN, float complex multiply (srfft.cc:52-56) */
    float nr = (k_re * root_re) - (k_im * root_im);
    k_im = k_re * root_im + k_im * root_re;
    k_re = nr;
    int kk = half - k;
    float c_re = (float)(0.5 * (data[2 * k] + data[len - 2 * k]));
    float c_im = (float)(0.5 * (data[2 * k + 1] - data[len - 2 * k + 1]));
    float d_re = (float)(0.5 * (data[2 * k + 1] + data[len - 2 * k + 1]));
    float d_im = (float)(-0.5 * (data[2 * k] - data[len - 2 * k]));
    data[2 * k] = c_re;
    data[2 * k + 1] = c_im;
    /* c += b*a with a = D_k, b = kN (srfft.cc:58-67) */
    data[2 * k] += k_re * d_re - k_im * d_im;
    data[2 * k + 1] += k_re * d_im + k_im * d_re;
    if (kk != k) {
      data[2 * kk] = c_re;
      data[2 * kk + 1] = -c_im;
      data[2 * kk] += (-k_re) * d_re - k_im * (-d_im);
      data[2 * kk + 1] += (-k_re) * (-d_im) + k_im * d_re;
    }
  }
  float z = data[0] + data[1], nyq = data[0] - data[1];
  data[0] = z;
  data[1] = nyq;
}

/* n transforms back to back (stride = real length): timing without one
 * foreign call per frame (tools/cpu_calibrate.py) */
ORC_EXPORT void orc_srfft_forward_n(const orc_srfft *f, float *data, int n, float *tmp) {
  for (int i = 0; i < n; ++i) orc_srfft_forward(f, data + (long)i * 2 * f->n_complex, tmp);
}

/* ------------------------------------------------------------------------ */
/* Fbank, restating src/fbank.cc.                                            */
/* ------------------------------------------------------------------------ */

typedef struct {
  orc_srfft *fft;
  float window[ORC_WINLEN];
  int mel_off[ORC_NMEL];
  int mel_len[ORC_NMEL];
  float mel_w[ORC_NMEL][ORC_PADDED / 2];
} orc_fbank;

static float orc_mel(float hz) { return 1127.0f * logf(1.0f + hz / 700.0f); }

/* src/fbank.cc:248-255 (window; note the truncated 2*pi of fbank.cc:19) and
 * src/fbank.cc:103-163 (mel triangles). */
ORC_EXPORT orc_fbank *orc_fbank_new(void) {
  orc_fbank *fb = (orc_fbank *)calloc(1, sizeof(orc_fbank));
  fb->fft = orc_srfft_new(ORC_PADDED);
  float a = (float)(6.28318530718 / (ORC_WINLEN - 1));
  for (int i = 0; i < ORC_WINLEN; ++i)
    fb->window[i] = (float)(0.54 - 0.46 * (double)cosf(a * (float)i));
  float fs = 16000.0f;
  int nbins = ORC_PADDED / 2;
  float width = fs / ORC_PADDED;
  float lo = orc_mel(20.0f), hi = orc_mel(8000.0f);
  float delta = (hi - lo) / (ORC_NMEL + 1);
  for (int b = 0; b < ORC_NMEL; ++b) {
    float l = lo + b * delta, c = lo + (b + 1) * delta, r = lo + (b + 2) * delta;
    int first = -1, last = -1;
    float tmp[ORC_PADDED / 2];
    for (int i = 0; i < nbins; ++i) {
      float mel = orc_mel(width * i);
      tmp[i] = 0.0f;
      if (mel > l && mel < r) {
        tmp[i] = mel <= c ? (mel - l) / (c - l) : (r - mel) / (r - c);
        if (first < 0) first = i;
        last = i;
      }
    }
    fb->mel_off[b] = first;
    fb->mel_len[b] = last + 1 - first;
    for (int i = 0; i < fb->mel_len[b]; ++i) fb->mel_w[b][i] = tmp[first + i];
  }
  return fb;
}

ORC_EXPORT void orc_fbank_free(orc_fbank *fb) {
  if (!fb) return;
  orc_srfft_free(fb->fft);
  free(fb);
}

/* Accessors for the host-generated tables (tests compare them with the
 * product's tables). */
ORC_EXPORT const float *orc_fbank_window(const orc_fbank *fb) { return fb->window; }
ORC_EXPORT int orc_fbank_mel(const orc_fbank *fb, int b, float *w, int *off) {
  *off = fb->mel_off[b];
  memcpy(w, fb->mel_w[b], sizeof(float) * (size_t)fb->mel_len[b]);
  return fb->mel_len[b];
}

/* src/fbank.cc:35-42 */
ORC_EXPORT int orc_fbank_num_frames(long n) {
  return n < ORC_WINLEN ? 0 : (int)(1 + (n - ORC_WINLEN) / ORC_SHIFT);
}

/* One frame: src/fbank.cc:74-100 (extract), 44-69 (DC, pre-emphasis, window),
 * 219-245 (FFT, power spectrum, mel, floor, log).  If mel_out != NULL the
 * pre-log mel energies are stored too. */
static void orc_fbank_frame(const orc_fbank *fb, const float *samples, float *feat,
                            float *mel_out) {
  float x[ORC_PADDED], tmp[ORC_PADDED];
  memcpy(x, samples, sizeof(float) * ORC_WINLEN);
  for (int i = ORC_WINLEN; i < ORC_PADDED; ++i) x[i] = 0.0f;
  float sum = 0.0f;
  for (int i = 0; i < ORC_WINLEN; ++i) sum += x[i];
  float mean = sum / ORC_WINLEN;
  for (int i = 0; i < ORC_WINLEN; ++i) x[i] -= mean;
  for (int i = ORC_WINLEN - 1; i > 0; --i) x[i] = (float)((double)x[i] - 0.97 * (double)x[i - 1]);
  x[0] = (float)((double)x[0] - 0.97 * (double)x[0]);
  for (int i = 0; i < ORC_WINLEN; ++i) x[i] *= fb->window[i];
  orc_srfft_forward(fb->fft, x, tmp);
  /* src/fbank.cc:193-211 */
  float p0 = x[0] * x[0], pn = x[1] * x[1];
  for (int i = 1; i < ORC_PADDED / 2; ++i) x[i] = x[2 * i] * x[2 * i] + x[2 * i + 1] * x[2 * i + 1];
  x[0] = p0;
  x[ORC_PADDED / 2] = pn;
  /* src/fbank.cc:165-184 + vector.cc:81-92 (sequential float dot) */
  for (int b = 0; b < ORC_NMEL; ++b) {
    float e = 0.0f;
    const float *w = fb->mel_w[b], *p = x + fb->mel_off[b];
    for (int i = 0; i < fb->mel_len[b]; ++i) e += w[i] * p[i];
    if (mel_out) mel_out[b] = e;
    /* vector.cc:166-184: floor at FLT_EPSILON, natural log (float) */
    if (e < FLT_EPSILON) e = FLT_EPSILON;
    feat[b] = logf(e);
  }
}

/* src/fbank.cc:265-314 over a whole utterance (one-shot).  Returns T. */
ORC_EXPORT int orc_fbank_compute(const orc_fbank *fb, const float *wave, long n, float *feats,
                                 float *mel_energies) {
  int t = orc_fbank_num_frames(n);
  for (int i = 0; i < t; ++i)
    orc_fbank_frame(fb, wave + (long)i * ORC_SHIFT, feats + (long)i * ORC_NMEL,
                    mel_energies ? mel_energies + (long)i * ORC_NMEL : NULL);
  return t;
}

/* ------------------------------------------------------------------------ */
/* Online CMVN, restating src/cmvn.cc:35-110.                                 */
/* ------------------------------------------------------------------------ */

/* global_stats: 41 floats (40 sums + count).  Frames are processed in order
 * 0..T-1 exactly like repeated GetFrame calls. */
ORC_EXPORT void orc_cmvn(const float *global_stats, const float *feats, int t_frames,
                         float *out) {
  float carry[ORC_NMEL + 1];
  for (int t = 0; t < t_frames; ++t) {
    double acc[ORC_NMEL + 1];
    /* ComputeStats (cmvn.cc:35-68): double temp, float carry */
    for (int d = 0; d <= ORC_NMEL; ++d) acc[d] = t > 0 ? (double)carry[d] : 0.0;
    const float *x = feats + (long)t * ORC_NMEL;
    for (int d = 0; d < ORC_NMEL; ++d) acc[d] += (double)x[d];
    acc[ORC_NMEL] += 1.0;
    if (t - ORC_CMVN_WINDOW >= 0) {
      const float *y = feats + (long)(t - ORC_CMVN_WINDOW) * ORC_NMEL;
      for (int d = 0; d < ORC_NMEL; ++d) acc[d] += -1.0 * (double)y[d];
      acc[ORC_NMEL] -= 1.0;
    }
    float st[ORC_NMEL + 1];
    for (int d = 0; d <= ORC_NMEL; ++d) carry[d] = st[d] = (float)acc[d];
    /* SmoothStats (cmvn.cc:70-89) */
    double cnt = st[ORC_NMEL];
    if (cnt < ORC_CMVN_WINDOW) {
      double from_global = ORC_CMVN_WINDOW - cnt;
      if (from_global > ORC_CMVN_GLOBAL) from_global = ORC_CMVN_GLOBAL;
      float alpha = (float)(from_global / (double)global_stats[ORC_NMEL]);
      for (int d = 0; d <= ORC_NMEL; ++d) {
        if (alpha != 1.0f) st[d] += alpha * global_stats[d];
        else st[d] += global_stats[d];
      }
    }
    /* Apply (cmvn.cc:91-98) */
    float scale = (float)(1 / (double)st[ORC_NMEL]);
    float neg = -scale;
    float *o = out + (long)t * ORC_NMEL;
    for (int d = 0; d < ORC_NMEL; ++d) {
      o[d] = x[d];
      if (neg != 1.0f) o[d] += neg * st[d];
      else o[d] += st[d];
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Nnet layers, restating src/nnet.cc.                                        */
/* ------------------------------------------------------------------------ */

/* SimpleMatMat order (src/matrix.cc:275-292): every C element is a float sum
 * over k in increasing order.  The i-k-j loop keeps that per-element order. */
ORC_EXPORT void orc_sgemm(int m, int n, int k, const float *a, int lda, const float *b, int ldb,
                          float *c, int ldc) {
  for (int i = 0; i < m; ++i) {
    float *ci = c + (long)i * ldc;
    for (int j = 0; j < n; ++j) ci[j] = 0.0f;
    const float *ai = a + (long)i * lda;
    for (int kk = 0; kk < k; ++kk) {
      float av = ai[kk];
      const float *bk = b + (long)kk * ldb;
      for (int j = 0; j < n; ++j) ci[j] += av * bk[j];
    }
  }
}

/* LinearLayer::Propagate (nnet.cc:22-36): C = A W, then += b row by row
 * (AddVec with alpha 1.0f takes the plain-add branch, vector.cc:249-257). */
ORC_EXPORT void orc_linear(int rows, int in_dim, int out_dim, const float *x, const float *w,
                           const float *bias, float *y) {
  orc_sgemm(rows, out_dim, in_dim, x, in_dim, w, out_dim, y, out_dim);
  for (int r = 0; r < rows; ++r)
    for (int j = 0; j < out_dim; ++j) y[(long)r * out_dim + j] += bias[j];
}

/* SpliceLayer::Propagate (nnet.cc:50-75): clamp each offset into the block. */
ORC_EXPORT void orc_splice(int rows, int dim, const float *x, int n_idx, const int *idx,
                           float *y) {
  for (int r = 0; r < rows; ++r)
    for (int s = 0; s < n_idx; ++s) {
      int src = r + idx[s];
      if (src < 0) src = 0;
      if (src > rows - 1) src = rows - 1;
      memcpy(y + ((long)r * n_idx + s) * dim, x + (long)src * dim, sizeof(float) * (size_t)dim);
    }
}

/* ReLULayer (nnet.cc:149-160) */
ORC_EXPORT void orc_relu(long count, float *x) {
  for (long i = 0; i < count; ++i)
    if (x[i] < 0.0f) x[i] = 0.0f;
}

/* BatchNormLayer (nnet.cc:106-117): MulElements then AddVec(1.0) -- two
 * roundings. */
ORC_EXPORT void orc_batchnorm(int rows, int dim, float *x, const float *scale, const float *offset) {
  for (int r = 0; r < rows; ++r) {
    float *v = x + (long)r * dim;
    for (int j = 0; j < dim; ++j) v[j] *= scale[j];
    for (int j = 0; j < dim; ++j) v[j] += offset[j];
  }
}

/* LogSoftmaxLayer (nnet.cc:137-146) -> ApplyLogSoftMax (vector.cc:109-122):
 * float sequential sum of expf, no max subtraction. */
ORC_EXPORT void orc_log_softmax(int rows, int dim, float *x) {
  for (int r = 0; r < rows; ++r) {
    float *v = x + (long)r * dim, sum = 0.0f;
    for (int j = 0; j < dim; ++j) sum += expf(v[j]);
    float ls = logf(sum);
    for (int j = 0; j < dim; ++j) v[j] -= ls;
  }
}

/* SoftmaxLayer (nnet.cc:125-134) -> ApplySoftMax (vector.cc:94-107) */
ORC_EXPORT void orc_softmax(int rows, int dim, float *x) {
  for (int r = 0; r < rows; ++r) {
    float *v = x + (long)r * dim, sum = 0.0f;
    for (int j = 0; j < dim; ++j) { v[j] = expf(v[j]); sum += v[j]; }
    for (int j = 0; j < dim; ++j) v[j] /= sum;
  }
}

/* NormalizeLayer (nnet.cc:163-178) */
ORC_EXPORT void orc_normalize(int rows, int dim, float *x) {
  for (int r = 0; r < rows; ++r) {
    float *v = x + (long)r * dim, ss = 0.0f;
    for (int j = 0; j < dim; ++j) ss += v[j] * v[j];
    float scale = (float)sqrt((double)(float)dim / (double)ss);
    for (int j = 0; j < dim; ++j) v[j] *= scale;
  }
}

/* ------------------------------------------------------------------------ */
/* int8 path: Quantize (src/matrix.cc:329-387) and MatMat_U8U8F32            */
/* (src/matrix.cc:389-420 -> gemmlowp eight_bit_int_gemm.cc:338-400).         */
/* ------------------------------------------------------------------------ */

ORC_EXPORT void orc_quant_params(long count, const float *x, float *scale_out, int32_t *zp_out) {
  float mn = FLT_MAX, mx = FLT_MIN; /* FLT_MIN: the reference's max init */
  for (long i = 0; i < count; ++i) {
    if (x[i] > mx) mx = x[i];
    if (x[i] < mn) mn = x[i];
  }
  double scale = (mx - mn) / 255.0;
  double fzp = -mn / scale;
  *zp_out = (int32_t)round(fzp);
  *scale_out = (float)scale;
}

/* The elementwise step of Quantize (src/matrix.cc:378-386):
 * std::max(0.0f, std::min(val, 255.0f)) spelled out as the standard library
 * defines it -- min(a, b) = (b < a) ? b : a, max(a, b) = (a < b) ? b : a --
 * so a NaN input becomes 0. */
ORC_EXPORT void orc_quantize_apply(long count, const float *x, float scale, int32_t zp, uint8_t *q) {
  for (long i = 0; i < count; ++i) {
    float v = x[i] / scale + (float)zp;
    v = (255.0f < v) ? 255.0f : v;
    v = (0.0f < v) ? v : 0.0f;
    q[i] = (uint8_t)roundf(v);
  }
}

ORC_EXPORT void orc_quantize(long count, const float *x, uint8_t *q, float *scale_out,
                             int32_t *zp_out) {
  orc_quant_params(count, x, scale_out, zp_out);
  orc_quantize_apply(count, x, *scale_out, *zp_out, q);
}

/* C[i][j] = float(int32( sum_k (A[i][k]-zpA)(B[k][j]-zpB) )) * (sA*sB).
 * The int32 accumulator is exact modulo 2^32 whatever the summation order,
 * so a 64-bit sum truncated to int32 equals gemmlowp's accumulator. */
ORC_EXPORT void orc_gemm_u8u8_i32(int m, int n, int k, const uint8_t *a, int32_t zpa,
                                  const uint8_t *b, int32_t zpb, int32_t *c) {
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) {
      int64_t acc = 0;
      for (int kk = 0; kk < k; ++kk)
        acc += (int64_t)((int32_t)a[(long)i * k + kk] - zpa) * ((int32_t)b[(long)kk * n + j] - zpb);
      c[(long)i * n + j] = (int32_t)(uint32_t)(uint64_t)acc;
    }
}

ORC_EXPORT void orc_gemm_u8u8f32(int m, int n, int k, const uint8_t *a, float sa, int32_t zpa,
                                 const uint8_t *b, float sb, int32_t zpb, float *c) {
  int32_t *acc = (int32_t *)malloc(sizeof(int32_t) * (size_t)m * (size_t)n);
  orc_gemm_u8u8_i32(m, n, k, a, zpa, b, zpb, acc);
  float s = sa * sb;
  for (long i = 0; i < (long)m * n; ++i) c[i] = (float)acc[i] * s;
  free(acc);
}
