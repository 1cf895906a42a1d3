// parse_fuzz.cc -- the model-file parsers under AddressSanitizer and
// UndefinedBehaviorSanitizer (CPU only; Makefile target
// build/bin/parse_fuzz_asan, run by tests/test_dropin.py):
//
//   * catears::read_nnet (catears_amd/csrc/model_io.cc, what
//     ce_gpu_model_load_mem / ce_gpu_nnet_check_mem run),
//   * pocketkaldi::Nnet::Read (the drop-in layer, catears_amd/host/src/nnet.cc)
//     over the compat VEC0 / MAT0 readers, and Configuration::Read.
//
// Inputs: a valid TDNN-shaped NN02 image (src/nnet.cc:221-293), every
// truncation of it, hand-made corruptions that must give the reference's
// messages (src/util.cc:123-153, src/vector.cc:267-300, src/matrix.cc:159-191,
// src/nnet.cc:259-264), headers declaring sections billions of bytes long,
// and seeded random byte / word corruptions.  Every input must end in OK, an
// IOError or a Corruption -- never a crash, an abort, an allocation of the
// declared size or a sanitizer report -- and both parsers must agree.
// Prints one line per check; exit status 0 when all pass.
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "configuration.h"
#include "model_io.h"
#include "nnet.h"

using namespace pocketkaldi;

static int failures = 0;
#define CHECK(cond, ...)          \
  do {                            \
    if (!(cond)) {                \
      printf("FAIL ");            \
      printf(__VA_ARGS__);        \
      printf("\n");               \
      ++failures;                 \
    }                             \
  } while (0)

// ---- NN02 image builder -------------------------------------------------

static void put(std::string *s, const void *p, size_t n) { s->append(static_cast<const char *>(p), n); }
static void put_i32(std::string *s, int32_t v) { put(s, &v, 4); }
static void put_vec(std::string *s, int n, float base) {
  put(s, "VEC0", 4);
  put_i32(s, 4 * n + 4);
  put_i32(s, n);
  for (int i = 0; i < n; ++i) {
    const float v = base + 0.01f * i;
    put(s, &v, 4);
  }
}
static void put_mat(std::string *s, int rows, int cols) {
  put(s, "MAT0", 4);
  put_i32(s, 8 + rows * (12 + 4 * cols));
  put_i32(s, rows);
  put_i32(s, cols);
  for (int r = 0; r < rows; ++r) put_vec(s, cols, 0.1f * r);
}
static void layer(std::string *s, int id) {
  put(s, "LAY0", 4);
  put_i32(s, id);
}

// Splice{-2..2} Narrow(2,2) Linear(5*4 -> 6) ReLU BatchNorm(6) Splice{-1,0,1}
// Narrow(1,1) Linear(18 -> 5) LogSoftmax: the converter's shape, small.
// Offsets of the interesting fields go to *at.
struct Marks {
  size_t splice_count, mat_rows, mat_cols, vec_dim, vec_section, layer_type, mat_row_dim;
};
static std::string nn02(Marks *at) {
  std::string s;
  put(&s, "NN02", 4);
  put_i32(&s, 3);
  put_i32(&s, 3);
  put_i32(&s, 9);
  layer(&s, catears::kSplice);
  at->splice_count = s.size();
  put_i32(&s, 5);
  for (int i = -2; i <= 2; ++i) put_i32(&s, i);
  layer(&s, catears::kNarrow);
  put_i32(&s, 2);
  put_i32(&s, 2);
  at->layer_type = s.size() + 4;
  layer(&s, catears::kLinear);
  const size_t m0 = s.size();  // "MAT0", section, rows, cols, then the rows
  at->mat_rows = m0 + 8;
  at->mat_cols = m0 + 12;
  at->mat_row_dim = m0 + 16 + 8;  // first row's VEC0 dim
  put_mat(&s, 20, 6);
  const size_t v0 = s.size();  // "VEC0", section, dim: the bias
  at->vec_section = v0 + 4;
  at->vec_dim = v0 + 8;
  put_vec(&s, 6, 0.5f);
  layer(&s, catears::kReLU);
  layer(&s, catears::kBatchNorm);
  put_vec(&s, 6, 1.0f);
  put_vec(&s, 6, -0.5f);
  layer(&s, catears::kSplice);
  put_i32(&s, 3);
  for (int i = -1; i <= 1; ++i) put_i32(&s, i);
  layer(&s, catears::kNarrow);
  put_i32(&s, 1);
  put_i32(&s, 1);
  layer(&s, catears::kLinear);
  put_mat(&s, 18, 5);
  put_vec(&s, 5, 0.0f);
  layer(&s, catears::kLogSoftmax);
  return s;
}

static void set_i32(std::string *s, size_t at, int32_t v) { memcpy(&(*s)[at], &v, 4); }

// ---- the two parsers ----------------------------------------------------

struct Result {
  int code;  // CE_GPU_OK / CE_GPU_EIO / CE_GPU_ECORRUPT
  std::string msg;
  int layers;
};

static Result parse_capi(const std::string &img) {
  catears::Reader rd;
  Result r{CE_GPU_OK, "", 0};
  int rc = rd.open_mem(img.data(), img.size(), "<nnet image>");
  std::vector<catears::RawLayer> layers;
  int hl = 0, hr = 0;
  if (rc == CE_GPU_OK) rc = catears::read_nnet(rd, &layers, &hl, &hr);
  r.code = rc;
  r.msg = rc == CE_GPU_OK ? "" : catears::last_error();
  r.layers = (int)layers.size();
  return r;
}

static Result parse_dropin(const std::string &path) {
  util::ReadableFile fd;
  Result r{CE_GPU_OK, "", 0};
  Status st = fd.Open(path);
  Nnet nnet;
  if (st.ok()) st = nnet.Read(&fd);
  if (!st.ok()) {
    r.msg = st.what();
    r.code = r.msg.rfind("IOError", 0) == 0 ? CE_GPU_EIO : r.msg.rfind("Corruption", 0) == 0 ? CE_GPU_ECORRUPT : -99;
  }
  return r;
}

static void write_file(const std::string &path, const std::string &data) {
  FILE *f = fopen(path.c_str(), "wb");
  fwrite(data.data(), 1, data.size(), f);
  fclose(f);
}

// Both parsers on one image: they must agree, and a failure must be one of
// the reference's two kinds.  Returns the image parser's result.
static Result both(const std::string &dir, const std::string &img, const char *what) {
  const std::string path = dir + "/fuzz.nnet";
  write_file(path, img);
  Result a = parse_capi(img), b = parse_dropin(path);
  CHECK(a.code == CE_GPU_OK || a.code == CE_GPU_EIO || a.code == CE_GPU_ECORRUPT, "%s: capi code %d", what, a.code);
  CHECK(a.code == b.code, "%s: capi %d '%s' vs drop-in %d '%s'", what, a.code, a.msg.c_str(), b.code, b.msg.c_str());
  if (a.code != CE_GPU_OK) CHECK(!a.msg.empty() && !b.msg.empty(), "%s: empty message", what);
  return a;
}

static bool has(const Result &r, const char *s) { return r.msg.find(s) != std::string::npos; }

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const int iters = argc > 2 ? atoi(argv[2]) : 20000;
  Marks at{};
  const std::string good = nn02(&at);

  Result r = both(dir, good, "valid image");
  CHECK(r.code == CE_GPU_OK && r.layers == 9, "valid image: code %d, %d layers", r.code, r.layers);
  printf("ok valid image (%zu bytes, %d layers)\n", good.size(), r.layers);

  // every truncation: the reference's truncated-file error
  int trunc_bad = 0;
  for (size_t n = 1; n < good.size(); ++n) {
    Result t = both(dir, good.substr(0, n), "truncation");
    if (t.code != CE_GPU_EIO || !has(t, "IOError: failed to read")) ++trunc_bad;
  }
  CHECK(trunc_bad == 0, "%d truncations did not fail as truncated files", trunc_bad);
  printf("ok %zu truncations\n", good.size() - 1);

  // the reference's messages
  std::string img = good;
  img[3] = '3';
  r = both(dir, img, "NN02 tag");
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "ReadAndVerifyString: 'NN02' expected but 'NN03' found"), "tag: %s",
        r.msg.c_str());
  img = good;
  set_i32(&img, at.layer_type, 42);
  r = both(dir, img, "layer type");
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "read_layer: unexpected layer type: 42"), "layer type: %s", r.msg.c_str());
  img = good;
  set_i32(&img, at.vec_section, 99);
  r = both(dir, img, "VEC0 section");
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "section_size = 6 * 4 + 4 expected, but 99 found"), "section: %s",
        r.msg.c_str());
  img = good;
  set_i32(&img, at.mat_cols, 7);
  r = both(dir, img, "MAT0 row width");
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "row_read.Dim() == 7 expected, but 6 found"), "row width: %s",
        r.msg.c_str());
  img = good;
  set_i32(&img, at.mat_rows, -1);
  r = both(dir, img, "MAT0 negative shape");
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "negative matrix shape"), "negative shape: %s", r.msg.c_str());
  img = good;
  set_i32(&img, at.splice_count, -3);
  r = both(dir, img, "Splice count");
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "SpliceLayer: unexpected num_indcies"), "splice: %s", r.msg.c_str());
  printf("ok reference messages\n");

  // sections declared billions of bytes long: refused before any allocation
  img = good;
  set_i32(&img, at.mat_rows, 0x7fffffff);
  set_i32(&img, at.mat_cols, 0x7fffffff);
  r = both(dir, img, "MAT0 2^31 x 2^31");
  // nothing is allocated from the shape: the first row is read, and its
  // width is the reference's error for these bytes
  CHECK(r.code == CE_GPU_ECORRUPT && has(r, "row_read.Dim() == 2147483647 expected, but 6 found"), "huge MAT0: %s",
        r.msg.c_str());
  img = good;
  set_i32(&img, at.mat_rows, 0x7fffffff);
  r = both(dir, img, "MAT0 2^31 rows");
  CHECK(r.code != CE_GPU_OK, "huge MAT0 rows: parsed");
  img = good;
  set_i32(&img, at.vec_dim, 0x1ffffffe);
  set_i32(&img, at.vec_section, 0x1ffffffe * 4 + 4);
  r = both(dir, img, "VEC0 2^29");
  CHECK(r.code == CE_GPU_EIO, "huge VEC0: %s", r.msg.c_str());
  img = good;
  set_i32(&img, at.splice_count, 0x7fffffff);
  r = both(dir, img, "Splice 2^31");
  CHECK(r.code == CE_GPU_EIO, "huge splice: %s", r.msg.c_str());
  img = good;
  set_i32(&img, 12, 0x7fffffff);  // layer count
  r = both(dir, img, "layer count 2^31");
  CHECK(r.code == CE_GPU_EIO, "huge layer count: %s", r.msg.c_str());
  printf("ok oversized sections\n");

  // seeded random corruptions: 1-4 bytes flipped, or one aligned word set to
  // a random / extreme value
  uint64_t st = 0x9e3779b97f4a7c15ull;
  auto next = [&st]() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
  };
  int counts[3] = {0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    img = good;
    if (it & 1) {
      const int k = 1 + (int)(next() % 4);
      for (int j = 0; j < k; ++j) img[next() % img.size()] ^= (char)(1 + next() % 255);
    } else {
      static const int32_t extreme[] = {0, -1, 1, 0x7fffffff, (int32_t)0x80000000, 0x40000000, 65536, 3};
      const size_t w = (next() % (img.size() / 4)) * 4;
      const int32_t v = (next() & 1) ? extreme[next() % 8] : (int32_t)next();
      set_i32(&img, w, v);
    }
    r = both(dir, img, "random corruption");
    counts[r.code == CE_GPU_OK ? 0 : r.code == CE_GPU_EIO ? 1 : 2]++;
  }
  printf("ok %d random corruptions: %d parsed, %d IOError, %d Corruption\n", iters, counts[0], counts[1], counts[2]);

  // compat Configuration::Read on garbage lines: an error or a parse, no crash
  for (int it = 0; it < 200; ++it) {
    std::string text;
    const int len = (int)(next() % 200);
    for (int j = 0; j < len; ++j) text.push_back((char)(next() % 128));
    write_file(dir + "/fuzz.conf", text);
    Configuration c;
    Status s = c.Read(dir + "/fuzz.conf");
    CHECK(s.ok() || !s.what().empty(), "configuration: empty error");
  }
  printf("ok 200 random configuration files\n");

  printf("%s\n", failures ? "FAILED" : "PASSED");
  return failures ? 1 : 0;
}
