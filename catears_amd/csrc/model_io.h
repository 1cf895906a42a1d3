// model_io.h -- host-only model readers of libcatears_hip: the reference's
// binary sections (VEC0 / MAT0 / NN02), its key = value configuration files,
// and the thread-local error record every C-ABI entry reports through.  No
// HIP here: tests/native/parse_fuzz.cc builds this file alone under
// AddressSanitizer / UndefinedBehaviorSanitizer and feeds it truncated and
// corrupted model images.
#pragma once

#include <stdint.h>
#include <stdio.h>

#include <map>
#include <string>
#include <vector>

#include "catears_gpu.h"

namespace catears {

// Records `msg` as this thread's last error and returns `code`.
int fail(int code, const std::string &msg);
const char *last_error();
std::string fmt(const char *f, ...) __attribute__((format(printf, 1, 2)));

// Little-endian binary reader with the reference's error strings
// (src/util.cc:123-153).  Every section length read from the file is checked
// against the bytes the file still holds before anything is allocated for
// it: a corrupt header (a VEC0 dim or MAT0 shape in the billions) fails as
// the truncated file it is -- "IOError: failed to read: <file>" -- instead of
// the reference's posix_memalign abort / std::bad_alloc, which must not cross
// the C-ABI.
struct Reader {
  FILE *f = nullptr;
  std::string name;
  int64_t size = 0;  // bytes in the file or image
  ~Reader();
  int open(const std::string &path);
  // The same over an in-memory image (ce_gpu_model_load_mem).
  int open_mem(const void *buf, size_t n, const char *label);
  int64_t remaining() const;
  int read(void *dst, size_t n);
  int i32(int32_t *v) { return read(v, 4); }
  int tag(const char *expect);
  // fails with the truncated-file error unless `n` more bytes are there
  int need(int64_t n);
  // Vector<Real>::Read (src/vector.cc:267-300), Real of size 4
  template <typename T>
  int vec(std::vector<T> *out) {
    static_assert(sizeof(T) == 4, "VEC0 payloads here are 4-byte");
    int32_t dim = 0;
    int rc = vec_head(&dim);
    if (rc != CE_GPU_OK) return rc;
    out->resize(dim);
    return read(out->data(), (size_t)dim * 4);
  }
  // Matrix<float>::Read (src/matrix.cc:159-191)
  int mat(std::vector<float> *out, int *rows, int *cols);

 private:
  // "VEC0", section size, dim: checked, and the payload known to be there
  int vec_head(int32_t *dim);
};

// Configuration::Read (src/configuration.cc:14-50): key = value, '#' comments,
// keys case-insensitive, paths relative to the config file's directory.
struct Config {
  std::string file;
  std::map<std::string, std::string> kv;
  int read(const std::string &path);
  int get(const std::string &key, std::string *v) const;
  int path(const std::string &key, std::string *v) const;
  int integer(const std::string &key, int *v) const;
};

// Layer ids (src/nnet.h:21-30).
enum LayerId { kLinear = 0, kReLU = 1, kNormalize = 2, kSoftmax = 3, kSplice = 6, kBatchNorm = 7,
               kLogSoftmax = 8, kNarrow = 9 };

struct RawLayer {
  int id = -1;
  std::vector<float> w, b, scale, offset;  // linear: w is in x out
  int rows = 0, cols = 0;
  std::vector<int32_t> idx;  // splice
  int left = 0, right = 0;   // narrow
};

// Nnet::Read / ReadLayer (src/nnet.cc:221-293): the NN02 header's left /
// right context in *hl / *hr, the layers in file order.
int read_nnet(Reader &rd, std::vector<RawLayer> *layers, int *hl, int *hr);

}  // namespace catears
