// model_io.cc -- host-only readers of the reference's model files (see
// model_io.h): VEC0 / MAT0 / NN02 sections with the reference's error
// strings, the key = value configuration, and the C-ABI's thread-local error
// record.
#include "model_io.h"

#include <ctype.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <fstream>

namespace catears {

// ---------------------------------------------------------------- errors --

static thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

const char *last_error() { return g_last_error.c_str(); }

std::string fmt(const char *f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

#define MIO_TRY(expr)                 \
  do {                                \
    int rc_ = (expr);                 \
    if (rc_ != CE_GPU_OK) return rc_; \
  } while (0)

// ---------------------------------------------------------------- Reader --

Reader::~Reader() {
  if (f) fclose(f);
}

int Reader::open(const std::string &path) {
  name = path;
  f = fopen(path.c_str(), "rb");
  if (!f) return fail(CE_GPU_EIO, "IOError: Unable to open " + path);
  if (fseek(f, 0, SEEK_END) != 0 || (size = ftell(f)) < 0 || fseek(f, 0, SEEK_SET) != 0)
    return fail(CE_GPU_EIO, "IOError: Unable to open " + path);
  return CE_GPU_OK;
}

int Reader::open_mem(const void *buf, size_t n, const char *label) {
  name = label;
  f = n ? fmemopen(const_cast<void *>(buf), n, "rb") : nullptr;
  if (!f) return fail(CE_GPU_EIO, std::string("IOError: Unable to open ") + label);
  size = (int64_t)n;
  return CE_GPU_OK;
}

int64_t Reader::remaining() const {
  const long at = f ? ftell(f) : -1;
  return at < 0 ? 0 : size - at;
}

int Reader::read(void *dst, size_t n) {
  if (n == 0) return CE_GPU_OK;
  if (!f || fread(dst, n, 1, f) != 1) return fail(CE_GPU_EIO, "IOError: failed to read: " + name);
  return CE_GPU_OK;
}

int Reader::need(int64_t n) {
  if (n < 0 || n > remaining()) return fail(CE_GPU_EIO, "IOError: failed to read: " + name);
  return CE_GPU_OK;
}

int Reader::tag(const char *expect) {
  char got[5] = {0};
  MIO_TRY(read(got, 4));
  if (memcmp(got, expect, 4) != 0)
    return fail(CE_GPU_ECORRUPT, fmt("Corruption: ReadAndVerifyString: '%s' expected but '%s' found in %s", expect,
                                     got, name.c_str()));
  return CE_GPU_OK;
}

int Reader::vec_head(int32_t *dim) {
  MIO_TRY(tag("VEC0"));
  int32_t section = 0, d = 0;
  MIO_TRY(i32(&section));
  MIO_TRY(i32(&d));
  if (d < 0 || (int64_t)d * 4 + 4 != section)
    return fail(CE_GPU_ECORRUPT,
                fmt("Corruption: section_size = %d * 4 + 4 expected, but %d found: %s", d, section, name.c_str()));
  MIO_TRY(need((int64_t)d * 4));
  *dim = d;
  return CE_GPU_OK;
}

int Reader::mat(std::vector<float> *out, int *rows, int *cols) {
  MIO_TRY(tag("MAT0"));
  int32_t section = 0, r = 0, c = 0;
  MIO_TRY(i32(&section));
  MIO_TRY(i32(&r));
  MIO_TRY(i32(&c));
  if (r < 0 || c < 0) return fail(CE_GPU_ECORRUPT, "Corruption: negative matrix shape in " + name);
  // The rows are appended as they are read rather than allocated from the
  // header's shape, so the storage never outgrows the file and every error
  // is the one the reference reports for the same bytes (a short row before
  // the end: the row width; the end first: the truncated file).
  out->clear();
  std::vector<float> row;
  for (int i = 0; i < r; ++i) {
    MIO_TRY(vec(&row));
    if ((int)row.size() != c)
      return fail(CE_GPU_ECORRUPT, fmt("Corruption: Matrix::Read: row_read.Dim() == %d expected, but %d found: %s",
                                       c, (int)row.size(), name.c_str()));
    out->insert(out->end(), row.begin(), row.end());
  }
  *rows = r;
  *cols = c;
  return CE_GPU_OK;
}

// ---------------------------------------------------------------- Config --

static std::string trim(const std::string &s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) ++a;
  while (b > a && isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

int Config::read(const std::string &path) {
  file = path;
  std::ifstream in(path);
  if (!in) return fail(CE_GPU_EIO, "IOError: Unable to open " + path);
  std::string line;
  while (std::getline(in, line)) {
    while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    size_t eq = line.find('=');
    if (eq == std::string::npos || line.find('=', eq + 1) != std::string::npos)
      return fail(CE_GPU_ECORRUPT, "Corruption: Unexpected line in " + path + ": " + line);
    std::string k = trim(line.substr(0, eq)), v = trim(line.substr(eq + 1));
    if (v.empty()) return fail(CE_GPU_ECORRUPT, "Corruption: Value cound not be empty: " + path);
    std::transform(k.begin(), k.end(), k.begin(), [](unsigned char ch) { return (char)tolower(ch); });
    kv[k] = v;
  }
  return CE_GPU_OK;
}

int Config::get(const std::string &key, std::string *v) const {
  auto it = kv.find(key);
  if (it == kv.end()) return fail(CE_GPU_ECORRUPT, "Corruption: Unable to find key '" + key + "' in '" + file + "'");
  *v = it->second;
  return CE_GPU_OK;
}

int Config::path(const std::string &key, std::string *v) const {
  MIO_TRY(get(key, v));
  if ((*v)[0] == '/') return CE_GPU_OK;
  size_t slash = file.rfind('/');
  if (slash != std::string::npos) *v = file.substr(0, slash + 1) + *v;
  return CE_GPU_OK;
}

int Config::integer(const std::string &key, int *v) const {
  std::string s;
  MIO_TRY(get(key, &s));
  char *end = nullptr;
  long x = strtol(s.c_str(), &end, 10);
  if (end == s.c_str()) return fail(CE_GPU_ECORRUPT, "Corruption: not an integer: " + key);
  *v = (int)x;
  return CE_GPU_OK;
}

// ------------------------------------------------------------------ NN02 --

int read_nnet(Reader &rd, std::vector<RawLayer> *layers, int *hl, int *hr) {
  const std::string &path = rd.name;
  MIO_TRY(rd.tag("NN02"));
  int32_t l = 0, r = 0, n = 0;
  MIO_TRY(rd.i32(&l));
  MIO_TRY(rd.i32(&r));
  MIO_TRY(rd.i32(&n));
  *hl = l;
  *hr = r;
  for (int i = 0; i < n; ++i) {
    RawLayer L;
    MIO_TRY(rd.tag("LAY0"));
    int32_t id = 0;
    MIO_TRY(rd.i32(&id));
    L.id = id;
    switch (id) {
      case kLinear:
        MIO_TRY(rd.mat(&L.w, &L.rows, &L.cols));
        MIO_TRY(rd.vec(&L.b));
        break;
      case kReLU:
      case kNormalize:
      case kSoftmax:
      case kLogSoftmax:
        break;
      case kSplice: {
        int32_t cnt = 0;
        MIO_TRY(rd.i32(&cnt));
        if (cnt < 0) return fail(CE_GPU_ECORRUPT, "Corruption: SpliceLayer: unexpected num_indcies");
        MIO_TRY(rd.need((int64_t)cnt * 4));
        L.idx.resize(cnt);
        for (int k = 0; k < cnt; ++k) MIO_TRY(rd.i32(&L.idx[k]));
        break;
      }
      case kBatchNorm:
        MIO_TRY(rd.vec(&L.scale));
        MIO_TRY(rd.vec(&L.offset));
        break;
      case kNarrow:
        MIO_TRY(rd.i32(&L.left));
        MIO_TRY(rd.i32(&L.right));
        break;
      default:
        return fail(CE_GPU_ECORRUPT,
                    fmt("Corruption: read_layer: unexpected layer type: %d (%s)", id, path.c_str()));
    }
    layers->push_back(std::move(L));
  }
  return CE_GPU_OK;
}

}  // namespace catears
