// compat_test.cc -- CPU test of the drop-in's stand-ins for the reference's
// container layer (catears_amd/host/compat): Configuration parsing and path
// resolution (src/configuration.cc:14-90), VEC0 / MAT0 readers with the
// reference's error strings (src/vector.cc:267-300, src/matrix.cc:159-191).
// Prints one line per check; tests/test_dropin.py runs it.
#include <stdio.h>
#include <string.h>

#include <string>

#include "configuration.h"
#include "matrix.h"
#include "vector.h"

using namespace pocketkaldi;

static int failures = 0;
#define CHECK(cond, what)                                   \
  do {                                                      \
    if (!(cond)) {                                          \
      printf("FAIL %s\n", what);                            \
      ++failures;                                           \
    } else {                                                \
      printf("ok %s\n", what);                              \
    }                                                       \
  } while (0)

static void write_file(const std::string &path, const void *data, size_t n) {
  FILE *f = fopen(path.c_str(), "wb");
  fwrite(data, 1, n, f);
  fclose(f);
}

static std::string vec0(const float *v, int n, int section_override = -1) {
  std::string s("VEC0");
  int32_t sec = section_override >= 0 ? section_override : 4 * n + 4, dim = n;
  s.append(reinterpret_cast<const char *>(&sec), 4);
  s.append(reinterpret_cast<const char *>(&dim), 4);
  s.append(reinterpret_cast<const char *>(v), 4 * (size_t)n);
  return s;
}

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  // Configuration
  const char *conf = "# comment\n  NNet = model.nnet \nprior=/abs/prior.vec\nleft_context = 10\n\n";
  write_file(dir + "/am.conf", conf, strlen(conf));
  Configuration c;
  CHECK(c.Read(dir + "/am.conf").ok(), "config read");
  std::string v;
  CHECK(c.GetPath("nnet", &v).ok() && v == dir + "/model.nnet", "relative path resolved, key case-insensitive");
  CHECK(c.GetPath("prior", &v).ok() && v == "/abs/prior.vec", "absolute path kept");
  int lc = 0;
  CHECK(c.GetInteger("left_context", &lc).ok() && lc == 10, "integer value");
  Status st = c.GetInteger("chunk_size", &lc);
  CHECK(!st.ok() && st.what().find("Unable to find key 'chunk_size'") != std::string::npos, "missing key error");
  const char *bad = "a = b = c\n";
  write_file(dir + "/bad.conf", bad, strlen(bad));
  Configuration c2;
  st = c2.Read(dir + "/bad.conf");
  CHECK(!st.ok() && st.what().rfind("Corruption: Unexpected line", 0) == 0, "malformed line rejected");
  Configuration c3;
  CHECK(!c3.Read(dir + "/absent.conf").ok(), "missing file is an error");

  // VEC0
  const float data[3] = {1.5f, -2.0f, 3.25f};
  std::string good = vec0(data, 3);
  write_file(dir + "/v.bin", good.data(), good.size());
  {
    util::ReadableFile fd;
    Vector<float> vv;
    CHECK(fd.Open(dir + "/v.bin").ok() && vv.Read(&fd).ok() && vv.Dim() == 3 && vv(2) == 3.25f, "VEC0 read");
  }
  std::string badsec = vec0(data, 3, 99);
  write_file(dir + "/vb.bin", badsec.data(), badsec.size());
  {
    util::ReadableFile fd;
    Vector<float> vv;
    fd.Open(dir + "/vb.bin");
    st = vv.Read(&fd);
    CHECK(!st.ok() && st.what().find("section_size = 3 * 4 + 4 expected, but 99 found") != std::string::npos,
          "VEC0 section size check");
  }
  std::string tag = "VECX" + good.substr(4);
  write_file(dir + "/vt.bin", tag.data(), tag.size());
  {
    util::ReadableFile fd;
    Vector<float> vv;
    fd.Open(dir + "/vt.bin");
    st = vv.Read(&fd);
    CHECK(!st.ok() && st.what().find("ReadAndVerifyString: 'VEC0' expected but 'VECX' found") != std::string::npos,
          "VEC0 tag check");
  }
  write_file(dir + "/vs.bin", good.data(), 10);
  {
    util::ReadableFile fd;
    Vector<float> vv;
    fd.Open(dir + "/vs.bin");
    st = vv.Read(&fd);
    CHECK(!st.ok() && st.what().find("failed to read") != std::string::npos, "truncated VEC0");
  }
  // MAT0: 2 x 3
  std::string m("MAT0");
  int32_t sec = 0, rows = 2, cols = 3;
  m.append(reinterpret_cast<const char *>(&sec), 4);
  m.append(reinterpret_cast<const char *>(&rows), 4);
  m.append(reinterpret_cast<const char *>(&cols), 4);
  m += vec0(data, 3);
  const float data2[3] = {4.0f, 5.0f, 6.0f};
  m += vec0(data2, 3);
  write_file(dir + "/m.bin", m.data(), m.size());
  {
    util::ReadableFile fd;
    Matrix<float> mm;
    CHECK(fd.Open(dir + "/m.bin").ok() && mm.Read(&fd).ok() && mm.NumRows() == 2 && mm(1, 2) == 6.0f, "MAT0 read");
  }
  std::string mbad = m.substr(0, 16) + vec0(data, 2) + vec0(data2, 3);
  write_file(dir + "/mb.bin", mbad.data(), mbad.size());
  {
    util::ReadableFile fd;
    Matrix<float> mm;
    fd.Open(dir + "/mb.bin");
    st = mm.Read(&fd);
    CHECK(!st.ok() && st.what().find("row_read.Dim() == 3 expected, but 2 found") != std::string::npos,
          "MAT0 row width check");
  }
  // SubMatrix / Row views share storage
  Matrix<float> a(3, 4);
  a(1, 2) = 7.0f;
  SubMatrix<float> sub = a.Range(1, 2, 1, 3);
  CHECK(sub(0, 1) == 7.0f && sub.Stride() == 4, "SubMatrix view");
  printf("%s\n", failures ? "FAILED" : "PASSED");
  return failures ? 1 : 0;
}
