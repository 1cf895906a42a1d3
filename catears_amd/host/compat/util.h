// util.h -- stand-in for the parts of pocketkaldi's util.h (reference
// src/util.h:35-175) that the hot-path classes and their callers use: the
// status macros, util::Format and util::ReadableFile.
#ifndef CATEARS_COMPAT_UTIL_H_
#define CATEARS_COMPAT_UTIL_H_

#include <assert.h>
#include <stdint.h>
#include <stdio.h>

#include <iostream>
#include <string>
#include <type_traits>
#include <vector>

#include "status.h"

#ifndef DISALLOW_COPY_AND_ASSIGN
#define DISALLOW_COPY_AND_ASSIGN(T) \
  T(const T &);                     \
  void operator=(const T &)
#endif

#define PK_UNUSED(x) (void)(x)
#define PK_MIN(a, b) ((a) < (b) ? (a) : (b))
#define PK_PATHMAX 1024

// Early-return on a failed Status (reference src/util.h:35-37).
#define PK_CHECK_STATUS(expr)               \
  {                                         \
    ::pocketkaldi::Status st_ = (expr);     \
    if (!st_.ok()) return st_;              \
  }

#define PK_INFO(msg) std::cout << __FILE__ << ": " << (msg) << std::endl;
#define PK_WARN(msg) std::cout << "WARN: " << __FILE__ << ": " << (msg) << std::endl;
#define PK_DEBUG(msg)

namespace pocketkaldi {
namespace util {

inline std::string ToString(const std::string &v) { return v; }
inline std::string ToString(const char *v) { return std::string(v); }
template <typename T, typename std::enable_if<std::is_arithmetic<T>::value, int>::type = 0>
inline std::string ToString(T v) {
  return std::to_string(v);
}

// "{}" placeholders filled left to right; extra arguments are ignored.
inline std::string Format(const std::string &fmt) { return fmt; }
template <typename T, typename... Rest>
inline std::string Format(const std::string &fmt, const T &first, const Rest &...rest) {
  std::string out = fmt;
  const size_t at = out.find("{}");
  if (at != std::string::npos) out.replace(at, 2, ToString(first));
  return Format(out, rest...);
}

std::string Trim(const std::string &str);
std::vector<std::string> Split(const std::string &str, const std::string &delim);
std::string Tolower(const std::string &str);
Status StringToLong(const std::string &str, long *val);

// Binary/text file reader with Status errors.  Owns the FILE* when opened by
// name, borrows it when constructed from one.
class ReadableFile {
 public:
  ReadableFile() = default;
  explicit ReadableFile(FILE *fd) : fd_(fd), owned_(false) {}
  ~ReadableFile();

  Status Open(const std::string &filename);
  Status Read(void *ptr, int size);
  Status ReadAndVerifyString(const std::string &expected);
  template <typename T>
  Status ReadValue(T *data) {
    return Read(data, sizeof(T));
  }
  // Fails as a truncated file ("failed to read: <file>") unless `bytes`
  // more bytes are left: a section length read from a corrupt header is
  // checked before anything is allocated for it (the reference would try
  // the allocation and abort).  A borrowed stream of unknown size passes.
  Status Need(int64_t bytes);
  bool ReadLine(std::string *line, Status *status);
  bool Eof() const;
  void Close();

  const std::string &filename() const { return filename_; }
  int64_t file_size() const { return file_size_; }

 private:
  std::string filename_;
  FILE *fd_ = nullptr;
  int64_t file_size_ = 0;
  bool owned_ = true;
  ReadableFile(const ReadableFile &) = delete;
  ReadableFile &operator=(const ReadableFile &) = delete;
};

}  // namespace util
}  // namespace pocketkaldi

#endif  // CATEARS_COMPAT_UTIL_H_
