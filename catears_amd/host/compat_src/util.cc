// util.cc -- stand-in implementations for compat/util.h (reference
// src/util.cc): string helpers and ReadableFile with the reference's error
// strings ("failed to read: <file>", "ReadAndVerifyString: ...").
#include "util.h"

#include <ctype.h>
#include <errno.h>
#include <stdlib.h>
#include <sys/stat.h>

#include <algorithm>

namespace pocketkaldi {
namespace util {

std::string Trim(const std::string &str) {
  size_t a = 0, b = str.size();
  while (a < b && isspace((unsigned char)str[a])) ++a;
  while (b > a && isspace((unsigned char)str[b - 1])) --b;
  return str.substr(a, b - a);
}

std::vector<std::string> Split(const std::string &str, const std::string &delim) {
  std::vector<std::string> out;
  size_t start = 0;
  for (;;) {
    const size_t at = str.find(delim, start);
    if (at == std::string::npos) {
      out.push_back(str.substr(start));
      return out;
    }
    out.push_back(str.substr(start, at - start));
    start = at + delim.size();
  }
}

std::string Tolower(const std::string &str) {
  std::string s = str;
  std::transform(s.begin(), s.end(), s.begin(), [](unsigned char c) { return (char)tolower(c); });
  return s;
}

Status StringToLong(const std::string &str, long *val) {
  errno = 0;
  char *end = nullptr;
  const long v = strtol(str.c_str(), &end, 0);
  if (errno != 0 || end == str.c_str() || *end != '\0')
    return Status::Corruption(Format("invalid integer string: {}", str));
  *val = v;
  return Status::OK();
}

ReadableFile::~ReadableFile() {
  if (owned_ && fd_) fclose(fd_);
}

Status ReadableFile::Open(const std::string &filename) {
  if (owned_ && fd_) fclose(fd_);
  owned_ = true;
  filename_ = filename;
  fd_ = fopen(filename.c_str(), "rb");
  if (!fd_) return Status::IOError(Format("Unable to open {}", filename));
  fseek(fd_, 0, SEEK_END);
  file_size_ = ftell(fd_);
  fseek(fd_, 0, SEEK_SET);
  return Status::OK();
}

Status ReadableFile::Read(void *ptr, int size) {
  if (size == 0) return Status::OK();
  if (!fd_ || fread(ptr, size, 1, fd_) != 1) return Status::IOError(Format("failed to read: {}", filename_));
  return Status::OK();
}

Status ReadableFile::ReadAndVerifyString(const std::string &expected) {
  std::string got(expected.size(), '\0');
  PK_CHECK_STATUS(Read(&got[0], (int)got.size()));
  got = got.c_str();  // stop at an embedded NUL like the reference's C string compare
  if (got != expected)
    return Status::Corruption(
        Format("ReadAndVerifyString: '{}' expected but '{}' found in {}", expected, got, filename_));
  return Status::OK();
}

Status ReadableFile::Need(int64_t bytes) {
  if (!fd_) return Status::IOError(Format("failed to read: {}", filename_));
  int64_t size = file_size_;
  if (!owned_) {
    struct stat st;
    if (fstat(fileno(fd_), &st) != 0 || !S_ISREG(st.st_mode)) return Status::OK();
    size = st.st_size;
  }
  const long at = ftell(fd_);
  if (at < 0) return Status::OK();
  if (bytes < 0 || bytes > size - at) return Status::IOError(Format("failed to read: {}", filename_));
  return Status::OK();
}

bool ReadableFile::ReadLine(std::string *line, Status *status) {
  line->clear();
  int c;
  bool any = false;
  while ((c = fgetc(fd_)) != EOF) {
    any = true;
    if (c == '\n') break;
    line->push_back((char)c);
  }
  if (!any) {
    if (ferror(fd_)) *status = Status::IOError(filename_);
    return false;
  }
  while (!line->empty() && (line->back() == '\r' || line->back() == '\n')) line->pop_back();
  return true;
}

bool ReadableFile::Eof() const { return fd_ == nullptr || feof(fd_) != 0; }

void ReadableFile::Close() {
  if (owned_ && fd_) fclose(fd_);
  fd_ = nullptr;
}

}  // namespace util
}  // namespace pocketkaldi
