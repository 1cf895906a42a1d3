// status.h -- stand-in for pocketkaldi's Status (reference src/status.h:37-104)
// used when the drop-in hot path is built outside the reference tree.  Inside
// the reference build the reference's own header is found first and this one
// is never seen.  Same observable contract: code 0 is success, what() carries
// a "Kind: " prefix.
#ifndef CATEARS_COMPAT_STATUS_H_
#define CATEARS_COMPAT_STATUS_H_

#include <string>
#include <utility>

namespace pocketkaldi {

class Status {
 public:
  Status() = default;

  static Status OK() { return Status(); }
  static Status IOError(const std::string &m) { return Status(1, "IOError: " + m); }
  static Status Corruption(const std::string &m) { return Status(2, "Corruption: " + m); }
  static Status RuntimeError(const std::string &m) { return Status(3, "RuntimeError: " + m); }
  static Status NotImplemented(const std::string &m) { return Status(4, "NotImplemented: " + m); }
  static Status Info(const std::string &m) { return Status(5, m); }

  bool ok() const { return code_ == 0; }
  int code() const { return code_; }
  const std::string &what() const { return text_; }

 private:
  Status(int code, std::string text) : code_(code), text_(std::move(text)) {}
  int code_ = 0;
  std::string text_;
};

}  // namespace pocketkaldi

#endif  // CATEARS_COMPAT_STATUS_H_
