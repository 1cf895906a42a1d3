// configuration.h -- stand-in for pocketkaldi's key=value configuration
// (reference src/configuration.h, src/configuration.cc:14-90): '#' comments,
// case-insensitive keys, paths relative to the file's directory.
#ifndef CATEARS_COMPAT_CONFIGURATION_H_
#define CATEARS_COMPAT_CONFIGURATION_H_

#include <limits.h>

#include <string>
#include <unordered_map>

#include "util.h"

namespace pocketkaldi {

class Configuration {
 public:
  Status Read(const std::string &filename);

  std::string GetPathOrElse(const std::string &key, const std::string &default_val) const;
  std::string GetStringOrElse(const std::string &key, const std::string &default_val) const;
  int GetIntegerOrElse(const std::string &key, int default_val) const;

  Status GetPath(const std::string &key, std::string *val) const;
  Status GetString(const std::string &key, std::string *val) const;
  Status GetInteger(const std::string &key, int *val) const;

  const std::string &filename() const { return filename_; }

 private:
  std::string filename_;
  std::unordered_map<std::string, std::string> table_;
  Status Missing(const std::string &key) const;
};

}  // namespace pocketkaldi

#endif  // CATEARS_COMPAT_CONFIGURATION_H_
