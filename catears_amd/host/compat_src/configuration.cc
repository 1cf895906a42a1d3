// configuration.cc -- stand-in for the reference's Configuration
// (src/configuration.cc:14-90).
#include "configuration.h"

namespace pocketkaldi {

Status Configuration::Read(const std::string &filename) {
  filename_ = filename;
  table_.clear();
  util::ReadableFile fd;
  PK_CHECK_STATUS(fd.Open(filename));
  std::string line;
  Status status;
  while (!fd.Eof() && fd.ReadLine(&line, &status)) {
    line = util::Trim(line);
    if (line.empty() || line[0] == '#') continue;
    const std::vector<std::string> kv = util::Split(line, "=");
    if (kv.size() != 2) return Status::Corruption(util::Format("Unexpected line in {}: {}", filename_, line));
    const std::string value = util::Trim(kv[1]);
    if (value.empty()) return Status::Corruption(util::Format("Value cound not be empty: {}", filename_));
    table_[util::Tolower(util::Trim(kv[0]))] = value;
  }
  return status;
}

std::string Configuration::GetStringOrElse(const std::string &key, const std::string &default_val) const {
  auto it = table_.find(util::Tolower(key));
  return it == table_.end() ? default_val : it->second;
}

std::string Configuration::GetPathOrElse(const std::string &key, const std::string &default_val) const {
  auto it = table_.find(util::Tolower(key));
  if (it == table_.end()) return default_val;
  const std::string &p = it->second;
  if (p[0] == '/') return p;
  const size_t slash = filename_.rfind('/');
  return slash == std::string::npos ? p : filename_.substr(0, slash + 1) + p;
}

int Configuration::GetIntegerOrElse(const std::string &key, int default_val) const {
  auto it = table_.find(util::Tolower(key));
  return it == table_.end() ? default_val : std::stoi(it->second);
}

Status Configuration::Missing(const std::string &key) const {
  return Status::Corruption(util::Format("Unable to find key '{}' in '{}'", key, filename_));
}

Status Configuration::GetPath(const std::string &key, std::string *val) const {
  if (!table_.count(util::Tolower(key))) return Missing(key);
  *val = GetPathOrElse(key, "");
  return Status::OK();
}

Status Configuration::GetString(const std::string &key, std::string *val) const {
  if (!table_.count(util::Tolower(key))) return Missing(key);
  *val = GetStringOrElse(key, "");
  return Status::OK();
}

Status Configuration::GetInteger(const std::string &key, int *val) const {
  if (!table_.count(util::Tolower(key))) return Missing(key);
  *val = GetIntegerOrElse(key, INT_MIN);
  return Status::OK();
}

}  // namespace pocketkaldi
