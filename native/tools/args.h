// Tiny `--key value` / `--flag` argument parser shared by the tk8s CLI tools.
#pragma once

#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>

namespace tk8s {

class Args {
 public:
  Args(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.rfind("--", 0) != 0) throw std::invalid_argument("unexpected argument: " + a);
      a = a.substr(2);
      const auto eq = a.find('=');
      if (eq != std::string::npos) {
        kv_[a.substr(0, eq)] = a.substr(eq + 1);
      } else if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) {
        kv_[a] = argv[++i];
      } else {
        kv_[a] = "1";
      }
    }
  }
  bool has(const std::string& k) const { return kv_.count(k) != 0; }
  std::string str(const std::string& k, const std::string& def = "") const {
    auto it = kv_.find(k);
    return it == kv_.end() ? def : it->second;
  }
  long long num(const std::string& k, long long def) const {
    auto it = kv_.find(k);
    return it == kv_.end() ? def : std::strtoll(it->second.c_str(), nullptr, 0);
  }

 private:
  std::map<std::string, std::string> kv_;
};

}  // namespace tk8s
