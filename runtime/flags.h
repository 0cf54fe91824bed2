// --key=value / --key value command-line flags (the gflags subset the
// reference's runtime binaries use).
#pragma once

#include <cstdlib>
#include <map>
#include <string>

struct Flags {
  std::map<std::string, std::string> kv;
  Flags(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a.rfind("--", 0) != 0) continue;
      a = a.substr(2);
      const size_t eq = a.find('=');
      if (eq != std::string::npos) {
        kv[a.substr(0, eq)] = a.substr(eq + 1);
      } else if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) {
        kv[a] = argv[++i];
      } else {
        kv[a] = "1";
      }
    }
  }
  bool has(const std::string& k) const { return kv.count(k) != 0; }
  std::string str(const std::string& k, const std::string& d) const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  int integer(const std::string& k, int d) const { return has(k) ? std::atoi(kv.at(k).c_str()) : d; }
  double real(const std::string& k, double d) const { return has(k) ? std::atof(kv.at(k).c_str()) : d; }
};
