// Command-line flags with environment overrides — the native replacement for the vendored
// CUDA-Samples CLI helpers (inc/helper_string.h:80-262: checkCmdLineFlag, getCmdLineArgumentInt/
// Float/String), which the reference includes but never calls (main() parses no argv, main.c:46-64).
//
// Accepted forms: --key=value, --key value, --flag (boolean true), --no-flag (boolean false).
// Every key can also be set through the environment as MOC_<KEY> (upper case, '-' -> '_');
// an explicit command-line value wins.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace moc {

class Flags {
 public:
  Flags() = default;
  // Parses argv; unknown positional arguments are kept in positional().
  Flags(int argc, char** argv);

  bool has(const std::string& key) const;
  std::string get(const std::string& key, const std::string& def) const;
  int64_t get_int(const std::string& key, int64_t def) const;
  double get_double(const std::string& key, double def) const;
  bool get_bool(const std::string& key, bool def) const;

  const std::vector<std::string>& positional() const { return positional_; }
  const std::map<std::string, std::string>& values() const { return values_; }
  // Keys given on the command line that are not in `known` (for a helpful error).
  std::vector<std::string> unknown(const std::vector<std::string>& known) const;

  void set(const std::string& key, const std::string& value) { values_[key] = value; }

 private:
  bool lookup(const std::string& key, std::string& out) const;
  std::map<std::string, std::string> values_;
  std::vector<std::string> positional_;
};

}  // namespace moc
