// Host runtime utilities: flags, logging, phase timer JSON, roctx ranges.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "moc/common.hpp"
#include "moc/runtime/flags.hpp"
#include "moc/runtime/log.hpp"
#include "moc/runtime/timer.hpp"
#include "moc/runtime/trace.hpp"
#include "moc/runtime/watchdog.hpp"

namespace moc {

// ---------------------------------------------------------------- flags
Flags::Flags(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.rfind("--", 0) != 0 || a.size() == 2) {
      positional_.push_back(a);
      continue;
    }
    a = a.substr(2);
    auto eq = a.find('=');
    if (eq != std::string::npos) {
      values_[a.substr(0, eq)] = a.substr(eq + 1);
    } else if (a.rfind("no-", 0) == 0) {
      values_[a.substr(3)] = "0";
    } else if (i + 1 < argc && std::strncmp(argv[i + 1], "--", 2) != 0) {
      values_[a] = argv[++i];
    } else {
      values_[a] = "1";
    }
  }
}

bool Flags::lookup(const std::string& key, std::string& out) const {
  auto it = values_.find(key);
  if (it != values_.end()) {
    out = it->second;
    return true;
  }
  std::string env = "MOC_";
  for (char c : key) env += (c == '-') ? '_' : static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  const char* v = std::getenv(env.c_str());
  if (v) {
    out = v;
    return true;
  }
  return false;
}

bool Flags::has(const std::string& key) const {
  std::string v;
  return lookup(key, v);
}

std::string Flags::get(const std::string& key, const std::string& def) const {
  std::string v;
  return lookup(key, v) ? v : def;
}

int64_t Flags::get_int(const std::string& key, int64_t def) const {
  std::string v;
  if (!lookup(key, v)) return def;
  char* end = nullptr;
  long long x = std::strtoll(v.c_str(), &end, 0);
  if (end == v.c_str() || *end != '\0') throw Error("flag --" + key + " expects an integer, got '" + v + "'");
  return x;
}

double Flags::get_double(const std::string& key, double def) const {
  std::string v;
  if (!lookup(key, v)) return def;
  char* end = nullptr;
  double x = std::strtod(v.c_str(), &end);
  if (end == v.c_str() || *end != '\0') throw Error("flag --" + key + " expects a number, got '" + v + "'");
  return x;
}

bool Flags::get_bool(const std::string& key, bool def) const {
  std::string v;
  if (!lookup(key, v)) return def;
  if (v == "1" || v == "true" || v == "yes" || v == "on") return true;
  if (v == "0" || v == "false" || v == "no" || v == "off") return false;
  throw Error("flag --" + key + " expects a boolean, got '" + v + "'");
}

std::vector<std::string> Flags::unknown(const std::vector<std::string>& known) const {
  std::vector<std::string> out;
  for (auto& kv : values_) {
    bool ok = false;
    for (auto& k : known) ok = ok || (k == kv.first);
    if (!ok) out.push_back(kv.first);
  }
  return out;
}

// ---------------------------------------------------------------- log
namespace {
LogLevel g_level = LogLevel::Warn;
int g_rank = -1;
}  // namespace

void log_set_level(LogLevel lvl) { g_level = lvl; }
void log_set_level(const std::string& name) {
  if (name == "error") g_level = LogLevel::Error;
  else if (name == "warn") g_level = LogLevel::Warn;
  else if (name == "info") g_level = LogLevel::Info;
  else if (name == "debug") g_level = LogLevel::Debug;
  else throw Error("unknown log level '" + name + "'");
}
void log_set_rank(int rank) {
  g_rank = rank;
  watchdog::set_rank(rank);
}
LogLevel log_level() { return g_level; }

void logf(LogLevel lvl, const char* fmt, ...) {
  if (static_cast<int>(lvl) > static_cast<int>(g_level)) return;
  static const char* names[] = {"E", "W", "I", "D"};
  char msg[2048];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(msg, sizeof msg, fmt, ap);
  va_end(ap);
  if (g_rank >= 0)
    std::fprintf(stderr, "[moc %s r%d] %s\n", names[static_cast<int>(lvl)], g_rank, msg);
  else
    std::fprintf(stderr, "[moc %s] %s\n", names[static_cast<int>(lvl)], msg);
}

// ---------------------------------------------------------------- trace
// roctx is resolved at the first range (dlopen of librocprofiler-sdk-roctx), so CPU-only runs of the
// host core never map any ROCm library. Entry points of the roctx C API (roctx.h).
namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  int (*name_thread)(const char*) = nullptr;
};
const Roctx& roctx() {
  static const Roctx r = [] {
    Roctx x;
    const char* v = std::getenv("MOC_TRACE");
    if (v && (std::strcmp(v, "0") == 0 || std::strcmp(v, "off") == 0)) return x;
    // default: only when a rocprofiler tool (rocprofv3) or the SDK is already in the process — ranges
    // are no-ops otherwise, and loading the library would cost every CPU-only run its start-up time
    const bool forced = v && (std::strcmp(v, "1") == 0 || std::strcmp(v, "on") == 0);
    const bool profiler = dlopen("librocprofiler-sdk-tool.so.1", RTLD_NOLOAD | RTLD_LAZY) ||
                          dlopen("librocprofiler-sdk.so.1", RTLD_NOLOAD | RTLD_LAZY);
    if (!forced && !profiler) return x;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return x;
    x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    x.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
    x.name_thread = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxNameOsThread"));
    return x;
  }();
  return r;
}
}  // namespace

bool trace_enabled() { return roctx().push != nullptr; }
void trace_push(const char* name) {
  if (roctx().push) roctx().push(name);
}
void trace_pop() {
  if (roctx().pop) roctx().pop();
}
void trace_mark(const char* name) {
  if (roctx().mark) roctx().mark(name);
}
void trace_name_thread(const char* name) {
  if (roctx().name_thread) roctx().name_thread(name);
}

// ---------------------------------------------------------------- timer
void PhaseTimer::begin(const std::string& name) {
  if (open_) end();
  cur_ = name;
  watchdog::set_phase(cur_.c_str());
  sw_.reset();
  sw_.start();
  trace_push(cur_.c_str());
  open_ = true;
}

void PhaseTimer::end() {
  if (!open_) return;
  sw_.stop();
  trace_pop();
  open_ = false;
  add(cur_, sw_.total_ms());
}

std::string PhaseTimer::json(const std::vector<std::pair<std::string, double>>& extra) const {
  std::ostringstream os;
  os.precision(6);
  os << std::fixed << "{";
  bool first = true;
  for (auto& p : phases_) {
    os << (first ? "" : ", ") << "\"" << p.first << "_ms\": " << p.second;
    first = false;
  }
  for (auto& p : extra) {
    os << (first ? "" : ", ") << "\"" << p.first << "\": " << p.second;
    first = false;
  }
  os << "}";
  return os.str();
}

}  // namespace moc
