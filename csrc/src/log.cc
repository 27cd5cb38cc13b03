#include "sda/log.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <ctime>
#include <mutex>

namespace sda {

namespace {
std::atomic<int> g_level{3};
std::mutex g_mu;
const char* name(int l) {
  switch (l) {
    case 1: return "CRIT";
    case 2: return "ERRO";
    case 3: return "WARN";
    case 4: return "INFO";
    case 5: return "DEBG";
    default: return "TRCE";
  }
}
}  // namespace

void set_log_level(int level) { g_level = level; }
int log_level() { return g_level; }

void log_at(int level, const std::string& msg) {
  if (level > g_level) return;
  auto now = std::chrono::system_clock::now();
  std::time_t t = std::chrono::system_clock::to_time_t(now);
  std::tm tm;
  gmtime_r(&t, &tm);
  char ts[32];
  std::strftime(ts, sizeof(ts), "%b %d %H:%M:%S", &tm);
  std::lock_guard<std::mutex> g(g_mu);
  std::fprintf(stderr, "%s %s %s\n", ts, name(level), msg.c_str());
}

}  // namespace sda
