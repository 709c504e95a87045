// roctx ranges, fault injection and the collective wait bound (see trace.h).
// The reference's only instrumentation is a chrono window printed on rank 0
// (kernel.cu:190,226-232) and its error paths return without MPI_Abort
// (kernel.cu:111-114); here stages carry roctx ranges and failures abort
// the whole group.
#include "stripe/trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <sstream>

#include "stripe/common.h"

namespace stripe {

namespace {

bool tracing_enabled() {
  // roctx calls are cheap without a tool attached; STRIPE_ROCTX=0 removes them
  static const bool on = [] {
    const char* e = std::getenv("STRIPE_ROCTX");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

}  // namespace

TraceRange::TraceRange(const char* name) : on_(tracing_enabled()) {
  if (on_) roctxRangePushA(name);
}

TraceRange::~TraceRange() {
  if (on_) roctxRangePop();
}

void trace_mark(const char* msg) {
  if (tracing_enabled()) roctxMarkA(msg);
}

void fault_point(const char* stage, int rank) {
  const char* env = std::getenv("STRIPE_FAULT");
  if (!env || !*env) return;
  std::stringstream ss(env);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    std::string mode = "throw";
    const size_t colon = item.find(':');
    if (colon != std::string::npos) {
      mode = item.substr(colon + 1);
      item = item.substr(0, colon);
    }
    std::string st = item, rk = "*";
    const size_t at = item.find('@');
    if (at != std::string::npos) {
      st = item.substr(0, at);
      rk = item.substr(at + 1);
    }
    if (st != stage) continue;
    if (rk != "*" && std::atoi(rk.c_str()) != rank) continue;
    std::ostringstream msg;
    msg << "injected fault (STRIPE_FAULT) at stage '" << stage << "' on rank " << rank;
    if (mode == "exit") {
      std::fprintf(stderr, "stripe: %s: exiting\n", msg.str().c_str());
      std::fflush(stderr);
      std::_Exit(3);
    }
    fail(msg.str());
  }
}

namespace {
std::atomic<int> g_log_level{-1};
std::mutex g_log_mu;

int parse_level() {
  const char* e = std::getenv("STRIPE_LOG");
  if (!e) return (int)LogLevel::Warning;
  std::string v(e);
  for (auto& ch : v) ch = (char)std::tolower((unsigned char)ch);
  if (v == "error" || v == "critical") return (int)LogLevel::Error;
  if (v == "info") return (int)LogLevel::Info;
  if (v == "debug") return (int)LogLevel::Debug;
  return (int)LogLevel::Warning;
}
}  // namespace

LogLevel log_level() {
  int l = g_log_level.load(std::memory_order_relaxed);
  if (l < 0) {
    l = parse_level();
    g_log_level.store(l);
  }
  return (LogLevel)l;
}

void set_log_level(LogLevel l) { g_log_level.store((int)l); }

void log_line(LogLevel l, int rank, const std::string& msg) {
  static const char tag[] = {'E', 'W', 'I', 'D'};
  const auto now = std::chrono::system_clock::now();
  const std::time_t t = std::chrono::system_clock::to_time_t(now);
  const int ms = (int)(std::chrono::duration_cast<std::chrono::milliseconds>(now.time_since_epoch()).count() % 1000);
  std::tm tmv{};
  localtime_r(&t, &tmv);
  char ts[32];
  std::strftime(ts, sizeof ts, "%H:%M:%S", &tmv);
  std::lock_guard<std::mutex> lk(g_log_mu);
  std::fprintf(stderr, "[r%d %s.%03d %c] %s\n", rank, ts, ms, tag[(int)l & 3], msg.c_str());
  std::fflush(stderr);
}

double comm_timeout_s() {
  const char* e = std::getenv("STRIPE_COMM_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : 600.0;
}

}  // namespace stripe
