// roctx ranges, fault injection and the collective wait bound (see trace.h).
// The reference's only instrumentation is a chrono window printed on rank 0
// (kernel.cu:190,226-232) and its error paths return without MPI_Abort
// (kernel.cu:111-114); here stages carry roctx ranges and failures abort
// the whole group.
#include "stripe/trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <sstream>
#include <thread>

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
    if (mode == "stall") {
      // a live peer that never answers (hung driver, stuck host thread): the
      // others must give up at their wait bound, not at this rank's exit
      const double s = 2.0 * comm_timeout_s() + 5.0;
      std::fprintf(stderr, "stripe: %s: stalling for %.0f s\n", msg.str().c_str(), s);
      std::fflush(stderr);
      std::this_thread::sleep_for(std::chrono::duration<double>(s));
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

namespace {
// last-words state: read by a signal handler, so only atomics and buffers
// that are never freed (a replaced line is leaked, a few KB per update)
struct LwText {
  const char* p;
  size_t n;
};
std::atomic<const LwText*> g_lw_text{nullptr};
std::atomic<int> g_lw_fd{-1};
std::atomic<int> g_lw_code{3};
std::atomic<bool> g_lw_written{false};
std::atomic<bool> g_lw_armed{false};
std::atomic<long> g_lw_gen{0};

bool lw_write_once() {
  if (g_lw_written.exchange(true)) return false;
  const int fd = g_lw_fd.load();
  const LwText* t = g_lw_text.load();
  if (!t) return true;
  const char* p = t->p;
  size_t n = t->n;
  while (fd >= 0 && p && n > 0) {
    const ssize_t w = ::write(fd, p, n);
    if (w <= 0) break;
    p += w;
    n -= (size_t)w;
  }
  return true;
}

void lw_on_sigterm(int) {
  lw_write_once();
  std::_Exit(g_lw_code.load());
}
}  // namespace

void last_words_arm(int fd, double deadline_s, int exit_code) {
  g_lw_fd.store(fd);
  g_lw_code.store(exit_code);
  g_lw_armed.store(true);
  const long gen = ++g_lw_gen;
  struct sigaction sa {};
  sa.sa_handler = lw_on_sigterm;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGTERM, &sa, nullptr);
  std::thread([deadline_s, gen] {
    const auto until = std::chrono::steady_clock::now() + std::chrono::duration<double>(deadline_s);
    while (std::chrono::steady_clock::now() < until) {
      if (!g_lw_armed.load() || g_lw_gen.load() != gen) return;
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
    }
    if (!g_lw_armed.load() || g_lw_gen.load() != gen) return;
    std::fprintf(stderr, "stripe: wall-time budget of %.0f s spent; writing the record so far and exiting\n",
                 deadline_s);
    std::fflush(stderr);
    if (lw_write_once()) std::_Exit(g_lw_code.load());
  }).detach();
}

void last_words_set(const std::string& line, int exit_code) {
  if (exit_code >= 0) g_lw_code.store(exit_code);
  if (line.empty()) return;
  std::string s = line;
  if (s.empty() || s.back() != '\n') s.push_back('\n');
  char* buf = new char[s.size()];  // never freed: a signal handler may be reading the previous one
  std::memcpy(buf, s.data(), s.size());
  g_lw_text.store(new LwText{buf, s.size()});
}

bool last_words_emit() { return lw_write_once(); }

void last_words_disarm() {
  g_lw_armed.store(false);
  signal(SIGTERM, SIG_DFL);
}

std::vector<std::string> mapped_libraries(const std::string& stem) {
  std::vector<std::string> out;
  std::FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return out;
  char line[4096];
  while (std::fgets(line, sizeof line, f)) {
    const char* path = std::strchr(line, '/');
    if (!path) continue;
    std::string p(path);
    while (!p.empty() && (p.back() == '\n' || p.back() == ' ')) p.pop_back();
    const size_t slash = p.rfind('/');
    const std::string base = p.substr(slash + 1);
    if (base.compare(0, stem.size(), stem) != 0 || base.find(".so") == std::string::npos) continue;
    // the stem must end the name part ("librccl" matches librccl.so.1, not librccl-net.so)
    const char next = base.size() > stem.size() ? base[stem.size()] : '\0';
    if (next != '.' && next != '\0') continue;
    if (std::find(out.begin(), out.end(), p) == out.end()) out.push_back(p);
  }
  std::fclose(f);
  return out;
}

double await_progress(const std::string& what, double limit_s, const std::function<Progress(std::string*)>& probe,
                      const std::function<bool()>& aborted, const std::function<void(const std::string&)>& give_up) {
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  for (;;) {
    std::string err;
    std::string why;
    if (aborted && aborted()) {
      why = "aborted while waiting for " + what;
    } else {
      const Progress p = probe(&err);
      if (p == Progress::Done) return elapsed() * 1e3;
      if (p == Progress::Failed) why = what + " failed: " + err;
      else if (elapsed() > limit_s)
        why = what + " did not complete within " + std::to_string(limit_s) + " s (STRIPE_COMM_TIMEOUT_S)";
    }
    if (!why.empty()) {
      if (give_up) give_up(why);
      fail(why);
    }
    // spin for the first millisecond (enqueue-only operations finish in
    // microseconds), then back off
    const double el = elapsed();
    if (el > 1e-3) std::this_thread::sleep_for(std::chrono::microseconds(el > 0.1 ? 1000 : 20));
  }
}

}  // namespace stripe
