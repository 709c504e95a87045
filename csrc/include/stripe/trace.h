// Observability and failure-path hooks.
//
// The reference has host wall-clock only (kernel.cu:190,226; kern.cpp:60,86),
// no error propagation between ranks (Q9: a failing rank returns 1 and the
// others hang in MPI) and no way to exercise its failure path.  Here:
//   * TraceRange: roctx ranges around every engine stage (load, scatter, halo,
//     compute, gather, store, h2d, d2h), visible in rocprofv3 --marker-trace;
//   * fault_point(): deterministic fault injection, STRIPE_FAULT="stage[@rank][:mode],...";
//   * comm_timeout_s(): the bound on every blocking wait for a collective
//     (STRIPE_COMM_TIMEOUT_S, default 600 s) after which the group aborts.
#pragma once

#include <sstream>
#include <string>

namespace stripe {

class TraceRange {
 public:
  explicit TraceRange(const char* name);
  explicit TraceRange(const std::string& name) : TraceRange(name.c_str()) {}
  ~TraceRange();
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_ = false;
};

void trace_mark(const char* msg);

// STRIPE_FAULT grammar: comma-separated "stage[@rank][:mode]".  stage is one of
// load, scatter, halo, compute, gather, store, e2e; rank an integer or '*'
// (default: every rank); mode "throw" (default: stripe::Error, which the group
// drivers turn into a collective abort) or "exit" (std::_Exit(3): a crashed
// process, for multi-process tests of the bounded waits).
void fault_point(const char* stage, int rank);

double comm_timeout_s();

// Leveled, rank-prefixed log lines on stderr (SURVEY §5 metrics / logging; the
// reference prints with std::cout from rank 0 only, kernel.cu:186-188,230-232).
// Level from STRIPE_LOG = error | warning | info | debug (default warning, the
// same variable the Python logger reads); `stripe --verbose` sets info.
enum class LogLevel : int { Error = 0, Warning = 1, Info = 2, Debug = 3 };
LogLevel log_level();
void set_log_level(LogLevel l);
void log_line(LogLevel l, int rank, const std::string& msg);  // "[r<rank> hh:mm:ss.mmm L] msg"

}  // namespace stripe

// STRIPE_LOG(Info, rank, "stripe rows " << n): the message is only formatted
// when the level is enabled
#define STRIPE_LOG(level, rank, expr)                                           \
  do {                                                                          \
    if ((int)::stripe::LogLevel::level <= (int)::stripe::log_level()) {         \
      std::ostringstream _ls;                                                   \
      _ls << expr;                                                              \
      ::stripe::log_line(::stripe::LogLevel::level, (rank), _ls.str());         \
    }                                                                           \
  } while (0)
