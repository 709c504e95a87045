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

#include <functional>
#include <sstream>
#include <string>
#include <vector>

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
// load, scatter, halo, compute, gather, store, e2e, dist (entry of the
// pipelined root-frame step, Engine::run_dist); rank an integer or '*'
// (default: every rank); mode "throw" (default: stripe::Error, which the group
// drivers turn into a collective abort), "exit" (std::_Exit(3): a crashed
// process, for multi-process tests of the bounded waits) or "stall" (sleep
// 2 x STRIPE_COMM_TIMEOUT_S + 5 s, then exit: a live peer that never answers).
void fault_point(const char* stage, int rank);

double comm_timeout_s();

// Bounded progress loop of an asynchronous communicator operation (RCCL
// non-blocking init / group end / finalize, a callback comm's posted group):
// `probe` is polled until it reports Done; Failed (its message in *err), the
// `aborted` flag raised by another thread, or `limit_s` elapsed end the loop
// by calling `give_up(message)` (which tears the communicator down) and
// raising stripe::Error.  Returns the milliseconds spent.  The reference's
// failure path is the hang this replaces (kernel.cu:111-114).
enum class Progress : int { Done = 0, Pending = 1, Failed = 2 };
// "Last words" of a benchmark process: one pre-formatted line that reaches
// `fd` exactly once -- from last_words_emit() on the normal path, or, if the
// run is still going at `deadline_s` (seconds from arming) or receives
// SIGTERM (torchrun stopping the group after a peer died), from a native
// watchdog thread / signal handler that writes it and ends the process with
// `exit_code`.  Native, so a rank blocked inside a long native call (which
// holds no Python frame to run a handler in) still reports.  The line is
// replaced with last_words_set() as results accumulate.
void last_words_arm(int fd, double deadline_s, int exit_code);
void last_words_set(const std::string& line, int exit_code = -1);  // exit_code < 0: keep
bool last_words_emit();  // writes the current line unless already written; true if this call wrote
void last_words_disarm();

// Paths of the shared objects mapped into this process whose file name starts
// with `stem` (e.g. "librccl"), from /proc/self/maps: which HIP runtime / RCCL
// copy a process actually runs (the benchmark record and a test pin it).
std::vector<std::string> mapped_libraries(const std::string& stem);
double await_progress(const std::string& what, double limit_s, const std::function<Progress(std::string*)>& probe,
                      const std::function<bool()>& aborted, const std::function<void(const std::string&)>& give_up);

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
