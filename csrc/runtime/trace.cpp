// roctx ranges, fault injection and the collective wait bound (see trace.h).
// The reference's only instrumentation is a chrono window printed on rank 0
// (kernel.cu:190,226-232) and its error paths return without MPI_Abort
// (kernel.cu:111-114); here stages carry roctx ranges and failures abort
// the whole group.
#include "stripe/trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

double comm_timeout_s() {
  const char* e = std::getenv("STRIPE_COMM_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : 600.0;
}

}  // namespace stripe
