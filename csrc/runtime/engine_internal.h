// Helpers shared by the engine's translation units (engine.cpp,
// engine_schedules.cpp, engine_tune.cpp, engine_transfer.cpp,
// engine_group.cpp); not part of the public API.
#pragma once

#include <chrono>
#include <cstdlib>
#include <cstring>

namespace stripe {

// STRIPE_SCHEDULE_EMU=split|pipe|split1 runs the multi-rank schedules on one
// rank (without the exchange) to time their launch/stream overhead on one GPU.
// Measured, gaussian5 on a 16384x2048 RGB stripe (the N=8 share): one launch
// 43.0 us/step; interior+boundary on one stream 46.9; the overlap schedule
// (cross-stream events around the exchange) 54.4; the pipelined schedule 51.5.
// Cross-queue event waits cost ~7 us per step on this stack, so the pipelined
// schedule (one cross-queue wait on the critical path) is the default.
inline int schedule_emu() {
  static const int v = [] {
    const char* e = std::getenv("STRIPE_SCHEDULE_EMU");
    if (!e) return 0;
    return std::strcmp(e, "split") == 0 ? 1 : std::strcmp(e, "pipe") == 0 ? 2 : std::strcmp(e, "split1") == 0 ? 3 : 0;
  }();
  return v;
}

// Global row of a self-halo stripe's first row inside its virtual frame
// (Engine::geom): beyond any stencil reach, a multiple of the MFMA passes'
// 32-row group grid.
constexpr int kSelfHaloRow0 = 4096;

// host wall clock in milliseconds
inline double host_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace stripe
