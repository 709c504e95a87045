// Fast host executor of compiled passes (the `host` backend and CPU ops).
//
// Same arithmetic as golden_pass (bit-identical output, tests/test_cpu_exec.py),
// organised for a CPU: the pointwise program becomes byte tables, every stencil
// tap is one auto-vectorised multiply-add sweep over a border-extended row of
// the whole width (x innermost, int32 accumulators), input rows are prologued
// once into a K-row ring, and row blocks run on a small thread pool.  The
// reference's CPU path (kern.cpp:58-77) ran OpenCV's SIMD cvtColor/filter2D;
// golden_pass stays the per-pixel oracle this path is checked against.
#pragma once

#include "stripe/golden.h"

namespace stripe {

// Threads a host pass may use: STRIPE_CPU_THREADS, else the hardware threads
// shared by `ranks_per_host` host ranks.
int cpu_threads(int ranks_per_host = 1);

// Compute output rows [y0, y1) (local) of one compiled pass on `threads` threads.
void cpu_pass(const Pass& p, ConstView in, MutView out, int W, RowGeom g, int y0, int y1, int threads);

// Whole-image helper (like golden_apply_plan).
Image cpu_apply_plan(const Image& in, const Plan& plan, int threads);

}  // namespace stripe
