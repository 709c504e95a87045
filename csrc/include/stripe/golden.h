// CPU golden path: a direct, obviously-correct implementation of the filter spec.
//
// It is (a) the oracle every HIP kernel is tested against bit-for-bit, and
// (b) the compute engine of the `host` backend (the reference's CPU variant,
// kern.cpp:58-77, which used OpenCV cvtColor/filter2D).  It never reads the
// x-margins of a padded buffer: borders are resolved by explicit index mapping,
// so it independently checks the margin bookkeeping of the device path.
#pragma once

#include <cstdint>
#include <vector>

#include "stripe/chain.h"
#include "stripe/image.h"

namespace stripe {

// A stripe buffer: row r (local) begins at origin + r*pitch, valid for local rows
// the caller guarantees (own rows plus halos).
struct ConstView {
  const uint8_t* origin = nullptr;
  int64_t pitch = 0;
};
struct MutView {
  uint8_t* origin = nullptr;
  int64_t pitch = 0;
};

// Geometry of the rows a pass sees: local row 0 is global row `row0` of an image
// of `Hg` rows (in no-halo/legacy mode: row0 = 0, Hg = stripe rows).
struct RowGeom {
  int row0 = 0;
  int Hg = 0;
};

// Compute output rows [y0, y1) (local) of one compiled pass.
void golden_pass(const Pass& p, ConstView in, MutView out, int W, RowGeom g, int y0, int y1);

// Whole-image helpers.
Image golden_apply_plan(const Image& in, const Plan& plan);
// Unfused: one op at a time (checks the chain compiler's fusion is exact).
Image golden_apply_ops(const Image& in, const std::vector<Op>& ops, Border default_border);

}  // namespace stripe
