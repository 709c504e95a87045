// Core types shared by every layer of the stripe runtime.
//
// The reference (kernel.cu / kern.cpp) has no error model: every failure prints and
// `return 1`s on one rank while the others deadlock in the next MPI call (SURVEY Q9,
// kernel.cu:111-114,148-206).  Here every failure is a C++ exception carrying a rank
// prefix; the comm layer turns an exception into a collective abort.
#pragma once

#include <cstddef>
#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

namespace stripe {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const std::string& msg) { throw Error(msg); }

#define STRIPE_CHECK(cond, msg)                                              \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::ostringstream _os;                                                \
      _os << __FILE__ << ":" << __LINE__ << ": " << msg;                     \
      ::stripe::fail(_os.str());                                             \
    }                                                                        \
  } while (0)

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
inline int64_t div_up(int64_t v, int64_t a) { return (v + a - 1) / a; }

// ---------------------------------------------------------------------------------
// Padded stripe layout (the invariant every buffer in the pipeline keeps).
//
//   row r (local, r in [-halo, rows + halo)) starts at  origin + r * pitch
//   byte b of a row (b in [-kMarginBytes, E + kMarginBytes)) is valid memory
//   E = W * C  (packed row bytes, pixels interleaved like PPM: R,G,B)
//
// The x-margins hold the border extension (reflect101 by default) of the row so
// stencil kernels read them like ordinary pixels; y-halo rows are filled by the
// neighbour halo exchange (or redirected by the kernel's scalar row mapping at the
// global image edges).  The reference has neither: it drops stripe edges (Q2, Q6).
// ---------------------------------------------------------------------------------
constexpr int kMarginBytes = 64;  // per side, 16-byte aligned
constexpr int kMaxRadius = 16;    // largest stencil radius any pass may use (K <= 33)

inline int64_t packed_row_bytes(int W, int C) { return (int64_t)W * C; }

inline int64_t padded_pitch(int W, int C) {
  // margin | data (rounded to 16 B chunks) | margin | spare for whole-chunk /
  // whole-16-pixel-group stores past the margin, 256 B rows
  return align_up(kMarginBytes + align_up((int64_t)W * C, 16) + kMarginBytes + 128, 256);
}

// Pixels of x-margin a C-channel buffer can hold (for gray 64 > kMaxRadius).
inline int margin_pixels(int C) {
  int m = kMarginBytes / C;
  return m < kMaxRadius ? m : kMaxRadius;
}

enum class Border : int {
  Reflect101 = 0,  // ...cb|abcd|cb...  OpenCV default (kern.cpp:75 filter2D)
  Replicate = 1,   // ...aa|abcd|dd...
  Constant = 2,    // ...00|abcd|00...
  Skip = 3,        // legacy ref-gpu: border pixels keep their (pre-stencil) value
                   // (kernel.cu:83 bounds test, minus its wrap/OOB row+col, Q2)
};

const char* border_name(Border b);
Border parse_border(const std::string& s);

// Map an out-of-range coordinate i (row or pixel column) into [0, n) for the
// given border mode.  Returns -1 for Constant.  Reflect101 is applied repeatedly
// so any i works even for tiny n (OpenCV borderInterpolate semantics).
inline int border_index(int i, int n, Border b) {
  if (i >= 0 && i < n) return i;
  switch (b) {
    case Border::Constant:
      return -1;
    case Border::Replicate:
      return i < 0 ? 0 : n - 1;
    default: {  // Reflect101 and Skip (skip pixels never use the value)
      if (n == 1) return 0;
      const int period = 2 * (n - 1);
      int j = i % period;
      if (j < 0) j += period;
      return j < n ? j : period - j;
    }
  }
}

}  // namespace stripe
