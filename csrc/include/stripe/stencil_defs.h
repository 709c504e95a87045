// Compile-time coefficient sets for the integer stencils.  Usable from host code
// (golden path / catalogue) and device code (kernels instantiate one template per
// filter so every tap is a literal and zero taps vanish; the reference instead
// keeps runtime-indexed private int[5][5] arrays per thread, kernel.cu:71-82,
// which spill to scratch on CDNA).
//
// Weights are correlation weights indexed [dy][dx] (dy = row offset + R).  The
// reference indexes filter[fx][fy] (kernel.cu:86-88) - transposed - but both of
// its filters are symmetric so the result is identical.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define STRIPE_HD __host__ __device__
#else
#define STRIPE_HD
#endif

namespace stripe {
namespace sdef {

struct Emboss3 {
  static constexpr bool BINOM = false;
  static constexpr int K = 3, R = 1, DIV = 1;
  static constexpr bool SEP = false, SOBEL = false;
  STRIPE_HD static constexpr int w(int dy, int dx) {
    constexpr int t[9] = {-2, -1, 0, -1, 1, 1, 0, 1, 2};  // kernel.cu:71-75
    return t[dy * 3 + dx];
  }
};

struct Emboss5 {
  static constexpr bool BINOM = false;
  static constexpr int K = 5, R = 2, DIV = 1;
  static constexpr bool SEP = false, SOBEL = false;
  STRIPE_HD static constexpr int w(int dy, int dx) {
    constexpr int d[5] = {4, 4, 1, -4, -4};  // kernel.cu:76-82 (diagonal)
    return dy == dx ? d[dy] : 0;
  }
};

struct Sharpen {
  static constexpr bool BINOM = false;
  static constexpr int K = 3, R = 1, DIV = 1;
  static constexpr bool SEP = false, SOBEL = false;
  STRIPE_HD static constexpr int w(int dy, int dx) {
    constexpr int t[9] = {0, -1, 0, -1, 5, -1, 0, -1, 0};
    return t[dy * 3 + dx];
  }
};

struct Laplace {
  static constexpr bool BINOM = false;
  static constexpr int K = 3, R = 1, DIV = 1;
  static constexpr bool SEP = false, SOBEL = false;
  STRIPE_HD static constexpr int w(int dy, int dx) {
    constexpr int t[9] = {0, 1, 0, 1, -4, 1, 0, 1, 0};
    return t[dy * 3 + dx];
  }
};

// Sobel: Gx = [1,2,1]^T (x) [-1,0,1],  Gy = [-1,0,1]^T (x) [1,2,1];  out = sat(|Gx|+|Gy|)
// Both kernels are rank one: the GPU runs it as a separable pair (vertical
// smoothing + difference rows, then horizontal difference + smoothing).
struct Sobel {
  static constexpr bool BINOM = false;
  static constexpr int K = 3, R = 1, DIV = 1;
  static constexpr bool SEP = true, SOBEL = true;
  STRIPE_HD static constexpr int g(int i) { return i == 1 ? 2 : 1; }
  STRIPE_HD static constexpr int wx(int dy, int dx) {
    constexpr int s[3] = {1, 2, 1}, d[3] = {-1, 0, 1};
    return s[dy] * d[dx];
  }
  STRIPE_HD static constexpr int wy(int dy, int dx) {
    constexpr int s[3] = {1, 2, 1}, d[3] = {-1, 0, 1};
    return d[dy] * s[dx];
  }
  STRIPE_HD static constexpr int w(int dy, int dx) { return wx(dy, dx); }
  static constexpr bool L2 = false;
};

// Sobel gradient magnitude: out = sat(round(sqrt(Gx^2 + Gy^2))), the L2 form of
// SURVEY §2.7's "sobel (|Gx|+|Gy| or L2)".  sqrt of an integer is never a
// half-integer, so the rounding is exact: round = k + (n > k^2 + k), k = isqrt(n).
struct SobelL2 : Sobel {
  static constexpr bool L2 = true;
};

// Separable integer smoothing filters: out = (sum + DIV/2) / DIV, sum >= 0.
struct Gaussian3 {  // binomial: cascade of K-1 two-tap sums
  static constexpr bool BINOM = true;
  static constexpr int K = 3, R = 1, DIV = 16;
  static constexpr bool SEP = true, SOBEL = false;
  STRIPE_HD static constexpr int g(int i) {
    constexpr int t[3] = {1, 2, 1};
    return t[i];
  }
  STRIPE_HD static constexpr int w(int dy, int dx) { return g(dy) * g(dx); }
};

struct Gaussian5 {  // binomial: cascade of K-1 two-tap sums
  static constexpr bool BINOM = true;
  static constexpr int K = 5, R = 2, DIV = 256;
  static constexpr bool SEP = true, SOBEL = false;
  STRIPE_HD static constexpr int g(int i) {
    constexpr int t[5] = {1, 4, 6, 4, 1};
    return t[i];
  }
  STRIPE_HD static constexpr int w(int dy, int dx) { return g(dy) * g(dx); }
};

struct Gaussian7 {  // binomial: cascade of K-1 two-tap sums
  static constexpr bool BINOM = true;
  static constexpr int K = 7, R = 3, DIV = 4096;
  static constexpr bool SEP = true, SOBEL = false;
  STRIPE_HD static constexpr int g(int i) {
    constexpr int t[7] = {1, 6, 15, 20, 15, 6, 1};
    return t[i];
  }
  STRIPE_HD static constexpr int w(int dy, int dx) { return g(dy) * g(dx); }
};

struct Box3 {
  static constexpr bool BINOM = false;
  static constexpr int K = 3, R = 1, DIV = 9;
  static constexpr bool SEP = true, SOBEL = false;
  STRIPE_HD static constexpr int g(int) { return 1; }
  STRIPE_HD static constexpr int w(int, int) { return 1; }
};

struct Box5 {
  static constexpr bool BINOM = false;
  static constexpr int K = 5, R = 2, DIV = 25;
  static constexpr bool SEP = true, SOBEL = false;
  STRIPE_HD static constexpr int g(int) { return 1; }
  STRIPE_HD static constexpr int w(int, int) { return 1; }
};

}  // namespace sdef
}  // namespace stripe
