// Filter catalogue: the exact numeric specification of every operation
// (SURVEY Appendix A).  Shared by the CPU golden path, the chain compiler and,
// through stencil_defs.h, the HIP kernels.
//
// Reference filters:
//   gray:ref      kernel.cu:31-44   Y = trunc(B*.11)+trunc(G*.59)+trunc(R*.3) (double)
//   gray:bt601    kern.cpp:73       OpenCV BGR2GRAY fixed point (>>14, rounded)
//   contrast:3.5  kernel.cu:49-58   trunc(clamp(3.5f*(p-128)+128))
//   contrast:3:cv kern.cpp:74       saturate_cast(3p-256) (OpenCV MatExpr folding)
//   emboss3/5     kernel.cu:64-94, kern.cpp:62-75
// North-star filters (BASELINE.json): invert, brightness, gaussian, sobel, sharpen,
// large-kernel blur.  Extras: gaussian3/7, box3/5, laplace, threshold, expand.
#pragma once

#include <string>
#include <vector>

#include "stripe/common.h"

namespace stripe {

enum class OpKind : int {
  Gray = 0,
  Contrast,
  Invert,
  Brightness,
  Threshold,
  Expand,   // 1 -> 3 channels (GRAY2BGR, kernel.cu:210)
  Stencil,  // integer stencil with compile-time coefficients (stencil_defs.h)
  Conv,     // float KxK convolution (blur:K, conv:...), MFMA path on GPU
};

enum class GrayMode : int { BT601 = 0, Ref = 1 };
enum class RoundMode : int { Trunc = 0, Nearest = 1 };

enum class StencilId : int {
  Emboss3 = 0,
  Emboss5,
  Gaussian3,
  Gaussian5,
  Gaussian7,
  Box3,
  Box5,
  Sharpen,
  Laplace,
  Sobel,
  SobelL2,
  kCount
};

struct StencilInfo {
  StencilId id;
  const char* name;
  int K;                 // window size (odd)
  bool separable;        // weights = w1 (x) w1
  bool sobel;            // sat(|Gx|+|Gy|), or with l2: sat(round(sqrt(Gx^2 + Gy^2)))
  bool l2 = false;
  int div;               // out = sat(floor((sum + div/2) / div)) (div==1: sat(sum))
  std::vector<int> w;    // K*K row-major [dy][dx] (correlation, like filter2D)
  std::vector<int> w1;   // separable 1-D taps
};

const StencilInfo& stencil_info(StencilId id);
bool stencil_from_name(const std::string& name, StencilId* out);

struct Op {
  OpKind kind = OpKind::Gray;
  GrayMode gray = GrayMode::BT601;
  RoundMode round = RoundMode::Trunc;
  float fval = 0.f;  // contrast factor
  int ival = 0;      // brightness delta / threshold
  StencilId sid = StencilId::Gaussian5;
  int K = 0;                  // conv window
  std::vector<float> weights; // conv: K*K f32 weights
  std::vector<float> sep_h, sep_v;  // conv: 1-D factors when weights[dy][dx] = sep_v[dy] * sep_h[dx]
  // conv precision on the MFMA path: 3 = weights as 24-bit fixed point (an
  // output differs from the f64 result only within ~1e-4 of a rounding tie),
  // 2 = 16-bit ("conv:K:w..:lsb", every output within 1 LSB, 2/3 of the MFMAs)
  int conv_digits = 3;
  std::string text;           // canonical spelling
  bool has_border = false;    // per-op border override ("gaussian5@replicate")
  Border border = Border::Reflect101;

  bool pointwise() const { return kind != OpKind::Stencil && kind != OpKind::Conv; }
  int radius() const;
  int channels_out(int cin) const;
};

// Parse "gray:ref,contrast:3.5,emboss3" (also presets "ref-gpu", "ref-cpu").
std::vector<Op> parse_chain(const std::string& spec);
std::string chain_to_string(const std::vector<Op>& ops);

// Gaussian weights exactly as specified for blur:K (OpenCV getGaussianKernel sigma rule).
std::vector<double> gaussian_1d(int K, double sigma);

// ---- pointwise semantics (u8 -> u8 per channel) ----
uint8_t apply_pointwise_u8(const Op& op, uint8_t p);
// Gray conversion of one pixel given semantic R, G, B (PPM order).
uint8_t gray_pixel(GrayMode m, uint8_t r, uint8_t g, uint8_t b);

// Exact integer replacement of trunc((double)x * w) for x in [0,255]:
// returns (mult, shift) with (x*mult)>>shift == trunc(x*w) for all x, or false.
bool find_trunc_magic(double w, uint32_t* mult, int* shift);

}  // namespace stripe
