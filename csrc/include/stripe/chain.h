// Chain compiler: turns the parsed filter list into fused passes.
//
// The reference launches one kernel per filter on the default stream
// (kernel.cu:192-195: gray, contrast, emboss = three full passes over the stripe,
// ~8 B/px of DRAM traffic).  Here every run of pointwise ops is folded into a
// 256-entry LUT program and fused into the load path (prologue) of the next
// stencil, or into the store path (epilogue) of the last one, so the reference's
// whole GPU chain becomes ONE kernel (3 B in + 1 B out per pixel).
#pragma once

#include <array>
#include <string>
#include <vector>

#include "stripe/filters.h"

namespace stripe {

// out = expand?( post( gray?( pre(p) ) ) )  -- all per-byte LUTs are exact u8 maps
struct PointwiseProgram {
  bool has_pre = false;
  std::array<uint8_t, 256> pre{};
  bool gray = false;
  GrayMode gmode = GrayMode::BT601;
  bool has_post = false;
  std::array<uint8_t, 256> post{};
  bool expand = false;

  bool identity() const { return !has_pre && !gray && !has_post && !expand; }
  bool lut_only() const { return !gray && !expand && !has_pre; }
  // Prologue of a stencil pass may gray-convert and LUT, but not pre-LUT or expand.
  bool prologue_ok() const { return !has_pre && !expand; }
  int channels_out(int cin) const { return expand ? 3 : (gray ? 1 : cin); }
  uint8_t apply_channel_lut(uint8_t v) const;  // post(pre(v)) when no gray
};

enum class PassKind : int { Pointwise = 0, Separable = 1, Direct = 2, Conv = 3 };

struct Pass {
  PassKind kind = PassKind::Pointwise;
  int cin = 3, cout = 3;   // channels read / written
  int cmid = 3;            // channels after the prologue (= stencil channel count)
  PointwiseProgram pro;    // Pointwise: the whole program; stencil: prologue
  bool has_epi = false;    // stencil epilogue LUT (channel count unchanged)
  std::array<uint8_t, 256> epi{};
  // stencil epilogue `expand`: the 1-channel result (after epi) is stored as 3
  // equal channels (cmid 1 -> cout 3), so gray -> stencil -> expand is one pass
  bool epi_expand = false;
  StencilId sid = StencilId::Gaussian5;
  int K = 1, R = 0;
  Border border = Border::Reflect101;
  std::vector<float> conv_w;  // Conv: K*K weights
  int conv_digits = 3;        // Conv: weight digits of the i8 MFMA path (Op::conv_digits)
  std::vector<float> sep_h, sep_v;  // Conv: 1-D factors of a rank-one window (separable MFMA path)
  // x-margin contract for the output (what the next stencil consumer needs)
  int out_margin_px = 0;
  Border out_margin_border = Border::Reflect101;
  // a gray:ref prologue's post LUT as clamp((a * v + b) >> k, 0, 255) when
  // that is exact for every v (contrast with a dyadic factor, brightness,
  // invert ...): the stencil kernels then map pixel pairs in packed i16
  // instead of LDS lookups
  bool post_aff = false;
  int post_a = 1, post_b = 0, post_k = 0;
  std::string desc;
};

struct Plan {
  std::string spec;
  int cin = 3, cout = 3;
  int max_radius = 0;
  int max_channels = 3;
  int in_margin_px = 0;                      // margins the input must carry
  Border in_margin_border = Border::Reflect101;
  std::vector<Pass> passes;
  std::string describe() const;
};

// default_border: border for every stencil without an explicit @mode suffix.
Plan compile_chain(const std::vector<Op>& ops, int cin, Border default_border,
                   bool fuse = true);

// Gray-conversion parameters in the form the kernels use.
// Find (a, b, k) with lut[v] == clamp((a * v + b) >> k, 0, 255) for every v
// in [0, 255], |a| * 255 + |b| < 2^15 (packed i16 arithmetic), smallest k.
bool lut_affine(const std::array<uint8_t, 256>& lut, int* a, int* b, int* k);

struct GrayParams {
  int mode = 0;           // 0 = bt601, 1 = ref (per-channel trunc magic)
  uint32_t mult[3] = {0, 0, 0};  // R, G, B
  int shift[3] = {0, 0, 0};
};
GrayParams gray_params(GrayMode m);

}  // namespace stripe
