// Filter catalogue and pointwise numerics.
#include "stripe/filters.h"

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>

#include "stripe/stencil_defs.h"

namespace stripe {

const char* border_name(Border b) {
  switch (b) {
    case Border::Reflect101: return "reflect101";
    case Border::Replicate: return "replicate";
    case Border::Constant: return "constant";
    case Border::Skip: return "skip";
  }
  return "?";
}

Border parse_border(const std::string& s) {
  if (s == "reflect101" || s == "reflect" || s == "default") return Border::Reflect101;
  if (s == "replicate" || s == "clamp") return Border::Replicate;
  if (s == "constant" || s == "zero") return Border::Constant;
  if (s == "skip" || s == "legacy") return Border::Skip;
  fail("unknown border mode '" + s + "' (reflect101|replicate|constant|skip)");
}

namespace {

template <class F>
StencilInfo make_info(StencilId id, const char* name) {
  StencilInfo s;
  s.id = id;
  s.name = name;
  s.K = F::K;
  s.separable = F::SEP;
  s.sobel = F::SOBEL;
  if constexpr (F::SOBEL) s.l2 = F::L2;
  s.div = F::DIV;
  for (int dy = 0; dy < F::K; ++dy)
    for (int dx = 0; dx < F::K; ++dx) s.w.push_back(F::w(dy, dx));
  return s;
}

template <class F>
StencilInfo make_sep(StencilId id, const char* name) {
  StencilInfo s = make_info<F>(id, name);
  for (int i = 0; i < F::K; ++i) s.w1.push_back(F::g(i));
  return s;
}

const std::vector<StencilInfo>& table() {
  static const std::vector<StencilInfo> t = [] {
    std::vector<StencilInfo> v((size_t)StencilId::kCount);
    v[(int)StencilId::Emboss3] = make_info<sdef::Emboss3>(StencilId::Emboss3, "emboss3");
    v[(int)StencilId::Emboss5] = make_info<sdef::Emboss5>(StencilId::Emboss5, "emboss5");
    v[(int)StencilId::Gaussian3] = make_sep<sdef::Gaussian3>(StencilId::Gaussian3, "gaussian3");
    v[(int)StencilId::Gaussian5] = make_sep<sdef::Gaussian5>(StencilId::Gaussian5, "gaussian5");
    v[(int)StencilId::Gaussian7] = make_sep<sdef::Gaussian7>(StencilId::Gaussian7, "gaussian7");
    v[(int)StencilId::Box3] = make_sep<sdef::Box3>(StencilId::Box3, "box3");
    v[(int)StencilId::Box5] = make_sep<sdef::Box5>(StencilId::Box5, "box5");
    v[(int)StencilId::Sharpen] = make_info<sdef::Sharpen>(StencilId::Sharpen, "sharpen");
    v[(int)StencilId::Laplace] = make_info<sdef::Laplace>(StencilId::Laplace, "laplace");
    v[(int)StencilId::Sobel] = make_info<sdef::Sobel>(StencilId::Sobel, "sobel");
    v[(int)StencilId::SobelL2] = make_info<sdef::SobelL2>(StencilId::SobelL2, "sobel_l2");
    return v;
  }();
  return t;
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) ++a;
  while (b > a && isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

double parse_num(const std::string& s, const std::string& ctx) {
  char* end = nullptr;
  double v = std::strtod(s.c_str(), &end);
  if (s.empty() || end == s.c_str() || *end != '\0') fail("bad number '" + s + "' in '" + ctx + "'");
  return v;
}

}  // namespace

const StencilInfo& stencil_info(StencilId id) {
  STRIPE_CHECK((int)id >= 0 && (int)id < (int)StencilId::kCount, "bad stencil id");
  return table()[(int)id];
}

bool stencil_from_name(const std::string& name, StencilId* out) {
  static const std::map<std::string, StencilId> alias = {
      {"emboss", StencilId::Emboss3},    {"emboss3", StencilId::Emboss3},
      {"emboss5", StencilId::Emboss5},   {"gaussian", StencilId::Gaussian5},
      {"gaussian3", StencilId::Gaussian3}, {"gaussian5", StencilId::Gaussian5},
      {"gaussian7", StencilId::Gaussian7}, {"gauss5", StencilId::Gaussian5},
      {"box3", StencilId::Box3},         {"box5", StencilId::Box5},
      {"sharpen", StencilId::Sharpen},   {"laplace", StencilId::Laplace},
      {"laplacian", StencilId::Laplace}, {"sobel", StencilId::Sobel},
      {"edge", StencilId::Sobel},        {"sobel_l2", StencilId::SobelL2},
      {"magnitude", StencilId::SobelL2},
  };
  auto it = alias.find(name);
  if (it == alias.end()) return false;
  *out = it->second;
  return true;
}

int Op::radius() const {
  if (kind == OpKind::Stencil) return stencil_info(sid).K / 2;
  if (kind == OpKind::Conv) return K / 2;
  return 0;
}

int Op::channels_out(int cin) const {
  if (kind == OpKind::Gray) return 1;
  if (kind == OpKind::Expand) return 3;
  return cin;
}

std::vector<double> gaussian_1d(int K, double sigma) {
  STRIPE_CHECK(K >= 1 && K % 2 == 1, "gaussian size must be odd, got " << K);
  if (sigma <= 0) sigma = 0.3 * ((K - 1) * 0.5 - 1) + 0.8;  // OpenCV getGaussianKernel rule
  std::vector<double> g(K);
  double s = 0;
  const int R = K / 2;
  for (int i = 0; i < K; ++i) {
    const double x = i - R;
    g[i] = std::exp(-(x * x) / (2 * sigma * sigma));
    s += g[i];
  }
  for (auto& v : g) v /= s;
  return g;
}

static Op make_conv_blur(int K, double sigma, const std::string& text) {
  STRIPE_CHECK(K >= 3 && K % 2 == 1 && K / 2 <= kMaxRadius,
               "blur:K needs odd K in [3, " << 2 * kMaxRadius + 1 << "], got " << K);
  Op op;
  op.kind = OpKind::Conv;
  op.K = K;
  auto g = gaussian_1d(K, sigma);
  op.weights.resize((size_t)K * K);
  for (int i = 0; i < K; ++i)
    for (int j = 0; j < K; ++j) op.weights[(size_t)i * K + j] = (float)(g[i] * g[j]);
  op.sep_h.resize((size_t)K);
  for (int i = 0; i < K; ++i) op.sep_h[(size_t)i] = (float)g[i];
  op.sep_v = op.sep_h;
  op.text = text;
  return op;
}

// Trailing ":exact" / ":lsb" of a float conv token (removed from parts):
// 3 = exact (the default), 2 = every output within 1 LSB of the f64 result.
static int take_precision(std::vector<std::string>& parts) {
  if (parts.size() < 2) return 3;
  const std::string last = trim(parts.back());
  if (last != "exact" && last != "lsb") return 3;
  parts.pop_back();
  return last == "lsb" ? 2 : 3;
}

std::vector<Op> parse_chain(const std::string& spec_in) {
  const std::string spec = trim(spec_in);
  std::vector<Op> ops;
  STRIPE_CHECK(!spec.empty(), "empty filter chain");
  for (const std::string& raw : split(spec, ',')) {
    std::string tok = trim(raw);
    STRIPE_CHECK(!tok.empty(), "empty token in chain '" << spec << "'");
    // presets (SURVEY Appendix A "presets") expand in place; halo/partition
    // flags of a preset are applied by the callers (CLI / models.PRESETS)
    if (tok == "ref-gpu" || tok == "ref-cpu") {
      auto sub = parse_chain(tok == "ref-gpu" ? "gray:ref,contrast:3.5,emboss3@skip"
                                              : "gray:bt601,contrast:3:cv,emboss3");
      ops.insert(ops.end(), sub.begin(), sub.end());
      continue;
    }
    Op op;
    // optional per-op border override: name[:args]@border
    auto at = tok.find('@');
    if (at != std::string::npos) {
      op.has_border = true;
      op.border = parse_border(tok.substr(at + 1));
      tok = tok.substr(0, at);
    }
    auto parts = split(tok, ':');
    const std::string name = parts[0];
    StencilId sid;
    if (name == "gray" || name == "grayscale" || name == "grey") {
      op.kind = OpKind::Gray;
      op.gray = GrayMode::BT601;
      if (parts.size() > 1) {
        if (parts[1] == "ref") op.gray = GrayMode::Ref;
        else if (parts[1] == "bt601" || parts[1] == "cv") op.gray = GrayMode::BT601;
        else fail("gray mode must be ref|bt601, got '" + parts[1] + "'");
      }
      op.text = op.gray == GrayMode::Ref ? "gray:ref" : "gray:bt601";
    } else if (name == "contrast") {
      op.kind = OpKind::Contrast;
      op.fval = parts.size() > 1 ? (float)parse_num(parts[1], tok) : 3.5f;
      op.round = RoundMode::Trunc;
      if (parts.size() > 2) {
        if (parts[2] == "cv" || parts[2] == "round") op.round = RoundMode::Nearest;
        else if (parts[2] == "ref" || parts[2] == "trunc") op.round = RoundMode::Trunc;
        else fail("contrast rounding must be ref|cv, got '" + parts[2] + "'");
      }
      std::ostringstream os;
      os << "contrast:" << op.fval << (op.round == RoundMode::Nearest ? ":cv" : "");
      op.text = os.str();
    } else if (name == "invert" || name == "negate") {
      op.kind = OpKind::Invert;
      op.text = "invert";
    } else if (name == "brightness" || name == "bright") {
      op.kind = OpKind::Brightness;
      STRIPE_CHECK(parts.size() > 1, "brightness needs a delta, e.g. brightness:40");
      op.ival = (int)parse_num(parts[1], tok);
      op.text = "brightness:" + std::to_string(op.ival);
    } else if (name == "threshold") {
      op.kind = OpKind::Threshold;
      op.ival = parts.size() > 1 ? (int)parse_num(parts[1], tok) : 128;
      op.text = "threshold:" + std::to_string(op.ival);
    } else if (name == "expand" || name == "gray2rgb") {
      op.kind = OpKind::Expand;
      op.text = "expand";
    } else if (name == "blur" || name == "gblur") {
      // blur:K[:sigma][:exact|:lsb]
      const int digits = take_precision(parts);
      STRIPE_CHECK(parts.size() <= 3, "blur syntax: blur:K[:sigma][:exact|:lsb]");
      const int K = parts.size() > 1 ? (int)parse_num(parts[1], tok) : 31;
      const double sigma = parts.size() > 2 ? parse_num(parts[2], tok) : 0.0;
      Op c = make_conv_blur(K, sigma, tok);
      c.has_border = op.has_border;
      c.border = op.border;
      c.conv_digits = digits;
      op = c;
    } else if (name == "conv") {
      // conv:K:w00;w01;...[:exact|:lsb]  (K*K weights, row-major, correlation)
      STRIPE_CHECK(parts.size() == 3 || parts.size() == 4, "conv syntax: conv:K:w0;w1;...;w(K*K-1)[:exact|:lsb]");
      if (parts.size() == 4) {
        const std::string prec = trim(parts[3]);
        STRIPE_CHECK(prec == "exact" || prec == "lsb", "conv precision must be exact or lsb, got '" << prec << "'");
        op.conv_digits = prec == "lsb" ? 2 : 3;
      }
      op.kind = OpKind::Conv;
      op.K = (int)parse_num(parts[1], tok);
      STRIPE_CHECK(op.K >= 1 && op.K % 2 == 1 && op.K / 2 <= kMaxRadius, "conv K must be odd <= 33");
      for (const auto& w : split(parts[2], ';')) op.weights.push_back((float)parse_num(trim(w), tok));
      STRIPE_CHECK((int)op.weights.size() == op.K * op.K,
                   "conv:" << op.K << " needs " << op.K * op.K << " weights, got " << op.weights.size());
      op.text = tok;
    } else if (name == "sepconv") {
      // sepconv:K:h0;...;h(K-1):v0;...;v(K-1)[:exact|:lsb]  rank-one KxK correlation
      // weights[dy][dx] = v[dy] * h[dx] (separable MFMA path on the GPU)
      op.conv_digits = take_precision(parts);
      STRIPE_CHECK(parts.size() == 4, "sepconv syntax: sepconv:K:h0;...;h(K-1):v0;...;v(K-1)[:exact|:lsb]");
      op.kind = OpKind::Conv;
      op.K = (int)parse_num(parts[1], tok);
      STRIPE_CHECK(op.K >= 1 && op.K % 2 == 1 && op.K / 2 <= kMaxRadius, "sepconv K must be odd <= 33");
      for (const auto& w : split(parts[2], ';')) op.sep_h.push_back((float)parse_num(trim(w), tok));
      for (const auto& w : split(parts[3], ';')) op.sep_v.push_back((float)parse_num(trim(w), tok));
      STRIPE_CHECK((int)op.sep_h.size() == op.K && (int)op.sep_v.size() == op.K,
                   "sepconv:" << op.K << " needs " << op.K << " horizontal and " << op.K << " vertical weights");
      op.weights.resize((size_t)op.K * op.K);
      for (int i = 0; i < op.K; ++i)
        for (int j = 0; j < op.K; ++j) op.weights[(size_t)i * op.K + j] = op.sep_v[(size_t)i] * op.sep_h[(size_t)j];
      op.text = tok;
    } else if (stencil_from_name(name, &sid)) {
      op.kind = OpKind::Stencil;
      op.sid = sid;
      op.text = stencil_info(sid).name;
    } else {
      fail("unknown filter '" + name +
           "' (gray[:ref|bt601], contrast:F[:cv], invert, brightness:D, threshold:T, expand, "
           "emboss3, emboss5, gaussian3/5/7, box3/5, sharpen, laplace, sobel, sobel_l2, blur:K[:sigma][:lsb], conv:K:w..[:lsb], sepconv:K:h..:v..[:lsb])");
    }
    if (op.has_border) op.text += std::string("@") + border_name(op.border);
    ops.push_back(op);
  }
  return ops;
}

std::string chain_to_string(const std::vector<Op>& ops) {
  std::string s;
  for (size_t i = 0; i < ops.size(); ++i) {
    if (i) s += ",";
    s += ops[i].text;
  }
  return s;
}

// ---------------------------------------------------------------------------
// Pointwise numerics
// ---------------------------------------------------------------------------

static inline uint8_t sat_i(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

#pragma clang fp contract(off)
uint8_t apply_pointwise_u8(const Op& op, uint8_t p) {
  switch (op.kind) {
    case OpKind::Invert:
      return (uint8_t)(255 - p);
    case OpKind::Brightness:
      return sat_i((int)p + op.ival);
    case OpKind::Threshold:
      return p >= op.ival ? 255 : 0;
    case OpKind::Contrast: {
      if (op.round == RoundMode::Trunc) {
        // kernel.cu:50,56: clamp(contrast * (p - 128) + 128) then (uchar) truncation.
        // Spec: f32 multiply then f32 add (no fma).
        volatile float prod = op.fval * (float)((int)p - 128);
        float v = prod + 128.0f;
        if (v < 0.f) v = 0.f;
        if (v > 255.f) v = 255.f;
        return (uint8_t)v;
      }
      // kern.cpp:74: OpenCV folds 3*(x-128)+128 into convertTo(alpha=f, beta=128-128f)
      // evaluated in f32 and saturate_cast (round half to even).
      const float alpha = op.fval;
      const float beta = (float)(128.0 - 128.0 * (double)op.fval);
      volatile float prod = (float)p * alpha;
      float v = prod + beta;
      float r = std::nearbyint(v);
      if (r < 0.f) r = 0.f;
      if (r > 255.f) r = 255.f;
      return (uint8_t)r;
    }
    default:
      fail("apply_pointwise_u8: not a per-channel LUT op: " + op.text);
  }
}

uint8_t gray_pixel(GrayMode m, uint8_t r, uint8_t g, uint8_t b) {
  if (m == GrayMode::Ref) {
    // kernel.cu:40-42 (BGR order there; weights are bound to semantic channels, Q5).
    // (float)x * 0.11 promotes to double; each term truncated to u8 separately.
    return (uint8_t)((uint8_t)((double)(float)b * 0.11) + (uint8_t)((double)(float)g * 0.59) +
                     (uint8_t)((double)(float)r * 0.3));
  }
  // OpenCV COLOR_BGR2GRAY, 8U: fixed point, yuv_shift 14, rounded (kern.cpp:73).
  return (uint8_t)((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14);
}
#pragma clang fp contract(on)

bool find_trunc_magic(double w, uint32_t* mult, int* shift) {
  for (int s = 8; s <= 24; ++s) {
    for (int bump = 0; bump <= 1; ++bump) {
      const uint32_t m = (uint32_t)std::floor(w * (double)(1u << s)) + (uint32_t)bump;
      bool ok = true;
      for (int x = 0; x < 256 && ok; ++x) {
        const uint32_t want = (uint32_t)(uint8_t)((double)(float)x * w);
        ok = ((uint32_t)x * m >> s) == want;
      }
      if (ok) {
        *mult = m;
        *shift = s;
        return true;
      }
    }
  }
  return false;
}

}  // namespace stripe
