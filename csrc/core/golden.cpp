// CPU golden implementation of compiled passes (the bit-exact oracle).
// It specifies every GPU kernel (the reference's grayscale/contrast/emboss,
// kernel.cu:31-94, race-free) and is the engine of the
// ref-cpu preset / host backend (the reference's OpenCV chain, kern.cpp:58-77).
#include "stripe/golden.h"

#include <cmath>
#include <cstring>

namespace stripe {

namespace {

inline uint8_t sat(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// Apply a pointwise program to one input pixel (cin channels) -> out (channels_out).
inline void apply_prog(const PointwiseProgram& pr, const uint8_t* px, int cin, uint8_t* out) {
  uint8_t v[3];
  for (int c = 0; c < cin; ++c) v[c] = pr.has_pre ? pr.pre[px[c]] : px[c];
  int n = cin;
  if (pr.gray) {
    STRIPE_CHECK(cin == 3, "gray needs 3 channels");
    v[0] = gray_pixel(pr.gmode, v[0], v[1], v[2]);
    n = 1;
  }
  if (pr.has_post)
    for (int c = 0; c < n; ++c) v[c] = pr.post[v[c]];
  if (pr.expand) {
    out[0] = out[1] = out[2] = v[0];
  } else {
    for (int c = 0; c < n; ++c) out[c] = v[c];
  }
}

// Prologue-applied rows with R pixels of border extension on each side.
struct RowCache {
  int W = 0, R = 0, C = 0, y_lo = 0;
  std::vector<std::vector<uint8_t>> rows;  // rows[y - y_lo][(x + R) * C + c]
  std::vector<bool> zero;                  // constant-border row outside the image

  const uint8_t* at(int y, int x) const { return rows[y - y_lo].data() + (size_t)(x + R) * C; }
};

RowCache build_cache(const Pass& p, ConstView in, int W, RowGeom g, int y_lo, int y_hi) {
  RowCache rc;
  rc.W = W;
  rc.R = p.R;
  rc.C = p.cmid;
  rc.y_lo = y_lo;
  const int R = p.R;
  const Border b = p.border;
  std::vector<uint8_t> px(p.cmid);
  for (int y = y_lo; y < y_hi; ++y) {
    std::vector<uint8_t> row((size_t)(W + 2 * R) * p.cmid, 0);
    int gy = g.row0 + y;
    bool zero_row = false;
    if (gy < 0 || gy >= g.Hg) {
      const int m = border_index(gy, g.Hg, b);
      if (m < 0) zero_row = true;
      else gy = m;
    }
    if (!zero_row) {
      const uint8_t* src = in.origin + (int64_t)(gy - g.row0) * in.pitch;
      for (int x = -R; x < W + R; ++x) {
        const int mx = border_index(x, W, b);
        if (mx < 0) continue;  // constant: zeros
        apply_prog(p.pro, src + (int64_t)mx * p.cin, p.cin, px.data());
        std::memcpy(row.data() + (size_t)(x + R) * p.cmid, px.data(), p.cmid);
      }
    }
    rc.rows.push_back(std::move(row));
  }
  return rc;
}

}  // namespace

// round(sqrt(n)) for n >= 0, exactly: sqrt of an integer is never k + 1/2.
static int isqrt_round(int n) {
  int k = (int)std::sqrt((double)n);
  while (k * k > n) --k;
  while ((k + 1) * (k + 1) <= n) ++k;
  return n > k * k + k ? k + 1 : k;
}

void golden_pass(const Pass& p, ConstView in, MutView out, int W, RowGeom g, int y0, int y1) {
  if (y1 <= y0) return;
  if (p.kind == PassKind::Pointwise) {
    std::vector<uint8_t> o(3);
    for (int y = y0; y < y1; ++y) {
      const uint8_t* src = in.origin + (int64_t)y * in.pitch;
      uint8_t* dst = out.origin + (int64_t)y * out.pitch;
      for (int x = 0; x < W; ++x) {
        apply_prog(p.pro, src + (int64_t)x * p.cin, p.cin, o.data());
        std::memcpy(dst + (int64_t)x * p.cout, o.data(), p.cout);
      }
    }
    return;
  }
  const int R = p.R, K = p.K, C = p.cmid;
  RowCache rc = build_cache(p, in, W, g, y0 - R, y1 + R);
  if (p.kind == PassKind::Conv) {
    for (int y = y0; y < y1; ++y) {
      uint8_t* dst = out.origin + (int64_t)y * out.pitch;
      for (int x = 0; x < W; ++x)
        for (int c = 0; c < C; ++c) {
          double s = 0;
          for (int dy = 0; dy < K; ++dy) {
            const uint8_t* r = rc.at(y + dy - R, x - R) + c;
            const float* w = p.conv_w.data() + (size_t)dy * K;
            for (int dx = 0; dx < K; ++dx) s += (double)w[dx] * (double)r[(size_t)dx * C];
          }
          dst[(int64_t)x * C + c] = sat((int)std::nearbyint(s));
        }
    }
    return;
  }
  const StencilInfo& si = stencil_info(p.sid);
  std::vector<int> wy;  // sobel's second kernel (transpose of Gx)
  if (si.sobel) {
    wy.resize((size_t)K * K);
    for (int dy = 0; dy < K; ++dy)
      for (int dx = 0; dx < K; ++dx) wy[(size_t)dy * K + dx] = si.w[(size_t)dx * K + dy];
  }
  for (int y = y0; y < y1; ++y) {
    uint8_t* dst = out.origin + (int64_t)y * out.pitch;
    const int gy = g.row0 + y;
    for (int x = 0; x < W; ++x) {
      // @skip: the reference processes o < x <= W-o, o < y <= H-o (kernel.cu:83).
      // Deliberate deviation at x = W-o and y = H-o: there the reference's window
      // reads column W (wrapping into the next row) or row H (past the buffer),
      // so those pixels keep their input value here, like the rest of the frame.
      const bool skip = p.border == Border::Skip &&
                        (x <= R || gy <= R || x >= W - R || gy >= g.Hg - R);
      for (int c = 0; c < C; ++c) {
        int v;
        if (skip) {
          v = rc.at(y, x)[c];
        } else {
          int s = 0, s2 = 0;
          for (int dy = 0; dy < K; ++dy) {
            const uint8_t* r = rc.at(y + dy - R, x - R) + c;
            for (int dx = 0; dx < K; ++dx) {
              const int pv = r[(size_t)dx * C];
              s += si.w[(size_t)dy * K + dx] * pv;
              if (si.sobel) s2 += wy[(size_t)dy * K + dx] * pv;
            }
          }
          if (si.sobel && si.l2) v = isqrt_round(s * s + s2 * s2);
          else if (si.sobel) v = std::abs(s) + std::abs(s2);
          else if (si.div > 1) v = (s + si.div / 2) / si.div;  // s >= 0 for smoothing filters
          else v = s;
          v = sat(v);
        }
        const uint8_t b = p.has_epi ? p.epi[v] : (uint8_t)v;
        if (p.epi_expand) {  // cmid 1 -> 3 equal channels
          dst[(int64_t)x * 3] = dst[(int64_t)x * 3 + 1] = dst[(int64_t)x * 3 + 2] = b;
        } else {
          dst[(int64_t)x * C + c] = b;
        }
      }
    }
  }
}

Image golden_apply_plan(const Image& in, const Plan& plan) {
  STRIPE_CHECK(in.C == plan.cin, "image has " << in.C << " channels, chain expects " << plan.cin);
  Image cur = in;
  for (const Pass& p : plan.passes) {
    Image nxt(in.W, in.H, p.cout);
    golden_pass(p, ConstView{cur.data.data(), cur.row_bytes()}, MutView{nxt.data.data(), nxt.row_bytes()},
                in.W, RowGeom{0, in.H}, 0, in.H);
    cur = std::move(nxt);
  }
  return cur;
}

Image golden_apply_ops(const Image& in, const std::vector<Op>& ops, Border default_border) {
  Image cur = in;
  for (const Op& op : ops) {
    Plan one = compile_chain({op}, cur.C, default_border, /*fuse=*/false);
    cur = golden_apply_plan(cur, one);
  }
  return cur;
}

}  // namespace stripe
