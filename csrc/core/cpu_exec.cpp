// Fast host executor (see cpu_exec.h).  Every formula mirrors golden_pass
// (golden.cpp) term for term; only the loop structure differs.
#include "stripe/cpu_exec.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>
#include <vector>

namespace stripe {

int cpu_threads(int ranks_per_host) {
  if (const char* e = std::getenv("STRIPE_CPU_THREADS")) return std::max(1, std::atoi(e));
  const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
  return std::max(1, std::min(64, hw / std::max(1, ranks_per_host)));
}

namespace {

inline uint8_t sat(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// round(sqrt(n)) for n >= 0, exactly (as golden.cpp)
inline int isqrt_round(int n) {
  int k = (int)std::sqrt((double)n);
  while (k * k > n) --k;
  while ((k + 1) * (k + 1) <= n) ++k;
  return n > k * k + k ? k + 1 : k;
}

// The pointwise program as byte tables: per pixel out = post(gray(pre(px))).
struct ProgTables {
  int cin = 3, cmid = 3;
  bool gray = false, ref = false, copy = false;
  uint8_t pre[256], lut[256];         // lut: post(pre(v)) (no gray) or post(v) (gray)
  uint8_t tr[256], tg[256], tb[256];  // gray:ref: the per-channel truncated terms of pre(v)

  ProgTables(const PointwiseProgram& pr, int cin_) : cin(cin_) {
    gray = pr.gray;
    cmid = gray ? 1 : cin;
    ref = pr.gmode == GrayMode::Ref;
    copy = !gray;
    for (int v = 0; v < 256; ++v) {
      pre[v] = pr.has_pre ? pr.pre[v] : (uint8_t)v;
      if (!gray) {
        lut[v] = pr.has_post ? pr.post[pre[v]] : pre[v];
        copy = copy && lut[v] == v;
      } else {
        lut[v] = pr.has_post ? pr.post[v] : (uint8_t)v;
        // gray_pixel(Ref, r, g, b) = trunc terms summed (<= 254): separable per channel
        tr[v] = gray_pixel(GrayMode::Ref, pre[v], 0, 0);
        tg[v] = gray_pixel(GrayMode::Ref, 0, pre[v], 0);
        tb[v] = gray_pixel(GrayMode::Ref, 0, 0, pre[v]);
      }
    }
  }

  // n pixels of cin bytes -> n pixels of cmid bytes
  void row(const uint8_t* src, int n, uint8_t* dst) const {
    if (!gray) {
      const int nb = n * cin;
      if (copy) {
        std::memcpy(dst, src, (size_t)nb);
      } else {
        for (int i = 0; i < nb; ++i) dst[i] = lut[src[i]];
      }
    } else if (ref) {
      for (int x = 0; x < n; ++x) dst[x] = lut[tr[src[3 * x]] + tg[src[3 * x + 1]] + tb[src[3 * x + 2]]];
    } else {
      for (int x = 0; x < n; ++x) {
        const int r = pre[src[3 * x]], g = pre[src[3 * x + 1]], b = pre[src[3 * x + 2]];
        dst[x] = lut[(r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14];
      }
    }
  }
};

// Run f(ya, yb) over [y0, y1) split into up to `threads` contiguous blocks
// (at least ~256 KiB of output each: thread start-up costs tens of us).
template <class F>
void parallel_rows(int y0, int y1, int64_t row_bytes, int threads, F&& f) {
  const int n = y1 - y0;
  if (n <= 0) return;
  const int64_t work = (int64_t)n * std::max<int64_t>(1, row_bytes);
  int T = (int)std::min<int64_t>({(int64_t)threads, (int64_t)n, std::max<int64_t>(1, work >> 18)});
  T = std::max(1, T);
  if (T == 1) {
    f(y0, y1);
    return;
  }
  // a worker's exception (or a thread that fails to start) must surface in
  // the caller as a C++ exception, not std::terminate: the first error is
  // kept and rethrown after every started worker has joined
  std::vector<std::exception_ptr> err((size_t)T);
  auto guarded = [&f, &err](int t, int ya, int yb) {
    try {
      f(ya, yb);
    } catch (...) {
      err[(size_t)t] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  th.reserve((size_t)T - 1);
  try {
    for (int t = 1; t < T; ++t)
      th.emplace_back(guarded, t, y0 + (int)((int64_t)n * t / T), y0 + (int)((int64_t)n * (t + 1) / T));
  } catch (...) {
    err[0] = std::current_exception();  // thread creation failed: the started workers still join
  }
  if (!err[0]) guarded(0, y0, y0 + (int)((int64_t)n / T));
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

// Prologued local row y with R border pixels each side ((W + 2R) * cmid bytes),
// all zeros for a constant-border row outside the image (golden build_cache).
void ext_row(const Pass& p, const ProgTables& pt, ConstView in, int W, RowGeom g, int y, uint8_t* dst) {
  const int R = p.R, C = p.cmid;
  const Border b = p.border;
  int gy = g.row0 + y;
  if (gy < 0 || gy >= g.Hg) {
    const int m = border_index(gy, g.Hg, b);
    if (m < 0) {
      std::memset(dst, 0, (size_t)(W + 2 * R) * C);
      return;
    }
    gy = m;
  }
  pt.row(in.origin + (int64_t)(gy - g.row0) * in.pitch, W, dst + (size_t)R * C);
  // the program is per pixel: the border pixel at x is the prologued pixel border_index(x)
  for (int k = 1; k <= R; ++k) {
    for (int side = 0; side < 2; ++side) {
      const int x = side ? W - 1 + k : -k;
      const int m = border_index(x, W, b);
      uint8_t* d = dst + (size_t)(x + R) * C;
      if (m < 0) std::memset(d, 0, (size_t)C);
      else std::memcpy(d, dst + (size_t)(m + R) * C, (size_t)C);
    }
  }
}

// Hot loops, each cloned for AVX2 and a baseline x86-64 target (the loader
// picks the AVX2 clone where the CPU has it; this file is host-only C++).
#define STRIPE_SIMD __attribute__((target_clones("avx2", "default")))

STRIPE_SIMD void tap_u8(int32_t* __restrict a, const uint8_t* __restrict s, int w, int n) {
  for (int i = 0; i < n; ++i) a[i] += w * (int32_t)s[i];
}
// unsigned 16-bit sums: the caller guarantees no wrap (non-negative taps, sum * 255 < 2^16)
STRIPE_SIMD void tap_u8_u16(uint16_t* __restrict a, const uint8_t* __restrict s, int w, int n) {
  for (int i = 0; i < n; ++i) a[i] = (uint16_t)(a[i] + (uint16_t)w * (uint16_t)s[i]);
}
STRIPE_SIMD void tap_u16(int32_t* __restrict a, const uint16_t* __restrict s, int w, int n) {
  for (int i = 0; i < n; ++i) a[i] += w * (int32_t)s[i];
}
STRIPE_SIMD void finish_shift(const int32_t* __restrict a, uint8_t* __restrict o, int h, int sh, int n) {
  for (int i = 0; i < n; ++i) {
    const int v = (a[i] + h) >> sh;  // sums >= 0: floor division by 2^sh
    o[i] = (uint8_t)(v > 255 ? 255 : v);
  }
}
STRIPE_SIMD void finish_sat(const int32_t* __restrict a, uint8_t* __restrict o, int n) {
  for (int i = 0; i < n; ++i) o[i] = (uint8_t)(a[i] < 0 ? 0 : (a[i] > 255 ? 255 : a[i]));
}
STRIPE_SIMD void finish_sobel(const int32_t* __restrict a, const int32_t* __restrict b, uint8_t* __restrict o, int n) {
  for (int i = 0; i < n; ++i) {
    const int v = (a[i] < 0 ? -a[i] : a[i]) + (b[i] < 0 ? -b[i] : b[i]);
    o[i] = (uint8_t)(v > 255 ? 255 : v);
  }
}

void stencil_rows(const Pass& p, const ProgTables& pt, ConstView in, MutView out, int W, RowGeom g, int ya, int yb) {
  const StencilInfo& si = stencil_info(p.sid);
  const int K = p.K, R = p.R, C = p.cmid;
  const int E = W * C, EW = (W + 2 * R) * C;
  std::vector<int> wy;
  if (si.sobel) {
    wy.resize((size_t)K * K);
    for (int dy = 0; dy < K; ++dy)
      for (int dx = 0; dx < K; ++dx) wy[(size_t)dy * K + dx] = si.w[(size_t)dx * K + dy];
  }
  // rank-one windows (gaussian / box): s = sum_dy w1[dy] sum_dx w1[dx] p, the same
  // integer as the K x K sum, as a vertical pass into u16 sums (no wrap: taps >= 0,
  // sum(w1) * 255 < 2^16) and a horizontal pass over them
  bool sep = si.separable && !si.sobel && (int)si.w1.size() == K;
  int w1sum = 0;
  for (int i = 0; sep && i < K; ++i) {
    sep = si.w1[(size_t)i] >= 0;
    w1sum += si.w1[(size_t)i];
    for (int j = 0; sep && j < K; ++j) sep = si.w[(size_t)i * K + j] == si.w1[(size_t)i] * si.w1[(size_t)j];
  }
  sep = sep && w1sum * 255 < 65536;
  int sh = -1;  // div as a shift when it is a power of two
  for (int k = 0; k < 31; ++k)
    if (si.div == (1 << k)) sh = k;

  std::vector<uint8_t> ring((size_t)K * EW);
  std::vector<int32_t> acc((size_t)E), acc2(si.sobel ? (size_t)E : 0);
  std::vector<uint16_t> vs(sep ? (size_t)EW : 0);
  std::vector<uint8_t> res((size_t)E);
  auto slot = [&](int y) { return ring.data() + (size_t)((y - (ya - R)) % K) * EW; };
  for (int y = ya - R; y < ya + R; ++y) ext_row(p, pt, in, W, g, y, slot(y));
  for (int y = ya; y < yb; ++y) {
    ext_row(p, pt, in, W, g, y + R, slot(y + R));
    std::fill(acc.begin(), acc.end(), 0);
    int32_t* a = acc.data();
    if (sep) {
      std::fill(vs.begin(), vs.end(), (uint16_t)0);
      for (int dy = 0; dy < K; ++dy) tap_u8_u16(vs.data(), slot(y + dy - R), si.w1[(size_t)dy], EW);
      for (int dx = 0; dx < K; ++dx) tap_u16(a, vs.data() + (size_t)dx * C, si.w1[(size_t)dx], E);
    } else {
      if (si.sobel) std::fill(acc2.begin(), acc2.end(), 0);
      for (int dy = 0; dy < K; ++dy) {
        const uint8_t* r = slot(y + dy - R);
        for (int dx = 0; dx < K; ++dx) {
          const uint8_t* s = r + (size_t)dx * C;
          const int w = si.w[(size_t)dy * K + dx];
          if (w != 0) tap_u8(a, s, w, E);
          if (si.sobel && wy[(size_t)dy * K + dx] != 0) tap_u8(acc2.data(), s, wy[(size_t)dy * K + dx], E);
        }
      }
    }
    uint8_t* o = res.data();
    const int32_t* a2 = acc2.data();
    if (si.sobel && si.l2) {
      for (int i = 0; i < E; ++i) o[i] = sat(isqrt_round(a[i] * a[i] + a2[i] * a2[i]));
    } else if (si.sobel) {
      finish_sobel(a, a2, o, E);
    } else if (si.div > 1 && sh >= 0) {
      finish_shift(a, o, si.div / 2, sh, E);
    } else if (si.div > 1) {
      const int d = si.div, h = si.div / 2;  // sums >= 0 for the smoothing filters
      for (int i = 0; i < E; ++i) o[i] = sat((a[i] + h) / d);
    } else {
      finish_sat(a, o, E);
    }
    if (p.border == Border::Skip) {  // golden.cpp:133 (the reference's interior-only bounds)
      const int gy = g.row0 + y;
      const uint8_t* center = slot(y) + (size_t)R * C;
      if (gy <= R || gy >= g.Hg - R) {
        std::memcpy(o, center, (size_t)E);
      } else {
        for (int x = 0; x < W; ++x)
          if (x <= R || x >= W - R) std::memcpy(o + (size_t)x * C, center + (size_t)x * C, (size_t)C);
      }
    }
    if (p.has_epi)
      for (int i = 0; i < E; ++i) o[i] = p.epi[o[i]];
    uint8_t* dst = out.origin + (int64_t)y * out.pitch;
    if (p.epi_expand) {
      for (int x = 0; x < W; ++x) dst[3 * x] = dst[3 * x + 1] = dst[3 * x + 2] = o[x];
    } else {
      std::memcpy(dst, o, (size_t)E);
    }
  }
}

void pointwise_rows(const Pass& p, const ProgTables& pt, ConstView in, MutView out, int W, int ya, int yb) {
  std::vector<uint8_t> tmp(p.pro.expand ? (size_t)W * pt.cmid : 0);
  for (int y = ya; y < yb; ++y) {
    const uint8_t* src = in.origin + (int64_t)y * in.pitch;
    uint8_t* dst = out.origin + (int64_t)y * out.pitch;
    if (!p.pro.expand) {
      pt.row(src, W, dst);
    } else {
      pt.row(src, W, tmp.data());  // expand follows a 1-channel program
      for (int x = 0; x < W; ++x) dst[3 * x] = dst[3 * x + 1] = dst[3 * x + 2] = tmp[(size_t)x];
    }
  }
}

}  // namespace

void cpu_pass(const Pass& p, ConstView in, MutView out, int W, RowGeom g, int y0, int y1, int threads) {
  if (y1 <= y0) return;
  const int64_t row_bytes = (int64_t)W * p.cout;
  if (p.kind == PassKind::Conv) {  // float windows: the golden f64 sums themselves, row-parallel
    parallel_rows(y0, y1, row_bytes * p.K * p.K, threads,
                  [&](int ya, int yb) { golden_pass(p, in, out, W, g, ya, yb); });
    return;
  }
  STRIPE_CHECK(!p.pro.gray || p.cin == 3, "gray needs 3 channels");
  STRIPE_CHECK(!p.pro.expand || p.kind == PassKind::Pointwise, "expand inside a stencil prologue");
  const ProgTables pt(p.pro, p.cin);
  if (p.kind == PassKind::Pointwise) {
    parallel_rows(y0, y1, row_bytes, threads, [&](int ya, int yb) { pointwise_rows(p, pt, in, out, W, ya, yb); });
    return;
  }
  STRIPE_CHECK(pt.cmid == p.cmid, "prologue channels " << pt.cmid << " != stencil channels " << p.cmid);
  parallel_rows(y0, y1, row_bytes * p.K, threads,
                [&](int ya, int yb) { stencil_rows(p, pt, in, out, W, g, ya, yb); });
}

Image cpu_apply_plan(const Image& in, const Plan& plan, int threads) {
  STRIPE_CHECK(in.C == plan.cin, "image has " << in.C << " channels, chain expects " << plan.cin);
  if (plan.passes.empty()) return in;
  Image cur;  // the first pass reads the input in place (no copy of the frame)
  const Image* src = &in;
  for (const Pass& p : plan.passes) {
    Image nxt(in.W, in.H, p.cout, NoInit{});  // cpu_pass writes every row of [0, H)
    cpu_pass(p, ConstView{src->data.data(), src->row_bytes()}, MutView{nxt.data.data(), nxt.row_bytes()}, in.W,
             RowGeom{0, in.H}, 0, in.H, threads);
    cur = std::move(nxt);
    src = &cur;
  }
  return cur;
}

}  // namespace stripe
