// Pass dispatch: one entry point for every compiled pass kind.
// Every launch is shape-checked before it runs and error-checked after (the
// reference launches three kernels with no checks, kernel.cu:192-195).
#include "stripe/kernels.h"

#include <algorithm>
#include <cstdlib>

#include "stripe/common.h"

namespace stripe {

namespace {

// Byte range of one buffer-descriptor view: the stencil / conv kernels address
// rows with 32-bit offsets and bias masked lanes by 2^31 (dev::kOOB), so a view
// must stay below 2 GiB (minus slack for the bias arithmetic).
// STRIPE_DESC_LIMIT (bytes) lowers it so tests can exercise the chunked path.
int64_t desc_limit() {
  static const int64_t v = [] {
    const char* e = std::getenv("STRIPE_DESC_LIMIT");
    const int64_t def = (1ll << 31) - (1ll << 20);
    return e ? std::max<int64_t>(1 << 16, std::min<int64_t>(def, std::atoll(e))) : def;
  }();
  return v;
}

int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// A stencil / conv pass over buffers larger than one descriptor view (an image
// that fits HBM but not 2 GiB: 32768^2 RGB is 3 GiB): split the output rows
// into chunks and re-base both views on each chunk.  Rows a chunk's kernels
// read past its own span (the 32-row groups of the MFMA blur, the 16*MT-row
// tiles of the MFMA conv round up) only feed outputs that are not stored; the
// Constant border's zero row becomes an out-of-range offset, which buffer loads
// return as zeros.
void launch_chunked(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  const int64_t lim = desc_limit();
  const int Rs = p.R + 64;
  const int64_t maxp = std::max(L.in_pitch, L.out_pitch);
  const int64_t cr = lim / maxp - 2 * Rs - 2;
  STRIPE_CHECK(cr >= 16, "rows too wide for " << lim << "-byte descriptor views (pitch " << maxp << ")");
  // local rows whose whole padded row lies inside each allocation
  const int64_t in_lo = floor_div(kMarginBytes - L.in_org + L.in_pitch - 1, L.in_pitch);
  const int64_t in_hi = floor_div(L.in_bytes - L.in_org + kMarginBytes, L.in_pitch);
  for (int r = 0; r < L.nrange; ++r) {
    for (int64_t c0 = L.ry[2 * r]; c0 < L.ry[2 * r + 1]; c0 += cr) {
      const int64_t c1 = std::min<int64_t>(c0 + cr, L.ry[2 * r + 1]);
      PassLaunch C = L;
      C.rebased = true;
      C.nrange = 1;
      C.ry[0] = (int)c0;
      C.ry[1] = (int)c1;
      const int64_t lo = std::max(c0 - Rs, in_lo), hi = std::min(c1 + Rs, in_hi);
      const int64_t ib = L.in_org + lo * L.in_pitch - kMarginBytes;
      C.in_base = L.in_base + ib;
      C.in_bytes = std::min((hi - lo) * L.in_pitch, L.in_bytes - ib);
      C.in_org = L.in_org - ib;
      C.in_zero = (int64_t)1 << 31;  // out of range: loads read zeros
      const int64_t ob = L.out_org + c0 * L.out_pitch - kMarginBytes;
      STRIPE_CHECK(ib >= 0 && ob >= 0 && ob + (c1 - c0) * L.out_pitch <= L.out_bytes + kMarginBytes,
                   "chunk outside its buffers");
      C.out_base = L.out_base + ob;
      C.out_bytes = std::min((c1 - c0) * L.out_pitch, L.out_bytes - ob);
      C.out_org = L.out_org - ob;
      if (p.kind == PassKind::Conv) launch_conv(p, pc, C, s);
      else launch_stencil(p, pc, C, s);
    }
  }
}

}  // namespace

void launch_pass(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  // host-side shape checks before any kernel touches memory
  STRIPE_CHECK(L.in && L.out && L.W >= 1 && L.rows >= 0, "bad pass launch");
  STRIPE_CHECK(L.nrange == 1 || L.nrange == 2, "nrange must be 1 or 2");
  STRIPE_CHECK(L.ext >= 0 && (L.ext == 0 || p.kind == PassKind::Separable || p.kind == PassKind::Direct ||
                               p.kind == PassKind::Pointwise),
               "halo-row outputs (ext) are for stencil and pointwise passes only");
  for (int r = 0; r < L.nrange; ++r)
    STRIPE_CHECK(-L.ext <= L.ry[2 * r] && L.ry[2 * r] <= L.ry[2 * r + 1] && L.ry[2 * r + 1] <= L.rows + L.ext,
                 "row range [" << L.ry[2 * r] << "," << L.ry[2 * r + 1] << ") outside stripe of " << L.rows
                               << " (+" << L.ext << " halo rows)");
  STRIPE_CHECK(L.in_pitch >= padded_pitch(L.W, p.cin) && L.out_pitch >= padded_pitch(L.W, p.cout),
               "pitch too small for the pass");
  STRIPE_CHECK(p.R <= kMaxRadius && p.out_margin_px <= margin_pixels(p.cout), "radius/margin too large");
  STRIPE_CHECK(L.Hg >= 1 && L.row0 >= 0 && L.row0 + L.rows <= L.Hg, "bad border geometry");
  STRIPE_CHECK(p.border != Border::Constant || L.zero_row != nullptr, "constant border needs a zero row");
  // hipGetLastError is sticky per thread and libraries (RCCL) may leave benign
  // errors behind: clear it so the post-launch check reports only our launch
  (void)hipGetLastError();
  if (p.kind != PassKind::Pointwise && (L.in_bytes > desc_limit() || L.out_bytes > desc_limit())) {
    launch_chunked(p, pc, L, s);
    return;
  }
  switch (p.kind) {
    case PassKind::Pointwise: launch_pointwise(p, pc, L, s); break;
    case PassKind::Separable:
    case PassKind::Direct: launch_stencil(p, pc, L, s); break;
    case PassKind::Conv: launch_conv(p, pc, L, s); break;
  }
}

}  // namespace stripe
