// Pass dispatch: one entry point for every compiled pass kind.
// Every launch is shape-checked before it runs and error-checked after (the
// reference launches three kernels with no checks, kernel.cu:192-195).
#include "stripe/kernels.h"

namespace stripe {

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
  switch (p.kind) {
    case PassKind::Pointwise: launch_pointwise(p, pc, L, s); break;
    case PassKind::Separable:
    case PassKind::Direct: launch_stencil(p, pc, L, s); break;
    case PassKind::Conv: launch_conv(p, pc, L, s); break;
  }
}

}  // namespace stripe
