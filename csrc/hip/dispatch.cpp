// Pass dispatch: one entry point for every compiled pass kind.
#include "stripe/kernels.h"

namespace stripe {

void launch_pass(const Pass& p, const PassConsts& pc, const PassLaunch& L, hipStream_t s) {
  switch (p.kind) {
    case PassKind::Pointwise: launch_pointwise(p, pc, L, s); break;
    case PassKind::Separable:
    case PassKind::Direct: launch_stencil(p, pc, L, s); break;
    case PassKind::Conv: launch_conv(p, pc, L, s); break;
  }
}

}  // namespace stripe
