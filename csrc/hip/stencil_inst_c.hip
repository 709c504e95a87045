// Stencil kernel instances: SobelL2, Emboss3, Emboss5 (see stencil_kernels.h).
#include "stencil_kernels.h"

namespace stripe {
namespace dev {

STRIPE_INSTANTIATE_LAUNCH_FILTER(SobelL2)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Emboss3)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Emboss5)

}  // namespace dev
}  // namespace stripe
