// Stencil kernel instances: Gaussian3, Gaussian5, Box3 (see stencil_kernels.h).
#include "stencil_kernels.h"

namespace stripe {
namespace dev {

STRIPE_INSTANTIATE_LAUNCH_FILTER(Gaussian3)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Gaussian5)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Box3)

}  // namespace dev
}  // namespace stripe
