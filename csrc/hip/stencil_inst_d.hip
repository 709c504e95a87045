// Stencil kernel instances: Sharpen, Laplace (see stencil_kernels.h).
#include "stencil_kernels.h"

namespace stripe {
namespace dev {

STRIPE_INSTANTIATE_LAUNCH_FILTER(Sharpen)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Laplace)

}  // namespace dev
}  // namespace stripe
