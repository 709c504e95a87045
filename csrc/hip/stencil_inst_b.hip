// Stencil kernel instances: Gaussian7, Box5, Sobel (see stencil_kernels.h).
#include "stencil_kernels.h"

namespace stripe {
namespace dev {

STRIPE_INSTANTIATE_LAUNCH_FILTER(Gaussian7)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Box5)
STRIPE_INSTANTIATE_LAUNCH_FILTER(Sobel)

}  // namespace dev
}  // namespace stripe
