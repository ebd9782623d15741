/* k_resid_l8.hip — instantiation of k_resid for LPC orders <= 8. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l8(const ResidArgs& a, bool wide, int rb, hipStream_t s) {
    return launch_resid_bucket<8>(a, wide, rb, s);
}
}  // namespace flacmi
