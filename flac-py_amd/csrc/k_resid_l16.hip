/* k_resid_l16.hip — instantiation of k_resid for LPC orders <= 16. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l16(const ResidArgs& a, bool wide, int rb, hipStream_t s) {
    return launch_resid_bucket<16>(a, wide, rb, s);
}
}  // namespace flacmi
