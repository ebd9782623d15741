/* k_resid_l12.hip — instantiation of k_resid for LPC orders <= 12. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l12(const ResidArgs& a, bool wide, int rb, hipStream_t s) {
    return launch_resid_bucket<12>(a, wide, rb, s);
}
}  // namespace flacmi
