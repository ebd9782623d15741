/* k_resid_l16.hip — instantiation of k_resid for LPC orders <= 16. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l16(const ResidArgs& a, int path, int rb, hipStream_t s) {
    return launch_resid_bucket<16>(a, path, rb, s);
}
}  // namespace flacmi
