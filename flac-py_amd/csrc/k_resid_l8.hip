/* k_resid_l8.hip — instantiation of k_resid for LPC orders <= 8. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l8(const ResidArgs& a, int path, int rb, hipStream_t s) {
    return launch_resid_bucket<8>(a, path, rb, s);
}
hipError_t launch_resid_retry_l8(const ResidArgs& a, hipStream_t s) { return launch_resid_list<8>(a, s); }
}  // namespace flacmi
