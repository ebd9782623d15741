/* k_resid_l12.hip — instantiation of k_resid for LPC orders <= 12. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l12(const ResidArgs& a, int path, int rb, hipStream_t s) {
    return launch_resid_bucket<12>(a, path, rb, s);
}
hipError_t launch_resid_retry_l12(const ResidArgs& a, hipStream_t s) { return launch_resid_list<12>(a, s); }
}  // namespace flacmi
