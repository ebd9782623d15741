/* k_resid_l32.hip — instantiation of k_resid for LPC orders <= 32. */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l32(const ResidArgs& a, int path, int rb, hipStream_t s) {
    return launch_resid_bucket<32>(a, path, rb, s);
}
}  // namespace flacmi
