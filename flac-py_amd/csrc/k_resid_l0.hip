/* k_resid_l0.hip — instantiation of k_resid for LPC orders <= 0 (fixed-only mode). */
#include "k_resid.h"

namespace flacmi {
hipError_t launch_resid_l0(const ResidArgs& a, int path, int rb, hipStream_t s) {
    return launch_resid_bucket<0>(a, path, rb, s);
}
}  // namespace flacmi
