// round_f32.hip -- k_round instantiations: float32 iterates over float32 rows (the throughput mode).
#include "kcommon.h"
#include "k_round.inc"

namespace dopt {

hipError_t launch_round_f32(int problem, int cpl, bool grad, bool met, const RoundArgs& a, int n_groups,
                            hipStream_t s) {
  return problem == 0 ? dispatch_cpl<float, float, 0>(cpl, grad, met, a, n_groups, s)
                      : dispatch_cpl<float, float, 1>(cpl, grad, met, a, n_groups, s);
}

}  // namespace dopt
