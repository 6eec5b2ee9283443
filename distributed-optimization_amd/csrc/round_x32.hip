// round_x32.hip -- k_round instantiations: float64 iterates and arithmetic over float32-stored rows (dopt_set_data_dtype).
#include "kcommon.h"
#include "k_round.inc"

namespace dopt {

hipError_t launch_round_x32(int problem, int cpl, bool grad, bool met, const RoundArgs& a, int n_groups,
                            hipStream_t s) {
  return problem == 0 ? dispatch_cpl<double, float, 0>(cpl, grad, met, a, n_groups, s)
                      : dispatch_cpl<double, float, 1>(cpl, grad, met, a, n_groups, s);
}

}  // namespace dopt
