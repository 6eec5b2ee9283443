// round_f64.hip -- k_round instantiations: float64 iterates over float64 rows (the reference's precision).
#include "kcommon.h"
#include "k_round.inc"

namespace dopt {

hipError_t launch_round_f64(int problem, int cpl, bool grad, bool met, const RoundArgs& a, int n_groups,
                            hipStream_t s) {
  return problem == 0 ? dispatch_cpl<double, double, 0>(cpl, grad, met, a, n_groups, s)
                      : dispatch_cpl<double, double, 1>(cpl, grad, met, a, n_groups, s);
}

}  // namespace dopt
