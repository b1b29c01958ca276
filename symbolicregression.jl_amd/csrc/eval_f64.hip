// eval_f64.hip — double variants of eval_kernel (see eval_kernel.h):
//   R = 4 rows per lane, kShallowSlots stack slots, basic or full operator set
//   R = 2 rows per lane, kMaxSlots stack slots (deep trees), full operator set
#include "eval_kernel.h"

namespace srhip {

template <>
hipError_t launch_eval<double>(const EvalPlan& plan, const EvalArgs<double>& a, int mode, hipStream_t stream) {
  if (plan.D == kMaxSlots) return launch_rd<double, 2, kMaxSlots, OPSET_FULL>(plan, a, mode, stream);
  if (plan.opset == OPSET_BASIC) return launch_rd<double, 4, kShallowSlots, OPSET_BASIC>(plan, a, mode, stream);
  return launch_rd<double, 4, kShallowSlots, OPSET_FULL>(plan, a, mode, stream);
}

}  // namespace srhip
