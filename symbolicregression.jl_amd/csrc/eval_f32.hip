// eval_f32.hip — float variants of eval_kernel (see eval_kernel.h):
//   R = 8 rows per lane, kShallowSlots stack slots, basic or full operator set
//   R = 4 rows per lane, kMaxSlots stack slots (deep trees), full operator set
#include "eval_kernel.h"


namespace srhip {

bool ti_compiled() { return SR_TI != 0; }

template <>
hipError_t launch_eval<float>(const EvalPlan& plan, const EvalArgs<float>& a, int mode, hipStream_t stream) {
  if (plan.D == kMaxSlots) return launch_rd<float, 4, kMaxSlots, OPSET_FULL>(plan, a, mode, stream);
  if (plan.opset == OPSET_BASIC) return launch_rd<float, SR_R32, kShallowSlots, OPSET_BASIC>(plan, a, mode, stream);
  return launch_rd<float, SR_R32, kShallowSlots, OPSET_FULL>(plan, a, mode, stream);
}

}  // namespace srhip
