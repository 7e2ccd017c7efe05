// rr_sk_fam_s9.hip — split-K kernel instantiations (rr_sk.hip dispatch): the int8 screen with ONE query piece (DT 9):
// bf16 storage's 32- and 64-slot blocks, fp32 storage's 32-slot blocks on large shards.
#include "rr_sk_kernel.h"

namespace rr {
namespace sk {
hipError_t fam_screen9(int metric, int ns, int kt, int grid, int qslots, const SkArgs& a, hipStream_t s) {
  if (qslots == 64) {
    // static schedule with the guided tail only: the 9-wave form's register budget (168) spills 10-39 VGPRs here
    if (a.full_lists == 2) return launch_metric<9, 2, 2, 0, 0, 2>(metric, ns, kt, grid, a, s);
    if (a.full_lists) return launch_metric<9, 2, 2, 0, 0, 1>(metric, ns, kt, grid, a, s);
    return launch_metric<9, 2, 2>(metric, ns, kt, grid, a, s);
  }
  const bool dyn = a.dyn && a.ctr && kt <= 16;
  if (a.full_lists == 2)
    return dyn ? launch_metric<9, 2, 1, 0, 1, 2>(metric, ns, kt, grid, a, s)
               : launch_metric<9, 2, 1, 0, 0, 2>(metric, ns, kt, grid, a, s);
  if (a.full_lists)
    return dyn ? launch_metric<9, 2, 1, 0, 1, 1>(metric, ns, kt, grid, a, s)
               : launch_metric<9, 2, 1, 0, 0, 1>(metric, ns, kt, grid, a, s);
  return dyn ? launch_metric<9, 2, 1, 0, 1>(metric, ns, kt, grid, a, s) : launch_metric<9, 2, 1>(metric, ns, kt, grid, a, s);
}
// Load this unit's code object on the current device now (rr_create, rr_preload_kernels): with the runtime's deferred
// loading the first launch of any of its kernels otherwise pays it — ~8 ms for a unit of split-K instantiations, inside
// the first search (measured: the first verify 8 ms after its screen, profiles/r06/preload/).
hipError_t preload_fam_screen9() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, (const void*)sk_score_kernel<9, 2, 16, true, 2, 1, 0, 1, 0>);
}
}  // namespace sk
}  // namespace rr
