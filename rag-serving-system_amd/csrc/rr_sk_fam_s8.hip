// rr_sk_fam_s8.hip — split-K kernel instantiations (rr_sk.hip dispatch): the int8 screen with two query pieces (DT 8,
// fp32 storage, 32 slots); dynamic schedule when the lists fit the 9-wave form's registers.
#include "rr_sk_kernel.h"

namespace rr {
namespace sk {
hipError_t fam_screen8(int metric, int ns, int kt, int grid, const SkArgs& a, hipStream_t s) {
  const bool dyn = a.dyn && a.ctr && kt <= 16;
  if (a.full_lists == 2)   // repair mode: full lists + per-chunk maxima of the bound
    return dyn ? launch_metric<8, 2, 1, 0, 1, 2>(metric, ns, kt, grid, a, s)
               : launch_metric<8, 2, 1, 0, 0, 2>(metric, ns, kt, grid, a, s);
  if (a.full_lists)
    return dyn ? launch_metric<8, 2, 1, 0, 1, 1>(metric, ns, kt, grid, a, s)
               : launch_metric<8, 2, 1, 0, 0, 1>(metric, ns, kt, grid, a, s);
  return dyn ? launch_metric<8, 2, 1, 0, 1>(metric, ns, kt, grid, a, s) : launch_metric<8, 2, 1>(metric, ns, kt, grid, a, s);
}
// Load this unit's code object on the current device now (rr_create, rr_preload_kernels): with the runtime's deferred
// loading the first launch of any of its kernels otherwise pays it — ~8 ms for a unit of split-K instantiations, inside
// the first search (measured: the first verify 8 ms after its screen, profiles/r06/preload/).
hipError_t preload_fam_screen8() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, (const void*)sk_score_kernel<8, 2, 16, true, 2, 1, 0, 1, 0>);
}
}  // namespace sk
}  // namespace rr
