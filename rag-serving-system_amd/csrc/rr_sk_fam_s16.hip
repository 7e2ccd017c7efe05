// rr_sk_fam_s16.hip — split-K kernel instantiations (rr_sk.hip dispatch): the f16 screens, DT 6 (over the fp32 rows) and
// DT 7 (over the f16 copy); dynamic schedule (the 9-wave form) when asked for and the lists fit its registers; short,
// full (FL 1) or repair-mode (FL 2: full lists + per-chunk maxima of the bound) per-lane lists.
#include "rr_sk_kernel.h"

namespace rr {
namespace sk {
template <int DT>
hipError_t screen16(int metric, int ns, int kt, int grid, const SkArgs& a, hipStream_t s) {
  const bool dyn = a.dyn && a.ctr && kt <= 16;
  if (a.full_lists == 2)
    return dyn ? launch_metric<DT, 2, 1, 0, 1, 2>(metric, ns, kt, grid, a, s)
               : launch_metric<DT, 2, 1, 0, 0, 2>(metric, ns, kt, grid, a, s);
  if (a.full_lists)
    return dyn ? launch_metric<DT, 2, 1, 0, 1, 1>(metric, ns, kt, grid, a, s)
               : launch_metric<DT, 2, 1, 0, 0, 1>(metric, ns, kt, grid, a, s);
  return dyn ? launch_metric<DT, 2, 1, 0, 1>(metric, ns, kt, grid, a, s)
             : launch_metric<DT, 2, 1>(metric, ns, kt, grid, a, s);
}

hipError_t fam_screen16(int sdt, int metric, int ns, int kt, int grid, const SkArgs& a, hipStream_t s) {
  return sdt == KDT_SCREEN16 ? screen16<7>(metric, ns, kt, grid, a, s) : screen16<6>(metric, ns, kt, grid, a, s);
}
// Load this unit's code object on the current device now (rr_create, rr_preload_kernels): with the runtime's deferred
// loading the first launch of any of its kernels otherwise pays it — ~8 ms for a unit of split-K instantiations, inside
// the first search (measured: the first verify 8 ms after its screen, profiles/r06/preload/).
hipError_t preload_fam_screen16() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, (const void*)sk_score_kernel<7, 2, 16, true, 2, 1, 0, 1, 0>);
}
}  // namespace sk
}  // namespace rr
