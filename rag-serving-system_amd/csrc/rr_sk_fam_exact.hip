// rr_sk_fam_exact.hip — split-K kernel instantiations (rr_sk.hip dispatch): the exact passes DT 0-3 (32 slots; bf16 and
// fp32-split also 64) and the screened search's verifies (MODE 1: DT 3 for fp32 storage, DT 1 for bf16).
#include "rr_sk_kernel.h"

namespace rr {
namespace sk {
hipError_t fam_exact(int sdt, int metric, int ns, int kt, int mode, int grid, int qslots, const SkArgs& a,
                     hipStream_t s) {
  if (mode == 1) {
    if (sdt == KDT_BF16) return launch_metric<1, 2, 1, 1>(metric, ns, kt, grid, a, s);
    return launch_metric<3, 2, 1, 1>(metric, ns, kt, grid, a, s);
  }
  if (qslots == 64) {   // one corpus pass for up to 64 queries: bf16 and fp32-split storage
    switch (sdt) {
      case 1: return launch_metric<1, 2, 2>(metric, ns, kt, grid, a, s);
      case 2: return launch_metric<2, 2, 2>(metric, ns, kt, grid, a, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (sdt) {
    case 0: return launch_metric<0, 2, 1>(metric, ns, kt, grid, a, s);
    case 1: return launch_metric<1, 2, 1>(metric, ns, kt, grid, a, s);
    case 2: return launch_metric<2, 2, 1>(metric, ns, kt, grid, a, s);
    case 3: return launch_metric<3, 2, 1>(metric, ns, kt, grid, a, s);
    default: return hipErrorInvalidValue;
  }
}
// Load this unit's code object on the current device now (rr_create, rr_preload_kernels): with the runtime's deferred
// loading the first launch of any of its kernels otherwise pays it — ~8 ms for a unit of split-K instantiations, inside
// the first search (measured: the first verify 8 ms after its screen, profiles/r06/preload/).
hipError_t preload_fam_exact() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, (const void*)sk_score_kernel<3, 4, 16, true, 2, 1, 1, 0, 0>);
}
}  // namespace sk
}  // namespace rr
