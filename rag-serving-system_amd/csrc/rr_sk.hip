// rr_sk.hip — dispatch of the split-K streaming kernel (rr_sk_kernel.h: the kernel, its contract and its dtypes).
// The instantiations live in four units compiled side by side (rr_sk_fam_exact.hip: DT 0-3 and the verifies;
// rr_sk_fam_s16.hip: the f16 screens DT 6 / 7; rr_sk_fam_s8.hip: DT 8; rr_sk_fam_s9.hip: DT 9) — one unit of all of
// them took ~8 minutes of hipcc. Diagnostic tools that include this file whole define RR_SK_ONE_UNIT (or
// RR_SK_NO_DISPATCH to instantiate one kernel themselves).
#include "rr_sk_kernel.h"

namespace rr {
namespace sk {
// validated by launch_sk_args; ns = slabs per wave of the storage the launch streams
hipError_t fam_exact(int sdt, int metric, int ns, int kt, int mode, int grid, int qslots, const SkArgs& a,
                     hipStream_t s);
hipError_t fam_screen16(int sdt, int metric, int ns, int kt, int grid, const SkArgs& a, hipStream_t s);
hipError_t fam_screen8(int metric, int ns, int kt, int grid, const SkArgs& a, hipStream_t s);
hipError_t fam_screen9(int metric, int ns, int kt, int grid, int qslots, const SkArgs& a, hipStream_t s);
hipError_t preload_fam_exact();
hipError_t preload_fam_screen16();
hipError_t preload_fam_screen8();
hipError_t preload_fam_screen9();
}  // namespace sk

size_t sk_lds_bytes(int sdt, bool cos, int ring, int qslots) {
  (void)cos;
  // + per-row factors [4][64] (the int8 screen: [4][192]), next-chunk words [4], query scalars [3][qslots], MODE 1
  // scratch: W [8][32] + akeys [32] keys, grow / gnorm / gvalid [32], xk [32] keys, the floors' and the list bounds'
  // maxima, 6 ints
  const size_t verify = (size_t)(kWaves * 32 + 32 + 32 + 8) * 8 + 3 * 32 * 4;
  const size_t factors = (size_t)4 * (sdt == KDT_SCREEN8 || sdt == KDT_SCREEN9 ? 192 : 64) * 4;
  return sk::ring_bytes(ring) + sk::red_bytes(ring, qslots / 32) + factors + 4 * 4 + 3 * qslots * 4 + verify;
}

bool sk_supports_64(int sdt) { return sdt == KDT_BF16 || sdt == KDT_F32_SPLIT; }
int sk_chunk_tiles(int sdt, int d, int ct8) {   // (the kernel's CT: CT0 by slabs per wave, or the int8 screen's ct8)
  const int ns = sk_slabs(sdt == KDT_SCREEN ? KDT_F32_X3 : sdt, d);
  if ((sdt == KDT_SCREEN8 || sdt == KDT_SCREEN9) && ct8 > 0) return ct8;
  return ns >= 4 ? 2 : ns == 3 ? 3 : ns == 2 ? 4 : 8;
}
int sk_slabs(int sdt, int d) {
  // (the int8 screen: kernel rows of two corpus rows, 2 d bytes)
  const int eb = sdt == KDT_BF16 || sdt == KDT_SCREEN16 || sdt == KDT_SCREEN8 || sdt == KDT_SCREEN9 ? 2 : 4;
  const int ks = d * eb / kWaves;   // row bytes per wave
  if (d <= 0 || ks % sk::kSlabRowBytes != 0) return 0;
  const int ns = ks / sk::kSlabRowBytes;
  return (ns >= 1 && ns <= (eb == 2 ? 2 : 4)) ? ns : 0;
}

#ifndef RR_SK_NO_DISPATCH   // (diagnostic tools that instantiate one kernel directly: tools/probe_screen.hip)
hipError_t preload_sk() {   // every split-K unit's code object on the current device
  for (hipError_t (*f)() : {sk::preload_fam_exact, sk::preload_fam_screen16, sk::preload_fam_screen8, sk::preload_fam_screen9})
    if (hipError_t e = f()) return e;
  return hipSuccess;
}

hipError_t launch_sk_args(int sdt, int metric, int kt, int mode, int grid, int qslots, const SkArgs& a_in,
                          hipStream_t s, int ring) {
  const int ns = sk_slabs(sdt == KDT_SCREEN ? KDT_F32_X3 : sdt, a_in.d);
  if (!ns || a_in.b < 1 || a_in.b > qslots || a_in.n < 1 || (qslots != 32 && qslots != 64)) return hipErrorInvalidValue;
  SkArgs a = a_in;
  // the kernel's chunk geometry (its CT: sk_chunk_tiles), here instead of in every workgroup (MODE 1 does not use it,
  // but would compute it)
  a.geo = chunk_geo((a.n + 31) / 32, sk_chunk_tiles(sdt, a.d, a.ct8), grid, !a.no_guided);
  a.geo_set = 1;
  if (ring == 0) ring = kSkRing;
  if (ring != 2) return hipErrorInvalidValue;
  if (mode == 1) {   // verify, one workgroup per query slot: exact fp32 arithmetic (32 slots) or bf16's (32 or 64)
    if (grid != qslots || kt > 16 + 16 * (qslots == 32)) return hipErrorInvalidValue;
    if (sdt != KDT_BF16 && (sdt != KDT_F32_X3 || qslots != 32)) return hipErrorInvalidValue;
    return sk::fam_exact(sdt, metric, ns, kt, 1, grid, qslots, a, s);
  }
  if (sdt == KDT_SCREEN || sdt == KDT_SCREEN16) {   // the f16 screens: over the fp32 rows, or the f16 copy
    const int ns16 = sdt == KDT_SCREEN16 ? sk_slabs(KDT_SCREEN16, a.d) : ns;
    if (qslots != 32 || !ns16) return hipErrorInvalidValue;
    return sk::fam_screen16(sdt, metric, ns16, kt, grid, a, s);
  }
  if (sdt == KDT_SCREEN8 || sdt == KDT_SCREEN9) {   // the int8 screens (a.corpus = the int8 copy, a.n = ceil(rows8 / 2))
    const int ns8 = sk_slabs(sdt, a.d);
    if (!ns8 || !a.q8 || !a.q8s || !a.sx8 || !a.e8 || a.n != (a.rows8 + 1) / 2 || (sdt == KDT_SCREEN8 && !a.q8p2))
      return hipErrorInvalidValue;
    if (sdt == KDT_SCREEN8) {
      if (qslots != 32) return hipErrorInvalidValue;
      return sk::fam_screen8(metric, ns8, kt, grid, a, s);
    }
    // ONE query piece (a.q8 [64][d], a.q8s [4][64]): bf16 storage's 32 or 64 slots, fp32 storage's 32 on large shards
    if (qslots == 64 && kt > 16) return hipErrorInvalidValue;
    return sk::fam_screen9(metric, ns8, kt, grid, qslots, a, s);
  }
  if (qslots == 64 && sdt != KDT_BF16 && sdt != KDT_F32_SPLIT) return hipErrorInvalidValue;
  if (sdt < 0 || sdt > 3) return hipErrorInvalidValue;
  return sk::fam_exact(sdt, metric, ns, kt, 0, grid, qslots, a, s);
}

hipError_t launch_sk(int sdt, int metric, int kt, int grid, const void* c, const float* nr, const float* rs,
                     const float* q, int64_t n, int d, int b, uint32_t base, uint64_t* cand, hipStream_t s, int ring,
                     int qslots, uint32_t* ctr) {
  SkArgs a{};
  a.ctr = ctr;
  a.dyn = ctr != nullptr;
  a.corpus = (const char*)c;
  a.norms = nr;
  a.rscale = rs;
  a.queries = q;
  a.n = n;
  a.d = d;
  a.b = b;
  a.idx_base = base;
  a.out = cand;
  return launch_sk_args(sdt, metric, kt, 0, grid, qslots, a, s, ring);
}

#endif   // RR_SK_NO_DISPATCH

}  // namespace rr

#ifdef RR_VERIFY_DIAG
extern "C" int rr_debug_verify(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(rr::sk::vdiag), sizeof(unsigned long long) * 32 * 8);
}
#endif

#ifdef RR_SK_ONE_UNIT   // (diagnostic tools: every instantiation in the including unit)
#include "rr_sk_fam_exact.hip"
#include "rr_sk_fam_s16.hip"
#include "rr_sk_fam_s8.hip"
#include "rr_sk_fam_s9.hip"
#endif
