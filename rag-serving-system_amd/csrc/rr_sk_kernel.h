// rr_sk_kernel.h — the split-K streaming kernel (template; rr_sk.hip dispatches, rr_sk_fam_*.hip instantiate):
// similarity + top-k in one corpus pass, the corpus staged through LDS by non-temporal LDS-DMA (gfx950 / MI355X).
//
// Same contract as fused_score_kernel (rr_kernels.hip; reference retriever.py:594-611 + :742-769): one
// workgroup per CU computes the (32 doc x 32 query) score blocks of its rows and keeps a top-KT per
// query; cand[blockIdx][32][KT] goes to merge_kernel. What changes is how the corpus reaches the MFMAs:
//
//   * The workgroup owns ONE contiguous row range and walks it in 32-row tiles. Wave w owns bytes
//     [w*KS, (w+1)*KS) of every row (KS = row bytes / 8): a split of the dot product's K dimension over
//     the 8 waves, so each wave's slice of all 32 queries fits in its VGPRs (no LDS query image).
//   * A wave moves its slice of a tile in 4-KiB slabs (32 rows x 128 contiguous bytes) with
//     `global_load_lds_dwordx4 ... nt`: 8 rows x 128 B per instruction. Measured on MI355X
//     (tools/kbench.hip): non-temporal loads of >= 128 contiguous bytes per row per instruction stream
//     at 6.9-7.1 TB/s, the default-policy / 32-byte-per-row register loads of fused_score_kernel at
//     6.2-6.3. The LDS image is source-swizzled (16-byte column c of row r lands at c ^ (r & 7)) so the
//     MFMA-shaped ds_read_b128 of 32 rows is conflict-free.
//   * Two slab slots per wave: slab s + 1 is in flight while slab s is read and multiplied (counted
//     vmcnt; LDS-DMA has no VGPR destination, so nothing hipcc allocates can be hit by a landing load).
//   * Per tile the 8 K-partials are summed through LDS (XOR-swizzled rows, conflict-free; double-buffered, one raw
//     s_barrier per tile)
//     in a fixed order; wave w then runs the metric epilogue for queries 4w..4w+3 (2 rows x 1 query
//     per lane) and a per-lane top-KT insert. At the end each query's 16 lane lists are merged with
//     shuffles.
//
// Kernel dtypes (template DT), all reading the storage formats rr_api.cpp writes:
//   0 fp32 rows (pair_unit order), v_mfma_f32_32x32x2_f32: a plain fmaf chain per K-slice.
//   1 bf16 rows (pair_unit order), v_mfma_f32_32x32x16_bf16 against the query's bf16 hi + lo.
//   2 split-f16 rows (hi/lo per 8 elements), 3 x v_mfma_f32_32x32x16_f16, exact 2^e rescale.
//   3 fp32 rows (pair_unit order), each fp32 value split EXACTLY into three bf16 (x = b0 + b1 + b2,
//     round-to-nearest splits), the query likewise; 6 bf16 MFMAs (b0c0 b0c1 b1c0 b1c1 b0c2 b2c0): every
//     partial product is exact in fp32 and the dropped terms (b1c2, b2c1, b2c2) are below 2^-23 |x q|
//     (unbiased), the size of one fp32 rounding per product, so a score carries fp32 summation error
//     only. Half of DT 0's matrix-core cycles (and no f32-MFMA clock throttling).
//   6 SCREEN over fp32 rows: x rounded to f16 (one v_cvt_pk_f16_f32 per pair), q = c0 + c1 in f16, two f16
//     MFMAs per K-step. Not a score: the key is an UPPER BOUND u >= the DT 3 score (see "Screened search").
//   7 SCREEN over the f16 copy of fp32 rows (the values DT 6 rounds to, stored: half the bytes), q as ONE f16
//     piece, one f16 MFMA per K-step (the wider bound of rr_api.cpp kScreen16EpsA/B covers q's rounding).
// The K order inside a wave's slice is a permutation applied identically to both operands.
//
// Screened search (fp32 storage, k <= 29; rr_api.cpp enqueue_block):
//   1. MODE 0, DT 6 over the shard: per doc and query an upper bound u = s~ + eps of the exact DT 3 score
//      (cosine: of the clipped quotient), eps = eps_a |x||q| + eps_b (sqrt(d) |x| + sum|q|) from the
//      f16 rounding of x (<= 2^-11 |x| + 2^-25 per element), of the query split (<= 2^-22 |q| + 2^-24.9) and
//      generous fp32 accumulation bounds for both computations (rr_api.cpp kScreenEpsA/B); top-KT
//      (KT >= k + 3) by u per workgroup. At half the matrix-core work and a tenth of the vector work of
//      DT 3 it streams at the LDS-DMA rate, also while the GPU's power management throttles the core
//      clock during its first ~40 launches out of idle (profiles/r02/kbench_transient_screen.log).
//   2. MODE 1, DT 3, one workgroup per query slot: merges the screen's lists into the global top-32 by u (one
//      MFMA tile of rows; KT until r5), gathers those rows and scores them with EXACTLY the DT 3 arithmetic (same K
//      split, MFMA order and wave-reduction order: bit-identical to a full DT 3 pass), keeps the exact top-k.
//      Complete when the exact k-th score is strictly above the 32nd upper bound (every other doc's exact score
//      is at most its u, which is at most that bound) — or when the shard has fewer than 32 docs. (Else the wide
//      phase, or in repair mode the repair pass; bf16 storage: DT 9 screen, DT 1 verify, the same steps.)
//   3. Otherwise (rare: > KT - k docs inside the bound's window) the verify raises the block's flag word
//      (a monotonic sequence number; exchanged with the candidates when shards exchange) and the host
//      re-runs that search with the exact one-pass kernel when it collects the results (rr_api.cpp).
//   Either way the results are those of the exact DT 3 path, for every shard layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rr_device.h"
#include "rr_internal.h"

namespace rr {
namespace sk {

// Phase timestamps per workgroup (s_memrealtime, 100 MHz) for tools/kbench.hip built with -DRR_SK_PROBE;
// compiled out of the product library.
#ifdef RR_SK_PROBE
__device__ unsigned long long probe[4096 * 8];
#define SK_PROBE(i)                                                   \
  do {                                                                \
    if (threadIdx.x == 0) probe[blockIdx.x * 8 + (i)] = wall_clock64(); \
  } while (0)
__device__ unsigned long long probe2[4096 * 8];   // verify list-merge sub-phases
#define SK_PROBE2(i)                                                   \
  do {                                                                 \
    if (threadIdx.x == 0) probe2[blockIdx.x * 8 + (i)] = wall_clock64(); \
  } while (0)
#else
#define SK_PROBE2(i) \
  do {               \
  } while (0)
#define SK_PROBE(i) \
  do {              \
  } while (0)
#endif
// Verify diagnostics (A/B builds with -DRR_VERIFY_DIAG only): per query slot of the last verify launch, [the k-th
// largest bound, the largest single-list bound, phase-1 exact k-th, phase-2 exact k-th, |R|, decision, complete]
#ifdef RR_VERIFY_DIAG
__device__ unsigned long long vdiag[32 * 8];
#define VDIAG(i, v)                                        \
  do {                                                     \
    vdiag[(vq & 31) * 8 + (i)] = (unsigned long long)(v);         \
  } while (0)
#else
#define VDIAG(i, v) \
  do {              \
  } while (0)
#endif

// Per-phase cycle counters per wave (diagnostic builds with RR_SK_DIAG & 4 only, tools/kbench_cfg5.hip):
// [workgroup][wave][slab wait, slab loop rest, barrier A, write + barrier B, partial reads, epilogue, tiles, -]
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 4)
__device__ unsigned long long phase_cycles[4096 * 9 * 8];
#define PH_NOW() ((unsigned long long)__builtin_amdgcn_s_memtime())
#define PH_ADD(i, v) (ph[i] += (v))
#else
#define PH_NOW() 0ull
#define PH_ADD(i, v) \
  do {              \
  } while (0)
#endif

constexpr int kSlabRowBytes = 128;                // contiguous bytes of one row per slab
constexpr int kSlabBytes = 32 * kSlabRowBytes;    // 4 KiB
constexpr int kRedStride = 36;                    // floats allocated per (wave, query) block of 32 rows
constexpr int kRedRow = 32;                       // ... of which the XOR-swizzled partial sums use 32
// MODE 1 wide verify: its candidate rows R (int32 local rows) in the slab ring after the list-merge scratch
constexpr int kWideListOff = 16384;
constexpr int kWideCap = (2 * 8 * kSlabBytes - kWideListOff) / 4;   // ring_bytes(2) - the offset, in rows

// Ring of RS slab slots per wave: RS - 1 slabs stay in flight while one is multiplied. With RS = 2 the
// K-partial block is double-buffered (one barrier per tile); with RS = 3 (2 x 32 KiB more ring) it is
// single-buffered to fit 160 KiB, and a second barrier before the next tile's partials are written
// (normally passed without waiting: a whole tile of MFMAs lies between it and the reads it guards).
// With 64 query slots (QH = 2 halves of 32) the partial block doubles, so it is single-buffered too.
__host__ __device__ constexpr size_t ring_bytes(int rs) { return (size_t)kWaves * rs * kSlabBytes; }
__host__ __device__ constexpr int red_bufs(int rs, int qh) { return rs == 2 && qh == 1 ? 2 : 1; }
__host__ __device__ constexpr size_t red_bytes(int rs, int qh) {
  return (size_t)red_bufs(rs, qh) * kWaves * (32 * qh) * kRedStride * 4;
}

// storage position P (16-byte unit of a pair_unit-ordered row) -> logical unit
__device__ __forceinline__ int inv_pair(int p) { return (p & ~3) | ((p & 1) << 1) | ((p >> 1) & 1); }

// One 16-byte-per-lane LDS-DMA load, non-temporal. M0 (the LDS destination base) is written and restored
// in the same statement (cdna_hip_programming.md, inline-asm rules). The leading lgkmcnt(0) retires this
// wave's ds_reads of the slot being overwritten (issued one iteration earlier).
__device__ __forceinline__ void glds16(const void* src, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// The same with a scalar base address and a per-lane 32-bit offset (global saddr form): the per-slab address
// arithmetic is then scalar; the lane offset is loop-invariant.
__device__ __forceinline__ void glds16s(const void* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

// One whole slab (4 x 8 rows x 128 B) from one scalar base: per-lane offsets v0..v3 (row groups 0, 8, 16, 24), LDS
// destinations lds, lds + 1 KiB, ... M0 is saved, stepped and restored inside the one statement, with one leading
// lgkmcnt(0) (this wave's ds_reads of the slot): a third of the scalar instructions of four glds16s calls.
__device__ __forceinline__ void glds16s_slab(const void* sbase, unsigned v0, unsigned v1, unsigned v2, unsigned v3,
                                             unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %5 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5 nt\n\t"
      "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(sbase), "s"(lds)
      : "memory", "scc");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// s_waitcnt vmcnt(n) for the n the issue sequence leaves (workgroup- or wave-uniform): 0, or one slab (4)
// plus wave 0's single-instruction extras (per-row factors: 1, the int8 screen's 3; chunk counter)
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    default: wait_vm<8>(); break;
  }
}
// One 4-byte-per-lane LDS-DMA load (the per-row factors of a tile: 64 lanes x 4 B), default policy.
__device__ __forceinline__ void glds4(const void* src, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// LDS writes of this wave visible, then the workgroup barrier (no vmcnt: slabs stay in flight across it)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// two fp32 -> packed bf16 (round to nearest even), a in the low half. A plain conversion: hipcc emits
// v_cvt_pk_bf16_f32 for it on gfx950 AND pads its hazards. (An inline-asm v_cvt_pk here fed the MFMAs
// with one wait state where a VALU write -> MFMA operand read needs two: hipcc pads asm outputs by one
// state only, and the MFMA intermittently read the previous value of the register — a ~1e-4 relative
// score error on a few launches.)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// x = b0 + b1 + b2 exactly: three round-to-nearest bf16 splits (b0 = bf16(x), b1 = bf16(x - b0),
// b2 = x - b0 - b1; each residual is exact in fp32 and the last one fits bf16's 8 significant bits).
// |b1| <= 2^-8 |x|, |b2| <= 2^-16 |x|. 11 VALU ops per pair of values.
__device__ __forceinline__ void split3(const float (&x)[8], bf16x8& b0, bf16x8& b1, bf16x8& b2) {
  u32x4 p0, p1, p2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i], b = x[2 * i + 1];
    p0[i] = cvt_pk_bf16(a, b);
    const float ra = a - __uint_as_float(p0[i] << 16), rb = b - __uint_as_float(p0[i] & 0xFFFF0000u);
    p1[i] = cvt_pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(p1[i] << 16), sb = rb - __uint_as_float(p1[i] & 0xFFFF0000u);
    p2[i] = cvt_pk_bf16(sa, sb);
  }
  b0 = __builtin_bit_cast(bf16x8, p0);
  b1 = __builtin_bit_cast(bf16x8, p1);
  b2 = __builtin_bit_cast(bf16x8, p2);
}

// All-ones / all-zeros lane mask the compiler cannot see through, and x AND-ed with it: the loads that
// feed it are then issued unconditionally (a select on the predicate gets turned into exec-masked branches
// around each load, which serialises their latencies). Exact zeros, whatever x holds.
__device__ __forceinline__ uint32_t opaque_mask(bool keep) {
  uint32_t m = keep ? 0xFFFFFFFFu : 0u;
  asm volatile("" : "+v"(m));
  return m;
}
__device__ __forceinline__ f32x4 zero_unless(f32x4 x, uint32_t m) {
  u32x4 u = __builtin_bit_cast(u32x4, x);
  u &= (u32x4){m, m, m, m};
  return __builtin_bit_cast(f32x4, u);
}

// Query operand (B) fragments of one wave's K-slice, per slab j and K-step.
template <int DT, int NS>
struct QFrag;
template <int NS>
struct QFrag<0, NS> { float v[NS][16]; };                     // per MFMA m: one fp32
template <int NS>
struct QFrag<1, NS> { bf16x8 hi[NS][4], lo[NS][4]; };         // 4 K-steps of 16 bf16 per slab
template <int NS>
struct QFrag<2, NS> { f16x8 hi[NS][2], lo[NS][2]; };          // 2 K-steps of 16 per slab
template <int NS>
struct QFrag<3, NS> { bf16x8 c0[NS][2], c1[NS][2], c2[NS][2]; };
template <int NS>
struct QFrag<6, NS> { f16x8 c0[NS][2], c1[NS][2]; };          // screen: q = c0 + c1 (+ <= 2^-22 |q|)
template <int NS>
struct QFrag<7, NS> { f16x8 c0[NS][4]; };   // screen over the f16 copy: 4 K-steps per slab, q as one f16 piece
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
template <int NS>
struct QFrag<8, NS> { i32x4 c1[NS][4], c2[NS][4]; };   // int8 screen: 4 K-steps of 32 per slab, two int8 pieces
template <int NS>
struct QFrag<9, NS> { i32x4 c1[NS][4]; };   // the bf16 storage's int8 screen: one int8 piece (64 slots fit)


// LDS byte offset (within a slot) of 16-byte column position cp of tile row r (swizzled image): column cp of row r sits
// at position cp ^ (r & 7) ^ ((r >> 3) & 1). A ds_read_b128 serves 16 lanes per pass — rows r .. r + 15 of one column
// position here — which must cover all 64 banks: the (r & 7) term spreads rows r .. r + 7 over 32 of them, the
// (r >> 3) & 1 term moves rows r + 8 .. r + 15 to the other 32. (r6: without it rows r and r + 8 shared their banks —
// 4 conflict cycles per fragment read, every SQ_LDS_BANK_CONFLICT cycle of the streaming kernels; profiles/r06/sq/.
// Round 4 had attributed them to the LDS-DMA landing.)
__device__ __forceinline__ int slab_off(int r, int cp) {
  return (r >> 3) * 1024 + (r & 7) * 128 + ((cp ^ (r & 7) ^ ((r >> 3) & 1)) << 4);
}

// Verify stage (MODE 1): the screen's [QS][nlists][KT] upper-bound lists -> this query's global top-NC by u
// in akeys[] (LDS, descending; NC = 32 >= KT: one whole MFMA tile of rows), by rank selection instead of NC rounds of
// wave-wide maxima:
//   1. thread l holds list l (sorted; lists beyond kThreads folded into thread l % kThreads's list);
//   2. H = the NC-th largest list head (its rank among the heads is NC - 1; 0 when fewer than NC heads are
//      non-empty). Every key of the global top-NC is >= H: NC distinct heads are >= H, so a key below H has
//      rank >= NC. Only the <= NC lists whose head is >= H can hold such keys: <= NC x KT candidates;
//   3. the non-empty keys >= H are appended to an LDS array, and the candidate of rank r < NC is akeys[r].
// Keys are unique (distinct row indices), so ranks are distinct. Each list of the screen carries its workgroup's
// floor after its KT keys (see KL in sk_score_kernel): their maximum goes to *floor_out (LDS; valid after the return).
// Keys a folded list loses (below the thread's list's last entry) join the floor maximum, so every key left out of
// akeys is at most max(akeys[NC - 1], *floor_out). Scratch: LDS free in MODE 1 (the slab ring): [kThreads] heads,
// [NC * KT] candidates, H, count, floor maximum.
// (r5: NC = 32 instead of KT — the first tile rescored 16 rows of its 32 — so the int8 screen's looser bound proves
// most slots without the wide phase.)
template <int KT, int NC = 32>
__device__ __forceinline__ void merge_lists_for_query(const uint64_t* __restrict__ in, int nlists, int qslots, int q,
                                                      uint64_t* scratch, uint64_t* akeys, uint64_t* floor_out,
                                                      uint64_t* tail_out) {
  const int tid = threadIdx.x;
  uint64_t* heads = scratch;
  uint64_t* cand = scratch + kThreads;
  uint64_t* hs = cand + NC * KT;
  int* cnt = (int*)(hs + 1);
  constexpr int LS = KT + 1;   // list stride: KT keys + the workgroup's floor
  static_assert(NC >= KT && NC <= 32, "the first verify tile rescores NC <= 32 rows");
  TopK<KT> tk;
  uint64_t fl = 0, tl = 0;     // floors; and every list's own bound, max(its KT-th key, its floor) (wide verify)
  if (tid < nlists) {
    const uint64_t* src = in + ((size_t)q * nlists + tid) * LS;   // query-major screen lists
#pragma unroll
    for (int i = 0; i < KT; ++i) tk.v[i] = src[i];
    fl = src[KT];
    tl = umax64(fl, tk.v[KT - 1]);
  } else {
    tk.init();
  }
  for (int l = tid + kThreads; l < nlists; l += kThreads) {   // lists beyond kThreads folded in (sorted input)
    const uint64_t* src = in + ((size_t)q * nlists + l) * LS;
    fl = umax64(fl, src[KT]);
    tl = umax64(tl, umax64(src[KT], src[KT - 1]));
    for (int i = 0; i < KT; ++i) {
      const uint64_t key = src[i];
      if (key <= tk.last()) {   // (this and the rest of the list are left out: the floor covers them)
        fl = umax64(fl, key);
        break;
      }
      fl = umax64(fl, tk.last());   // the entry the insert pushes out
      tk.insert(key);
    }
  }
  SK_PROBE2(0);   // lists loaded (this thread's)
  const int nl = nlists < kThreads ? nlists : kThreads;
  const int nlp = (nl + 7) & ~7;   // heads padded with empty keys to whole 8-key groups
  const int lane = tid & 63, wv = tid >> 6;
  uint64_t* fw = hs + 4;             // [kWaves] per-wave floor maxima, then [kWaves] list-bound maxima
  uint64_t* tw = fw + kWaves;
  if (tid == 0) {
    hs[0] = 0;
    cnt[0] = 0;
  }
  if (tid < nlp) heads[tid] = tk.v[0];   // (threads past the lists hold empty lists)
  // the floors' and the list bounds' maxima: a wave-wide max, one LDS word per wave (not one LDS atomic per list on a
  // single address: 2 x 256 of those serialised to ~7 us)
  const uint64_t fwv = wave_max_u64(fl), twv = wave_max_u64(tl);
  if (lane == 0 && wv < kWaves) {   // (a carried verify's 9th wave, the screen's scheduler, only passes the barriers)
    fw[wv] = fwv;
    tw[wv] = twv;
  }
  __syncthreads();
  SK_PROBE2(1);   // heads in LDS
  // each head's rank among the heads: 8 heads per step from broadcast 16-byte LDS reads; with <= 256 lists two threads
  // per head, each scanning half of them (every wave busy), their counts added through LDS
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  const u64x2* hv = (const u64x2*)heads;
  // (16 heads per step while the range allows — eight reads in flight per LDS latency — then 8)
  auto count_above = [&](uint64_t me, int j0, int j1) {
    int rank = 0;
    int j = j0;
    for (; j + 8 <= j1; j += 8) {
      u64x2 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = hv[j + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) rank += (x[u][0] > me ? 1 : 0) + (x[u][1] > me ? 1 : 0);
    }
    if (j < j1) {   // (j1 - j0 is a multiple of 4)
      u64x2 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = hv[j + u];
#pragma unroll
      for (int u = 0; u < 4; ++u) rank += (x[u][0] > me ? 1 : 0) + (x[u][1] > me ? 1 : 0);
    }
    return rank;
  };
  if (nlp <= kThreads / 2) {
    int* part = (int*)(tw + kWaves);   // [kThreads / 2] the second half's counts
    const int hh = tid & (kThreads / 2 - 1), half = tid / (kThreads / 2);
    const uint64_t me = heads[hh];
    const int g8 = nlp / 16 * 4;       // the first half's end, in 16-byte units (multiple of 4)
    int rank = 0;
    if (hh < nl && me != 0) rank = half ? count_above(me, g8, nlp / 2) : count_above(me, 0, g8);
    if (half == 1) part[hh] = rank;
    __syncthreads();
    if (!half && hh < nl && me != 0 && rank + part[hh] == NC - 1) hs[0] = me;
  } else if (tid < nl && tk.v[0] != 0) {
    if (count_above(tk.v[0], 0, nlp / 2) == NC - 1) hs[0] = tk.v[0];
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t f = 0, t = 0;
    for (int i = 0; i < kWaves; ++i) {
      f = umax64(f, fw[i]);
      t = umax64(t, tw[i]);
    }
    *floor_out = f;
    *tail_out = t;
  }
  SK_PROBE2(2);   // H known
  const uint64_t th = hs[0];
  if (tid < nl && tk.v[0] != 0 && tk.v[0] >= th) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < KT; ++i) c += tk.v[i] != 0 && tk.v[i] >= th ? 1 : 0;   // a prefix of the sorted list
    const int pos = atomicAdd(cnt, c);
#pragma unroll
    for (int i = 0; i < KT; ++i)
      if (i < c) cand[pos + i] = tk.v[i];
  }
  __syncthreads();
  SK_PROBE2(3);   // candidates appended
  const int m = cnt[0];
  if (tid < NC && tid >= m) akeys[tid] = 0;   // fewer than NC keys in all: empty tail
  for (int c = tid; c < m; c += kThreads) {
    const uint64_t me = cand[c];
    int rank = 0;
    for (int j = 0; j < m; ++j) rank += cand[j] > me ? 1 : 0;
    if (rank < NC) akeys[rank] = me;
  }
  __syncthreads();
}

// The wide phase's bar (MODE 1 and the fused verify; ords of keys). vtail = the largest bound of any single list:
// every key missing from every list is at most vtail. Two cases prove the block with one more pass over the lists:
//   * the first pass's exact k-th key ek lies above vtail: the true k-th score is at least ek's, so only rows whose
//     bound reaches ek can be in the top-k — and all of them are list entries (anything else is <= vtail < ek). R =
//     the entries with bound >= ek: typically a few rows more than KT, where the bound is looser than KT - k
//     ranks of the score distribution (the int8 screen, or a crowded top);
//   * else, when the k-th largest bound lies above vtail (near-duplicate clusters): R = every entry above vtail.
// Either way the exact k-th key of R is above vtail and the block is complete.
__device__ __forceinline__ uint32_t wide_bar(uint64_t ek, uint64_t tb) {
  const uint32_t e = (uint32_t)(ek >> 32), t = (uint32_t)(tb >> 32);
  return ek != 0 && e > t ? e : t + 1;
}

// QH = query halves: 32 * QH query slots per pass (64 for the batch-64 configs: one corpus pass serves
// them all; each A fragment then feeds the MFMAs of both halves).
// MODE 0: top-KT per query over this workgroup's rows (DT 6: by upper bound).
// MODE 1: verify (DT 3, QH 1): block q = query slot q; see "Screened search" above.
template <int DT, int NS, int KT, bool COS, int RS, int QH, int MODE, int SCHED, int FL>
__global__ __launch_bounds__(SCHED ? 576 : 512, 1) void sk_score_kernel(const SkArgs a) {
  static_assert(RS == 2, "two slab slots per wave: one in flight while one is multiplied (the waits assume it)");
  static_assert(QH == 1 || QH == 2, "32 or 64 query slots");
  static_assert(MODE == 0 || ((DT == 3 || DT == 1) && QH == 1),
                "the verify stage runs the storage's exact arithmetic: fp32 (DT 3) or bf16 (DT 1)");
  static_assert(SCHED == 0 || (MODE == 0 && QH == 1), "the scheduler wave serves the 32-slot streaming pass");
  constexpr int QS = 32 * QH;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SK_PROBE(0);
  if constexpr (MODE == 0) {   // the exchanged flag word this block's verify may raise starts at 0
    if (a.clear_word && blockIdx.x == 0 && threadIdx.x == 0) *a.clear_word = 0;
  }
  if constexpr (MODE == 0 && FL == 2) {   // repair mode: this block's chunk marks start empty (the verify sets them)
    for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < a.rbits_words; i += (int)(gridDim.x * blockDim.x))
      a.rbits[i] = 0u;
  }
  const char* __restrict__ corpus = a.corpus;
  const float* __restrict__ norms = a.norms;
  const float* __restrict__ rscale = a.rscale;
  const float* __restrict__ queries = a.queries;
  const int64_t n = a.n;
  const int d = a.d, b = a.b;
  const uint32_t idx_base = a.idx_base;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  constexpr bool SCR = DT == 6 || DT == 7 || DT == 8 || DT == 9;   // the screen (upper bounds, "Screened search")
  constexpr bool I8 = DT == 8 || DT == 9;                          // ... over an int8 copy (kernel rows of two rows)
  // The screen's per-lane lists hold KL keys, not KT: a query's LPQ lanes together still hold >= KT, and a lane drops
  // a key only below its own last entry. The workgroup reports the largest last entry of its full lanes as its FLOOR
  // (no key missing from its list is above max(the list's KT-th key, the floor)); the verify adds the floors to its
  // completeness bound. The branch-free insert, the epilogue's largest VALU item, then costs KL compare-selects.
  // (FL = 1: full lists, KL = KT — the handle switches to them when the short lists' floors stop the verify's
  // proofs, e.g. near-duplicate clusters whose copies crowd a few lanes; rr_api.cpp observe_settled)
  constexpr int KL = SCR && KT > 4 && !FL ? 4 : KT;
  constexpr int EB = DT == 1 || DT == 7 ? 2 : I8 ? 1 : 4;   // storage bytes per element
  // the int8 screen reads two corpus rows as one kernel row (waves 0-3 the first, 4-7 the second): its tiles then
  // carry 64 KiB like the f16 copy's, 64 corpus rows each (int8 tiles of 32 rows would halve every per-tile cost's
  // share of the bytes it pays for)
  constexpr int RPK = I8 ? 2 : 1;
  const int row_bytes = d * EB * RPK;
  constexpr int KS = NS * kSlabRowBytes;                        // bytes of a row per wave
  const int p0 = w * (KS / 16);                                 // first 16-byte storage unit of the slice

  float* red = (float*)(smem + ring_bytes(RS));
  constexpr int SW = (COS || SCR ? 1 : 0) + (DT == 2 ? 1 : 0);   // per-row factors (norm, split scale)
  // LDS-DMA instructions per tile for them: one (64 lanes: 2 factors x 32 rows), or the int8 screen's three (norm,
  // scale, error norm of 64 corpus rows)
  constexpr int FX = I8 ? 3 : SW > 0 ? 1 : 0;
  constexpr int TRS = I8 ? 192 : 64;                            // floats per factor slot
  float* trow = (float*)(smem + ring_bytes(RS) + red_bytes(RS, QH));   // [4 tiles][TRS]
  int* nxt = (int*)(trow + 4 * TRS);                            // [2] next chunk (dynamic schedule), + pad
  float* qinfo = (float*)(nxt + 4);                             // [QS] |q|, [QS] 2^-e / sum|q| / max|q|, [QS] int e
  int* qexp = (int*)(qinfo + 2 * QS);

  // ---- MODE 1: the candidate rows of query slot vq ---------------------------------------------------------
  // (LDS after qexp: merge scratch W [8][KT], akeys [KT], grow [32], gnorm [32], gvalid [32], xk [KT])
  const int vq = MODE == 1 ? (int)blockIdx.x : 0;
  // (the bf16 screen's verify serves 64 slots: slot vq's data — query row, lists, chunk maxima, results — at vq, its
  // place in this workgroup's 32-column lane mapping and query scalars at vql)
  const int vql = vq & 31;
  uint64_t* vW = (uint64_t*)(qexp + QS);
  uint64_t* akeys = vW + kWaves * KT;   // [32]: the first tile's candidates (merge_lists_for_query NC)
  int* grow = (int*)(akeys + 32);
  float* gnorm = (float*)(grow + 32);
  int* gvalid = (int*)(gnorm + 32);
  uint64_t* xk = (uint64_t*)(gvalid + 32);
  uint64_t* vfloor = xk + KT;   // MODE 1: the largest floor of the screen's lists (see KL)
  uint64_t* vtail = vfloor + 1; // MODE 1: the largest bound of any single list, max(KT-th key, floor) (wide verify)
  int* vstate = (int*)(vtail + 1);   // MODE 1: [0] what the leader decided after the first check, [1] |R|, [4] R's bar,
                                     // [5] the slot needs the repair pass, [6] its bar (an ord)
  // MODE 1 reads its 32 gathered rows straight into registers (all loads issued at once: one latency), the
  // exact fragments the LDS image would give: lane (r, h) takes 16-byte units 4(i>>1) + 2h + (i&1) of slab j
  f32x4 vrow[MODE == 1 ? NS : 1][4];
  // (bf16, DT 1: K-step t's unit 2t + h)
  auto vunit = [&](int i) { return DT == 1 ? 2 * i + h : 4 * (i >> 1) + 2 * h + (i & 1); };
  if constexpr (MODE == 1) {
    if (vq >= b) {   // padding slot: keep the exchange buffer uniform
      if (a.out_keys && tid < KT) a.out_keys[(size_t)vq * KT + tid] = 0;
      return;
    }
  }

  // ---- MODE 0 work: 32-row tiles in chunks of CT tiles (about 8 slabs, 256 KiB of corpus per workgroup).
  // Workgroup g takes chunk g, then (SCHED) the next free chunk from a device counter — workgroups on CUs that
  // get a larger share of the HBM bandwidth take more chunks, so all of them finish together — or (static)
  // chunks g + G, g + 2G, ...
  constexpr int CT0 = NS >= 4 ? 2 : NS == 3 ? 3 : NS == 2 ? 4 : 8;
  // the int8 screen: a.ct8 tiles (of 64 corpus rows) per chunk — 2 on small shards, where a 4-tile chunk is a large
  // share of a workgroup's work and the last ones leave a tail (profiles/r04/ab/ab_ct8.txt), else 4
  const int CT = I8 && a.ct8 > 0 ? a.ct8 : CT0;
  const int64_t G = gridDim.x, g = blockIdx.x;
  // Guided tail: chunks of CT tiles, then (CT > 2) the last ~2 G tiles in 2-tile chunks, so the launch's last chunks —
  // the tail where workgroups finish at different times — are short (tools/probe_screen.hip: the 1M-row int8 screen's
  // workgroups ended over 9 us with 4-tile chunks throughout; +4-5 % for the screen alone at 1M rows,
  // profiles/r05/ab_guided.txt). Chunk c: first tile cbase(c), ctiles(c) tiles; every chunk but the last has >= 2 tiles
  // (the scheduler wave's next-chunk word is read at a chunk's last tile).
  // The repair pass (a.rlist: MODE 0 over the fp32 rows, static schedule) instead walks the screen chunks listed in
  // rlist: chunk j = the corpus rows of screen chunk rlist[j] (rs: the screen's geometry, rs_rows rows per screen tile).
  const bool REP = MODE == 0 && !SCR && SCHED == 0 && a.rlist != nullptr;
  const ChunkGeo geo = a.geo_set ? a.geo : chunk_geo((n + 31) / 32, CT, G, !a.no_guided);   // (host-computed: launch_sk_args)
  const int64_t T = geo.T;
  const int64_t C = REP ? (int64_t)*a.rcount : geo.C;
  auto rep_rows = [&](int64_t j, int64_t* r0, int64_t* r1) {
    const int64_t sc = a.rlist[j];
    *r0 = chunk_tile0(a.rs, sc) * a.rs_rows;
    const int64_t e = *r0 + (int64_t)chunk_ntiles(a.rs, sc) * a.rs_rows;
    *r1 = e < n ? e : n;
  };
  auto cbase = [&](int64_t c) -> int64_t {
    if (REP) {
      int64_t r0, r1;
      rep_rows(c, &r0, &r1);
      return r0 / 32;
    }
    return chunk_tile0(geo, c);
  };
  auto ctiles = [&](int64_t c) -> int {
    if (REP) {
      int64_t r0, r1;
      rep_rows(c, &r0, &r1);
      return (int)((r1 - r0 + 31) / 32);
    }
    return chunk_ntiles(geo, c);
  };

  // LDS-DMA lane mapping: instruction i of a slab covers tile rows 8i + lane/8, 16-byte column
  // (lane % 8) ^ (lane / 8) ^ (i & 1) of the slab — so the image holds column c of row r at c ^ (r & 7) ^ ((r >> 3) & 1)
  // (slab_off)
  const int rl = lane >> 3, cl = lane & 7;
  const unsigned ring_lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(smem + (size_t)w * RS * kSlabBytes));
  const unsigned trow_lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)trow);
  const char* ring = smem + (size_t)w * RS * kSlabBytes;
  const char* lane_src = corpus + (size_t)w * KS + ((cl ^ rl) << 4);        // row groups 0, 16 (instructions 0, 2)
  const char* lane_srcx = corpus + (size_t)w * KS + ((cl ^ rl ^ 1) << 4);   // row groups 8, 24 (instructions 1, 3)

  // per-lane part of a slab address: row rl of each 8-row group, swizzled 16-byte column (< 8 rows: 32-bit)
  const unsigned lane_off = (unsigned)(rl * row_bytes + ((cl ^ rl) << 4));
  const unsigned lane_offx = (unsigned)(rl * row_bytes + ((cl ^ rl ^ 1) << 4));
  const unsigned row8 = (unsigned)(8 * row_bytes);   // (row groups 8, 16, 24 of a tile: offsets < 2^32)
  const char* wave_src = corpus + (size_t)w * KS;
  auto issue = [&](int64_t base, int j, int slot) {   // slab j (this wave's K-slice) of the tile at row base
    if (base + 32 <= n) {   // whole tile (workgroup-uniform): scalar addresses
      const int64_t sb = __builtin_amdgcn_readfirstlane((int)(base >> 32)) * 0x100000000ll +
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)base);
#ifndef RR_SK_SLAB_ASM
#define RR_SK_SLAB_ASM 1   // one inline-asm statement per slab; A/B (r4, profiles/r04/ab_slab.txt): window +1.5 %, steady +0.8 %
#endif
      if constexpr (RR_SK_SLAB_ASM) {
        glds16s_slab(wave_src + sb * row_bytes + j * kSlabRowBytes, lane_off, lane_offx + row8, lane_off + 2 * row8,
                     lane_offx + 3 * row8, ring_lds + slot * kSlabBytes);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          glds16s(wave_src + (sb + 8 * i) * row_bytes + j * kSlabRowBytes, (i & 1) ? lane_offx : lane_off,
                  ring_lds + slot * kSlabBytes + i * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int64_t row = base + 8 * i + rl;
        row = row < n ? row : n - 1;                    // partial last tile: re-read a valid row
        glds16(((i & 1) ? lane_srcx : lane_src) + row * row_bytes + j * kSlabRowBytes, ring_lds + slot * kSlabBytes + i * 1024);
      }
    }
  };
  // wave 0: the per-row factors of the tile at row base into factor slot ts (lanes 0-31: the norm, or the
  // split scale when there is no norm; lanes 32-63: the split scale next to a norm)
  auto issue_factors = [&](int64_t base, int ts) {
    if constexpr (I8) {   // corpus rows 2 base + lane: norm, scale, error norm
      int64_t row = 2 * base + lane;
      row = row < a.rows8 ? row : a.rows8 - 1;
      glds4(norms + row, trow_lds + ts * TRS * 4);
      glds4(a.sx8 + row, trow_lds + ts * TRS * 4 + 256);
      glds4(a.e8 + row, trow_lds + ts * TRS * 4 + 512);
    } else {
      int64_t row = base + (lane & 31);
      row = row < n ? row : n - 1;
      const float* src = ((SW == 2 && lane >= 32) || (DT == 2 && !COS)) ? rscale : norms;
      glds4(src + row, trow_lds + ts * 256);
    }
  };

  if constexpr (SCHED) {
    if (w == kWaves) {
      // The scheduler wave (a 9th wave: no corpus, no query, no inline-asm loads, so hipcc's own waits around
      // its atomic drain nothing else). Per chunk it takes the next free chunk from the counter and publishes
      // it in nxt[] before the chunk's first reduction barrier; the streaming waves read it at the chunk's last
      // step. It passes exactly the barriers the streaming waves pass: one after the query scalars, one per tile.
      __syncthreads();
      int64_t ck = g;
      int cp = 0;
      while (ck < C) {
        const int tic = ctiles(ck);
        if (ck != C - 1 && lane == 0) {   // every chunk but the last asks once: C - 1 dequeues per launch
          const uint32_t old = __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const int64_t nc = G + (int64_t)old;
          nxt[cp] = (int)(nc < C ? nc : C);
          // the launch's last dequeue resets the counter for the next launch on this stream
          if ((int64_t)old == C - 2) __hip_atomic_store(a.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int t = 0; t < tic; ++t) lds_barrier();
        if (ck == C - 1) break;
        ck = nxt[cp];
        cp ^= 1;
      }
      return;
    }
  }

  // Slabs in flight per wave: LA = 2 when a tile has at least two slabs — slab i + 2 is issued into slab i's
  // slot as soon as slab i's fragments are in registers (before its MFMAs), so two slabs stay in flight through
  // the MFMAs and the epilogue — else 1 (slab i + 1 issued before waiting for slab i).
#ifndef RR_SK_LOOKAHEAD
#define RR_SK_LOOKAHEAD 2
#endif
#ifndef RR_SK_LA64
#define RR_SK_LA64 1
#endif
  constexpr int LA = NS >= 2 ? (QH == 1 || I8 ? RR_SK_LOOKAHEAD : RR_SK_LA64) : 1;   // (64-slot bf16: measured faster with 1)
  int pend = 0;   // LA 2: vector-memory ops this wave issued after the slab it waits for next
  int64_t chunk = g, base = cbase(chunk) * 32;
  if constexpr (MODE == 0) {
    if (chunk < C) {   // prologue: the first tile's factors and slab 0 (and 1)
      if (FX && w == 0) issue_factors(base, 0);
      issue(base, 0, 0);
      if constexpr (LA == 2) {
        issue(base, 1, 1);
        pend = 4;
      }
    }
  }
  // ---- query side: this wave's K-slice of every query as MFMA B operands, |q| and split exponents.
  // Runs while the prologue slabs above are in flight (their latency overlaps the query loads).
  QFrag<DT, NS> qfs[QH];
  // the screen's per-query scalars from the fragments' own loads (SCR): this lane's sum of x^2 and of |x| over the
  // query values it converts (its part of the wave's K-slice)
  float scr_ss = 0.f, scr_sa = 0.f;
  auto build_frags = [&]() {
    // lane: query r (+ 32 per half), K half h
#pragma unroll
    for (int qh = 0; qh < QH; ++qh) {
      QFrag<DT, NS>& qf = qfs[qh];
      // MODE 1 puts query vq in every column: each output element depends only on its own column's operands,
      // so column vq's scores are bit-identical to a full pass's, and every lane loads the same 4 KB
      const int rq = MODE == 1 ? vq : r + 32 * qh;
      const bool qv = rq < b;
      const float* qrow = queries + (size_t)(qv ? rq : 0) * d;
      const uint32_t qmask = opaque_mask(qv);
      // 16-byte loads of 4 consecutive elements (e % 4 == 0), unconditional (rows >= b read row 0) and
      // zeroed by a select: no per-element exec-masked branches around the loads
      auto qvec = [&](int e) -> f32x4 { return zero_unless(*(const f32x4*)(qrow + e), qmask); };
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        if constexpr (DT == 0) {
          // MFMA m of slab j: lane half h holds position 4h + (m >> 2), element m & 3
#pragma unroll
          for (int m4 = 0; m4 < 4; ++m4) {
            const f32x4 v = qvec(4 * inv_pair(p0 + 8 * j + 4 * h + m4));
#pragma unroll
            for (int e = 0; e < 4; ++e) qf.v[j][4 * m4 + e] = v[e];
          }
        } else if constexpr (DT == 1) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {   // K-step t: lane half h reads position 2t + h (8 bf16)
            const int L = inv_pair(p0 + 8 * j + 2 * t + h);
            const f32x4 va = qvec(8 * L), vb = qvec(8 * L + 4);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = e < 4 ? va[e] : vb[e - 4];
              const __bf16 bh = (__bf16)x;
              qf.hi[j][t][e] = bh;
              qf.lo[j][t][e] = (__bf16)(x - (float)bh);
            }
          }
        } else if constexpr (DT == 8) {
          // the query prep kernel's int8 pieces (natural element order, padding slots zero): wave w's K-slice of the
          // two-row kernel row is elements (w % 4) KS .. + KS of its corpus row; K-step t, lane half h: 16 elements
          // at 32 t + 16 h of slab j — the 16-byte column 2t + h of the LDS image, as DT 7
          const int8_t* p1 = a.q8 + (size_t)rq * d;
          const int8_t* p2 = a.q8p2 + (size_t)rq * d;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e0 = (w & (kWaves / 2 - 1)) * KS + j * kSlabRowBytes + 32 * t + 16 * h;
            qf.c1[j][t] = *(const i32x4*)(p1 + e0);
            qf.c2[j][t] = *(const i32x4*)(p2 + e0);
          }
        } else if constexpr (DT == 9) {
          // one piece per query (slot rq = r + 32 qh), the same element mapping as DT 8
          const int8_t* p1 = a.q8 + (size_t)rq * d;
#pragma unroll
          for (int t = 0; t < 4; ++t)
            qf.c1[j][t] = *(const i32x4*)(p1 + (w & (kWaves / 2 - 1)) * KS + j * kSlabRowBytes + 32 * t + 16 * h);
        } else if constexpr (DT == 7) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {   // the bf16 layout (position 2t + h, 8 elements), f16 pieces c0 + c1
            const int L = inv_pair(p0 + 8 * j + 2 * t + h);
            const f32x4 va = qvec(8 * L), vb = qvec(8 * L + 4);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = e < 4 ? va[e] : vb[e - 4];
              qf.c0[j][t][e] = (_Float16)x;
              scr_ss = fmaf(x, x, scr_ss);
              scr_sa += fabsf(x);
            }
          }
        } else if constexpr (DT == 2) {
          const int ex = qv ? qexp[rq] : 0;
#pragma unroll
          for (int t = 0; t < 2; ++t) {   // K-step t: lane half h reads units 4t + 2h (hi), + 1 (lo)
            const int g8 = (p0 + 8 * j + 4 * t + 2 * h) >> 1;   // 8-element group
            const f32x4 va = qvec(8 * g8), vb = qvec(8 * g8 + 4);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float xs = ldexpf(e < 4 ? va[e] : vb[e - 4], ex);
              const _Float16 fh = (_Float16)xs;
              qf.hi[j][t][e] = fh;
              qf.lo[j][t][e] = (_Float16)(xs - (float)fh);
            }
          }
        } else {
#pragma unroll
          for (int t = 0; t < 2; ++t) {   // K-step t: lane half h reads positions 4t + 2h, 4t + 2h + 1
            float x[8];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const f32x4 v = qvec(4 * inv_pair(p0 + 8 * j + 4 * t + 2 * h + u));
#pragma unroll
              for (int e = 0; e < 4; ++e) x[4 * u + e] = v[e];
            }
            if constexpr (DT == 3) {
              split3(x, qf.c0[j][t], qf.c1[j][t], qf.c2[j][t]);
            } else {   // DT 6: q = c0 + c1 in f16 (RNE), residual exact in fp32
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const _Float16 c0 = (_Float16)x[e];
                qf.c0[j][t][e] = c0;
                qf.c1[j][t][e] = (_Float16)(x[e] - (float)c0);
                scr_ss = fmaf(x[e], x[e], scr_ss);
                scr_sa += fabsf(x[e]);
              }
            }
          }
        }
      }
    }
  };
  // Pin the fragments: an empty asm that "rewrites" each one makes them opaque values, so they stay in VGPRs
  // for the whole launch. Without it hipcc kept the fp32 query values instead and re-derived the fragments
  // (mask, bf16 / f16 splits) inside the tile loop for every slab — the 64-slot bf16 kernel's main VALU cost.
  auto pin_frags = [&]() {
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        if constexpr (DT == 0) {
#pragma unroll
          for (int m = 0; m < 16; ++m) asm volatile("" : "+v"(qfs[qh].v[j][m]));
        } else if constexpr (DT == 1) {
#pragma unroll
          for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(qfs[qh].hi[j][t]), "+v"(qfs[qh].lo[j][t]));
        } else if constexpr (DT == 2) {
#pragma unroll
          for (int t = 0; t < 2; ++t) asm volatile("" : "+v"(qfs[qh].hi[j][t]), "+v"(qfs[qh].lo[j][t]));
        } else if constexpr (DT == 3) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
            asm volatile("" : "+v"(qfs[qh].c0[j][t]), "+v"(qfs[qh].c1[j][t]), "+v"(qfs[qh].c2[j][t]));
        } else if constexpr (DT == 7) {
#pragma unroll
          for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(qfs[qh].c0[j][t]));
        } else if constexpr (DT == 8) {
#pragma unroll
          for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(qfs[qh].c1[j][t]), "+v"(qfs[qh].c2[j][t]));
        } else if constexpr (DT == 9) {
#pragma unroll
          for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(qfs[qh].c1[j][t]));
        } else {
#pragma unroll
          for (int t = 0; t < 2; ++t) asm volatile("" : "+v"(qfs[qh].c0[j][t]), "+v"(qfs[qh].c1[j][t]));
        }
      }
  };
  // the int8 screen's per-query scalars of this lane's epilogue query (qe below), loaded with the fragments: one
  // latency before the first barrier instead of a second one after it
  float q8pre[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (I8) {   // (the staged scalars [6][stride]: |q|, sum|q|, then DT 8's scale / 64 and two-piece residual
                        // norm, or DT 9's scale and one-piece residual norm — rr_device.h q8_stage_row)
    const int qe0 = 4 * QH * w + lane / (16 / QH);
    const size_t st = (size_t)a.q8s_stride;
#pragma unroll
    for (int i = 0; i < 4; ++i) q8pre[i] = a.q8s[(i < 2 || DT == 8 ? i : i + 2) * st + qe0];
  }
  if constexpr (MODE == 0) SK_PROBE(6);   // (diagnostic builds: prologue issued, before the fragments)
  if constexpr (DT != 2) {
    build_frags();
    pin_frags();
  }
  if constexpr (MODE == 0) SK_PROBE(7);   // (fragments in registers)
  // ---- per-query scalars: |q| (cosine, fp32 as cp.linalg.norm, retriever.py:602), split exponents (DT 2),
  // sum |q| (DT 6 bound), max |q| (MODE 1: the screen's f16 range). All loads of a group of 4 queries are
  // issued before any is used (one L2/HBM latency per group, not one per query); the sums are the same
  // lane-strided fmaf chains + xor tree in the same order.
  if constexpr (MODE == 1) {   // |q| and max |q| of query vq only, by wave 0
    if (w == 0) {
      const int nc = d >> 2;
      f32x4 v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cc = lane + 64 * c;
        v[c] = zero_unless(((const f32x4*)queries)[(size_t)vq * nc + (cc < nc ? cc : 0)], opaque_mask(cc < nc));
      }
      float ss = 0.f, m = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (lane + 64 * c < nc) {
          const f32x4 x = v[c];
          ss = fmaf(x.x, x.x, ss); ss = fmaf(x.y, x.y, ss); ss = fmaf(x.z, x.z, ss); ss = fmaf(x.w, x.w, ss);
          m = fmaxf(m, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
        }
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {   // the same xor tree as the full pass's |q|
        ss += __shfl_xor(ss, off, 64);
        m = fmaxf(m, __shfl_xor(m, off, 64));
      }
      if (lane == 0) {
        qinfo[vql] = sqrtf(ss);
        qinfo[QS + vql] = m;
      }
    }
    __syncthreads();
  } else if constexpr (SCR) {
    // The screen's |q| and sum|q| from the values the fragments were built from (each wave holds its K-slice of
    // every query; lanes r and r + 32 the two halves): per-wave partials in the verify scratch (unused in MODE 0),
    // summed per query in wave order below. No second read of the query rows: every workgroup re-reading all 32
    // rows from L2 was the larger part of the launch's start-up (8-10 us). The order of these sums differs from
    // the exact path's |q|, so the bound takes a 2^-18 relative bump for it (rr_sk.hip epilogue).
    if constexpr (!I8) {   // (the int8 screens' scalars come from the query prep kernel)
      const float ss = scr_ss + __shfl_xor(scr_ss, 32, 64), sa = scr_sa + __shfl_xor(scr_sa, 32, 64);
      float* part = (float*)vW;
      if (lane < 32) {
        part[w * 32 + lane] = ss;
        part[kWaves * 32 + w * 32 + lane] = sa;
      }
    }
    __syncthreads();
  } else if (COS || DT == 2) {
    const int nc = d >> 2;                      // float4 per row (d <= 1024 on this kernel: <= 4 per lane)
#pragma unroll
    for (int g4 = 0; g4 < QH; ++g4) {
      f32x4 v[4][4];
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        const int q = w * 4 * QH + 4 * g4 + qi;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int cc = lane + 64 * c;
          const f32x4 x = ((const f32x4*)queries)[(size_t)(q < b ? q : 0) * nc + (cc < nc ? cc : 0)];
          v[qi][c] = zero_unless(x, opaque_mask(q < b && cc < nc));
        }
      }
#pragma unroll
      for (int qi = 0; qi < 4; ++qi) {
        const int q = w * 4 * QH + 4 * g4 + qi;
        float ss = 0.f, m = 0.f, sa = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (lane + 64 * c < nc) {
            const f32x4 x = v[qi][c];
            ss = fmaf(x.x, x.x, ss); ss = fmaf(x.y, x.y, ss); ss = fmaf(x.z, x.z, ss); ss = fmaf(x.w, x.w, ss);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
            if constexpr (SCR) sa += (fabsf(x.x) + fabsf(x.y)) + (fabsf(x.z) + fabsf(x.w));
          }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          ss += __shfl_xor(ss, off, 64);
          m = fmaxf(m, __shfl_xor(m, off, 64));
          if constexpr (SCR) sa += __shfl_xor(sa, off, 64);
        }
        int E = 0;
        if (m > 0.f) frexpf(m, &E);
        const int ex = m > 0.f ? 15 - E : 0;
        if (lane == 0) {
          qinfo[q] = sqrtf(ss);
          qinfo[QS + q] = DT == 2 ? ldexpf(1.0f, -ex) : SCR ? sa * (1.0f + 0x1p-20f) : m;
          qexp[q] = ex;
        }
      }
    }
    __syncthreads();
  }

  if constexpr (DT == 2) {
    build_frags();
    pin_frags();
  }

  // ---- MODE 1: this query's candidates (the queries' fragments and scalars above are already built, so
  // their loads overlapped the list loads), then their rows straight into registers ---------------------------
  if constexpr (MODE == 1) {
    static_assert((size_t)(kThreads + 32 * KT + 4 + 2 * kWaves) * 8 + kThreads / 2 * 4 <= kWideListOff,
                  "verify merge scratch in the slab ring");
    SK_PROBE(6);
    merge_lists_for_query<KT>(a.vin, a.nlists, QS, vq, (uint64_t*)smem, akeys, vfloor, vtail);
    SK_PROBE(7);
    if (tid < 32) {
      const uint64_t k0 = akeys[0];
      const uint64_t key = akeys[tid];
      const int64_t first = k0 ? (int64_t)(0xFFFFFFFFu - (uint32_t)k0) - idx_base : 0;
      const int64_t row = key ? (int64_t)(0xFFFFFFFFu - (uint32_t)key) - idx_base : first;
      grow[tid] = (int)row;
      gvalid[tid] = key != 0;
      gnorm[tid] = COS ? norms[row] : 0.f;
    }
    __syncthreads();
    SK_PROBE(3);
    const char* src = corpus + (int64_t)grow[r] * row_bytes + (size_t)w * KS;
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        vrow[j][i] = *(const f32x4*)(src + j * kSlabRowBytes + (vunit(i) << 4));
  }


  // epilogue lane mapping: wave w owns queries 4·QH·w + [0, 4·QH); LPQ lanes per query, each with DPL
  // consecutive tile rows (QH 1: 16 lanes x 2 rows, QH 2: 8 lanes x 4 rows)
  constexpr int LPQ = 16 / QH, DPL = 2 * QH;
  constexpr int DPO = DPL * RPK;
  constexpr int NIA = DT == 8 ? 2 : DT == 9 ? QH : 1;   // int32 accumulators (DT 8: pieces p1, p2; DT 9: query halves)   // scores per lane and tile (the int8 screen: the two corpus rows of each kernel row)
  constexpr int J = (KT + LPQ - 1) / LPQ;   // (the epilogue's tighter bar: each lane's J-th list entry)
  static_assert(J <= KL, "the tighter bar reads each lane's J-th entry");
  const int qe = 4 * QH * w + lane / LPQ, er = DPL * (lane % LPQ);
  const bool qev = MODE == 1 ? qe == vql : qe < b;
  float qn = COS && !SCR ? qinfo[qe] : 0.f;
  const float qs = DT == 2 ? qinfo[QS + qe] : 1.f;
  float qsa = 0.f, q8sc = 0.f, q8e1 = 0.f, q8e2 = 0.f, q8e3 = 0.f;
  if constexpr (I8) {
    qn = q8pre[0];   // (a.q8s[i * QS + qe], loaded before the first barrier)
    qsa = q8pre[1];
    q8sc = q8pre[2];
    // the bound's slack e Q1 + |x| Q2 + Q3 (see the epilogue), its per-query factors once: all terms are positive and
    // each is rounded a few times, which the 1.001 margin covers
    const float eq = q8pre[3];
    q8e1 = (qn + eq) * 1.001f;
    q8e2 = (eq + fmaf(a.eps_a, qn, a.eps_b * a.sqrt_d)) * 1.001f;
    // + 2^-110 absolute: the exact DT 3 score's products that fall below fp32's normal range, and every rounding of
    // this bound's own arithmetic in the subnormal range, for rows and queries both tiny; + Q2 2^-69: the row norm |x|
    // (fp32 sum of squares) reads short by at most sqrt(d) 2^-74.5 when the squares underflow
    q8e3 = fmaf(q8e2, 0x1p-69f, fmaf(a.eps_b * qsa, 1.001f, 0x1p-110f));
  } else if constexpr (SCR) {
    const float* part = (const float*)vW;
    float s2 = 0.f, s1 = 0.f;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {
      s2 += part[ww * 32 + qe];
      s1 += part[kWaves * 32 + ww * 32 + qe];
    }
    qn = sqrtf(s2);
    // (+ what eps_b >= 2^-25 turns into the int8 screen's absolute terms, q8e3: 2^-110 for subnormal products and
    // roundings, and (eps_a |q| + eps_b sqrt(d)) 2^-69 for a row norm whose squares underflowed — eps_a / eps_b < 2^14)
    qsa = fmaf(s1, 1.0f + 0x1p-18f, fmaf(qn, 0x1p-55f, 0x1p-63f));
  }

  TopK<KL> tk;
  tk.init();
  float umax = -INFINITY;   // repair mode (FL 2): this lane's largest bound in the current chunk
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 4)
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // phase cycles; [7] = insert executions (wave-wide)
#endif

  // The metric epilogue of one tile: its summed scores svp (this lane's DPL rows), its first row bse and its factor
  // slot tsl. (Issuing it one tile late, in the next tile's MFMA shadow, measured -2 % on the 64-slot bf16 kernel
  // and neutral on the screen: profiles/r03/a/ab_pipelined_epilogue_rejected.txt.)
  auto epilogue = [&](const float (&svp)[DPO], int64_t bse, int tsl) {
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 1)
      // diagnostic builds only (tools/kbench_cfg5.hip): no epilogue, the sums kept live by one compare each
#pragma unroll
      for (int e = 0; e < DPL; ++e)
        if (svp[e] > 1e30f) tk.insert(make_key(svp[e], (uint32_t)(bse + er + e)));
      return;
#endif
      // Cosine prefilter: a score whose estimate dot * rcp(den) (within a few ulp of the quotient) is below
      // the lane's current k-th score minus a 2^-20 relative margin cannot enter the list, so only the
      // few that pass pay the exact IEEE division (the list only grows inside the loop: the threshold
      // taken here is conservative).
      // full-key output (a.all_keys; the 32-wide instantiation, for the full-sort path): every key goes to HBM
      constexpr bool DUMP = MODE == 0 && KT == 32 && QH == 1 && SCHED == 0 && !SCR;
      // The bar a key must clear: the largest last entry of the query's LPQ lane lists (once full). A key at or
      // below it cannot be in this workgroup's top-KT for the query (that lane alone holds KT keys above it), so
      // no lane keeps it — the merged lists are the same as without the bar, but lanes insert ~LPQ x less often
      // (the branch-free insert is the epilogue's largest VALU cost, and it runs for the whole wave whenever
      // any of its lanes inserts). For the large-k floors: a key dropped here is below a full lane's last entry.
      // A tighter bar, as valid: when each of the group's LPQ lanes holds J = ceil(KT / LPQ) keys of at least y, the
      // group holds LPQ * J >= KT keys >= y, so no key below y is in the workgroup's top-KT. y = the smallest of the
      // lanes' J-th entries (0 while a lane holds fewer) — about the group's KT-th key, where the largest last entry
      // is about its (LPQ x KT)-th: far fewer keys pass, and the insert runs far less often. Not for the large-k output
      // (its lists must hold the workgroup's top wide_k > KT); the screen's short lists hold J (<= KL) too, and a key it
      // drops below y is below the workgroup's KT-th key or a full lane's last (its floor): either way inside the
      // verify's bound.
      uint32_t th = group_max_u32<LPQ>((uint32_t)(tk.last() >> 32));
      if (MODE == 1 || a.wide_k == 0) {
        const uint32_t tmin = group_min_u32<LPQ>((uint32_t)(tk.v[J - 1] >> 32));
        th = th > tmin ? th : tmin;
      }
      // Keys whose score ord is below th are dropped; ties on the score go on to the insert, whose 64-bit compares
      // place them exactly (inserting a key at or below a list's last leaves it unchanged).
      float thr = -INFINITY;
      if constexpr (SCR) {
        // the screen compares in the bound's own (float) domain, and only the keys that pass are formed — one
        // compare per score instead of a key and a 64-bit compare
        if (th != 0) thr = float_of_ord(th);
      } else if constexpr (COS) {
        if (th != 0) {
          const float t = float_of_ord(th);
          thr = t - fabsf(t) * 0x1p-20f - 0x1p-100f;
        }
      }
      // rows of this tile (scalar; 32 except in the last tile): the screen's validity test is one 32-bit compare
      // (the int8 screen: corpus rows of this 64-row tile, lane rows 2 er .. 2 er + 3)
      const int rem = I8 ? (int)(a.rows8 - 2 * bse < 64 ? a.rows8 - 2 * bse : 64)
                              : MODE == 0 ? (int)(n - bse < 32 ? n - bse : 32) : 32;
      const uint32_t key_base = MODE == 0 ? idx_base + (uint32_t)(RPK * bse) : 0u;
      const int ero = RPK * er;   // this lane's first tile row
      // the exact paths' prefilter, rcp-free: s / den >= thr  <=  s >= thr * den (den > 0), evaluated as one fma of
      // per-tile terms; within 2^-20 relative of the quotient's own rounding, like the margin above
      float thq = 0.f, th8 = -INFINITY;
      if constexpr (COS && !SCR) {
        if (th != 0) {
          thq = thr * qn;
          th8 = thr * 1e-8f;
        }
      }
      const float thf = th != 0 ? float_of_ord(th) : -INFINITY;   // dot: the bar's float (ord order = float order)
      // this lane's per-row factors, one vector LDS read each (factor 0 at [0, 32), factor 1 at [32, 64))
      float fac0[DPO], fac1[DPO], fac2[DPO];
      if constexpr (I8) {   // norm, scale, error norm of corpus rows 2 er .. 2 er + DPO - 1 (16-byte aligned)
        const float* tf = trow + tsl * TRS + ero;
#pragma unroll
        for (int e4 = 0; e4 < DPO; e4 += 4) {
          const f32x4 v0 = *(const f32x4*)(tf + e4), v1 = *(const f32x4*)(tf + 64 + e4), v2 = *(const f32x4*)(tf + 128 + e4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            fac0[e4 + e] = v0[e];
            fac1[e4 + e] = v1[e];
            fac2[e4 + e] = v2[e];
          }
        }
      } else if constexpr (MODE == 0 && (COS || SCR || DT == 2)) {
        const float* tf = trow + tsl * 64 + er;
        if constexpr (DPL == 4) {
          const f32x4 v0 = *(const f32x4*)tf;
#pragma unroll
          for (int e = 0; e < 4; ++e) fac0[e] = v0[e];
          if constexpr (DT == 2 && COS) {
            const f32x4 v1 = *(const f32x4*)(tf + 32);
#pragma unroll
            for (int e = 0; e < 4; ++e) fac1[e] = v1[e];
          }
        } else {
          const float2 v0 = *(const float2*)tf;
          fac0[0] = v0.x;
          fac0[1] = v0.y;
          if constexpr (DT == 2 && COS) {
            const float2 v1 = *(const float2*)(tf + 32);
            fac1[0] = v1.x;
            fac1[1] = v1.y;
          }
        }
      }
      bool pass[DPO];
      float sc[DPO], ndv[DPO];
      int64_t rows[DPO];
      bool anyp = false;
#pragma unroll
      for (int e = 0; e < DPO; ++e) {
        int64_t row;
        bool valid;
        float nd = 1.f;
        float s = svp[e];
        pass[e] = false;
        if constexpr (MODE == 1) {
          row = grow[er + e];
          valid = qev && gvalid[er + e];
          if constexpr (COS) nd = gnorm[er + e];
        } else {
          row = RPK * bse + ero + e;
          // (the screen keeps lists for padding query slots too: nobody reads them)
          valid = SCR ? ero + e < rem : qev && ero + e < rem;
          if constexpr (DT == 2) s = s * (COS ? fac1[e] : fac0[e]) * qs;   // exact 2^e rescales
          if constexpr (COS || SCR) nd = fac0[e];
        }
        rows[e] = row;
        sc[e] = s;
        ndv[e] = nd;
        if constexpr (SCR) {
          // upper bound of the exact (DT 3) score, see "Screened search"; the relative bumps cover the
          // roundings of the bound's own arithmetic and of the reciprocal (<= 1 ulp)
          float v;
          if constexpr (I8) {
            // int8 screen: s = x8 . (64 p1 + p2) exactly (DT 9: x8 . p1) (int32, rounded once to fp32); x . q = sx s scale + q~ . rx
            // + eq . x with |q~ . rx| <= (|q| + eq) e and |eq . x| <= eq |x|, plus the exact DT 3 score's own error
            // (eps_a |x||q| + eps_b (sqrt(d) |x| + sum|q|), rr_api.cpp kScreen8EpsA/B; eps_b sum|q| also covers
            // residuals whose squares underflow fp32 in e, |r| < 2^-63); x 1.001 for the roundings of
            // |q| and of these products, 2^-21 |est| for the three roundings of est
            const float est = (s * fac1[e]) * q8sc;
            // = ((|q| + eq) e + eq |x| + eps_a |x||q| + eps_b (sqrt(d) |x| + sum|q|)) x 1.001, factored per query
            const float eps = fmaf(fac2[e], q8e1, fmaf(nd, q8e2, q8e3));
            v = est + fmaf(fabsf(est), 0x1p-21f, eps);
          } else {
            const float eps = fmaf(a.eps_a * nd, qn, a.eps_b * fmaf(a.sqrt_d, nd, qsa));
            v = s + eps;
          }
          v += fabsf(v) * 0x1p-22f;
          float u;
          if constexpr (COS) {
            u = v * __builtin_amdgcn_rcpf(cos_den(qn, nd));
            u += fabsf(u) * 0x1p-18f + 0x1p-126f;   // (+ |q| in another summation order than the exact path's)
            // the exact score is clipped to [-1, 1] (retriever.py:609). The min comes first: a NaN bound (inf * 0 or
            // inf - inf in the bound's own arithmetic) becomes +1, never a value below the exact score. (rr_api.cpp
            // keeps rows and queries where that arithmetic stays finite; this is the kernel's own guard.)
            u = fmaxf(fminf(u, 1.0f), -1.0f);
          } else {
            u = v;
          }
          if (valid && u >= thr) tk.insert(make_key(u, key_base + (uint32_t)(ero + e)));   // (NaN: never)
          if constexpr (FL == 2) {   // repair mode: the largest bound of the chunk's rows (NaN-free: u is clipped)
            if (valid) umax = fmaxf(umax, u);
          }
        } else if constexpr (COS) {
          // dot / (|q|*|d| + 1e-8), then clip to [-1, 1]   (retriever.py:605-609)
          if (DUMP && a.all_keys) {
            if (valid) {
              const float den = cos_den(qn, nd);
              a.all_keys[(size_t)qe * n + row] = make_key(fminf(fmaxf(s / den, -1.0f), 1.0f), idx_base + (uint32_t)row);
            }
          } else {
            pass[e] = valid && s >= fmaf(thq, nd, th8);
          }
        } else {
          if (DUMP && a.all_keys) {
            if (valid) a.all_keys[(size_t)qe * n + row] = make_key(s, idx_base + (uint32_t)row);
          } else {
            pass[e] = valid && s >= thf;
          }
        }
        if constexpr (!SCR && KT > 16) {
          // (32-entry lists: the insert right here — keeping the scores for a later pass spills those kernels)
          if (pass[e]) {
            float c = s;
            if constexpr (COS) {
              c = c / cos_den(qn, nd);
              c = fminf(fmaxf(c, -1.0f), 1.0f);
            }
            const uint64_t key = make_key(c, idx_base + (uint32_t)row);
            if ((uint32_t)(key >> 32) >= th) tk.insert(key);
          }
          pass[e] = false;
        }
        anyp = anyp || pass[e];
      }
      if constexpr (!SCR && KT <= 16) {
        // the few scores that pass: their exact keys (IEEE division for cosine, as the reference's elementwise
        // kernel), inserted when at or above the bar (ties on the score go on to the insert's 64-bit compares)
        if (anyp) {
#pragma unroll
          for (int e = 0; e < DPL; ++e) {
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 4)
            if (__builtin_amdgcn_ballot_w64(pass[e]) != 0) PH_ADD(7, 1);
#endif
            if (pass[e]) {
              float c = sc[e];
              if constexpr (COS) {
                c = c / cos_den(qn, ndv[e]);
                c = fminf(fmaxf(c, -1.0f), 1.0f);
              }
              const uint64_t key = make_key(c, idx_base + (uint32_t)rows[e]);
              if ((uint32_t)(key >> 32) >= th) tk.insert(key);
            }
          }
        }
      }
  };

  // Stagger (streaming passes): waves 4-7 — the SIMD partners of waves 0-3 — run each tile's epilogue one tile
  // late, after issuing the next tile's MFMAs, its summed scores kept in registers across the barrier. Partners
  // that reach the same phase together (matrix work, epilogue, barrier) leave the matrix core idle while both run
  // the epilogue's vector work; staggered, one wave's epilogue runs beside its partner's MFMAs. The lists see the
  // same inserts in the same order: results are unchanged.
#ifndef RR_SK_STAGGER
#define RR_SK_STAGGER 2   // 0 off, 1 the 64-slot pass only, 2 every streaming pass
#endif
#ifndef RR_SK_STAGGER8
#define RR_SK_STAGGER8 0   // 1: the int8 screen too — its 9-wave form then spills 6 VGPRs and measured 4-8 % slower
                           // (profiles/r04/ab/ab_i8_stagger.txt)
#endif
  // (Rejected and removed: exchanging a tile's K-partials one tile late behind the next tile's MFMAs, -2 % on the
  // 64-slot pass, profiles/r03/b/ab_pipelined_exchange_rejected.txt; deferring the odd waves instead of 4-7.)
  constexpr bool STG = MODE == 0 && FL != 2 && !(QH == 2 && DT == 2) && DT != 6 && (!I8 || RR_SK_STAGGER8) &&
                       KT <= 16 &&   // (measured)
                       (RR_SK_STAGGER == 2 || (RR_SK_STAGGER == 1 && QH == 2));
  const bool defer = STG && w >= 4;
  float svd[DPO];
  int64_t bsd = -1;   // first row of the deferred tile (-1: none)
  int tsd = 0;        // its factor slot (4 slots: wave 0 refills a slot three tiles after its tile at the earliest)

  // ---- sum the 8 K-partials of a tile (fixed order), then the metric epilogue --------------------------
  auto write_partials = [&](float* rb, const f32x16 (&accs)[QH]) {
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int a4 = 0; a4 < 4; ++a4) {   // C/D map: acc[4a + i] = (doc 8a + 4h + i, query r)
        const f32x4 v = {accs[qh][4 * a4], accs[qh][4 * a4 + 1], accs[qh][4 * a4 + 2], accs[qh][4 * a4 + 3]};
        // 32 floats per (wave, query) row, its eight 16-byte chunks XOR-swizzled by the query index: the 8-lane
        // groups of this ds_write_b128 and the epilogue's ds_read_b64 / ds_read_b128 groups are conflict-free
        // (the +4-float padding it replaced left the reads 2-way conflicted: 1.6e8 of 5.0e8 LDS cycles at B = 64)
        const int rq = 32 * qh + r;
        *(f32x4*)(rb + (w * QS + rq) * kRedRow + 4 * ((2 * a4 + h) ^ (rq & 7))) = v;
      }
  };
  // int8 screen: each wave's two accumulators (pieces p1, p2) combined exactly, 64 a1 + a2 (|.| < 2^29), as int32 bits
  auto write_partials8 = [&](float* rb, const i32x16 (&ia)[2]) {
#pragma unroll
    for (int a4 = 0; a4 < 4; ++a4) {
      i32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = ia[0][4 * a4 + i] * 64 + ia[1][4 * a4 + i];
      *(i32x4*)(rb + (w * QS + r) * kRedRow + 4 * ((2 * a4 + h) ^ (r & 7))) = v;
    }
  };
  // DT 9: each query half's accumulator as int32 bits (|.| < 2^23), the 64-slot layout of write_partials
  auto write_partials9 = [&](float* rb, const i32x16 (&ia)[NIA]) {
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int a4 = 0; a4 < 4; ++a4) {
        const i32x4 v = {ia[qh][4 * a4], ia[qh][4 * a4 + 1], ia[qh][4 * a4 + 2], ia[qh][4 * a4 + 3]};
        const int rq = 32 * qh + r;
        *(i32x4*)(rb + (w * QS + rq) * kRedRow + 4 * ((2 * a4 + h) ^ (rq & 7))) = v;
      }
  };
  // ... and summed exactly in int32 (|sum| < 2^31): waves 0-3 give the kernel rows' first corpus rows, 4-7 the second;
  // sv = corpus rows 2 er, 2 er + 1, ..., 2 (er + DPL) - 1, each rounded once to fp32
  auto read_partials8 = [&](const float* rb, float (&sv)[DPO]) {
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    typedef int i32xd __attribute__((ext_vector_type(DPL)));
    i32xd ev, od;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {
      const i32xd p = *(const i32xd*)(rb + (ww * QS + qe) * kRedRow + 4 * ((er >> 2) ^ (qe & 7)) + (er & 3));
      if (ww == 0) ev = p;
      else if (ww < kWaves / 2) ev += p;
      else if (ww == kWaves / 2) od = p;
      else od += p;
    }
#pragma unroll
    for (int i = 0; i < DPL; ++i) {
      sv[2 * i] = (float)ev[i];
      sv[2 * i + 1] = (float)od[i];
    }
  };
  // (two-float vectors: packed adds, each element summed in the same wave order)
  auto read_partials = [&](const float* rb, float (&sv)[DPL]) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 acc2[DPL / 2];
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {   // fixed wave order: the same sums for any QH (wave 0's partial first)
      const float* src = rb + (ww * QS + qe) * kRedRow + 4 * ((er >> 2) ^ (qe & 7)) + (er & 3);
      if constexpr (DPL == 2) {
        const f32x2 p = *(const f32x2*)src;
        acc2[0] = ww ? acc2[0] + p : p;
      } else {
        const f32x4 p = *(const f32x4*)src;
        const f32x2 p0 = {p[0], p[1]}, p1 = {p[2], p[3]};
        acc2[0] = ww ? acc2[0] + p0 : p0;
        acc2[1] = ww ? acc2[1] + p1 : p1;
      }
    }
#pragma unroll
    for (int e = 0; e < DPL; ++e) sv[e] = acc2[e >> 1][e & 1];
  };
  // Static issue priority for waves 4-7 (the second-dispatched half, the arbitration loser of every VALU/MFMA issue
  // contest with its SIMD partner; MI355X_MICROARCH.md "Two waves per SIMD" item 4): config-5 shard +1.2 % with the
  // stagger (tools/kbench_cfg5.hip; waves 0-3 instead: null). 0 off, 1 waves 4-7, 2 waves 0-3 (A/B).
#ifndef RR_SK_PRIO
#define RR_SK_PRIO 1
#endif
  // (not the int8 screen, which runs without the stagger: +1.5-3 % without it, profiles/r04/ab/ab_i8_prio.txt)
  if (MODE == 0 && !I8 && ((RR_SK_PRIO == 1 && w >= 4) || (RR_SK_PRIO == 2 && w < 4))) __builtin_amdgcn_s_setprio(1);
  unsigned long long ph_t = PH_NOW();
  (void)ph_t;
  SK_PROBE(1);
  int slot = 0, ti = 0, cpar = 0, ts = 0;   // ring slot, tile of the chunk, nxt parity, factor slot
  int64_t tcount = 0;                       // tiles done (reduction buffer parity)
  bool run = MODE == 1 || chunk < C;
  while (run) {
    const int tic = MODE == 1 ? 1 : ctiles(chunk);   // tiles in this chunk
    const bool last_in_chunk = ti + 1 == tic;
    int64_t next_chunk = C, next_base = -1;
    f32x16 accs[QH];
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int i = 0; i < 16; ++i) accs[qh][i] = 0.f;
    i32x16 iacc[NIA];   // the int8 screens' accumulators (DT 8: pieces p1, p2; DT 9: the query halves)
    if constexpr (I8)
#pragma unroll
      for (int u = 0; u < NIA; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) iacc[u][i] = 0;
    // LA 2: after slab j's fragments are read, its slot takes slab j + 2 — of this tile, or slab 0 / 1 of the
    // next tile (found at slab NS - 2; wave 0 issues that tile's factors before its slab 0)
    auto issue_ahead = [&](auto jc) {
      constexpr int j = decltype(jc)::value;
      int n_is = 0;
      if constexpr (j + 2 < NS) {
        issue(base, j + 2, slot);
        n_is = 4;
      } else if constexpr (j + 2 == NS) {
        if (!last_in_chunk) {
          next_base = base + 32;
        } else {   // (SCHED: nxt[] was published before this chunk's first tile barrier; a chunk with a
                   // successor has >= 2 tiles, so that barrier is behind us)
          next_chunk = !SCHED ? chunk + G : chunk == C - 1 ? C : (int64_t)nxt[cpar];
          next_base = next_chunk < C ? cbase(next_chunk) * 32 : -1;
        }
        if (next_base >= 0) {
          if (FX && w == 0) {
            issue_factors(next_base, (ts + 1) & 3);
            n_is += FX;
          }
          issue(next_base, 0, slot);
          n_is += 4;
        }
      } else {
        if (next_base >= 0) {
          issue(next_base, 1, slot);
          n_is = 4;
        }
      }
      pend = n_is;
    };
    static_for<0, NS>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      if constexpr (MODE == 0 && LA == 2) {
        const unsigned long long pw0 = PH_NOW();
        wait_vm_n(pend);   // slab j landed (loads complete in order; the pend ops issued after it may not have)
        PH_ADD(0, PH_NOW() - pw0);
      } else if constexpr (MODE == 0) {
        // keep one slab in flight: issue the next slab (of this tile, or slab 0 of the next tile with wave 0
        // issuing that tile's factors first) into the slot consumed last, then wait for this one. Wave 0's
        // counted wait includes its single-instruction extras issued after this slab (factors, counter).
        int nw = 0, extra0 = 0;
        if (j + 1 < NS) {
          issue(base, j + 1, slot ^ 1);
          nw = 4;
        } else {
          if (!last_in_chunk) {
            next_base = base + 32;
          } else {
            next_chunk = !SCHED ? chunk + G : chunk == C - 1 ? C : (int64_t)nxt[cpar];
            next_base = next_chunk < C ? cbase(next_chunk) * 32 : -1;
          }
          if (next_base >= 0) {
            if (FX && w == 0) {
              issue_factors(next_base, (ts + 1) & 3);
              extra0 += FX;
            }
            issue(next_base, 0, slot ^ 1);
            nw = 4;
          }
        }
        if (nw) nw += w == 0 ? extra0 : 0;
        const unsigned long long pw0 = PH_NOW();
        wait_vm_n(nw);
        PH_ADD(0, PH_NOW() - pw0);
      }
      const char* sl = ring + slot * kSlabBytes;
      if constexpr (DT == 0) {
        f32x4 av[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = *(const f32x4*)(sl + slab_off(r, 4 * h + i));
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int m = 0; m < 16; ++m)
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m >> 2][m & 3], qfs[qh].v[j][m], accs[qh], 0, 0, 0);
      } else if constexpr (DT == 1) {
        bf16x8 av[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
          av[t] = MODE == 1 ? __builtin_bit_cast(bf16x8, vrow[MODE == 1 ? j : 0][t]) : *(const bf16x8*)(sl + slab_off(r, 2 * t + h));
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[t], qfs[qh].hi[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[t], qfs[qh].lo[j][t], accs[qh], 0, 0, 0);
        }
      } else if constexpr (DT == 7) {   // screen over the f16 copy: x exactly as DT 6 rounds it, half the bytes
        f16x8 av[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = *(const f16x8*)(sl + slab_off(r, 2 * t + h));
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t], qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
        }
      } else if constexpr (DT == 8) {   // int8 screen: 32 K per MFMA, both query pieces
        i32x4 av[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = *(const i32x4*)(sl + slab_off(r, 2 * t + h));
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          iacc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[t], qfs[0].c1[j][t], iacc[0], 0, 0, 0);
          iacc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[t], qfs[0].c2[j][t], iacc[1], 0, 0, 0);
        }
      } else if constexpr (DT == 9) {   // bf16 storage's int8 screen: one piece per query, both query halves
        i32x4 av[4];
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 8)
        // diagnostic builds only (profiles/r06/sq): no slab fragment reads (the LDS-DMA still lands)
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = (i32x4){lane, t, j, (int)tcount};
#else
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = *(const i32x4*)(sl + slab_off(r, 2 * t + h));
#endif
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          for (int qh = 0; qh < QH; ++qh) iacc[qh] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[t], qfs[qh].c1[j][t], iacc[qh], 0, 0, 0);
      } else if constexpr (DT == 2) {
        f16x8 ah[2], al[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          ah[t] = *(const f16x8*)(sl + slab_off(r, 4 * t + 2 * h));
          al[t] = *(const f16x8*)(sl + slab_off(r, 4 * t + 2 * h + 1));
        }
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], qfs[qh].hi[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], qfs[qh].lo[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[t], qfs[qh].hi[j][t], accs[qh], 0, 0, 0);
        }
      } else {
        f32x4 av[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          av[i] = MODE == 1 ? vrow[MODE == 1 ? j : 0][i] : *(const f32x4*)(sl + slab_off(r, 4 * (i >> 1) + 2 * h + (i & 1)));
        if constexpr (MODE == 0 && LA == 2) issue_ahead(jc);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const float x[8] = {av[2 * t].x, av[2 * t].y, av[2 * t].z, av[2 * t].w,
                              av[2 * t + 1].x, av[2 * t + 1].y, av[2 * t + 1].z, av[2 * t + 1].w};
          if constexpr (DT == 3) {
            bf16x8 b0, b1, b2;
            split3(x, b0, b1, b2);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c2[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
          } else {   // DT 6: x rounded to f16 (RNE), two f16 MFMAs
            f16x8 hx;
#pragma unroll
            for (int e = 0; e < 8; ++e) hx[e] = (_Float16)x[e];
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(hx, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(hx, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
          }
        }
      }
      slot ^= 1;
    });
    unsigned long long pt1 = PH_NOW();
    (void)pt1;
    PH_ADD(1, pt1 - ph_t);
    if (defer && bsd >= 0) {   // the previous tile's epilogue, beside this tile's MFMAs
      epilogue(svd, bsd, tsd);
      bsd = -1;
      const unsigned long long pe = PH_NOW();
      PH_ADD(5, pe - pt1);
      pt1 = pe;
    }

    float* rb = red + (red_bufs(RS, QH) == 2 ? (size_t)(tcount & 1) * kWaves * QS * kRedStride : 0);
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 2)
    if (MODE == 0) {   // diagnostic builds only: no K-partial exchange (the barrier stays), this wave's own partials
      lds_barrier();
      float sv[DPO];
#pragma unroll
      for (int e = 0; e < DPO; ++e) {
        if constexpr (I8) sv[e] = (float)iacc[e % NIA][e];
        else sv[e] = accs[e % QH][e];
      }
      epilogue(sv, base, ts);
      ++tcount;
      ts = (ts + 1) & 3;
      if (!last_in_chunk) {
        ++ti;
        base += 32;
        continue;
      }
      if (next_chunk >= C) break;
      chunk = next_chunk;
      ti = 0;
      cpar ^= 1;
      base = cbase(chunk) * 32;
      continue;
    }
#endif
    {
      if constexpr (red_bufs(RS, QH) == 1) {
        if (tcount > 0) lds_barrier();   // every wave has read the previous tile's partials
      }
      const unsigned long long pt2 = PH_NOW();
      if constexpr (DT == 8) write_partials8(rb, iacc);
      else if constexpr (DT == 9) write_partials9(rb, iacc);
      else write_partials(rb, accs);
      lds_barrier();   // (also publishes wave 0's LDS-DMA factors and its next-chunk word)
      const unsigned long long pt3 = PH_NOW();
      float sv[DPO];
      if constexpr (I8) read_partials8(rb, sv);
      else read_partials(rb, sv);
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 4)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (int e = 0; e < DPL; ++e) asm volatile("" : "+v"(sv[e]));
#endif
      const unsigned long long pt4 = PH_NOW();
      if (defer) {
#pragma unroll
        for (int e = 0; e < DPO; ++e) svd[e] = sv[e];
        bsd = base;
        tsd = ts;
      } else {
        epilogue(sv, base, ts);
      }
      if constexpr (SCR && FL == 2) {   // repair mode: the chunk's largest bound per query, at its last tile
        if (last_in_chunk) {
          const uint32_t m = group_max_u32<LPQ>(ord_of(umax));
          if (lane % LPQ == 0) a.cmax[(size_t)chunk * QS + qe] = m;
          umax = -INFINITY;
        }
      }
      const unsigned long long pt5 = PH_NOW();
      PH_ADD(2, pt2 - pt1);
      PH_ADD(3, pt3 - pt2);
      PH_ADD(4, pt4 - pt3);
      PH_ADD(5, pt5 - pt4);
      PH_ADD(6, 1);
      ph_t = pt5;
    }
    if (tcount == 0) SK_PROBE(2);
    if (MODE == 0 && tcount == 1) SK_PROBE(3);
    ++tcount;
    if constexpr (MODE == 1) break;
    ts = (ts + 1) & 3;
    if (!last_in_chunk) {
      ++ti;
      base += 32;
    } else {
      if (next_chunk >= C) break;
      chunk = next_chunk;
      ti = 0;
      cpar ^= 1;
      base = cbase(chunk) * 32;
    }
  }
  if (defer && bsd >= 0) epilogue(svd, bsd, tsd);   // the last tile's deferred epilogue
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 4)
  if (MODE == 0 && lane == 0)
    for (int i = 0; i < 8; ++i) phase_cycles[((size_t)blockIdx.x * 9 + w) * 8 + i] = ph[i];
#endif
  SK_PROBE(4);

  // ---- per query: merge its LPQ lane lists (KT rounds of an LPQ-lane max; keys are unique) -------------
  if constexpr (MODE == 0 && KT == 32 && QH == 1 && SCHED == 0 && !SCR) {
    if (a.all_keys) return;
    if (a.wide_k > 0) {
      // Large k: the query's top-wide_k of its LPQ lane lists. The lists go to LDS (the ring and the partial
      // blocks are free once every wave is past its last tile) and each round's winner advances its own head
      // from there. Floor: a lane whose list is full dropped only keys below its last; the workgroup drops
      // the keys left after wide_k rounds — the floor is the largest of those bounds (0: nothing dropped).
      static_assert((size_t)kQSlots * LPQ * (KT + 1) * 8 <= ring_bytes(RS) + red_bytes(RS, QH), "LDS lists");
      __syncthreads();
      const int li = lane % LPQ;
      uint64_t* mine = (uint64_t*)smem + (size_t)(qe * LPQ + li) * (KT + 1);
#pragma unroll
      for (int i = 0; i < KT; ++i) mine[i] = tk.v[i];
      const uint64_t lane_floor = tk.v[KT - 1];
      uint64_t head = tk.v[0];
      int hp = 0;
      uint64_t* dst = a.out + ((size_t)g * QS + qe) * a.wide_k;
#pragma unroll 1
      for (int rnd = 0; rnd < a.wide_k; ++rnd) {
        const uint64_t m = group_max_u64<LPQ>(head);
        if (m != 0 && head == m) {   // keys are unique: exactly one owner advances
          ++hp;
          head = hp < KT ? mine[hp] : 0;
        }
        if (li == 0) dst[rnd] = m;
      }
      const uint64_t fl = umax64(group_max_u64<LPQ>(lane_floor), group_max_u64<LPQ>(head));
      if (li == 0) a.floors[(size_t)g * QS + qe] = fl;
      return;
    }
  }
  if constexpr (MODE == 0) {
    // the screen's lists go query-major, [QS][grid][KT + 1] — KT keys, then the workgroup's floor (see KL): each
    // verify workgroup then reads its query's lists as one contiguous block (the other paths' merge_kernel reads
    // [grid][QS][KT])
    uint64_t* dst = a.out + (SCR ? ((size_t)qe * gridDim.x + blockIdx.x) * (KT + 1)
                                 : ((size_t)blockIdx.x * QS + qe) * KT);
    if constexpr (SCR) {   // before any pop: a full lane's last entry bounds every key it dropped
      const uint64_t fl = group_max_u64<LPQ>(tk.v[KL - 1]);
      if (lane % LPQ == 0) dst[KT] = KL < KT ? fl : 0;   // (KL = KT: the lists are the exact top-KT)
    }
#pragma unroll 1
    for (int rnd = 0; rnd < KT; ++rnd) {
      const uint64_t m = group_max_u64<LPQ>(tk.v[0]);
      if (m != 0 && tk.v[0] == m) tk.pop();
      if (lane % LPQ == 0) dst[rnd] = m;
    }
  } else if constexpr (MODE == 1) {
    // The wave that owns query slot vq (QH 1: queries 4w..4w+3) merges its lanes' lists into xk; its leader lane
    // checks completeness and writes the results. Every wave stays: a second, wide phase may follow.
    const bool owner = w == vql / 4;
    const bool leader = owner && qe == vql && lane % LPQ == 0;
    auto lane_merge = [&]() {
      if (owner) {
#pragma unroll 1
        for (int rnd = 0; rnd < KT; ++rnd) {
          const uint64_t m = group_max_u64<LPQ>(tk.v[0]);
          if (m != 0 && tk.v[0] == m) tk.pop();
          if (qe == vql && lane % LPQ == 0) xk[rnd] = m;
        }
      }
    };
    // The leader's verdict and the results (xk); an incomplete block raises the flag word (the host re-runs it).
    // Repair mode (a.rbits: the block's screen recorded per-chunk maxima of the bound): a slot the bound cannot prove
    // is not flagged — its exact k-th key ek bars the chunks to rescore, since every row that can be in its top-k has
    // bound >= its exact score >= the true k-th score >= ek's; they are marked in rbits (mark, every thread, below) and
    // the repair pass merges their exact keys with xk (written to out_keys). Returns whether the slot needs it.
    auto finish = [&](bool complete) -> bool {
      // the query inside the screen's range: max|q| < 2^15 (the f16 screens read q as f16; with it |q| <= 2^15 sqrt(d)
      // keeps every screen's bound arithmetic finite) and |q| finite (false for a NaN element, which max|q| drops)
      const bool range = qinfo[QS + vql] < 32768.0f && qinfo[vql] <= 3.0e38f && !a.force_incomplete;
      const bool repair = a.rbits != nullptr && !complete && range;
      complete = complete && range;
      if (!complete && !repair) {   // the first query slot to flag the block also counts it
        if (__hip_atomic_fetch_max(a.flag, (uint64_t)a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
            (uint64_t)a.seq)
          __hip_atomic_fetch_add(a.count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (repair && a.repair_count) __hip_atomic_fetch_add(a.repair_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (vq == 0) __hip_atomic_fetch_add(a.count + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // done
      if (a.out_keys)
        for (int i = 0; i < KT; ++i) a.out_keys[(size_t)vq * KT + i] = xk[i];
      if (a.out_scores)
        for (int i = 0; i < a.k_out; ++i) {
          const uint64_t key = xk[i];
          a.out_scores[(size_t)vq * a.k_out + i] = key ? float_of_ord((uint32_t)(key >> 32)) : -INFINITY;
          a.out_idx[(size_t)vq * a.k_out + i] = key ? (int64_t)(0xFFFFFFFFu - (uint32_t)key) : -1;
        }
      return repair;
    };
    // repair mode: every chunk whose largest bound for this slot reaches bar (an ord), marked for the repair pass
    auto mark = [&](uint32_t bar) {
      for (int64_t c = tid; c < a.nchunks; c += kThreads)
        if (a.cmax[(size_t)c * (a.cslots ? a.cslots : 32) + vq] >= bar) atomicOr(&a.rbits[c >> 5], 1u << (c & 31));
    };
    lane_merge();
    if (leader) {
      // Every key not rescored is at most the 32nd candidate's bound, or — left out of its list — at most that list's
      // KT-th key or its workgroup's floor, both within vtail (0, 0: fewer than 32 docs here and nothing dropped). With
      // 32 candidates from lists of KT < 32 the 32nd can lie below a list's KT-th (a cluster filling one list): vtail
      // must be checked, where the KT-th candidate bounded every list's KT-th by itself.
      const uint64_t ukt = umax64(akeys[31], *vtail);
      const uint64_t ek = xk[a.k_out - 1];         // the exact k-th key
      const bool complete = ukt == 0 || (ek != 0 && (uint32_t)(ek >> 32) > (uint32_t)(ukt >> 32));
      // Not proven: the wide phase can still prove it when the k-th largest bound of all lies above the largest
      // bound of any single list (vtail): every key left out of every list is below that.
      const uint64_t tb = *vtail;
      const uint32_t rbar = wide_bar(ek, tb);
      const bool wide = !complete && a.wide_verify && !a.force_incomplete && qinfo[QS + vql] < 32768.0f &&
                        qinfo[vql] <= 3.0e38f &&
                        ((uint32_t)(ek >> 32) > (uint32_t)(tb >> 32) ||
                         (uint32_t)(akeys[a.k_out - 1] >> 32) > (uint32_t)(tb >> 32));
      vstate[0] = wide ? 1 : 0;
      vstate[4] = (int)rbar;
      VDIAG(0, akeys[a.k_out - 1]);
      VDIAG(1, tb);
      VDIAG(2, ek);
      VDIAG(3, 0);
      VDIAG(4, 0);
      VDIAG(5, complete ? 0 : wide ? 1 : 2);
      VDIAG(6, complete);
      vstate[5] = !wide && finish(complete) ? 1 : 0;
      vstate[6] = (int)(uint32_t)(ek >> 32);   // (0 with fewer than k candidates: every chunk)
    }
    __syncthreads();
    if (vstate[5]) {
      mark((uint32_t)vstate[6]);
      return;
    }
    if (vstate[0] != 1) return;

    // ---- wide phase: R = every list entry whose bound reaches R's bar (wide_bar; every key left out of the lists is
    // at most vtail, below the bar), rescored with exactly the arithmetic of the first tile (same K split, MFMA order,
    // wave order, epilogue), 32 rows a tile; complete when the exact k-th key is above vtail. Lists are disjoint (each
    // workgroup its own rows). The first tile's rows — akeys, the 32 largest list entries when no list was folded
    // (nlists <= kThreads) — are not rescored (r6): their exact keys (the first tile's top-KT, xk) go back into the
    // owner lanes' lists, and R's other entries follow. The top-k of exact keys over that superset of R is the same.
    int* wl = (int*)(smem + kWideListOff);
    const uint32_t tb_ord = (uint32_t)(*vtail >> 32);
    const uint32_t rbar = (uint32_t)vstate[4];
    // list entries at or above done_from were the first tile's rows (keys are unique; akeys[31] = 0: every entry was)
    const uint64_t done_from = a.nlists <= kThreads ? (akeys[31] ? akeys[31] : 1ull) : ~0ull;
    if (tid == 0) vstate[1] = 0;
    __syncthreads();
    for (int l = tid; l < a.nlists; l += kThreads) {
      const uint64_t* src = a.vin + ((size_t)vq * a.nlists + l) * (KT + 1);
      int c = 0;
      while (c < KT && (uint32_t)(src[c] >> 32) >= rbar) ++c;   // a prefix of the sorted list
      int c0 = 0;
      while (c0 < c && src[c0] >= done_from) ++c0;              // ... whose first c0 entries were scored already
      if (c > c0) {
        const int pos = atomicAdd(&vstate[1], c - c0);
        for (int i = c0; i < c; ++i)
          if (pos + i - c0 < kWideCap) wl[pos + i - c0] = (int)((int64_t)(0xFFFFFFFFu - (uint32_t)src[i]) - idx_base);
      }
    }
    __syncthreads();
    const int nr = vstate[1];
    if (nr > kWideCap) {   // (cannot happen while lists x KT <= kWideCap; kept as a guard)
      if (leader) {
        vstate[5] = finish(false) ? 1 : 0;
        vstate[6] = (int)(uint32_t)(xk[a.k_out - 1] >> 32);
      }
      __syncthreads();
      if (vstate[5]) mark((uint32_t)vstate[6]);
      return;
    }
    tk.init();
    if (done_from != ~0ull && owner && qe == vql) {   // the first tile's exact top-KT, spread over the query's LPQ lanes
#pragma unroll
      for (int i = 0; i < KT; ++i)
        if (i % LPQ == lane % LPQ && xk[i] != 0) tk.insert(xk[i]);
    }
    const int ntiles = (nr + 31) / 32;
    for (int t = 0; t < ntiles; ++t) {
      // this lane's MFMA row (r) and its epilogue rows (er + e)
      const int ri = 32 * t + r;
      const char* src = corpus + (int64_t)wl[ri < nr ? ri : 0] * row_bytes + (size_t)w * KS;
#pragma unroll
      for (int j = 0; j < NS; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          vrow[j][i] = *(const f32x4*)(src + j * kSlabRowBytes + (vunit(i) << 4));
      int erow[DPL];
      float end[DPL];
#pragma unroll
      for (int e = 0; e < DPL; ++e) {
        const int ei = 32 * t + er + e;
        erow[e] = ei < nr ? wl[ei] : -1;
        end[e] = COS ? norms[erow[e] >= 0 ? erow[e] : 0] : 1.f;
      }
      f32x16 acc;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        if constexpr (DT == 1) {   // the bf16 pass's MFMAs: per K-step, hi then lo
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const bf16x8 ab = __builtin_bit_cast(bf16x8, vrow[j][tt]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, qfs[0].hi[j][tt], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, qfs[0].lo[j][tt], acc, 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) {
            const f32x4 v0 = vrow[j][2 * tt], v1 = vrow[j][2 * tt + 1];
            const float x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            bf16x8 b0, b1, b2;
            split3(x, b0, b1, b2);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[0].c0[j][tt], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[0].c1[j][tt], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[0].c0[j][tt], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[0].c1[j][tt], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[0].c2[j][tt], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, qfs[0].c0[j][tt], acc, 0, 0, 0);
          }
        }
      }
      // K-partials through LDS in the fixed wave order (the first tile used buffer 0: alternate from 1)
      float* rb = red + (size_t)((t + 1) & 1) * kWaves * QS * kRedStride;
#pragma unroll
      for (int a4 = 0; a4 < 4; ++a4) {
        const f32x4 v = {acc[4 * a4], acc[4 * a4 + 1], acc[4 * a4 + 2], acc[4 * a4 + 3]};
        *(f32x4*)(rb + (w * QS + r) * kRedRow + 4 * ((2 * a4 + h) ^ (r & 7))) = v;
      }
      lds_barrier();
      float sv[DPL];
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) {
        const float2 p = *(const float2*)(rb + (ww * QS + qe) * kRedRow + 4 * ((er >> 2) ^ (qe & 7)) + (er & 3));
        sv[0] = ww ? sv[0] + p.x : p.x;
        sv[1] = ww ? sv[1] + p.y : p.y;
      }
      // the same threshold as the first tile's epilogue (score ords; ties go on to the exact insert)
      uint32_t th = group_max_u32<LPQ>((uint32_t)(tk.last() >> 32));
      {
        const uint32_t tmin = group_min_u32<LPQ>((uint32_t)(tk.v[J - 1] >> 32));
        th = th > tmin ? th : tmin;
      }
      float thr = -INFINITY;
      if constexpr (COS) {
        if (th != 0) {
          const float tt = float_of_ord(th);
          thr = tt - fabsf(tt) * 0x1p-20f - 0x1p-100f;
        }
      }
#pragma unroll
      for (int e = 0; e < DPL; ++e) {
        const bool valid = qev && erow[e] >= 0;
        const float s = sv[e];
        if constexpr (COS) {
          const float den = cos_den(qn, end[e]);
          if (valid && s * __builtin_amdgcn_rcpf(den) >= thr) {
            float c = s / den;   // IEEE division, as the first tile and the full pass
            c = fminf(fmaxf(c, -1.0f), 1.0f);
            const uint64_t key = make_key(c, idx_base + (uint32_t)erow[e]);
            if ((uint32_t)(key >> 32) >= th) tk.insert(key);
          }
        } else {
          const uint64_t key = make_key(s, idx_base + (uint32_t)erow[e]);
          if (valid && (uint32_t)(key >> 32) >= th) tk.insert(key);
        }
      }
    }
    lane_merge();
    if (leader) {
      const uint64_t ek = xk[a.k_out - 1];
      const bool complete = tb_ord == 0 || (ek != 0 && (uint32_t)(ek >> 32) > tb_ord);
      VDIAG(3, ek);
      VDIAG(4, nr);
      VDIAG(6, complete);
      if (complete && a.wide_count) __hip_atomic_fetch_add(a.wide_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      vstate[5] = finish(complete) ? 1 : 0;
      vstate[6] = (int)(uint32_t)(ek >> 32);
    }
    __syncthreads();
    if (vstate[5]) mark((uint32_t)vstate[6]);
  }
  SK_PROBE(5);
}

template <int DT, int NS, int KT, bool COS, int RS, int QH, int MODE, int SCHED, int FL>
hipError_t launch_t(int grid, const SkArgs& a, hipStream_t s) {
  auto kern = sk_score_kernel<DT, NS, KT, COS, RS, QH, MODE, SCHED, FL>;
  static bool attr_set = false;   // the dynamic-LDS ceiling is a per-function attribute: set it once
  const size_t lds = sk_lds_bytes(DT, COS, RS, 32 * QH);
  if (!attr_set) {
    if (hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
      return e;
    attr_set = true;
  }
  RR_LAUNCH(kern, dim3(grid), dim3(kThreads + (SCHED ? 64 : 0)), lds, s, a);
  return hipGetLastError();
}

template <int DT, int NS, bool COS, int RS, int QH, int MODE, int SCHED, int FL>
hipError_t launch_kt(int kt, int grid, const SkArgs& a, hipStream_t s) {
  switch (kt) {
    case 4: return launch_t<DT, NS, 4, COS, RS, QH, MODE, SCHED, FL>(grid, a, s);
    case 8: return launch_t<DT, NS, 8, COS, RS, QH, MODE, SCHED, FL>(grid, a, s);
    case 16: return launch_t<DT, NS, 16, COS, RS, QH, MODE, SCHED, FL>(grid, a, s);
    // 64 slots x KT 32 spills (served as two 32-slot passes); the 9-wave form's register budget (168) does not
    // hold KT 32 lists
    case 32: if constexpr (QH == 1 && SCHED == 0) return launch_t<DT, NS, 32, COS, RS, QH, MODE, 0, FL>(grid, a, s);
             else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int DT, bool COS, int RS, int QH, int MODE, int SCHED, int FL>
hipError_t launch_ns(int ns, int kt, int grid, const SkArgs& a, hipStream_t s) {
  switch (ns) {
    case 1: return launch_kt<DT, 1, COS, RS, QH, MODE, SCHED, FL>(kt, grid, a, s);
    case 2: return launch_kt<DT, 2, COS, RS, QH, MODE, SCHED, FL>(kt, grid, a, s);
    case 3: if constexpr (DT != 1 && DT != 7 && DT != 8 && DT != 9) return launch_kt<DT, 3, COS, RS, QH, MODE, SCHED, FL>(kt, grid, a, s);
            else return hipErrorInvalidValue;
    case 4: if constexpr (DT != 1 && DT != 7 && DT != 8 && DT != 9) return launch_kt<DT, 4, COS, RS, QH, MODE, SCHED, FL>(kt, grid, a, s);
            else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int DT, int RS, int QH, int MODE = 0, int SCHED = 0, int FL = 0>
hipError_t launch_metric(int metric, int ns, int kt, int grid, const SkArgs& a, hipStream_t s) {
  return metric ? launch_ns<DT, true, RS, QH, MODE, SCHED, FL>(ns, kt, grid, a, s)
                : launch_ns<DT, false, RS, QH, MODE, SCHED, FL>(ns, kt, grid, a, s);
}

}  // namespace sk
}  // namespace rr
