// rr_sk.hip — split-K streaming kernel: similarity + top-k in one corpus pass, the corpus staged through
// LDS by non-temporal LDS-DMA (gfx950 / MI355X).
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
//   * Per tile the 8 K-partials are summed through LDS (double-buffered, one raw s_barrier per tile)
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
// The K order inside a wave's slice is a permutation applied identically to both operands.
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
#else
#define SK_PROBE(i) \
  do {              \
  } while (0)
#endif

constexpr int kSlabRowBytes = 128;                // contiguous bytes of one row per slab
constexpr int kSlabBytes = 32 * kSlabRowBytes;    // 4 KiB
constexpr int kRedStride = 36;                    // floats per (wave, query) block of 32 rows (+4 pad)
constexpr int kSegRows = 1024;                    // rows of per-doc factors held in LDS at a time

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

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
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

// x = b0 + b1 + r with |r| <= 2^-16 |x| (the first two splits of split3; r dropped). 6 VALU per pair.
__device__ __forceinline__ void split2(const float (&x)[8], bf16x8& b0, bf16x8& b1) {
  u32x4 p0, p1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i], b = x[2 * i + 1];
    p0[i] = cvt_pk_bf16(a, b);
    const float ra = a - __uint_as_float(p0[i] << 16), rb = b - __uint_as_float(p0[i] & 0xFFFF0000u);
    p1[i] = cvt_pk_bf16(ra, rb);
  }
  b0 = __builtin_bit_cast(bf16x8, p0);
  b1 = __builtin_bit_cast(bf16x8, p1);
}
__device__ __forceinline__ bf16x8 split1(const float (&x)[8]) {
  u32x4 p0;
#pragma unroll
  for (int i = 0; i < 4; ++i) p0[i] = cvt_pk_bf16(x[2 * i], x[2 * i + 1]);
  return __builtin_bit_cast(bf16x8, p0);
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
struct QFrag<4, NS> { bf16x8 c0[NS][2], c1[NS][2]; };
template <int NS>
struct QFrag<5, NS> { bf16x8 c0[NS][2], c1[NS][2]; };


// LDS byte offset (within a slot) of 16-byte column position cp of tile row r (swizzled image)
__device__ __forceinline__ int slab_off(int r, int cp) { return (r >> 3) * 1024 + (r & 7) * 128 + ((cp ^ (r & 7)) << 4); }

// QH = query halves: 32 * QH query slots per pass (64 for the batch-64 configs: one corpus pass serves
// them all; each A fragment then feeds the MFMAs of both halves).
template <int DT, int NS, int KT, bool COS, int RS, int QH>
__global__ __launch_bounds__(512, 1) void sk_score_kernel(const char* __restrict__ corpus,
                                                          const float* __restrict__ norms,
                                                          const float* __restrict__ rscale,
                                                          const float* __restrict__ queries, int64_t n, int d,
                                                          int b, uint32_t idx_base, uint64_t* __restrict__ out) {
  static_assert(RS == 2 || RS == 3, "ring depth 2 or 3 (the tail waits are written for these)");
  static_assert(QH == 1 || QH == 2, "32 or 64 query slots");
  constexpr int QS = 32 * QH;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  SK_PROBE(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  constexpr int EB = DT == 1 ? 2 : 4;                           // storage bytes per element
  const int row_bytes = d * EB;
  constexpr int KS = NS * kSlabRowBytes;                        // bytes of a row per wave
  const int p0 = w * (KS / 16);                                 // first 16-byte storage unit of the slice

  float* red = (float*)(smem + ring_bytes(RS));
  constexpr int SW = (COS ? 1 : 0) + (DT == 2 ? 1 : 0);          // per-doc floats in the segment
  float* seg = (float*)(smem + ring_bytes(RS) + red_bytes(RS, QH));
  float* qinfo = seg + kSegRows * (SW > 0 ? SW : 1);            // [QS] |q|, [QS] 2^-e (split), [QS] int e
  int* qexp = (int*)(qinfo + 2 * QS);

  // ---- this workgroup's rows ----------------------------------------------------------------------------
  const int64_t G = gridDim.x, g = blockIdx.x;
  const int64_t per = n / G, rem = n % G;
  const int64_t r0 = g * per + (g < rem ? g : rem);
  const int64_t r1 = r0 + per + (g < rem ? 1 : 0);
  const int64_t ntile = (r1 - r0 + 31) / 32;

  // LDS-DMA lane mapping: instruction i of a slab covers tile rows 8i + lane/8, 16-byte column
  // (lane % 8) ^ (lane / 8) of the slab — so the image holds column c of row r at c ^ (r & 7)
  const int rl = lane >> 3, cl = lane & 7;
  const unsigned ring_lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(smem + (size_t)w * RS * kSlabBytes));
  const char* ring = smem + (size_t)w * RS * kSlabBytes;
  const char* lane_src = corpus + (size_t)w * KS + ((cl ^ rl) << 4);

  auto issue = [&](int64_t tile, int j, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t row = r0 + tile * 32 + 8 * i + rl;
      row = row < r1 ? row : r1 - 1;                  // partial last tile: re-read a valid row
      glds16(lane_src + row * row_bytes + j * kSlabRowBytes, ring_lds + slot * kSlabBytes + i * 1024);
    }
  };

  const int64_t total = ntile * NS;                   // slabs this wave consumes
  // prologue: the first RS - 1 slabs (slab p = tile p / NS, column block p % NS, slot p)
#pragma unroll
  for (int p = 0; p < RS - 1; ++p)
    if (p < total) issue(p / NS, p % NS, p);
  // ---- query side: this wave's K-slice of every query as MFMA B operands, |q| and split exponents.
  // Runs while the prologue slabs above are in flight (their latency overlaps the query loads).
  QFrag<DT, NS> qfs[QH];
  auto build_frags = [&]() {
    // lane: query r (+ 32 per half), K half h
#pragma unroll
    for (int qh = 0; qh < QH; ++qh) {
      QFrag<DT, NS>& qf = qfs[qh];
      const int rq = r + 32 * qh;
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
            if constexpr (DT == 3) split3(x, qf.c0[j][t], qf.c1[j][t], qf.c2[j][t]);
            else split2(x, qf.c0[j][t], qf.c1[j][t]);
          }
        }
      }
    }
  };
  if constexpr (DT != 2) build_frags();
  // ---- per-query scalars: |q| (cosine, fp32 as cp.linalg.norm, retriever.py:602) and split exponents.
  // All loads of a group of 4 queries are issued before any is used (one L2/HBM latency per group, not
  // one per query); the sums are the same lane-strided fmaf chains + xor tree in the same order.
  if (COS || DT == 2) {
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
        float ss = 0.f, m = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (lane + 64 * c < nc) {
            const f32x4 x = v[qi][c];
            ss = fmaf(x.x, x.x, ss); ss = fmaf(x.y, x.y, ss); ss = fmaf(x.z, x.z, ss); ss = fmaf(x.w, x.w, ss);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
          }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          ss += __shfl_xor(ss, off, 64);
          m = fmaxf(m, __shfl_xor(m, off, 64));
        }
        int E = 0;
        if (m > 0.f) frexpf(m, &E);
        const int ex = m > 0.f ? 15 - E : 0;
        if (lane == 0) {
          qinfo[q] = sqrtf(ss);
          qinfo[QS + q] = ldexpf(1.0f, -ex);
          qexp[q] = ex;
        }
      }
    }
    __syncthreads();
  }

  if constexpr (DT == 2) build_frags();

  // epilogue lane mapping: wave w owns queries 4·QH·w + [0, 4·QH); LPQ lanes per query, each with DPL
  // consecutive tile rows (QH 1: 16 lanes x 2 rows, QH 2: 8 lanes x 4 rows)
  constexpr int LPQ = 16 / QH, DPL = 2 * QH;
  const int qe = 4 * QH * w + lane / LPQ, er = DPL * (lane % LPQ);
  const bool qev = qe < b;
  const float qn = COS ? qinfo[qe] : 0.f;
  const float qs = DT == 2 ? qinfo[QS + qe] : 1.f;

  TopK<KT> tk;
  tk.init();

  SK_PROBE(1);
  int64_t seg_lo = INT64_MIN / 2;
  int slot = 0;                                       // slot of the slab being consumed
  for (int64_t tile = 0; tile < ntile; ++tile) {
    f32x16 accs[QH];
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int i = 0; i < 16; ++i) accs[qh][i] = 0.f;
    static_for<0, NS>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      // keep RS - 1 slabs in flight: issue slab s + RS - 1 into the slot consumed last, then wait for
      // slab s (4 LDS-DMA instructions per slab; the younger ones stay outstanding)
      constexpr int jn = j + RS - 1;
      const int64_t tn = tile + jn / NS;
      int nslot = slot + RS - 1;
      nslot -= nslot >= RS ? RS : 0;
      if (tn < ntile) {
        issue(tn, jn % NS, nslot);
        wait_vm<4 * (RS - 1)>();
      } else if (RS == 3 && tile * NS + j + 2 == total) {   // tail: one younger slab still in flight
        wait_vm<4>();
      } else {
        wait_vm<0>();
      }
      const char* sl = ring + slot * kSlabBytes;
      if constexpr (DT == 0) {
        f32x4 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *(const f32x4*)(sl + slab_off(r, 4 * h + i));
#pragma unroll
        for (int m = 0; m < 16; ++m)
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[m >> 2][m & 3], qfs[qh].v[j][m], accs[qh], 0, 0, 0);
      } else if constexpr (DT == 1) {
        bf16x8 a[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) a[t] = *(const bf16x8*)(sl + slab_off(r, 2 * t + h));
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], qfs[qh].hi[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], qfs[qh].lo[j][t], accs[qh], 0, 0, 0);
        }
      } else if constexpr (DT == 2) {
        f16x8 ah[2], al[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          ah[t] = *(const f16x8*)(sl + slab_off(r, 4 * t + 2 * h));
          al[t] = *(const f16x8*)(sl + slab_off(r, 4 * t + 2 * h + 1));
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], qfs[qh].hi[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], qfs[qh].lo[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[t], qfs[qh].hi[j][t], accs[qh], 0, 0, 0);
        }
      } else {
        f32x4 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *(const f32x4*)(sl + slab_off(r, 4 * (i >> 1) + 2 * h + (i & 1)));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const float x[8] = {a[2 * t].x, a[2 * t].y, a[2 * t].z, a[2 * t].w,
                              a[2 * t + 1].x, a[2 * t + 1].y, a[2 * t + 1].z, a[2 * t + 1].w};
          if constexpr (DT == 4) {
            bf16x8 b0, b1;
            split2(x, b0, b1);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
          } else if constexpr (DT == 5) {
            const bf16x8 b0 = split1(x);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
            for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
          } else {
          bf16x8 b0, b1, b2;
          split3(x, b0, b1, b2);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b1, qfs[qh].c1[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b0, qfs[qh].c2[j][t], accs[qh], 0, 0, 0);
          for (int qh = 0; qh < QH; ++qh) accs[qh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b2, qfs[qh].c0[j][t], accs[qh], 0, 0, 0);
          }
        }
      }
      slot = slot + 1 == RS ? 0 : slot + 1;
    });

    // ---- sum the 8 K-partials of this tile (fixed order), then the metric epilogue --------------------
    float* rb = red + (red_bufs(RS, QH) == 2 ? (size_t)(tile & 1) * kWaves * QS * kRedStride : 0);
    if constexpr (red_bufs(RS, QH) == 1) {
      if (tile > 0) lds_barrier();   // every wave has read the previous tile's partials
    }
#pragma unroll
    for (int qh = 0; qh < QH; ++qh)
#pragma unroll
      for (int a4 = 0; a4 < 4; ++a4) {   // C/D map: acc[4a + i] = (doc 8a + 4h + i, query r)
        const f32x4 v = {accs[qh][4 * a4], accs[qh][4 * a4 + 1], accs[qh][4 * a4 + 2], accs[qh][4 * a4 + 3]};
        *(f32x4*)(rb + (w * QS + 32 * qh + r) * kRedStride + 8 * a4 + 4 * h) = v;
      }
    lds_barrier();
    const int64_t tb = r0 + tile * 32;
    if constexpr (SW > 0) {
      if (tb < seg_lo || tb + 32 > seg_lo + kSegRows) {   // workgroup-uniform: refill the per-doc factors
        seg_lo = tb;
        for (int i = tid; i < kSegRows; i += kThreads) {
          int64_t row = tb + i;
          row = row < r1 ? row : r1 - 1;
          if constexpr (COS && DT == 2) {
            seg[2 * i] = norms[row];
            seg[2 * i + 1] = rscale[row];
          } else if constexpr (COS) {
            seg[i] = norms[row];
          } else {
            seg[i] = rscale[row];
          }
        }
        lds_barrier();
      }
    }
    float sv[DPL];
#pragma unroll
    for (int e = 0; e < DPL; ++e) sv[e] = 0.f;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {   // fixed wave order: the same sums for any QH
      const float* src = rb + (ww * QS + qe) * kRedStride + er;
      if constexpr (DPL == 2) {
        const float2 p = *(const float2*)src;
        sv[0] += p.x;
        sv[1] += p.y;
      } else {
        const f32x4 p = *(const f32x4*)src;
#pragma unroll
        for (int e = 0; e < 4; ++e) sv[e] += p[e];
      }
    }
    // Cosine prefilter: a score whose estimate dot * rcp(den) (within a few ulp of the quotient) is below
    // the lane's current k-th score minus a 2^-20 relative margin cannot enter the list, so only the
    // few that pass pay the exact IEEE division (the list only grows inside the loop: the threshold
    // taken here is conservative).
    float thr = -INFINITY;
    if constexpr (COS) {
      const uint64_t last = tk.last();
      if (last != 0) {
        const float t = float_of_ord((uint32_t)(last >> 32));
        thr = t - fabsf(t) * 0x1p-20f - 0x1p-100f;
      }
    }
#pragma unroll
    for (int e = 0; e < DPL; ++e) {
      const int64_t row = tb + er + e;
      float s = sv[e];
      const int64_t li = row - seg_lo;
      if constexpr (DT == 2) s = s * (COS ? seg[2 * li + 1] : seg[li]) * qs;   // exact 2^e rescales
      const bool valid = qev && row < r1;
      if constexpr (COS) {
        // dot / (|q|*|d| + 1e-8), then clip to [-1, 1]   (retriever.py:605-609)
        const float nd = DT == 2 ? seg[2 * li] : seg[li];
        const float den = cos_den(qn, nd);
        if (valid && s * __builtin_amdgcn_rcpf(den) >= thr) {
          float c = s / den;   // IEEE division, as the reference's elementwise kernel
          c = fminf(fmaxf(c, -1.0f), 1.0f);
          const uint64_t key = make_key(c, idx_base + (uint32_t)row);
          if (key > tk.last()) tk.insert(key);
        }
      } else {
        const uint64_t key = make_key(s, idx_base + (uint32_t)row);
        if (valid && key > tk.last()) tk.insert(key);
      }
    }
    if (tile == 0) SK_PROBE(2);
    if (tile == 1) SK_PROBE(3);
  }
  SK_PROBE(4);

  // ---- per query: merge its LPQ lane lists (KT rounds of an LPQ-lane max; keys are unique) -------------
  uint64_t* dst = out + ((size_t)g * QS + qe) * KT;
#pragma unroll 1
  for (int rnd = 0; rnd < KT; ++rnd) {
    uint64_t m = tk.v[0];
#pragma unroll
    for (int off = LPQ / 2; off >= 1; off >>= 1) {
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)m, off, 64);
      const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(m >> 32), off, 64);
      m = umax64(m, ((uint64_t)hi << 32) | lo);
    }
    if (m != 0 && tk.v[0] == m) tk.pop();
    if (lane % LPQ == 0) dst[rnd] = m;
  }
  SK_PROBE(5);
}

template <int DT, int NS, int KT, bool COS, int RS, int QH>
hipError_t launch_t(int grid, const void* c, const float* nr, const float* rs, const float* q, int64_t n, int d,
                    int b, uint32_t base, uint64_t* out, hipStream_t s) {
  auto kern = sk_score_kernel<DT, NS, KT, COS, RS, QH>;
  const size_t lds = sk_lds_bytes(DT, COS, RS, 32 * QH);
  if (hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
    return e;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, s, (const char*)c, nr, rs, q, n, d, b, base, out);
  return hipGetLastError();
}

template <int DT, int NS, bool COS, int RS, int QH>
hipError_t launch_kt(int kt, int grid, const void* c, const float* nr, const float* rs, const float* q, int64_t n,
                     int d, int b, uint32_t base, uint64_t* out, hipStream_t s) {
  switch (kt) {
    case 4: return launch_t<DT, NS, 4, COS, RS, QH>(grid, c, nr, rs, q, n, d, b, base, out, s);
    case 8: return launch_t<DT, NS, 8, COS, RS, QH>(grid, c, nr, rs, q, n, d, b, base, out, s);
    case 16: return launch_t<DT, NS, 16, COS, RS, QH>(grid, c, nr, rs, q, n, d, b, base, out, s);
    case 32: if constexpr (QH == 1) return launch_t<DT, NS, 32, COS, RS, QH>(grid, c, nr, rs, q, n, d, b, base, out, s);
             else return hipErrorInvalidValue;   // 64 slots x KT 32 spills: served as two 32-slot passes
    default: return hipErrorInvalidValue;
  }
}

template <int DT, bool COS, int RS, int QH>
hipError_t launch_ns(int ns, int kt, int grid, const void* c, const float* nr, const float* rs, const float* q,
                     int64_t n, int d, int b, uint32_t base, uint64_t* out, hipStream_t s) {
  switch (ns) {
    case 1: return launch_kt<DT, 1, COS, RS, QH>(kt, grid, c, nr, rs, q, n, d, b, base, out, s);
    case 2: return launch_kt<DT, 2, COS, RS, QH>(kt, grid, c, nr, rs, q, n, d, b, base, out, s);
    case 3: if constexpr (DT != 1) return launch_kt<DT, 3, COS, RS, QH>(kt, grid, c, nr, rs, q, n, d, b, base, out, s);
            else return hipErrorInvalidValue;
    case 4: if constexpr (DT != 1) return launch_kt<DT, 4, COS, RS, QH>(kt, grid, c, nr, rs, q, n, d, b, base, out, s);
            else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int DT, int RS, int QH>
hipError_t launch_metric(int metric, int ns, int kt, int grid, const void* c, const float* nr, const float* rs,
                         const float* q, int64_t n, int d, int b, uint32_t base, uint64_t* out, hipStream_t s) {
  return metric ? launch_ns<DT, true, RS, QH>(ns, kt, grid, c, nr, rs, q, n, d, b, base, out, s)
                : launch_ns<DT, false, RS, QH>(ns, kt, grid, c, nr, rs, q, n, d, b, base, out, s);
}

}  // namespace sk

size_t sk_lds_bytes(int sdt, bool cos, int ring, int qslots) {
  const int sw = (cos ? 1 : 0) + (sdt == 2 ? 1 : 0);
  return sk::ring_bytes(ring) + sk::red_bytes(ring, qslots / 32) + (size_t)sk::kSegRows * (sw > 0 ? sw : 1) * 4 +
         3 * qslots * 4;
}

bool sk_supports_64(int sdt) { return sdt == KDT_BF16 || sdt == KDT_F32_SPLIT; }
int sk_slabs(int sdt, int d) {
  const int eb = sdt == 1 ? 2 : 4;
  const int ks = d * eb / kWaves;   // row bytes per wave
  if (d <= 0 || ks % sk::kSlabRowBytes != 0) return 0;
  const int ns = ks / sk::kSlabRowBytes;
  return (ns >= 1 && ns <= (sdt == 1 ? 2 : 4)) ? ns : 0;
}

hipError_t launch_sk(int sdt, int metric, int kt, int grid, const void* c, const float* nr, const float* rs,
                     const float* q, int64_t n, int d, int b, uint32_t base, uint64_t* cand, hipStream_t s, int ring,
                     int qslots) {
  const int ns = sk_slabs(sdt, d);
  if (!ns || b < 1 || b > qslots || n < 1 || (qslots != 32 && qslots != 64)) return hipErrorInvalidValue;
  if (ring == 0) ring = kSkRing;
  if (qslots == 64) {   // one corpus pass for up to 64 queries: bf16 and fp32-split storage, ring 2
    if (ring != 2) return hipErrorInvalidValue;
    switch (sdt) {
      case 1: return sk::launch_metric<1, 2, 2>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 2: return sk::launch_metric<2, 2, 2>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (ring == 2) {
    switch (sdt) {
      case 0: return sk::launch_metric<0, 2, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 1: return sk::launch_metric<1, 2, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 2: return sk::launch_metric<2, 2, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 3: return sk::launch_metric<3, 2, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
#ifdef RR_SK_SCREEN_PROBE
      case 4: return sk::launch_metric<4, 2, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 5: return sk::launch_metric<5, 2, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
#endif
      default: return hipErrorInvalidValue;
    }
  }
#ifdef RR_SK_RING3   // A/B builds only (tools/kbench.hip): measured no faster, see kSkRing
  if (ring == 3) {   // (the f32-MFMA form DT 0 is a kbench reference only: ring 2)
    switch (sdt) {
      case 1: return sk::launch_metric<1, 3, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 2: return sk::launch_metric<2, 3, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      case 3: return sk::launch_metric<3, 3, 1>(metric, ns, kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
      default: return hipErrorInvalidValue;
    }
  }
#endif
  return hipErrorInvalidValue;
}

}  // namespace rr
