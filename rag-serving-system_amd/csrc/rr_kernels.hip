// rr_kernels.hip — hand-written CDNA4 (gfx950, wave64) kernels for the batched dense-retrieval hot path.
//
// Reference behaviour being replaced (ngray0/RAG-Serving-System, rag_service/core/retriever.py):
//   CupyRetriever.distance_cosine  :594-611  (B,N) dot GEMM + norm passes + divide + clip, all materialised
//   CupyRetriever.batch_retrieve   :742-769  per-row argpartition + argsort loop (B launches)
//   SimpleRetriever.retrieve       :112-120  fp32 matvec + argpartition + descending argsort
// Here the whole thing is ONE streaming pass over the corpus: the (B x N) score matrix never reaches
// HBM. Each wave owns a 32-document tile, computes the 32(doc) x 32(query) score block with MFMA
// directly from 16-byte-per-lane corpus loads (the corpus is read exactly once, so it is not staged
// through LDS — only the queries, which every wave re-reads, live in LDS), applies the metric
// epilogue in registers and folds the 16 scores per lane into a per-lane sorted top-KT list.
// Lists are merged per workgroup in LDS; a second tiny kernel merges the per-workgroup lists.
//
// Score/index keys. A candidate is one uint64: high 32 bits = order-preserving image of the fp32
// score, low 32 bits = 0xFFFFFFFF - global_index. Unsigned key order == (score desc, index asc), the
// deterministic tie rule of this implementation (the reference's tie order is implementation
// defined: numpy introselect / CUB). Key 0 = empty slot.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "rr_internal.h"
#include "rr_device.h"

namespace rr {

// 16-byte corpus loads of one pipeline group (U loads at 32-byte stride).
// LM 0: plain loads, waits placed by hipcc.
// LM 1: inline-asm global_load_dwordx4, waits counted by hand (wait_group): hipcc does not see these
//       loads, so it cannot drain the prefetch queue with its own conservative vmcnt(0) at the loop
//       head. Any vector-memory op hipcc adds only makes a counted wait stricter, never looser.
// LM 2: as LM 1 with the non-temporal hint (`nt`): the corpus is streamed once per search.
// 16-byte unit offset of load u inside a group. Every row layout pairs the two 16-byte pieces a lane
// consumes back to back: split-f16 rows store a chunk's hi and lo pieces adjacent; fp32 and bf16 rows
// store chunks 2m and 2m+1 adjacent (pair_unit layout). A lane reads 32 contiguous bytes and the two
// lane halves 64 contiguous bytes of a row per load pair.
template <int DT>
__device__ __forceinline__ constexpr int group_off(int u) { return 4 * (u >> 1) + (u & 1); }

template <int LM, int DT, int U, int u>
__device__ __forceinline__ void load_one(u32x4 (&dst)[U], const u32x4* src) {
  constexpr int off = 16 * group_off<DT>(u);
  if constexpr (LM == 1)
    asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(dst[u]) : "v"(src), "i"(off));
  else
    asm volatile("global_load_dwordx4 %0, %1, off offset:%2 nt" : "=v"(dst[u]) : "v"(src), "i"(off));
  if constexpr (u + 1 < U) load_one<LM, DT, U, u + 1>(dst, src);
}

template <int LM, int U, int DT>
__device__ __forceinline__ void load_group(u32x4 (&dst)[U], const u32x4* src) {
  if constexpr (LM == 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) dst[u] = src[group_off<DT>(u)];
  } else {
    load_one<LM, DT, U, 0>(dst, src);
  }
}
// Before the MFMAs read dst[u] of the OLDEST group: `younger` groups of U loads were issued after it.
template <int LM, int U, int N>
__device__ __forceinline__ void wait_vm(u32x4& v) {
  if constexpr (LM != 0) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v) : "i"(N));
}
// Drain of the corpus pipeline: vmcnt(0) in the first statement, and every buffer named as a
// read-write operand of that or a later statement, so each in-flight destination stays allocated
// until the loads have landed.
#define RR_B8(s, o) "+v"(b[s][o + 0]), "+v"(b[s][o + 1]), "+v"(b[s][o + 2]), "+v"(b[s][o + 3]), \
                    "+v"(b[s][o + 4]), "+v"(b[s][o + 5]), "+v"(b[s][o + 6]), "+v"(b[s][o + 7])
#define RR_B4(s, o) "+v"(b[s][o + 0]), "+v"(b[s][o + 1]), "+v"(b[s][o + 2]), "+v"(b[s][o + 3])
#define RR_KEEP(s)                                                              \
  if constexpr (U == 4) asm volatile("" : RR_B4(s, 0));                         \
  else if constexpr (U == 8) asm volatile("" : RR_B8(s, 0));                    \
  else { asm volatile("" : RR_B8(s, 0)); asm volatile("" : RR_B8(s, 8)); }
template <int LM, int NB, int U>
__device__ __forceinline__ void drain_group_loads(u32x4 (&b)[NB][U]) {
  if constexpr (LM != 0) {
    static_assert((U == 4 || U == 8 || U == 16) && NB >= 2 && NB <= 4, "drain written for U 4/8/16, NB 2-4");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (the wait above is ordered before these by `volatile`; the operands keep every buffer live up
    // to here, i.e. past the wait)
    RR_KEEP(0)
    RR_KEEP(1)
    if constexpr (NB > 2) { RR_KEEP(2) }
    if constexpr (NB > 3) { RR_KEEP(3) }
  }
}
#undef RR_KEEP
#undef RR_B4
#undef RR_B8

// ------------------------------------------------------------------------------------------------
// fused similarity + top-k
// ------------------------------------------------------------------------------------------------
// DT: 0 = fp32 corpus  (chunk = 8 k-values: lane half h holds k = 8c + 4h + {0..3}; 4 x
//                       v_mfma_f32_32x32x2_f32, A = doc value, B = query value)
//     1 = bf16 corpus  (chunk = 16 k-values: lane half h holds k = 16c + 8h + {0..7}; 2 x
//                       v_mfma_f32_32x32x16_bf16 against the query's bf16 hi and lo parts)
// The k permutation inside a chunk is applied identically to both operands, so the dot is exact up
// to fp32 accumulation order (fp32 path: a plain fmaf chain per (doc, query)).
// LDS image: query operand for (chunk c, half h, query slot q) at 16-byte slot (2c + h) * 32 + q —
// one wave's ds_read_b128 covers 1 KiB contiguous: conflict-free.
// MODE 0: per-lane top-KT, merged per workgroup -> cand[blockIdx][32][KT]
// MODE 1: every key written to keys[q][doc] (the k > RR_FUSED_KMAX path)
template <int DT, int KT, bool COS, int MODE, int NB = 2, int LM = 0, int AS = 0, int DBG = 0, int U = kGroupChunks>
__global__ __launch_bounds__(kThreads) void fused_score_kernel(
    const u32x4* __restrict__ corpus, const float* __restrict__ norms, const float* __restrict__ rscale,
    const float* __restrict__ queries, int64_t n, int d, int b, uint32_t idx_base, uint64_t* __restrict__ out,
    int seg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 31, h = lane >> 5;

  const int d4 = d >> 2;                          // float4 per query row
  const int nchunk = DT == 0 ? (d >> 3) : (d >> 4);
  constexpr int CPG = DT == 2 ? U / 2 : U;         // chunks per pipeline group (split-f16: 2 loads/chunk)
  const int ngroup = nchunk / CPG;
  const size_t qimg_bytes = (size_t)nchunk * 2 * kQSlots * 16;  // per image
  float* qnorm = (float*)(smem + (DT == 0 ? qimg_bytes : 2 * qimg_bytes));
  float* qinv = qnorm + kQSlots;                    // split-f16: 2^-e of each query's scaling
  // Per-doc factors in LDS: each wave keeps a `seg`-row stretch of its rows (its own segment of the
  // region after the query image) of |d| (cosine) and, for split-f16, the row scale; refilled when its
  // tiles walk past the end (ordinary loads: hipcc drains the vector-memory queue once per refill).
  constexpr bool SEG = COS || DT == 2;
  constexpr int SW = (COS && DT == 2) ? 2 : 1;      // floats per row in the segment
  float* const wseg = qinv + kQSlots + wid * seg * SW;
  int64_t seg_lo = INT64_MIN / 2;

  // ---- stage the queries into LDS (zero rows for unused slots) --------------------------------
  if constexpr (DT == 0) {
    f32x4* Q4 = (f32x4*)smem;
    // query slot fastest across lanes: consecutive lanes write consecutive 16-byte LDS slots
    for (int e = tid; e < kQSlots * d4; e += kThreads) {
      const int q = e & (kQSlots - 1), c4 = e / kQSlots;   // c4 = 2 * chunk + half
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (q < b) v = ((const f32x4*)queries)[(size_t)q * d4 + c4];
      Q4[c4 * kQSlots + q] = v;
    }
  } else if constexpr (DT == 1) {
    bf16x8* Qhi = (bf16x8*)smem;
    bf16x8* Qlo = (bf16x8*)(smem + qimg_bytes);
    const int d8 = d >> 3;                       // 8-element groups per row = 2 * chunk + half
    for (int e = tid; e < kQSlots * d8; e += kThreads) {
      const int q = e & (kQSlots - 1), c8 = e / kQSlots;
      bf16x8 hi, lo;
      if (q < b) {
        const f32x4* src = (const f32x4*)(queries + (size_t)q * d + c8 * 8);
        const f32x4 x0 = src[0], x1 = src[1];
        const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const __bf16 bh = (__bf16)xs[j];
          hi[j] = bh;
          lo[j] = (__bf16)(xs[j] - (float)bh);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { hi[j] = (__bf16)0.f; lo[j] = (__bf16)0.f; }
      }
      Qhi[c8 * kQSlots + q] = hi;
      Qlo[c8 * kQSlots + q] = lo;
    }
  } else {
    // split-f16: q * 2^e = hi + lo to 2^-22 relative (22-bit significand), hi and lo f16, with 2^e putting the
    // row's max |q| in [2^14, 2^15) (every f16 part normal down to 2^-18 of the max)
    int* qexp = (int*)qinv;
    for (int q = wid; q < kQSlots; q += kWaves) {
      float m = 0.f;
      if (q < b)
        for (int c = lane; c < d4; c += 64) {
          const f32x4 v = ((const f32x4*)queries)[(size_t)q * d4 + c];
          m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      int E = 0;
      if (m > 0.f) frexpf(m, &E);
      if (lane == 0) qexp[q] = m > 0.f ? 15 - E : 0;
    }
    __syncthreads();
    f16x8* Qhi = (f16x8*)smem;
    f16x8* Qlo = (f16x8*)(smem + qimg_bytes);
    const int d8 = d >> 3;
    for (int e = tid; e < kQSlots * d8; e += kThreads) {
      const int q = e & (kQSlots - 1), c8 = e / kQSlots;
      f16x8 hi, lo;
      if (q < b) {
        const int ex = qexp[q];
        const f32x4* src = (const f32x4*)(queries + (size_t)q * d + c8 * 8);
        const f32x4 x0 = src[0], x1 = src[1];
        const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xsj = ldexpf(xs[j], ex);
          const _Float16 fh = (_Float16)xsj;
          hi[j] = fh;
          lo[j] = (_Float16)(xsj - (float)fh);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { hi[j] = (_Float16)0.f; lo[j] = (_Float16)0.f; }
      }
      Qhi[c8 * kQSlots + q] = hi;
      Qlo[c8 * kQSlots + q] = lo;
    }
    __syncthreads();                              // qexp read above; now overwrite with 2^-e
    if (tid < kQSlots) qinv[tid] = ldexpf(1.0f, -qexp[tid]);
  }
  if constexpr (COS) {
    // |q| in fp32 from the original fp32 queries (cp.linalg.norm(X, axis=1), retriever.py:602)
    for (int q = wid; q < kQSlots; q += kWaves) {
      float s = 0.f;
      if (q < b)
        for (int c = lane; c < d4; c += 64) {
          const f32x4 v = ((const f32x4*)queries)[(size_t)q * d4 + c];
          s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
        }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
      if (lane == 0) qnorm[q] = sqrtf(s);
    }
  }
  __syncthreads();

  const bool qvalid = r < b;
  const float qn = COS ? qnorm[r] : 0.f;
  const float qs = DT == 2 ? qinv[r] : 1.f;
  const int64_t rstride = DT == 1 ? (int64_t)(d >> 3) : (int64_t)(d >> 2);  // 16-byte units per corpus row

  TopK<KT> tk;
  tk.init();

  // Work split over the grid's waves. A wave walks 32-row tiles starting at row `base0`, `bstep`
  // rows apart, until `limit` (exclusive; also the bound for valid documents).
  //   AS 0: tiles dealt round-robin over all waves.
  //   AS 1: each wave owns one contiguous, balanced row range (equal bytes per wave, no tail of
  //         whole tiles); the last tile of a range is partial and its loads stay inside the range.
  const int64_t nwave = (int64_t)gridDim.x * kWaves;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wid;
  int64_t base0, limit, bstep;
  if constexpr (AS == 0) {
    base0 = gw * kTileDocs;
    limit = n;
    bstep = nwave * kTileDocs;
  } else {
    const int64_t per = n / nwave, rem = n % nwave;
    base0 = gw * per + (gw < rem ? gw : rem);
    limit = base0 + per + (gw < rem ? 1 : 0);
    bstep = kTileDocs;
  }
  if (base0 < limit) {
    auto rowp = [&](int64_t base) -> const u32x4* {
      int64_t row = base + r;
      row = row < limit ? row : limit - 1;
      return corpus + row * rstride + 2 * h;
    };
    auto compute = [&](u32x4 (&buf)[U], int g, f32x16& acc) {
      if constexpr (DT == 2) {
        static_for<0, U / 2>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          // oldest group in flight: (NB-1) younger groups of U loads were issued after it
          wait_vm<LM, U, (NB - 1) * U + (U - 1 - 2 * j)>(buf[2 * j]);
          wait_vm<LM, U, (NB - 1) * U + (U - 2 - 2 * j)>(buf[2 * j + 1]);
          const int slot = (2 * (g * CPG + j) + h) * kQSlots + r;
          if constexpr (DBG == 1) {
            acc[j & 15] += __builtin_bit_cast(f32x4, buf[2 * j]).x + __builtin_bit_cast(f32x4, buf[2 * j + 1]).x;
          } else {
            const f16x8 ah = __builtin_bit_cast(f16x8, buf[2 * j]);
            const f16x8 al = __builtin_bit_cast(f16x8, buf[2 * j + 1]);
            const f16x8 qh = ((const f16x8*)smem)[slot];
            const f16x8 ql = ((const f16x8*)(smem + qimg_bytes))[slot];
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, qh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ql, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, qh, acc, 0, 0, 0);
          }
        });
      } else {
        static_for<0, U>([&](auto uc) {
          constexpr int u = decltype(uc)::value;
          wait_vm<LM, U, (NB - 1) * U + (U - 1 - u)>(buf[u]);
          const int slot = (2 * (g * U + u) + h) * kQSlots + r;
          if constexpr (DBG == 1) {   // diagnostic: no MFMA, keep the loaded bytes live
            acc[u & 15] += __builtin_bit_cast(f32x4, buf[u]).x;
          } else if constexpr (DT == 0) {
            const f32x4 a = __builtin_bit_cast(f32x4, buf[u]);
            const f32x4 q = ((const f32x4*)smem)[slot];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, q.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, q.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, q.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, q.w, acc, 0, 0, 0);
          } else {
            const bf16x8 a = __builtin_bit_cast(bf16x8, buf[u]);
            const bf16x8 qh = ((const bf16x8*)smem)[slot];
            const bf16x8 ql = ((const bf16x8*)(smem + qimg_bytes))[slot];
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, ql, acc, 0, 0, 0);
          }
        });
      }
    };
    auto epilogue = [&](int64_t base, const f32x16& acc) {
      if constexpr (DBG == 2) {   // diagnostic: no epilogue, keep acc live
        asm volatile("" :: "v"(acc[0]), "v"(acc[15]));
        return;
      }
      if constexpr (SEG) {
        if (base < seg_lo || base + kTileDocs > seg_lo + seg) {   // wave-uniform
          seg_lo = base;
#pragma unroll 1
          for (int i = lane; i < seg; i += 64) {
            int64_t row = base + i;
            row = row < limit ? row : limit - 1;
            if constexpr (COS && DT == 2) {
              wseg[2 * i] = norms[row];
              wseg[2 * i + 1] = rscale[row];
            } else if constexpr (COS) {
              wseg[i] = norms[row];
            } else {
              wseg[i] = rscale[row];
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      // Cosine prefilter (top-k mode): a score whose quick estimate acc * rcp(den) (within 3 ulp of
      // the exact quotient) is below the lane's current k-th score minus a 2^-20 relative margin cannot
      // enter the list, so only the few that pass pay the exact IEEE division.
      float thr = -INFINITY;
      if constexpr (COS && MODE == 0) {
        const uint64_t last = tk.last();
        if (last != 0) {
          const float t = float_of_ord((uint32_t)(last >> 32));
          thr = t - fabsf(t) * 0x1p-20f - 0x1p-100f;
        }
      }
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int dl = (v & 3) + 8 * (v >> 2) + 4 * h;   // C/D row map of the 32x32 MFMA
        const int64_t doc = base + dl;
        float s = acc[v];
        if constexpr (DT == 2) {   // undo the two exact power-of-two scalings
          const float rs = COS ? wseg[2 * (doc - seg_lo) + 1] : wseg[doc - seg_lo];
          s = s * rs * qs;
        }
        const bool valid = qvalid && doc < limit;
        if constexpr (COS) {
          // dot / (|q|*|d| + 1e-8), then clip to [-1, 1]   (retriever.py:605-609)
          const float nd = DT == 2 ? wseg[2 * (doc - seg_lo)] : wseg[doc - seg_lo];
          const float den = cos_den(qn, nd);
          if constexpr (MODE == 0) {
            if (valid && s * __builtin_amdgcn_rcpf(den) >= thr) {
              float c = s / den;   // IEEE division, as the reference's elementwise kernel
              c = fminf(fmaxf(c, -1.0f), 1.0f);
              const uint64_t key = make_key(c, idx_base + (uint32_t)doc);
              if (key > tk.last()) tk.insert(key);
            }
          } else {
            float c = s / den;
            c = fminf(fmaxf(c, -1.0f), 1.0f);
            if (valid) out[(size_t)r * (size_t)n + (size_t)doc] = make_key(c, idx_base + (uint32_t)doc);
          }
        } else if constexpr (MODE == 0) {
          if (valid) {
            const uint64_t key = make_key(s, idx_base + (uint32_t)doc);
            if (key > tk.last()) tk.insert(key);
          }
        } else {
          if (valid) out[(size_t)r * (size_t)n + (size_t)doc] = make_key(s, idx_base + (uint32_t)doc);
        }
      }
    };

    // Software pipeline: the load cursor runs NB-1 groups (NB-1 x U x 16 B per lane) ahead of the
    // compute cursor; both walk this wave's tiles in order, so the prefetch crosses tile boundaries.
    // Past the wave's last tile the loads re-read a valid address instead of branching around them.
    u32x4 buf[NB][U];
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    int64_t cbase = base0, lrow = base0;
    int cg = 0, lg = 0;
    const u32x4* lptr = rowp(base0);
    const u32x4* const safe = lptr;
    auto issue = [&](u32x4 (&dst)[U]) {
      const u32x4* src = lrow < limit ? lptr + 2 * U * lg : safe;
      load_group<LM, U, DT>(dst, src);
      if (++lg == ngroup) {
        lg = 0;
        lrow += bstep;
        if (lrow < limit) lptr = rowp(lrow);
      }
    };
    auto consume = [&](u32x4 (&src)[U]) -> bool {
      compute(src, cg, acc);
      if (++cg < ngroup) return true;
      epilogue(cbase, acc);
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.f;
      cg = 0;
      cbase += bstep;
      if (cbase >= limit) return false;
      return true;
    };
#pragma unroll
    for (int s = 0; s < NB - 1; ++s) issue(buf[s]);
    for (;;) {
#pragma unroll
      for (int s = 0; s < NB; ++s) {
        issue(buf[(s + NB - 1) % NB]);
        // keep the prefetch ahead of the MFMAs (hipcc otherwise sinks the loads below them)
        __builtin_amdgcn_sched_barrier(0);
        if (!consume(buf[s])) goto wave_done;
      }
    }
  wave_done:
    // The loop leaves prefetches in flight (the dummy loads that keep the hand counts exact). Their
    // destination registers must stay allocated until they land, or hipcc may hand them to later code
    // and the late data would overwrite it: one drain that names every buffer as an operand.
    drain_group_loads<LM, NB, U>(buf);
  }

  if constexpr (MODE == 0) {
    // ---- workgroup merge: 16 lists (8 waves x 2 halves) per query slot -> top-KT -----------------
    __syncthreads();                      // query image no longer needed: reuse LDS
    uint64_t* L = (uint64_t*)smem;        // [32 q][16 lists][KT]
    const int list = wid * 2 + h;
#pragma unroll
    for (int i = 0; i < KT; ++i) L[((size_t)r * 16 + list) * KT + i] = tk.v[i];
    __syncthreads();
    constexpr int IT = (16 * KT) / 64;
    for (int q = wid; q < kQSlots; q += kWaves) {
      const uint64_t* src = L + (size_t)q * 16 * KT;
      uint64_t it[IT];
#pragma unroll
      for (int i = 0; i < IT; ++i) it[i] = src[lane + 64 * i];
      uint64_t* dst = out + ((size_t)blockIdx.x * kQSlots + q) * KT;
      for (int rnd = 0; rnd < KT; ++rnd) {
        uint64_t best = 0;
#pragma unroll
        for (int i = 0; i < IT; ++i) best = umax64(best, it[i]);
        best = wave_max_u64(best);
#pragma unroll
        for (int i = 0; i < IT; ++i) it[i] = (it[i] == best) ? 0 : it[i];
        if (lane == 0) dst[rnd] = best;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// merge of candidate lists: in [nlists][slots][in_kt] -> top-KT per query slot
// ------------------------------------------------------------------------------------------------
// One workgroup per query slot. Every input list is already sorted (descending), so: thread t takes
// list t (lists beyond 256 are folded in by insertion), each wave extracts its top-KT by KT rounds of a
// wave-wide max over the lanes' list heads (the winning lane advances its head from LDS; no barrier),
// and wave 0 merges the 4 per-wave winner lists the same way.
template <int KT>
__global__ __launch_bounds__(256) void merge_kernel(const uint64_t* __restrict__ in, int nlists, int slots, int b,
                                                    int k_out, uint64_t* __restrict__ out_keys,
                                                    float* __restrict__ out_scores,
                                                    int64_t* __restrict__ out_idx, int64_t stride,
                                                    uint64_t* __restrict__ flag_out,
                                                    uint64_t* __restrict__ clear_word) {
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (clear_word && q == 0 && tid == 0) *clear_word = 0;
  if (flag_out && q == 0 && tid < 64) {   // the shards' screened-search flags (one word after each list)
    uint64_t f = 0;
    for (int l = tid; l < nlists; l += 64) f = umax64(f, in[(size_t)l * stride + (size_t)slots * KT]);
    f = wave_max_u64(f);
    if (tid == 0 && f > *flag_out) *flag_out = f;   // the word only grows; stream order serialises writers
  }
  __shared__ uint64_t L[256][KT];
  __shared__ uint64_t W[4 * KT];
  TopK<KT> tk;
  if (tid < nlists) {
    const uint64_t* src = in + (size_t)tid * stride + (size_t)q * KT;
#pragma unroll
    for (int i = 0; i < KT; ++i) tk.v[i] = src[i];
  } else {
    tk.init();
  }
  for (int l = tid + 256; l < nlists; l += 256) {
    const uint64_t* src = in + (size_t)l * stride + (size_t)q * KT;
    for (int i = 0; i < KT; ++i) {
      const uint64_t key = src[i];
      if (key <= tk.last()) break;            // sorted input: nothing further can enter
      bool dup = false;                       // (the same key in two lists: a repaired row the verify also scored)
#pragma unroll
      for (int j = 0; j < KT; ++j) dup = dup || tk.v[j] == key;
      if (!dup) tk.insert(key);
    }
  }
#pragma unroll
  for (int i = 0; i < KT; ++i) L[tid][i] = tk.v[i];
  uint64_t head = tk.v[0];
  int p = 0;
  for (int rnd = 0; rnd < KT; ++rnd) {
    const uint64_t m = wave_max_u64(head);
    if (lane == 0) W[wid * KT + rnd] = m;
    if (m != 0 && head == m) {                 // every owner of m advances (a key in two lists is emitted once)
      ++p;
      head = p < KT ? L[tid][p] : 0;
    }
  }
  __syncthreads();
  if (wid != 0) return;
  uint64_t a = lane < 4 * KT ? W[lane] : 0, c = lane + 64 < 4 * KT ? W[lane + 64] : 0;
  uint64_t mine = 0;
  for (int rnd = 0; rnd < KT; ++rnd) {
    const uint64_t m = wave_max_u64(umax64(a, c));
    if (m != 0) {   // every copy of m leaves (equal keys from different lists: one result)
      if (a == m) a = 0;
      if (c == m) c = 0;
    }
    if (lane == rnd) mine = m;
  }
  if (lane < KT) {
    if (out_keys) out_keys[(size_t)q * KT + lane] = mine;
    if (out_scores && q < b && lane < k_out) {
      float sc = -INFINITY;
      int64_t ix = -1;
      if (mine != 0) {
        sc = float_of_ord((uint32_t)(mine >> 32));
        ix = (int64_t)(0xFFFFFFFFu - (uint32_t)mine);
      }
      out_scores[(size_t)q * k_out + lane] = sc;
      out_idx[(size_t)q * k_out + lane] = ix;
    }
  }
}

__global__ void decode_kernel(const uint64_t* __restrict__ keys, int64_t count, float* __restrict__ scores,
                              int64_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint64_t key = keys[i];
  float s = -INFINITY;
  int64_t ix = -1;
  if (key != 0) {
    s = float_of_ord((uint32_t)(key >> 32));
    ix = (int64_t)(0xFFFFFFFFu - (uint32_t)key);
  }
  scores[i] = s;
  idx[i] = ix;
}

// sorted [b][seg] -> out [32 slots][k] (rows >= b untouched)
__global__ void regroup_kernel(const uint64_t* __restrict__ in, int world, int k, uint64_t* __restrict__ out) {
  const int q = blockIdx.y;
  const int total = world * k;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int g = i / k, j = i - g * k;
    out[(size_t)q * total + i] = in[((size_t)g * kQSlots + q) * k + j];
  }
}

// ------------------------------------------------------------------------------------------------
// top-k selection for 32 < k <= 256 (rr_api.cpp large-k path): radix select, no sort of all keys
// ------------------------------------------------------------------------------------------------
// Workgroup (q, part): the keys of lists [part * lpp, (part + 1) * lpp) for query slot q (element (l, pos) at
// in[l * lstride + q * qstride + pos], pos < kin; order inside a list does not matter), PER per thread in
// registers. The k-th largest key is found one byte at a time from the top: a 256-bin histogram (LDS
// atomics) of the keys that match the bytes fixed so far, the bin holding the k-th, repeat — until the
// bin is taken whole. Keys are unique, so exactly min(k, nonzero) keys have a masked value >= the prefix;
// they are collected in LDS and (sort) ordered by a bitonic network. Stage 1 (parts > 1) leaves each
// part's top-k unsorted for stage 2 (parts = 1). Completeness (floors): every list l < nfloors dropped only
// keys below floors[l * fstride + q]; the result is exact when the largest floor is below the k-th key.
constexpr int kSelThreads = 1024;
constexpr int kSelMax = 256;   // k <= 256

template <int PER>
__global__ __launch_bounds__(kSelThreads) void select_kernel(const SelArgs a) {
  const int q = blockIdx.x, part = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int k = a.k;
  __shared__ int hist[256];
  __shared__ uint64_t sel[kSelMax];
  __shared__ int s_nz, s_cnt, s_digit, s_need, s_binc;
  __shared__ uint64_t s_floor;
  uint64_t* out_keys = a.out_keys ? a.out_keys + ((size_t)q * a.parts + part) * k : nullptr;
  if (a.xoff >= 0 && q == 0 && part == 0 && tid < 64) {   // the exchanged lists' flag words
    uint64_t f = 0;
    for (int l = tid; l < a.nlists; l += 64) f = umax64(f, a.in[(size_t)l * a.lstride + a.xoff]);
    f = wave_max_u64(f);
    if (tid == 0 && f > *a.flag) *a.flag = f;   // the word only grows; stream order serialises writers
  }
  if (q >= a.b) {   // padding slot: uniform exchange buffers
    if (out_keys)
      for (int i = tid; i < k; i += kSelThreads) out_keys[i] = 0;
    return;
  }
  const int lpp = (a.nlists + a.parts - 1) / a.parts;
  const int l0 = part * lpp, nl = max(0, min(a.nlists, l0 + lpp) - l0);
  const int total = nl * a.kin;
  uint64_t kv[PER];
  int nz = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = tid + kSelThreads * i;
    uint64_t key = 0;
    if (e < total) {
      const int l = e / a.kin, pos = e - l * a.kin;
      key = a.in[(size_t)(l0 + l) * a.lstride + (size_t)q * a.qstride + pos];
    }
    kv[i] = key;
    nz += key != 0;
  }
  if (tid == 0) {
    s_nz = 0;
    s_cnt = 0;
    s_floor = 0;
  }
  for (int i = tid; i < kSelMax; i += kSelThreads) sel[i] = 0;
  __syncthreads();
  if (nz) atomicAdd(&s_nz, nz);
  if (a.floors)
    for (int l = tid; l < a.nfloors; l += kSelThreads) {
      const uint64_t f = a.floors[(size_t)l * a.fstride + q];
      if (f) __hip_atomic_fetch_max(&s_floor, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  __syncthreads();
  const int m = min(k, s_nz);
  uint64_t prefix = 0, mask = 0;
  int need = m;
  for (int shift = 56; shift >= 0 && need > 0; shift -= 8) {
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (kv[i] != 0 && (kv[i] & mask) == prefix) atomicAdd(&hist[(int)(kv[i] >> shift) & 255], 1);
    __syncthreads();
    if (tid < 64) {   // lane L: bins 255 - 4L .. 252 - 4L, highest first
      int c[4], s4 = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - 4 * lane - j];
        s4 += c[j];
      }
      int incl = s4;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
      }
      int run = incl - s4;
      if (run < need && need <= incl) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (run < need && need <= run + c[j]) {
            s_digit = 255 - 4 * lane - j;
            s_need = need - run;
            s_binc = c[j];
          }
          run += c[j];
        }
      }
    }
    __syncthreads();
    prefix |= (uint64_t)s_digit << shift;
    mask |= (uint64_t)0xFF << shift;
    need = s_need;
    if (s_binc == need) break;   // the whole bin is in the top-k (uniform)
  }
  if (m > 0) {
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (kv[i] != 0 && (kv[i] & mask) >= prefix) sel[atomicAdd(&s_cnt, 1)] = kv[i];
  }
  __syncthreads();
  if (a.sort) {   // bitonic network over 256 entries (zeros sink), descending
    for (int size = 2; size <= kSelMax; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        if (tid < kSelMax / 2) {
          const int i = 2 * tid - (tid & (stride - 1)), j = i + stride;
          const bool desc = (i & size) == 0;
          const uint64_t x = sel[i], y = sel[j];
          if ((x < y) == desc) {
            sel[i] = y;
            sel[j] = x;
          }
        }
        __syncthreads();
      }
  }
  if (a.floors && tid == 0) {
    const uint64_t kth = s_nz >= k ? sel[k - 1] : 0;   // sorted: the k-th key
    const bool complete = (s_floor == 0 || s_floor < kth) && !a.force_incomplete;
    if (!complete)   // the first query slot to flag the block also counts it
      if (__hip_atomic_fetch_max(a.flag, (uint64_t)a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
          (uint64_t)a.seq && a.count)
        __hip_atomic_fetch_add(a.count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int i = tid; i < k; i += kSelThreads) {
    const uint64_t key = i < kSelMax ? sel[i] : 0;
    if (out_keys) out_keys[i] = key;
    if (a.out_scores) {
      a.out_scores[(size_t)q * k + i] = key ? float_of_ord((uint32_t)(key >> 32)) : -INFINITY;
      a.out_idx[(size_t)q * k + i] = key ? (int64_t)(0xFFFFFFFFu - (uint32_t)key) : -1;
    }
  }
  (void)lane;
}

// ------------------------------------------------------------------------------------------------
// corpus preparation
// ------------------------------------------------------------------------------------------------
// fp32 and bf16 row storage in 16-byte units: unit g = 2c + h of a row (chunk c, lane half h; fp32:
// elements 8c + 4h + {0..3}, bf16: 16c + 8h + {0..7}) lives at unit 4(c >> 1) + 2h + (c & 1), so the two
// chunks a lane loads back to back are adjacent (32 contiguous bytes per lane, 64 per row).
__device__ __forceinline__ int pair_unit(int g) {
  const int c = g >> 1, h = g & 1;
  return 4 * (c >> 1) + 2 * h + (c & 1);
}

// fp32 rows -> pair_unit layout (one 16-byte unit per thread), and back.
__global__ void permute_f32_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t nrows, int d,
                                   int inverse) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int upr = d >> 2;
  if (i >= nrows * upr) return;
  const int64_t row = i / upr;
  const int g = (int)(i - row * upr);
  if (inverse) out[i] = in[row * upr + pair_unit(g)];
  else out[row * upr + pair_unit(g)] = in[i];
}

template <bool F16>
__global__ void f32_to_16_kernel(const float* __restrict__ in, u32x4* __restrict__ out, int64_t nrows, int d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // one 8-element group
  const int gpr = d >> 3;
  if (i >= nrows * gpr) return;
  const int64_t row = i / gpr;
  const int g = (int)(i - row * gpr);
  const f32x4 x0 = ((const f32x4*)in)[2 * i], x1 = ((const f32x4*)in)[2 * i + 1];
  const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  if constexpr (F16) {
    f16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (_Float16)xs[j];
    out[row * gpr + pair_unit(g)] = __builtin_bit_cast(u32x4, v);
  } else {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)xs[j];
    out[row * gpr + pair_unit(g)] = __builtin_bit_cast(u32x4, v);
  }
}

__global__ void bf16_to_f32_kernel(const u32x4* __restrict__ in, float* __restrict__ out, int64_t nrows, int d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int gpr = d >> 3;
  if (i >= nrows * gpr) return;
  const int64_t row = i / gpr;
  const int g = (int)(i - row * gpr);
  const bf16x8 v = __builtin_bit_cast(bf16x8, in[row * gpr + pair_unit(g)]);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[i * 8 + j] = (float)v[j];
}

// fp32 rows -> split-f16 storage: per 8-element group g of a row, 16 bytes of hi then 16 bytes of lo
// (byte offset 32 g), where x * 2^e = hi + lo to 2^-22 relative and 2^e puts the row's max |x| in
// [2^14, 2^15). Also |row|_2 of the ORIGINAL fp32 values and rscale = 2^-e. One wave per row.
__global__ __launch_bounds__(256) void split_f32_kernel(const float* __restrict__ in, int64_t n, int d,
                                                        u32x4* __restrict__ out, float* __restrict__ norms,
                                                        float* __restrict__ rscale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const f32x4* src = (const f32x4*)(in + row * d);
  float m = 0.f, ss = 0.f;
  for (int c = lane; c < (d >> 2); c += 64) {
    const f32x4 v = src[c];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    ss = fmaf(v.x, v.x, ss); ss = fmaf(v.y, v.y, ss); ss = fmaf(v.z, v.z, ss); ss = fmaf(v.w, v.w, ss);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    m = fmaxf(m, __shfl_xor(m, off, 64));
    ss += __shfl_xor(ss, off, 64);
  }
  int E = 0;
  if (m > 0.f) frexpf(m, &E);
  const int ex = m > 0.f ? 15 - E : 0;
  if (lane == 0) {
    norms[row] = sqrtf(ss);
    rscale[row] = ldexpf(1.0f, -ex);
  }
  u32x4* dst = out + row * (d >> 2);
  for (int g = lane; g < (d >> 3); g += 64) {
    const f32x4 x0 = src[2 * g], x1 = src[2 * g + 1];
    const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    f16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xsj = ldexpf(xs[j], ex);
      const _Float16 fh = (_Float16)xsj;
      hi[j] = fh;
      lo[j] = (_Float16)(xsj - (float)fh);
    }
    dst[2 * g] = __builtin_bit_cast(u32x4, hi);
    dst[2 * g + 1] = __builtin_bit_cast(u32x4, lo);
  }
}

// fp32 rows (natural element order) -> the int8 screen copy (rr_sk.hip DT 8), one wave per row:
//   sx = max|x| / 127 (0 for a zero row), x8 = clamp(rint(t), -127, 127) with t = x / sx — any x8 is valid, the bound
//   uses e — and e >= |x - sx x8|_2 (real arithmetic), computed in the scale's units so that no square underflows:
//   t - x8 is exact, and x / sx - t is within 2^-24 |t| (IEEE division; 2^-149 if t is subnormal), so
//   |x - sx x8|_2 <= sx |t - x8|_2 + 2^-24 (1 + 2^-23) |x|_2 + sx sqrt(d) 2^-149, |x|_2 <= sqrt(d) max|x|. The sum of
//   squares of t - x8 (in [-1/2, 1/2]: <= d / 4 + 6 roundings a chain, squares below 2^-126 add <= 2^-116 in all) and
//   the sqrt and product within 2^-14, covered by the 2^-12 relative bump; 2^-22 sqrt(d) max|x| covers the division
//   term 4x over, and 2^-140 what the products round away when max|x| is itself near fp32's underflow.
// bf16: quantise the rows' bf16 roundings (RNE) — the values bf16 storage holds — instead of the fp32 values.
__device__ __forceinline__ f32x4 bf16_round4(f32x4 v) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (float)(__bf16)v[j];
  return v;
}
__global__ __launch_bounds__(256) void f32_to_i8_kernel(const float* __restrict__ in, int64_t n, int d,
                                                        uint32_t* __restrict__ out, float* __restrict__ sx,
                                                        float* __restrict__ e8, int bf16) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const f32x4* src = (const f32x4*)(in + row * d);
  float m = 0.f;
  for (int c = lane; c < (d >> 2); c += 64) {
    const f32x4 v = bf16 ? bf16_round4(src[c]) : src[c];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  const float s = m > 0.f ? m / 127.0f : 0.f;
  float ss = 0.f;
  uint32_t* dst = out + row * (d >> 2);
  for (int c = lane; c < (d >> 2); c += 64) {
    const f32x4 v = bf16 ? bf16_round4(src[c]) : src[c];
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = s > 0.f ? v[j] / s : 0.f;
      const float q = fminf(fmaxf(rintf(t), -127.0f), 127.0f);
      const float r = t - q;   // exact
      ss = fmaf(r, r, ss);
      packed |= ((uint32_t)(int)q & 0xFFu) << (8 * j);
    }
    dst[c] = packed;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if (lane == 0) {
    sx[row] = s;
    e8[row] = fmaf(s * sqrtf(ss), 1.0f + 0x1p-12f, fmaf(m, sqrtf((float)d) * 0x1p-22f, 0x1p-140f));
  }
}

// The int8 screens' query pieces of a staged batch: one 64-lane workgroup per query row (rr_device.h q8_stage_row) over
// every row a block reads (the rows past b zeroed: any block's padding slots read zeros), where the batch is staged.
__global__ __launch_bounds__(64) void q8_stage_kernel(const float* __restrict__ q, int b, int d, int8_t* __restrict__ q8,
                                                      int qc, float* __restrict__ q8s, float* __restrict__ qcopy) {
  q8_stage_row(q, b, d, q8, q8 + (size_t)qc * d, q8s, qc, qcopy, (int)blockIdx.x, (int)threadIdx.x);
}

// Repair pass (rr_sk.hip "Repair"): the set bits of `bits` -> their indices in ascending order (list) and their count,
// one 1024-thread workgroup: per pass of 1024 words, a block-wide scan of the words' popcounts gives each thread its
// output position.
__global__ __launch_bounds__(1024) void compact_bits_kernel(const uint32_t* __restrict__ bits, int words,
                                                            int* __restrict__ list, int* __restrict__ count) {
  __shared__ int pre[1024];
  const int t = threadIdx.x;
  int total = 0;
  for (int w0 = 0; w0 < words; w0 += 1024) {
    const int w = w0 + t;
    const uint32_t v = w < words ? bits[w] : 0u;
    const int c = __popc(v);
    pre[t] = c;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {   // inclusive scan
      const int x = t >= off ? pre[t - off] : 0;
      __syncthreads();
      pre[t] += x;
      __syncthreads();
    }
    int pos = total + pre[t] - c;
    for (uint32_t x = v; x; x &= x - 1) list[pos++] = (w << 5) + (__ffs(x) - 1);
    total += pre[1023];
    __syncthreads();
  }
  if (t == 0) *count = total;
}

__global__ void unsplit_f32_kernel(const u32x4* __restrict__ in, const float* __restrict__ rscale, int64_t n,
                                   int d, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // one 8-element group
  if (i >= n * (d >> 3)) return;
  const int64_t row = i / (d >> 3);
  const f16x8 hi = __builtin_bit_cast(f16x8, in[2 * i]);
  const f16x8 lo = __builtin_bit_cast(f16x8, in[2 * i + 1]);
  const float rs = rscale[row];
#pragma unroll
  for (int j = 0; j < 8; ++j) out[i * 8 + j] = ((float)hi[j] + (float)lo[j]) * rs;
}

// One wave per row: |row|_2 in fp32 (the reference recomputes cp.linalg.norm(Y, axis=1) every call,
// retriever.py:603; here it is computed once at load).
template <int DT>
__global__ __launch_bounds__(256) void row_norms_kernel(const void* __restrict__ corpus, int64_t n, int d,
                                                         float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  float s = 0.f;
  if constexpr (DT == 0) {
    const f32x4* p = (const f32x4*)((const float*)corpus + row * d);
    for (int c = lane; c < (d >> 2); c += 64) {
      const f32x4 v = p[c];
      s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
    }
  } else {
    const __bf16* p = (const __bf16*)corpus + row * d;
    for (int c = lane; c < d; c += 64) { const float v = (float)p[c]; s = fmaf(v, v, s); }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) norms[row] = sqrtf(s);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// kind 0: ((h mod 255) - 127) / 128 ; kind 1: Irwin-Hall(4) * sqrt(3) (unnormalised)
__global__ void synth_kernel(int kind, uint64_t seed, int64_t row_begin, int64_t n_rows, int d,
                             float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows * (int64_t)d) return;
  const uint64_t gi = (uint64_t)(row_begin * (int64_t)d) + (uint64_t)i;
  const uint64_t z = splitmix64(seed, gi);
  float v;
  if (kind == 0) {
    v = (float)((int)(z % 255ull) - 127) * 0.0078125f;
  } else {
    const float u = (float)(z & 0xFFFF) + (float)((z >> 16) & 0xFFFF) + (float)((z >> 32) & 0xFFFF) +
                    (float)(z >> 48);
    v = (u * (1.0f / 65536.0f) - 2.0f) * 1.7320508f;
  }
  out[i] = v;
}

__global__ __launch_bounds__(256) void normalize_rows_kernel(float* __restrict__ x, int64_t n, int d) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  float* p = x + row * d;
  float s = 0.f;
  for (int c = lane; c < d; c += 64) s = fmaf(p[c], p[c], s);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  const float inv = 1.0f / sqrtf(s);
  for (int c = lane; c < d; c += 64) p[c] = p[c] * inv;
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
int fused_kt(int k) {
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 16) return 16;
  if (k <= 32) return 32;
  return 0;
}

// LDS of the query image (fp32: one 4-byte image; bf16 / split-f16: hi + lo 2-byte images) plus the
// per-query scalars, or of the end-of-kernel merge if larger.
size_t fused_lds_bytes(int d, int kt, int kdt) {
  (void)kdt;
  const size_t qimg = (size_t)kQSlots * d * 4 + 2 * kQSlots * sizeof(float);
  const size_t merge = (size_t)kQSlots * 16 * (kt > 0 ? kt : 1) * 8;
  return qimg > merge ? qimg : merge;
}

// Rows of each wave's per-doc segment (|d| and/or the split-f16 row scale, `sw` floats per row): what
// fits next to the query image, a multiple of 32, capped at 2048 rows (64 tiles between refills).
static int segment_rows(int d, int sw) {
  const size_t base = (size_t)kQSlots * d * 4 + 2 * kQSlots * sizeof(float);
  const int64_t rows = (int64_t)((160 * 1024 - base) / (4 * sw) / kWaves) / kTileDocs * kTileDocs;
  return (int)(rows > 2048 ? 2048 : rows);
}

// Pipeline depth and load form of the shipped kernel (chosen by tools/kbench.hip A/B runs on MI355X).
constexpr int kPipeNB = 2;
constexpr int kLoadMode = 1;
constexpr int kAssign = 1;

template <int DT, int KT, bool COS, int MODE, int NB = kPipeNB, int LM = kLoadMode, int AS = kAssign, int DBG = 0,
          int U = (KT >= 32 ? kGroupChunks / 2 : kGroupChunks)>   // KT 32: fewer buffers, no spills
hipError_t launch_fused_t(int grid, const void* corpus, const float* norms, const float* rscale,
                          const float* queries, int64_t n, int d, int b, uint32_t idx_base, uint64_t* out,
                          hipStream_t s) {
  constexpr int sw = (COS && DT == 2) ? 2 : 1;
  const int seg = (COS || DT == 2) ? segment_rows(d, sw) : 0;
  size_t lds = fused_lds_bytes(d, MODE == 0 ? KT : 1, DT);
  const size_t lds_seg = (size_t)kQSlots * d * 4 + 2 * kQSlots * sizeof(float) + (size_t)seg * sw * kWaves * 4;
  if (lds_seg > lds) lds = lds_seg;
  auto kern = fused_score_kernel<DT, KT, COS, MODE, NB, LM, AS, DBG, U>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, s, (const u32x4*)corpus, norms, rscale, queries, n,
                     d, b, idx_base, out, seg);
  return hipGetLastError();
}

template <int DT, bool COS>
static hipError_t launch_fused_k(int kt, int grid, const void* c, const float* nr, const float* rs,
                                 const float* q, int64_t n, int d, int b, uint32_t base, uint64_t* o,
                                 hipStream_t s) {
  switch (kt) {
    case 4: return launch_fused_t<DT, 4, COS, 0>(grid, c, nr, rs, q, n, d, b, base, o, s);
    case 8: return launch_fused_t<DT, 8, COS, 0>(grid, c, nr, rs, q, n, d, b, base, o, s);
    case 16: return launch_fused_t<DT, 16, COS, 0>(grid, c, nr, rs, q, n, d, b, base, o, s);
    case 32: return launch_fused_t<DT, 32, COS, 0>(grid, c, nr, rs, q, n, d, b, base, o, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fused(int kdt, int metric, int kt, int grid, const void* c, const float* nr, const float* rs,
                        const float* q, int64_t n, int d, int b, uint32_t base, uint64_t* cand, hipStream_t s) {
  switch (kdt) {
    case KDT_F32_MFMA:
      return metric ? launch_fused_k<0, true>(kt, grid, c, nr, rs, q, n, d, b, base, cand, s)
                    : launch_fused_k<0, false>(kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
    case KDT_BF16:
      return metric ? launch_fused_k<1, true>(kt, grid, c, nr, rs, q, n, d, b, base, cand, s)
                    : launch_fused_k<1, false>(kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
    case KDT_F32_SPLIT:
      return metric ? launch_fused_k<2, true>(kt, grid, c, nr, rs, q, n, d, b, base, cand, s)
                    : launch_fused_k<2, false>(kt, grid, c, nr, rs, q, n, d, b, base, cand, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_full_keys(int kdt, int metric, int grid, const void* c, const float* nr, const float* rs,
                            const float* q, int64_t n, int d, int b, uint32_t base, uint64_t* keys, hipStream_t s) {
  switch (kdt) {
    case KDT_F32_MFMA:
      return metric ? launch_fused_t<0, 4, true, 1>(grid, c, nr, rs, q, n, d, b, base, keys, s)
                    : launch_fused_t<0, 4, false, 1>(grid, c, nr, rs, q, n, d, b, base, keys, s);
    case KDT_BF16:
      return metric ? launch_fused_t<1, 4, true, 1>(grid, c, nr, rs, q, n, d, b, base, keys, s)
                    : launch_fused_t<1, 4, false, 1>(grid, c, nr, rs, q, n, d, b, base, keys, s);
    case KDT_F32_SPLIT:
      return metric ? launch_fused_t<2, 4, true, 1>(grid, c, nr, rs, q, n, d, b, base, keys, s)
                    : launch_fused_t<2, 4, false, 1>(grid, c, nr, rs, q, n, d, b, base, keys, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_merge(int kt, const uint64_t* in, int nlists, int in_kt, int b, int k_out, uint64_t* out_keys,
                        float* out_scores, int64_t* out_idx, hipStream_t s, int slots, int64_t list_stride,
                        uint64_t* flag_out, uint64_t* clear_word) {
  if (list_stride == 0) list_stride = (int64_t)slots * in_kt;
  if (in_kt != kt) return hipErrorInvalidValue;   // lists are always produced at the kernel's KT
  // Rows >= b of out_keys are still produced (from the zero-filled slots) so the buffer is uniform.
  if (b > slots) return hipErrorInvalidValue;
  const int grid = out_keys ? slots : b;
  switch (kt) {
    case 4: RR_LAUNCH(merge_kernel<4>, dim3(grid), dim3(256), 0, s, in, nlists, slots, b, k_out, out_keys, out_scores, out_idx, list_stride, flag_out, clear_word); break;
    case 8: RR_LAUNCH(merge_kernel<8>, dim3(grid), dim3(256), 0, s, in, nlists, slots, b, k_out, out_keys, out_scores, out_idx, list_stride, flag_out, clear_word); break;
    case 16: RR_LAUNCH(merge_kernel<16>, dim3(grid), dim3(256), 0, s, in, nlists, slots, b, k_out, out_keys, out_scores, out_idx, list_stride, flag_out, clear_word); break;
    case 32: RR_LAUNCH(merge_kernel<32>, dim3(grid), dim3(256), 0, s, in, nlists, slots, b, k_out, out_keys, out_scores, out_idx, list_stride, flag_out, clear_word); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_compact_bits(const uint32_t* rbits, int words, int* list, int* count, hipStream_t s) {
  hipLaunchKernelGGL(compact_bits_kernel, dim3(1), dim3(1024), 0, s, rbits, words, list, count);
  return hipGetLastError();
}

hipError_t launch_regroup(const uint64_t* gathered, int world, int k, int b, uint64_t* out, hipStream_t s) {
  const int64_t seg = (int64_t)world * k;
  hipLaunchKernelGGL(regroup_kernel, dim3((unsigned)((seg + 255) / 256), b), dim3(256), 0, s, gathered, world, k, out);
  return hipGetLastError();
}

hipError_t launch_select(const SelArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kSelMax || a.parts < 1 || a.nlists < 1 || a.kin < 1 || a.b < 1 || a.b > kQSlots)
    return hipErrorInvalidValue;
  const int64_t per_part = (int64_t)((a.nlists + a.parts - 1) / a.parts) * a.kin;
  const dim3 grid(kQSlots, a.parts);
  if (per_part <= 1 * kSelThreads) hipLaunchKernelGGL(select_kernel<1>, grid, dim3(kSelThreads), 0, s, a);
  else if (per_part <= 2 * kSelThreads) hipLaunchKernelGGL(select_kernel<2>, grid, dim3(kSelThreads), 0, s, a);
  else if (per_part <= 4 * kSelThreads) hipLaunchKernelGGL(select_kernel<4>, grid, dim3(kSelThreads), 0, s, a);
  else if (per_part <= 8 * kSelThreads) hipLaunchKernelGGL(select_kernel<8>, grid, dim3(kSelThreads), 0, s, a);
  else if (per_part <= 16 * kSelThreads) hipLaunchKernelGGL(select_kernel<16>, grid, dim3(kSelThreads), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_decode(const uint64_t* keys, int b, int k, float* scores, int64_t* idx, hipStream_t s) {
  const int64_t count = (int64_t)b * k;
  hipLaunchKernelGGL(decode_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, keys, count, scores, idx);
  return hipGetLastError();
}

hipError_t launch_permute_f32(const float* in, float* out, int64_t nrows, int d, int inverse, hipStream_t s) {
  const int64_t units = nrows * (d >> 2);
  hipLaunchKernelGGL(permute_f32_kernel, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, s, (const u32x4*)in,
                     (u32x4*)out, nrows, d, inverse);
  return hipGetLastError();
}

hipError_t launch_f32_to_bf16(const float* in, uint16_t* out, int64_t nrows, int d, hipStream_t s) {
  const int64_t groups = nrows * (d >> 3);
  hipLaunchKernelGGL(f32_to_16_kernel<false>, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, in,
                     (u32x4*)out, nrows, d);
  return hipGetLastError();
}

hipError_t launch_f32_to_f16(const float* in, uint16_t* out, int64_t nrows, int d, hipStream_t s) {
  const int64_t groups = nrows * (d >> 3);
  hipLaunchKernelGGL(f32_to_16_kernel<true>, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, in,
                     (u32x4*)out, nrows, d);
  return hipGetLastError();
}

namespace {
thread_local LaunchEvents g_launch_events;
}  // namespace
void set_launch_events(hipEvent_t start, hipEvent_t stop) { g_launch_events = LaunchEvents{start, stop}; }
LaunchEvents take_launch_events() {
  const LaunchEvents e = g_launch_events;
  g_launch_events = LaunchEvents{};
  return e;
}

hipError_t launch_f32_to_i8(const float* in, int64_t nrows, int d, int8_t* out, float* sx, float* e, hipStream_t s,
                            int bf16) {
  if (nrows < 1 || d % 4 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(f32_to_i8_kernel, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, s, in, nrows, d,
                     (uint32_t*)out, sx, e, bf16);
  return hipGetLastError();
}

// Every kernel unit's code object on the current device (rr_create): deferred loading otherwise loads a unit at the first
// launch of one of its kernels — inside the first search (~8 ms for a split-K unit, profiles/r06/preload/).
hipError_t preload_kernels() {
  hipFuncAttributes fa;
  if (hipError_t e = hipFuncGetAttributes(&fa, (const void*)q8_stage_kernel)) return e;
  if (hipError_t e = preload_topk()) return e;
  return preload_sk();
}

hipError_t launch_q8_stage(const float* q, int b, int d, int8_t* q8, int qc, float* q8s, float* qcopy, hipStream_t s) {
  // the rows any block reads: 32-slot blocks for b <= 32, else round_up(b, 64) (64-slot blocks, or 32-slot pairs)
  const int rows = b <= 32 ? 32 : (b + 63) / 64 * 64;
  if (b < 1 || d < 1 || d % 4 != 0 || rows > qc) return hipErrorInvalidValue;
  RR_LAUNCH(q8_stage_kernel, dim3(rows), dim3(64), 0, s, q, b, d, q8, qc, q8s, qcopy);
  return hipGetLastError();
}

hipError_t launch_bf16_to_f32(const uint16_t* in, float* out, int64_t nrows, int d, hipStream_t s) {
  const int64_t groups = nrows * (d >> 3);
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s,
                     (const u32x4*)in, out, nrows, d);
  return hipGetLastError();
}

hipError_t launch_split_f32(const float* in, int64_t n, int d, void* out, float* norms, float* rscale,
                            hipStream_t s) {
  hipLaunchKernelGGL(split_f32_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, in, n, d, (u32x4*)out, norms,
                     rscale);
  return hipGetLastError();
}

hipError_t launch_unsplit_f32(const void* in, const float* rscale, int64_t n, int d, float* out, hipStream_t s) {
  const int64_t groups = n * (d >> 3);
  hipLaunchKernelGGL(unsplit_f32_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s, (const u32x4*)in,
                     rscale, n, d, out);
  return hipGetLastError();
}

hipError_t launch_row_norms(int dtype, const void* corpus, int64_t n, int d, float* norms, hipStream_t s) {
  const unsigned grid = (unsigned)((n + 3) / 4);
  if (dtype == 0) hipLaunchKernelGGL(row_norms_kernel<0>, dim3(grid), dim3(256), 0, s, corpus, n, d, norms);
  else hipLaunchKernelGGL(row_norms_kernel<1>, dim3(grid), dim3(256), 0, s, corpus, n, d, norms);
  return hipGetLastError();
}

__global__ void absmax_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
  {
    const float v = fabsf(x[i]);
    m = fmaxf(m, v != v ? INFINITY : v);   // (fmaxf drops NaN: a NaN counts as infinite here, so range checks fail)
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax((int*)out, __float_as_int(m));   // non-negative: int order = float order
}

hipError_t launch_absmax(const float* x, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(absmax_kernel, dim3(1024), dim3(256), 0, s, x, n, out);
  return hipGetLastError();
}

// A/B stand-in for a slower exchange (the 8-GPU all-gather's latency, on one GPU): one workgroup that occupies a CU
// for `ticks` of the 100 MHz wall clock (bounded: it ends after ticks whatever happens), as an RCCL kernel does.
__global__ void delay_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

hipError_t launch_delay(int us, hipStream_t s) {
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, (uint64_t)us * 100);
  return hipGetLastError();
}

// Diagnostic: the address of the hardware (AQL) queue this launch was dispatched from, into *out (rr_stream_queues).
__global__ void queue_probe_kernel(uint64_t* out) {
  if (threadIdx.x == 0) *out = (uint64_t)(uintptr_t)__builtin_amdgcn_queue_ptr();
}

hipError_t launch_queue_probe(uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(queue_probe_kernel, dim3(1), dim3(64), 0, s, out);
  return hipGetLastError();
}

hipError_t launch_synth(int kind, uint64_t seed, int64_t row_begin, int64_t n_rows, int d, float* out,
                        hipStream_t s) {
  const int64_t count = n_rows * (int64_t)d;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, kind, seed, row_begin,
                     n_rows, d, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || kind == 0) return e;
  hipLaunchKernelGGL(normalize_rows_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, s, out, n_rows, d);
  return hipGetLastError();
}

}  // namespace rr
