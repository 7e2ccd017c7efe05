// rr_device.h — device-side helpers shared by the retrieval kernels (rr_kernels.hip, rr_sk.hip):
// vector types, a compile-time loop, the 64-bit (score, index) keys and the per-lane top-KT list.
//
// Score/index keys. A candidate is one uint64: high 32 bits = order-preserving image of the fp32
// score, low 32 bits = 0xFFFFFFFF - global_index. Unsigned key order == (score desc, index asc), the
// deterministic tie rule of this implementation (the reference's tie order is implementation
// defined: numpy introselect / CUB). Key 0 = empty slot.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace rr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ------------------------------------------------------------------------------------------------
// keys
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord_of(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float float_of_ord(uint32_t o) {
  const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}
__device__ __forceinline__ uint64_t make_key(float s, uint32_t gidx) {
  return ((uint64_t)ord_of(s) << 32) | (uint64_t)(0xFFFFFFFFu - gidx);
}
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// Cosine denominator |q|*|d| + 1e-8 with the product rounded BEFORE the add, as the reference computes it
// (norm_X @ norm_Y.T, then + 1e-8 elementwise; retriever.py:605-607): no FMA contraction here.
__device__ __forceinline__ float cos_den(float qn, float nd) {
#pragma clang fp contract(off)
  return qn * nd + 1e-8f;
}

// Per-lane sorted (descending) list of the KT best keys, fully in registers (static indexing only).
template <int KT>
struct TopK {
  uint64_t v[KT];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int i = 0; i < KT; ++i) v[i] = 0;
  }
  __device__ __forceinline__ uint64_t last() const { return v[KT - 1]; }
  // Branch-free insertion of x (caller checked x > last()).
  __device__ __forceinline__ void insert(uint64_t x) {
#pragma unroll
    for (int i = KT - 1; i > 0; --i) {
      const uint64_t up = v[i - 1];
      v[i] = (x > up) ? up : umax64(x, v[i]);
    }
    v[0] = umax64(x, v[0]);
  }
  __device__ __forceinline__ void pop() {
#pragma unroll
    for (int i = 0; i < KT - 1; ++i) v[i] = v[i + 1];
    v[KT - 1] = 0;
  }
};

// ------------------------------------------------------------------------------------------------
// cross-lane max of 64-bit keys with DPP (row ops take a VALU slot each; no LDS round trip as the
// ds_swizzle / ds_bpermute forms of __shfl_xor do): the high words first, then the low words of the
// lanes that hold the high maximum.
// ------------------------------------------------------------------------------------------------
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp_max_u32(uint32_t v) {
  if constexpr (ROW_MASK == 0xF) {
    // every lane reads a valid source lane (quad_perm / row mirrors): a plain DPP move, which the compiler folds
    // into the max itself (v_max_u32_dpp: one VALU instead of a copy, the DPP move and the max)
    const uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
    return v > t ? v : t;
  } else {
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xF, false);
    return v > t ? v : t;
  }
}
// max over aligned groups of G lanes (G = 2, 4, 8, 16), every lane of the group gets it
template <int G>
__device__ __forceinline__ uint32_t group_max_u32(uint32_t v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "DPP row groups");
  v = dpp_max_u32<0xB1>(v);                        // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v = dpp_max_u32<0x4E>(v);  // quad_perm [2,3,0,1]
  if constexpr (G >= 8) v = dpp_max_u32<0x141>(v); // row_half_mirror
  if constexpr (G >= 16) v = dpp_max_u32<0x140>(v); // row_mirror
  return v;
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_min_u32(uint32_t v) {
  const uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
  return v < t ? v : t;
}
// min over aligned groups of G lanes (G = 2, 4, 8, 16), every lane of the group gets it
template <int G>
__device__ __forceinline__ uint32_t group_min_u32(uint32_t v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "DPP row groups");
  v = dpp_min_u32<0xB1>(v);
  if constexpr (G >= 4) v = dpp_min_u32<0x4E>(v);
  if constexpr (G >= 8) v = dpp_min_u32<0x141>(v);
  if constexpr (G >= 16) v = dpp_min_u32<0x140>(v);
  return v;
}
// max over the 64 lanes, returned in every lane
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = group_max_u32<16>(v);
  v = dpp_max_u32<0x142, 0xA>(v);                   // row_bcast:15 into rows 1, 3
  v = dpp_max_u32<0x143, 0xC>(v);                   // row_bcast:31 into rows 2, 3: lane 63 has the max
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
template <int G>
__device__ __forceinline__ uint64_t group_max_u64(uint64_t x) {
  const uint32_t hi = group_max_u32<G>((uint32_t)(x >> 32));
  const uint32_t lo = group_max_u32<G>((uint32_t)(x >> 32) == hi ? (uint32_t)x : 0u);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
  const uint32_t hi = wave_max_u32((uint32_t)(x >> 32));
  const uint32_t lo = wave_max_u32((uint32_t)(x >> 32) == hi ? (uint32_t)x : 0u);
  return ((uint64_t)hi << 32) | lo;
}

// The int8 screen's query pieces, one wave per query slot: s = max|q| / 127, t = q / s, p1 = clamp(rint(t)), p2 =
// clamp(rint((t - p1) * 64)) — q ~ s (p1 + p2 / 64), the MFMAs' sum being x8 . (64 p1 + p2) — and eq >= the
// residual's norm (real arithmetic), in the scale's units as f32_to_i8_kernel: t - p1 - p2 / 64 is exact (each step
// by Sterbenz), so |q - s (p1 + p2 / 64)|_2 <= s |t - p1 - p2/64|_2 (x 1 + 2^-12) + 2^-21 sqrt(d) max|q| + 2^-140.
// |q| and sum|q| in fp32 (the bound bumps for their summation order). One wave (64 lanes) per query slot `slot`;
// slots >= b get zero pieces and scalars. Run by q8_prep_kernel / q9_prep_kernel (rr_kernels.hip) in front of the
// screen on its stream. (Quantising in every screen workgroup instead — each redoing all 32 queries,
// two L2 passes — measured 8-13 us longer per launch: profiles/r04/ab/int8/.)
// PIECES = 1 (the bf16-storage screen, DT 9: q ~ s p1, pieces [QS][d], scalars [4][QS] with the scale s itself; up to 64
// slots) or 2 (DT 8: q ~ s (p1 + p2 / 64), pieces [2][32][d], scale s / 64).
template <int PIECES = 2, int kQS = 32>
__device__ __forceinline__ void q8_prep_slot(const float* __restrict__ q, int b, int d, int8_t* __restrict__ q8,
                                             float* __restrict__ q8s, int slot, int lane) {
  int8_t* p1 = q8 + (size_t)slot * d;
  int8_t* p2 = q8 + (size_t)(kQS + slot) * d;
  if (slot >= b) {
    for (int e = 4 * lane; e < d; e += 256) {
      *(uint32_t*)(p1 + e) = 0;
      if constexpr (PIECES == 2) *(uint32_t*)(p2 + e) = 0;
    }
    if (lane < 4) q8s[lane * kQS + slot] = 0.f;
    return;
  }
  (void)p2;
  const f32x4* src = (const f32x4*)(q + (size_t)slot * d);
  // d <= 1024 (every d the int8 copy serves): the lane's <= 4 float4 loaded once, all issued before the first use —
  // one memory latency for both passes instead of one per float4 per pass (the same values in the same order)
  constexpr int kRegC = 4;
  const bool in_regs = d <= 64 * 4 * kRegC;
  f32x4 vr[kRegC];
  if (in_regs) {
#pragma unroll
    for (int i = 0; i < kRegC; ++i) {
      const int c = lane + 64 * i;
      vr[i] = c < (d >> 2) ? src[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float m = 0.f, s2 = 0.f, s1 = 0.f;
  auto pass1 = [&](const f32x4 v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      m = fmaxf(m, fabsf(v[j]));
      s2 = fmaf(v[j], v[j], s2);
      s1 += fabsf(v[j]);
    }
  };
  if (in_regs) {
#pragma unroll
    for (int i = 0; i < kRegC; ++i)
      if (lane + 64 * i < (d >> 2)) pass1(vr[i]);
  } else {
    for (int c = lane; c < (d >> 2); c += 64) pass1(src[c]);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    m = fmaxf(m, __shfl_xor(m, off, 64));
    s2 += __shfl_xor(s2, off, 64);
    s1 += __shfl_xor(s1, off, 64);
  }
  const float s = m > 0.f ? m / 127.0f : 0.f;
  float se = 0.f;
  auto pass2 = [&](const f32x4 v, int c) {
    uint32_t w1 = 0, w2 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = 0.f, cc = 0.f, r = 0.f;
      if (s > 0.f) {
        const float t = v[j] / s;
        a = fminf(fmaxf(rintf(t), -127.0f), 127.0f);
        const float ta = t - a;   // exact
        if constexpr (PIECES == 2) {
          cc = fminf(fmaxf(rintf(ta * 64.0f), -127.0f), 127.0f);
          r = ta - cc * 0x1p-6f;    // exact
        } else {
          r = ta;
        }
      }
      w1 |= ((uint32_t)(int)a & 0xFFu) << (8 * j);
      w2 |= ((uint32_t)(int)cc & 0xFFu) << (8 * j);
      se = fmaf(r, r, se);
    }
    *(uint32_t*)(p1 + 4 * c) = w1;
    if constexpr (PIECES == 2) *(uint32_t*)(p2 + 4 * c) = w2;
  };
  if (in_regs) {
#pragma unroll
    for (int i = 0; i < kRegC; ++i)
      if (lane + 64 * i < (d >> 2)) pass2(vr[i], lane + 64 * i);
  } else {
    for (int c = lane; c < (d >> 2); c += 64) pass2(src[c], c);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) se += __shfl_xor(se, off, 64);
  if (lane == 0) {
    q8s[slot] = sqrtf(s2);
    q8s[kQS + slot] = s1 * (1.0f + 0x1p-18f);
    q8s[2 * kQS + slot] = PIECES == 2 ? s * 0x1p-6f : s;
    q8s[3 * kQS + slot] = fmaf(s * sqrtf(se), 1.0f + 0x1p-12f, fmaf(m, sqrtf((float)d) * 0x1p-21f, 0x1p-140f));
  }
}

}  // namespace rr
