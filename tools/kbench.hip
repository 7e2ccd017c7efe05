// kbench.hip — A/B microbenchmark of fused-kernel variants (pipeline depth NB, load form LM) on one
// device, interleaved in one process (cdna_hip_programming.md §5.4 rule 24). Development tool, not
// part of the product; it compiles the product kernel source directly.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I rag-serving-system_amd/csrc \
//         tools/kbench.hip -o tools/kbench && tools/kbench [n_docs] [rounds]
#include "../rag-serving-system_amd/csrc/rr_kernels.hip"
#define RR_SK_ONE_UNIT   // (every split-K instantiation in this unit: rr_sk.hip includes rr_sk_fam_*.hip)
#include "../rag-serving-system_amd/csrc/rr_sk.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>
#include <unistd.h>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

using namespace rr;

// Memory-side ceilings for the corpus stream, no MFMA: (a) the fused kernel's fragment pattern (each
// lane a row, 2 lanes x 16 B per row per instruction, U loads per lane in flight); (b) lane-linear
// 1 KiB per wave-instruction. Each wave reduces what it read into one word so nothing is dead.
template <int U>
__global__ __launch_bounds__(512) void stream_frag(const u32x4* __restrict__ c, int64_t n, int d, unsigned* out) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t nwave = (int64_t)gridDim.x * 8, gw = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int64_t per = n / nwave, b0 = gw * per;
  const int rs = d >> 2, ng = (d >> 3) / U;
  unsigned acc = 0;
  for (int64_t base = b0; base < b0 + per; base += 32) {
    int64_t row = base + r < b0 + per ? base + r : b0 + per - 1;
    const u32x4* p = c + row * rs + h;
    for (int g = 0; g < ng; ++g) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[2 * (g * U + u)];
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  out[gw * 64 + lane] = acc;
}
__global__ __launch_bounds__(512) void stream_lin(const u32x4* __restrict__ c, int64_t n16, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwave = (int64_t)gridDim.x * 8, gw = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int64_t per = n16 / nwave, b0 = gw * per;
  unsigned acc = 0;
  for (int64_t i = b0 + lane; i + 64 * 7 < b0 + per; i += 64 * 8) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = c[i + 64 * u];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  out[gw * 64 + lane] = acc;
}

// (c) LDS-DMA stream: each wave moves 1 KiB pieces of its contiguous range into its own LDS ring with
// global_load_lds_dwordx4 (R pieces in flight, counted vmcnt), then reads each piece back (ds_read_b128).
template <int R, int NT>
__global__ __launch_bounds__(512) void stream_glds(const u32x4* __restrict__ c, int64_t n16, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char ring_smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nwave = (int64_t)gridDim.x * 8, gw = (int64_t)blockIdx.x * 8 + wid;
  const int64_t per = n16 / nwave / 64 * 64, b0 = gw * per;   // 16-byte units, whole pieces
  const int64_t npieces = per / 64;
  u32x4* ring = (u32x4*)ring_smem + wid * R * 64;
  const unsigned ring_base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)ring);
  unsigned acc = 0;
  auto issue = [&](int64_t p) {
    const u32x4* src = c + b0 + p * 64 + lane;
    const unsigned dst = ring_base + (unsigned)((p % R) * 1024);
    unsigned keep;
    if constexpr (NT)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  for (int64_t p = 0; p < R - 1 && p < npieces; ++p) issue(p);
  for (int64_t p = 0; p < npieces; ++p) {
    if (p + R - 1 < npieces) {
      issue(p + R - 1);
      asm volatile("s_waitcnt vmcnt(%0)" :: "i"(R - 1) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const u32x4 v = ring[(p % R) * 64 + lane];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[gw * 64 + lane] = acc;
}
template <int NT>
__global__ __launch_bounds__(512) void stream_lin_nt(const u32x4* __restrict__ c, int64_t n16, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const int64_t nwave = (int64_t)gridDim.x * 8, gw = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int64_t per = n16 / nwave, b0 = gw * per;
  unsigned acc = 0;
  for (int64_t i = b0 + lane; i + 64 * 7 < b0 + per; i += 64 * 8) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(c + i + 64 * u);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  out[gw * 64 + lane] = acc;
}

// (d) nt loads with LPR lanes per row (16*LPR contiguous bytes of a row per instruction, 64/LPR rows),
// a wave sweeping a block of rows column-chunk by column-chunk (U instructions in flight).
template <int LPR, int NT>
__global__ __launch_bounds__(512) void stream_pat(const u32x4* __restrict__ c, int64_t n, int d, unsigned* out) {
  const int lane = threadIdx.x & 63;
  constexpr int RPI = 64 / LPR;                  // rows per instruction
  const int upr = d >> 2;                        // 16-byte units per row
  const int64_t nwave = (int64_t)gridDim.x * 8, gw = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int64_t per = n / nwave / 32 * 32, b0 = gw * per;
  unsigned acc = 0;
  const int rl = lane / LPR, cl = lane % LPR;
  for (int64_t base = b0; base < b0 + per; base += 32) {
    // 32 rows x upr units: instruction i covers rows (i % (32/RPI))*RPI + rl, column chunk (i / (32/RPI))
    constexpr int RB = 32 / RPI;
    const int nin = RB * (upr / LPR);
    for (int i0 = 0; i0 < nin; i0 += 8) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u;
        const int64_t row = base + (i % RB) * RPI + rl;
        const u32x4* p = c + row * upr + (i / RB) * LPR + cl;
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  out[gw * 64 + lane] = acc;
}

// (e) split-K streaming skeleton: a workgroup walks its contiguous rows in 32-row tiles; wave w owns bytes
// [w*KS, (w+1)*KS) of every row and moves them in 4-KiB slabs (32 rows x 128 B, 4 LDS-DMA instructions of
// 8 rows x 128 B, source-swizzled) through an RS-slot LDS ring, then reads MFMA-shaped fragments
// (lane (r, h): 16 B of row r) back with ds_read_b128. A raw s_barrier per tile stands in for the
// cross-wave reduction.
__device__ __forceinline__ void glds16(const void* src, unsigned lds, int nt) {
  unsigned keep;
  if (nt)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
template <int RS, int NT, int BAR>
__global__ __launch_bounds__(512) void stream_sk(const char* __restrict__ c, int64_t n, int row_bytes, unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char sk_smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int KS = row_bytes / 8, nslab = KS / 128;
  const int64_t per = n / gridDim.x / 32 * 32, b0 = (int64_t)blockIdx.x * per;
  const int64_t ntile = per / 32, total = ntile * nslab;
  char* ring = sk_smem + wid * RS * 4096;
  const unsigned ring_lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)ring);
  const int rl = lane >> 3, cl = lane & 7;
  auto issue = [&](int64_t s) {
    const int64_t t = s / nslab;
    const int j = (int)(s - t * nslab);
    const unsigned slot = ring_lds + (unsigned)((s % RS) * 4096);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = b0 + t * 32 + 8 * i + rl;
      const char* src = c + row * row_bytes + wid * KS + j * 128 + ((cl ^ rl) << 4);
      glds16(src, slot + i * 1024, NT);
    }
  };
  unsigned acc = 0;
  const int r = lane & 31, h = lane >> 5;
  for (int64_t s = 0; s < RS - 1 && s < total; ++s) issue(s);
  for (int64_t s = 0; s < total; ++s) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // previous slab's ds_reads done (slot reuse)
    if (s + RS - 1 < total) {
      issue(s + RS - 1);
      asm volatile("s_waitcnt vmcnt(%0)" :: "i"(4 * (RS - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const char* slot = ring + (s % RS) * 4096;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int chunk = 2 * cc + h;
      const u32x4 v = *(const u32x4*)(slot + (r >> 3) * 1024 + (r & 7) * 128 + ((chunk ^ (r & 7)) << 4));
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (BAR && (s % nslab) == nslab - 1) __builtin_amdgcn_s_barrier();
  }
  out[((int64_t)blockIdx.x * 8 + wid) * 64 + lane] = acc;
}

struct Variant {
  std::string name;
  int dtype;
  std::function<hipError_t(const void*, uint64_t*)> run;
  std::vector<double> ms;
};

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const int reps = 10;
  const int d = 1024, b = 32, kt = 8;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float *c32, *norms, *q;
  uint16_t* c16;
  CK(hipMalloc(&c32, (size_t)n * d * 4));
  CK(hipMalloc(&c16, (size_t)n * d * 2));
  CK(hipMalloc(&norms, (size_t)(n + 64) * 4));
  CK(hipMalloc(&q, (size_t)b * d * 4));
  CK(launch_synth(1, 1234, 0, n, d, c32, s));
  CK(launch_synth(1, 99, 0, b, d, q, s));
  CK(launch_f32_to_bf16(c32, c16, n, d, s));
  uint16_t* cf16;   // the f16 screening copy (DT 7)
  CK(hipMalloc(&cf16, (size_t)n * d * 2));
  CK(launch_f32_to_f16(c32, cf16, n, d, s));
  CK(launch_row_norms(0, c32, n, d, norms, s));
  float *csplit, *norms2, *rscale;
  CK(hipMalloc(&csplit, (size_t)n * d * 4));
  CK(hipMalloc(&norms2, (size_t)(n + 64) * 4));
  CK(hipMalloc(&rscale, (size_t)(n + 64) * 4));
  CK(launch_split_f32(c32, n, d, csplit, norms2, rscale, s));
  {  // the fp32-MFMA kernel reads rows in the pair_unit layout
    float* cperm;
    CK(hipMalloc(&cperm, (size_t)n * d * 4));
    CK(launch_permute_f32(c32, cperm, n, d, 0, s));
    CK(hipStreamSynchronize(s));
    CK(hipFree(c32));
    c32 = cperm;
  }
  const int grid = cus;
  uint64_t *cand, *ref32, *ref16;
  const size_t cand_elems = (size_t)grid * kQSlots * kt;
  CK(hipMalloc(&cand, cand_elems * 8));
  std::vector<uint64_t> h_ref32(cand_elems), h_ref16(cand_elems), h_out(cand_elems);

  uint64_t* fin;
  CK(hipMalloc(&fin, kQSlots * kt * 8));
  unsigned* sink;
  CK(hipMalloc(&sink, (size_t)grid * 4 * 8 * 64 * 4));  // room for the x4 grid
#ifdef RR_SK_PROBE
  if (argc > 3 && strcmp(argv[3], "probe") == 0) {   // per-workgroup phase timestamps of the split-K kernel
    struct P { const char* name; int dt; int cos; const void* c; const float* nr; };
    const P ps[] = {{"sk f16 screen copy (DT 7) cos", 7, 1, cf16, norms}, {"sk fp32 (DT 3) cos", 3, 1, c32, norms},
                    {"sk bf16 (DT 1) cos", 1, 1, c16, norms}, {"sk fp32 (DT 3) dot", 3, 0, c32, norms}};
    std::vector<unsigned long long> h((size_t)grid * 8);
    for (const P& p : ps) {
      for (int rep = 0; rep < 4; ++rep) {
        CK(launch_sk(p.dt, p.cos, 8, grid, p.c, p.nr, rscale, q, n, d, b, 0, cand, s, 2));
        CK(hipStreamSynchronize(s));
      }
      CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(rr::sk::probe), h.size() * 8));
      unsigned long long t0min = ~0ull, t0max = 0, t5max = 0;
      for (int g = 0; g < grid; ++g) {
        t0min = std::min(t0min, h[g * 8]); t0max = std::max(t0max, h[g * 8]); t5max = std::max(t5max, h[g * 8 + 5]);
      }
      printf("{\"probe\": \"%s\", \"n\": %lld, \"start_spread_us\": %.2f, \"span_us\": %.2f", p.name, (long long)n,
             (t0max - t0min) / 100.0, (t5max - t0min) / 100.0);
      const char* ph[] = {"prep", "tile0", "tile1", "rest", "merge"};
      for (int i = 1; i <= 5; ++i) {
        std::vector<double> v;
        for (int g = 0; g < grid; ++g) v.push_back((double)(h[g * 8 + i] - h[g * 8 + i - 1]) / 100.0);
        std::sort(v.begin(), v.end());
        printf(", \"%s_us\": [%.2f, %.2f, %.2f]", ph[i - 1], v[0], v[v.size() / 2], v.back());
      }
      std::vector<double> e;
      for (int g = 0; g < grid; ++g) e.push_back((double)(h[g * 8 + 5] - t0min) / 100.0);
      std::sort(e.begin(), e.end());
      printf(", \"end_us_min_med_max\": [%.2f, %.2f, %.2f]}\n", e[0], e[e.size() / 2], e.back());
    }
    return 0;
  }
#endif
#define V32(NB, LM, AS, COS, DBG, U) Variant{"fp32 NB=" #NB " LM=" #LM " AS=" #AS " COS=" #COS " DBG=" #DBG " U=" #U, 0, \
    [&](const void* c, uint64_t* o) { return launch_fused_t<0, 8, COS, 0, NB, LM, AS, DBG, U>(grid, c, norms, rscale, q, n, d, b, 0, o, s); }, {}}
#define V16(NB, LM, AS, COS, DBG, U) Variant{"bf16 NB=" #NB " LM=" #LM " AS=" #AS " COS=" #COS " DBG=" #DBG " U=" #U, 1, \
    [&](const void* c, uint64_t* o) { return launch_fused_t<1, 8, COS, 0, NB, LM, AS, DBG, U>(grid, c, norms, rscale, q, n, d, b, 0, o, s); }, {}}
#define VS(NB, LM, AS, COS, DBG, U) Variant{"fp32-split NB=" #NB " LM=" #LM " AS=" #AS " COS=" #COS " DBG=" #DBG " U=" #U, 2, \
    [&](const void* c, uint64_t* o) { return launch_fused_t<2, 8, COS, 0, NB, LM, AS, DBG, U>(grid, c, norms2, rscale, q, n, d, b, 0, o, s); }, {}}
#define VK(DT, BUF, COS, RS) Variant{"sk DT=" #DT " COS=" #COS " ring=" #RS, BUF, \
    [&](const void* c, uint64_t* o) { return launch_sk(DT, COS, 8, grid, c, DT == 2 ? norms2 : norms, rscale, q, n, d, b, 0, o, s, RS); }, {}}
  std::vector<Variant> vs = {V32(2, 1, 1, true, 0, 8), VS(2, 1, 1, true, 0, 8), V16(2, 1, 1, true, 0, 8),
                             VK(3, 0, 1, 2), VK(6, 0, 1, 2), VK(2, 2, 1, 2), VK(1, 1, 1, 2), VK(3, 0, 0, 2)};
  std::vector<Variant> streams = {
      Variant{"stream frag U=8 fp32", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL(stream_frag<8>, dim3(grid), dim3(512), 0, s, (const u32x4*)c, n, d, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream frag U=16 fp32", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL(stream_frag<16>, dim3(grid), dim3(512), 0, s, (const u32x4*)c, n, d, sink);
        return hipGetLastError(); }, {}},
      Variant{"merge_kernel KT=8 (256 lists)", 0, [&](const void*, uint64_t*) {
        return launch_merge(kt, cand, grid, kt, b, 5, fin, nullptr, nullptr, s); }, {}},
      Variant{"stream lin fp32", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL(stream_lin, dim3(grid), dim3(512), 0, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream glds R=8 default", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_glds<8, 0>), dim3(grid), dim3(512), 8 * 8 * 1024, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream glds R=8 nt", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_glds<8, 1>), dim3(grid), dim3(512), 8 * 8 * 1024, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream glds R=16 nt", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_glds<16, 1>), dim3(grid), dim3(512), 8 * 16 * 1024, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream glds R=4 nt", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_glds<4, 1>), dim3(grid), dim3(512), 8 * 4 * 1024, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream lin nt-builtin", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL(stream_lin_nt<1>, dim3(grid), dim3(512), 0, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk RS=2 nt=1 bar=1", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<2, 1, 1>), dim3(grid), dim3(512), 8 * 2 * 4096, s, (const char*)c, n, d * 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk bf16 RS=2 nt=1 bar=1", 1, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<2, 1, 1>), dim3(grid), dim3(512), 8 * 2 * 4096, s, (const char*)c, n, d * 2, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk RS=3 nt=1 bar=1", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<3, 1, 1>), dim3(grid), dim3(512), 8 * 3 * 4096, s, (const char*)c, n, d * 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk bf16 RS=3 nt=1 bar=1", 1, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<3, 1, 1>), dim3(grid), dim3(512), 8 * 3 * 4096, s, (const char*)c, n, d * 2, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk RS=4 nt=1 bar=1", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<4, 1, 1>), dim3(grid), dim3(512), 8 * 4 * 4096, s, (const char*)c, n, d * 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk bf16 RS=4 nt=1 bar=1", 1, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<4, 1, 1>), dim3(grid), dim3(512), 8 * 4 * 4096, s, (const char*)c, n, d * 2, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk RS=2 nt=0 bar=1", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<2, 0, 1>), dim3(grid), dim3(512), 8 * 2 * 4096, s, (const char*)c, n, d * 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk bf16 RS=2 nt=0 bar=1", 1, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<2, 0, 1>), dim3(grid), dim3(512), 8 * 2 * 4096, s, (const char*)c, n, d * 2, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk RS=3 nt=1 bar=0", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<3, 1, 0>), dim3(grid), dim3(512), 8 * 3 * 4096, s, (const char*)c, n, d * 4, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream sk bf16 RS=3 nt=1 bar=0", 1, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL((stream_sk<3, 1, 0>), dim3(grid), dim3(512), 8 * 3 * 4096, s, (const char*)c, n, d * 2, sink);
        return hipGetLastError(); }, {}},
      Variant{"stream lin x4grid fp32", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL(stream_lin, dim3(grid * 4), dim3(512), 0, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
  };
  if (argc > 3 && strcmp(argv[3], "transient") == 0) {
    // Per-launch durations from an idle GPU: each variant after `idle` seconds without work, `count`
    // launches timed one by one (HIP events), so the clock/power transient shows per kernel form.
    const int count = argc > 4 ? atoi(argv[4]) : 40;
    const int idle_ms = argc > 5 ? atoi(argv[5]) : 3000;
    CK(hipFuncSetAttribute((const void*)stream_sk<3, 1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 3 * 4096));
    std::vector<Variant> tv = {VK(3, 0, 1, 2), VK(6, 0, 1, 2), VK(2, 2, 1, 2), streams[9], VK(6, 0, 1, 2),
                               VK(3, 0, 1, 2)};
    std::vector<hipEvent_t> ev(2 * count);
    for (auto& e : ev) CK(hipEventCreate(&e));
    for (auto& v : tv) {
      const void* c = v.dtype == 1 ? (const void*)c16 : v.dtype == 2 ? (const void*)csplit : (const void*)c32;
      CK(hipStreamSynchronize(s));
      usleep(idle_ms * 1000);
      for (int i = 0; i < count; ++i) {
        CK(hipEventRecord(ev[2 * i], s));
        CK(v.run(c, cand));
        CK(hipEventRecord(ev[2 * i + 1], s));
      }
      CK(hipStreamSynchronize(s));
      printf("{\"transient\": \"%s\", \"us\": [", v.name.c_str());
      for (int i = 0; i < count; ++i) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
        printf("%s%.0f", i ? ", " : "", ms * 1e3);
      }
      printf("]}\n");
      fflush(stdout);
    }
    return 0;
  }
  CK(hipFuncSetAttribute((const void*)stream_glds<16, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 16 * 1024));
  CK(hipFuncSetAttribute((const void*)stream_sk<3, 1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 3 * 4096));
  CK(hipFuncSetAttribute((const void*)stream_sk<3, 1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 3 * 4096));
  CK(hipFuncSetAttribute((const void*)stream_sk<4, 1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 4 * 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // reference outputs (first variant of each dtype) and correctness of the others
  bool have32 = false, have16 = false;
  h_out.resize(kQSlots * kt);
  h_ref32.resize(kQSlots * kt);
  h_ref16.resize(kQSlots * kt);
  for (auto& v : vs) {
    CK(hipMemsetAsync(cand, 0, cand_elems * 8, s));
    CK(v.run(v.dtype == 1 ? (const void*)c16 : v.dtype == 2 ? (const void*)csplit : (const void*)c32, cand));
    CK(launch_merge(kt, cand, grid, kt, b, kt, fin, nullptr, nullptr, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h_out.data(), fin, kQSlots * kt * 8, hipMemcpyDeviceToHost));
    auto& ref = h_ref32;
    bool& have = have32;
    if (!have) { ref = h_out; have = true; }
    int same_idx = 0;
    for (size_t i = 0; i < ref.size(); ++i) same_idx += (uint32_t)ref[i] == (uint32_t)h_out[i];
    printf("{\"variant\": \"%s\", \"same_index_frac_vs_first\": %.4f, \"bitwise\": %s}\n", v.name.c_str(),
           same_idx / (double)ref.size(), memcmp(ref.data(), h_out.data(), ref.size() * 8) == 0 ? "true" : "false");
  }
  const size_t nvar = vs.size();
  for (auto& v : streams) vs.push_back(v);
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      const void* c = v.dtype == 1 ? (const void*)c16 : v.dtype == 2 ? (const void*)csplit : (const void*)c32;
      CK(v.run(c, cand));   // warm
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) CK(v.run(c, cand));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / reps);
    }
  }
  for (auto& v : vs) {
    std::vector<double> m = v.ms;
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2], best = m[0];
    const bool is_stream = (size_t)(&v - &vs[0]) >= nvar;
    const double bytes = (double)n * d * (v.dtype == 1 ? 2 : 4) + (is_stream ? 0.0 : n * 4.0 + b * d * 4.0);
    printf("{\"variant\": \"%s\", \"median_us\": %.1f, \"min_us\": %.1f, \"GBps_median\": %.0f, \"frac_8TBs\": %.3f}\n",
           v.name.c_str(), med * 1e3, best * 1e3, bytes / (med * 1e-3) / 1e9, bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
