// kbench_cfg5.hip — decomposition of the 64-slot bf16 pass (config 5's per-GPU shard) on one device: the product
// kernel as built with the RR_SK_DIAG knob of rr_sk.hip (0 full; 1 no epilogue; 3 no epilogue and no K-partial
// exchange), the 32-slot bf16 pass on the same rows, and the slab-streaming skeleton (LDS-DMA only). Development
// tool, not part of the product; it compiles the product kernel source directly.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I rag-serving-system_amd/csrc [-DRR_SK_DIAG=n] \
//         tools/kbench_cfg5.hip -o tools/kbench_cfg5 && tools/kbench_cfg5 [n_docs] [rounds]
#include "../rag-serving-system_amd/csrc/rr_kernels.hip"
#define RR_SK_ONE_UNIT   // (every split-K instantiation in this unit: rr_sk.hip includes rr_sk_fam_*.hip)
#include "../rag-serving-system_amd/csrc/rr_sk.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

#ifndef RR_SK_DIAG
#define RR_SK_DIAG_NAME 0
#else
#define RR_SK_DIAG_NAME RR_SK_DIAG
#endif

using namespace rr;

// the split-K kernel's corpus movement alone: 4-KiB slabs per wave through a 2-slot LDS ring (one in flight while
// one is read back with the MFMA-shaped ds_read_b128), one barrier per 32-row tile
__global__ __launch_bounds__(512) void stream_slabs(const char* __restrict__ c, int64_t n, int row_bytes,
                                                    unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char ss_smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int KS = row_bytes / 8, nslab = KS / 128;
  const int64_t per = n / gridDim.x / 32 * 32, b0 = (int64_t)blockIdx.x * per;
  const int64_t total = per / 32 * nslab;
  char* ring = ss_smem + wid * 2 * 4096;
  const unsigned ring_lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)ring);
  const int rl = lane >> 3, cl = lane & 7, r = lane & 31, h = lane >> 5;
  auto issue = [&](int64_t s) {
    const int64_t t = s / nslab;
    const int j = (int)(s - t * nslab);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const char* src = c + (b0 + t * 32 + 8 * i + rl) * row_bytes + wid * KS + j * 128 + ((cl ^ rl) << 4);
      sk::glds16(src, ring_lds + (unsigned)((s & 1) * 4096) + i * 1024);
    }
  };
  unsigned acc = 0;
  if (total > 0) issue(0);
  for (int64_t s = 0; s < total; ++s) {
    if (s + 1 < total) {
      issue(s + 1);
      sk::wait_vm<4>();
    } else {
      sk::wait_vm<0>();
    }
    const char* slot = ring + (s & 1) * 4096;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const u32x4 v = *(const u32x4*)(slot + sk::slab_off(r, 2 * cc + h));
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if ((s % nslab) == nslab - 1) __builtin_amdgcn_s_barrier();
  }
  out[((int64_t)blockIdx.x * 8 + wid) * 64 + lane] = acc;
}

struct Variant {
  std::string name;
  double bytes;
  std::function<hipError_t()> run;
  std::vector<double> ms;
};

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 6250000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7;
  const int reps = 5, d = 1024;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  uint16_t* c16;
  float *norms, *q, *tmp;
  const int64_t chunk = 1 << 20;
  CK(hipMalloc(&c16, (size_t)n * d * 2));
  CK(hipMalloc(&norms, (size_t)(n + 64) * 4));
  CK(hipMalloc(&q, (size_t)64 * d * 4));
  CK(hipMalloc(&tmp, (size_t)chunk * d * 4));
  for (int64_t r0 = 0; r0 < n; r0 += chunk) {   // unit-norm rows, bf16 storage, norms of the stored values
    const int64_t nr = std::min(chunk, n - r0);
    CK(launch_synth(1, 1234, r0, nr, d, tmp, s));
    CK(launch_f32_to_bf16(tmp, c16 + r0 * d, nr, d, s));
  }
  CK(launch_row_norms(1, c16, n, d, norms, s));
  CK(launch_synth(1, 99, 0, 64, d, q, s));
  CK(hipStreamSynchronize(s));
  CK(hipFree(tmp));
  const int grid = cus;
  uint64_t* cand;
  CK(hipMalloc(&cand, (size_t)grid * 64 * 32 * 8));
  unsigned* sink;
  CK(hipMalloc(&sink, (size_t)grid * 8 * 64 * 4));
  CK(hipFuncSetAttribute((const void*)stream_slabs, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 2 * 4096));
  const double bytes = (double)n * d * 2 + n * 4.0;
  std::vector<Variant> vs = {
      {"64-slot bf16 cos kt16 diag=" + std::to_string(RR_SK_DIAG_NAME), bytes,
       [&] { return launch_sk(KDT_BF16, 1, 16, grid, c16, norms, nullptr, q, n, d, 64, 0, cand, s, 2, 64); }, {}},
      {"32-slot bf16 cos kt16 diag=" + std::to_string(RR_SK_DIAG_NAME), bytes,
       [&] { return launch_sk(KDT_BF16, 1, 16, grid, c16, norms, nullptr, q, n, d, 32, 0, cand, s, 2, 32); }, {}},
      {"slab stream only (LDS-DMA, 2 slots, barrier per tile)", (double)n * d * 2, [&] {
         hipLaunchKernelGGL(stream_slabs, dim3(grid), dim3(512), 8 * 2 * 4096, s, (const char*)c16, n, d * 2, sink);
         return hipGetLastError();
       }, {}},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) CK(v.run());   // warm, attributes
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) CK(v.run());
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / reps);
    }
#if defined(RR_SK_DIAG) && (RR_SK_DIAG & 4)
  // per-phase cycles per tile and wave (s_memtime around each phase; the timers themselves cost a little)
  for (int vi = 0; vi < 2; ++vi) {
    CK(vs[vi].run());
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h((size_t)grid * 9 * 8);
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(rr::sk::phase_cycles), h.size() * 8));
    for (int grp = 0; grp < 2; ++grp) {   // waves 0-3, waves 4-7 (the stagger defers the second group)
      double acc[8] = {0};
      for (int g = 0; g < grid; ++g)
        for (int w = 4 * grp; w < 4 * grp + 4; ++w)
          for (int i = 0; i < 8; ++i) acc[i] += (double)h[((size_t)g * 9 + w) * 8 + i];
      const double tiles = acc[6] > 0 ? acc[6] : 1;
      printf("{\"phases\": \"%s\", \"waves\": \"%d-%d\", \"cycles_per_tile_wave\": {\"slab_wait\": %.0f, "
             "\"slab_loop_incl_wait\": %.0f, \"barrier_A\": %.0f, \"write_barrier_B\": %.0f, \"partial_reads\": %.0f, "
             "\"epilogue\": %.0f}, \"insert_executions_per_tile_wave\": %.3f, \"tiles_per_wave\": %.1f}\n",
             vs[vi].name.c_str(), 4 * grp, 4 * grp + 3, acc[0] / tiles, acc[1] / tiles, acc[2] / tiles, acc[3] / tiles,
             acc[4] / tiles, acc[5] / tiles, acc[7] / tiles, tiles / (grid * 4.0));
    }
  }
#endif
  for (auto& v : vs) {
    std::vector<double> m = v.ms;
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    printf("{\"variant\": \"%s\", \"n\": %lld, \"median_us\": %.1f, \"min_us\": %.1f, \"frac_8TBs\": %.4f}\n",
           v.name.c_str(), (long long)n, med * 1e3, m[0] * 1e3, v.bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
