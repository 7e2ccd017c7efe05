// kbench.hip — A/B microbenchmark of fused-kernel variants (pipeline depth NB, load form LM) on one
// device, interleaved in one process (cdna_hip_programming.md §5.4 rule 24). Development tool, not
// part of the product; it compiles the product kernel source directly.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I rag-serving-system_amd/csrc \
//         tools/kbench.hip -o tools/kbench && tools/kbench [n_docs] [rounds]
#include "../rag-serving-system_amd/csrc/rr_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
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
#define V32(NB, LM, AS, COS, DBG, U) Variant{"fp32 NB=" #NB " LM=" #LM " AS=" #AS " COS=" #COS " DBG=" #DBG " U=" #U, 0, \
    [&](const void* c, uint64_t* o) { return launch_fused_t<0, 8, COS, 0, NB, LM, AS, DBG, U>(grid, c, norms, rscale, q, n, d, b, 0, o, s); }, {}}
#define V16(NB, LM, AS, COS, DBG, U) Variant{"bf16 NB=" #NB " LM=" #LM " AS=" #AS " COS=" #COS " DBG=" #DBG " U=" #U, 1, \
    [&](const void* c, uint64_t* o) { return launch_fused_t<1, 8, COS, 0, NB, LM, AS, DBG, U>(grid, c, norms, rscale, q, n, d, b, 0, o, s); }, {}}
#define VS(NB, LM, AS, COS, DBG, U) Variant{"fp32-split NB=" #NB " LM=" #LM " AS=" #AS " COS=" #COS " DBG=" #DBG " U=" #U, 2, \
    [&](const void* c, uint64_t* o) { return launch_fused_t<2, 8, COS, 0, NB, LM, AS, DBG, U>(grid, c, norms2, rscale, q, n, d, b, 0, o, s); }, {}}
  std::vector<Variant> vs = {V32(2, 1, 1, true, 0, 8), V32(2, 1, 1, true, 1, 8), V32(3, 1, 1, true, 0, 8), V32(2, 1, 1, true, 0, 4), VS(2, 1, 1, true, 0, 8), VS(2, 1, 1, false, 0, 8),
                             VS(2, 1, 1, true, 2, 8), V16(2, 1, 1, true, 0, 8), V16(3, 1, 1, true, 0, 8),
                             V16(2, 1, 1, false, 0, 8), V16(2, 1, 1, true, 1, 8)};
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
      Variant{"stream lin x4grid fp32", 0, [&](const void* c, uint64_t*) {
        hipLaunchKernelGGL(stream_lin, dim3(grid * 4), dim3(512), 0, s, (const u32x4*)c, n * d / 4, sink);
        return hipGetLastError(); }, {}},
  };
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
