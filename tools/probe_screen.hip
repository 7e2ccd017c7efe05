// probe_screen.hip — per-workgroup phase timestamps (s_memrealtime, 100 MHz) of ONE screen launch of the product
// kernel (rr_sk.hip built with -DRR_SK_PROBE), for the small-shard fixed-cost analysis. Development
// tool, not part of the product: it compiles the product kernel source directly, instantiating only the kernels it
// launches (RR_SK_NO_DISPATCH).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DRR_SK_PROBE -DRR_SK_NO_DISPATCH -I include \
//         -I rag-serving-system_amd/csrc tools/probe_screen.hip -o tools/probe_screen
//   tools/probe_screen [rows=125000] [grid=256] [ct8=2] [unused=0] [guided=1] [streams_test=0] [pieces=2]
// (pieces: 2 = DT 8, the two-piece int8 screen; 1 = DT 9, one piece. The chunk geometry is computed on the host, as
// launch_sk_args does since r6.)
// (argument 4 was the rejected joiner prep, removed from the product kernel in r5; kept as a placeholder)
// Phases per workgroup: start -> (1) prologue + query fragments -> (2) first tile -> (3) second tile -> (4) the rest of
// its tiles -> (5) list merge and write. Printed: min / median / max over the workgroups, and the launch span.
#include "../rag-serving-system_amd/csrc/rr_kernels.hip"
#include "../rag-serving-system_amd/csrc/rr_sk.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);        \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)

using namespace rr;

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 125000;
  int grid = argc > 2 ? atoi(argv[2]) : 256;
  const int ct8 = argc > 3 ? atoi(argv[3]) : 2;
  const int prep = argc > 4 ? atoi(argv[4]) : 0;
  const int guided = argc > 5 ? atoi(argv[5]) : 1;
  const int d = 1024, b = 32;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int64_t r2 = (n + 1) / 2 * 2;
  float *c32, *norms, *q, *sx, *e8, *q8s;
  int8_t *c8, *q8;
  uint64_t* cand;
  uint32_t* ctr;
  CK(hipMalloc(&c32, (size_t)n * d * 4));
  CK(hipMalloc(&c8, (size_t)r2 * d));
  CK(hipMalloc(&sx, (size_t)r2 * 4));
  CK(hipMalloc(&e8, (size_t)r2 * 4));
  CK(hipMalloc(&norms, (size_t)(n + 64) * 4));
  CK(hipMalloc(&q, (size_t)b * d * 4));
  CK(hipMalloc(&q8, (size_t)2 * 64 * d));   // (launch_q8_stage: p1 [64][d], p2 [64][d])
  CK(hipMalloc(&q8s, (size_t)kQ8Scalars * 64 * 4));
  CK(hipMalloc(&cand, (size_t)(grid + 64) * 64 * 32 * 8));
  CK(hipMalloc(&ctr, 512));
  CK(hipMemset(ctr, 0, 512));
  uint64_t* flag;
  CK(hipMalloc(&flag, 8));
  CK(hipMemset(flag, 0, 8));
  CK(hipMemset(c8 + (size_t)n * d, 0, (size_t)(r2 - n) * d));
  CK(launch_synth(1, 1234, 0, n, d, c32, s));
  CK(launch_synth(1, 99, 0, b, d, q, s));
  CK(launch_row_norms(0, c32, n, d, norms, s));
  CK(launch_f32_to_i8(c32, n, d, c8, sx, e8, s));
  CK(launch_q8_stage(q, b, d, q8, 64, q8s, nullptr, s));
  CK(hipStreamSynchronize(s));
  SkArgs a{};
  a.corpus = (const char*)c8;
  a.norms = norms;
  a.queries = q;
  a.n = r2 / 2;
  a.rows8 = n;
  a.d = d;
  a.b = b;
  a.out = cand;
  a.ctr = ctr;
  a.dyn = 1;
  a.sqrt_d = 32.0f * (1.0f + 0x1p-20f);
  a.eps_a = 6e-5f;
  a.eps_b = 4e-8f;
  a.q8 = q8;
  a.q8p2 = q8 + (size_t)64 * d;
  a.q8s = q8s;
  a.q8s_stride = 64;
  a.sx8 = sx;
  a.e8 = e8;
  a.ct8 = ct8;
  const int pieces = argc > 7 ? atoi(argv[7]) : 2;
  auto kern = pieces == 1 ? sk::sk_score_kernel<9, 2, 16, true, 2, 1, 0, 1, 0> : sk::sk_score_kernel<8, 2, 16, true, 2, 1, 0, 1, 0>;
  const int sdt = pieces == 1 ? KDT_SCREEN9 : KDT_SCREEN8;
  const size_t lds = sk_lds_bytes(sdt, true, 2, 32);
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  std::vector<unsigned long long> h((size_t)grid * 8);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  a.no_guided = !guided;
  a.geo = chunk_geo((a.n + 31) / 32, sk_chunk_tiles(sdt, a.d, a.ct8), grid, !a.no_guided);
  a.geo_set = 1;
  for (int rep = 0; rep < 30; ++rep) {
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads + 64), lds, s, a);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
  }
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  if (argc > 6 && atoi(argv[6]) > 0) {
    // back-to-back throughput of the same screen (no prep, no verify): 1 stream vs 2 alternating streams (own counters
    // and candidate buffers), 200 launches each, interleaved twice — the launch-to-launch overlap available per block
    const int nl = 200;
    hipStream_t s2;
    CK(hipStreamCreate(&s2));
    uint32_t* ctr2;
    uint64_t* cand2;
    CK(hipMalloc(&ctr2, 512));
    CK(hipMemset(ctr2, 0, 512));
    CK(hipMalloc(&cand2, (size_t)(grid + 64) * 64 * 32 * 8));
    SkArgs b2 = a;
    b2.ctr = ctr2;
    b2.out = cand2;
    for (int round = 0; round < 2; ++round)
      for (int two = 0; two < 2; ++two) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < nl; ++i) {
          const bool odd = two && (i & 1);
          hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads + 64), lds, odd ? s2 : s, odd ? b2 : a);
        }
        hipEvent_t j;
        CK(hipEventCreate(&j));
        CK(hipEventRecord(j, s2));
        CK(hipStreamWaitEvent(s, j, 0));
        CK(hipEventRecord(e1, s));
        CK(hipDeviceSynchronize());
        float tm = 0;
        CK(hipEventElapsedTime(&tm, e0, e1));
        printf("{\"rows\": %lld, \"grid\": %d, \"streams\": %d, \"us_per_launch\": %.2f}\n", (long long)n, grid,
               two ? 2 : 1, tm * 1e3 / nl);
      }
    return 0;
  }
  CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(rr::sk::probe), h.size() * 8));
  unsigned long long t0min = ~0ull, t0max = 0, t5max = 0;
  for (int g = 0; g < grid; ++g) {
    t0min = std::min(t0min, h[g * 8]);
    t0max = std::max(t0max, h[g * 8]);
    t5max = std::max(t5max, h[g * 8 + 5]);
  }
  unsigned long long hf = 0;
  CK(hipMemcpy(&hf, flag, 8, hipMemcpyDeviceToHost));
  printf("{\"pieces\": %d, \"guided\": %d, \"prep\": %d, \"flag\": %llu, \"rows\": %lld, \"grid\": %d, \"ct8\": %d, \"event_us\": %.2f, \"start_spread_us\": %.2f, \"span_us\": %.2f",
         pieces, guided, prep, hf, (long long)n, grid, ct8, ms * 1e3, (t0max - t0min) / 100.0, (t5max - t0min) / 100.0);
  const char* ph[] = {"prologue", "tile0", "tile1", "rest", "merge"};
  for (int i = 1; i <= 5; ++i) {
    std::vector<double> v;
    for (int g = 0; g < grid; ++g) v.push_back((double)(h[g * 8 + i] - h[g * 8 + i - 1]) / 100.0);
    std::sort(v.begin(), v.end());
    printf(", \"%s_us\": [%.2f, %.2f, %.2f]", ph[i - 1], v[0], v[v.size() / 2], v.back());
  }
  {
    // the prologue's sub-phases: start -> prologue issued (6) -> fragments in registers (7) -> loop start (1)
    const int sub[4] = {0, 6, 7, 1};
    const char* nm[3] = {"issue", "frags", "barrier_scalars"};
    for (int i = 0; i < 3; ++i) {
      std::vector<double> v;
      for (int g = 0; g < grid; ++g) v.push_back((double)(h[g * 8 + sub[i + 1]] - h[g * 8 + sub[i]]) / 100.0);
      std::sort(v.begin(), v.end());
      printf(", \"pro_%s_us\": [%.2f, %.2f, %.2f]", nm[i], v[0], v[v.size() / 2], v.back());
    }
  }
  std::vector<double> st, e;
  for (int g = 0; g < grid; ++g) {
    st.push_back((double)(h[g * 8] - t0min) / 100.0);
    e.push_back((double)(h[g * 8 + 5] - t0min) / 100.0);
  }
  std::sort(e.begin(), e.end());
  std::sort(st.begin(), st.end());
  printf(", \"start_us_p10_p50_p90\": [%.2f, %.2f, %.2f]", st[grid / 10], st[grid / 2], st[grid * 9 / 10]);
  printf(", \"end_us_min_p10_med_p90_max\": [%.2f, %.2f, %.2f, %.2f, %.2f]}\n", e[0], e[grid / 10], e[grid / 2],
         e[grid * 9 / 10], e.back());
  return 0;
}
