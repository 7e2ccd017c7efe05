// verify_probe.hip — per-phase timestamps of the screened search's verify kernel (development probe).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DRR_SK_PROBE -I include -I rag-serving-system_amd/csrc \
//         tools/verify_probe.hip -o tools/verify_probe && tools/verify_probe [n_docs] [int8=1]
// int8 = 1: the verify of an int8 screen (DT 8 over the int8 copy, wide phase on) — the headline path; 0: the DT 6 screen.
#include "../rag-serving-system_amd/csrc/rr_kernels.hip"
#define RR_SK_ONE_UNIT   // (every split-K instantiation in this unit: rr_sk.hip includes rr_sk_fam_*.hip)
#include "../rag-serving-system_amd/csrc/rr_sk.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);          \
      exit(2);                                                                                    \
    }                                                                                             \
  } while (0)

using namespace rr;

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int i8 = argc > 2 ? atoi(argv[2]) : 1;
  const int d = 1024, b = 32, k = 5;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float *tmp, *c32, *norms, *q, *osc;
  int64_t* oix;
  uint64_t *cand, *flag;
  int* count;
  CK(hipMalloc(&tmp, (size_t)n * d * 4));
  CK(hipMalloc(&c32, (size_t)n * d * 4));
  CK(hipMalloc(&norms, (size_t)(n + 64) * 4));
  CK(hipMalloc(&q, (size_t)b * d * 4));
  CK(hipMalloc(&osc, b * k * 4));
  CK(hipMalloc(&oix, b * k * 8));
  CK(hipMalloc(&cand, (size_t)cus * 32 * 32 * 8));
  CK(hipMalloc(&flag, 64));
  CK(hipMalloc(&count, 64));
  CK(hipMemset(flag, 0, 64));
  CK(launch_synth(1, 1234, 0, n, d, tmp, s));
  CK(launch_permute_f32(tmp, c32, n, d, 0, s));
  CK(launch_row_norms(0, c32, n, d, norms, s));
  CK(launch_synth(1, 99, 0, b, d, q, s));
  const int64_t r2 = (n + 1) / 2 * 2;
  int8_t *c8, *q8;
  float *sx, *e8, *q8s;
  uint32_t* ctr;
  int* wcount;
  CK(hipMalloc(&c8, (size_t)r2 * d));
  CK(hipMalloc(&sx, (size_t)r2 * 4));
  CK(hipMalloc(&e8, (size_t)r2 * 4));
  CK(hipMalloc(&q8, (size_t)2 * 64 * d));   // (launch_q8_stage: p1 [64][d], p2 [64][d])
  CK(hipMalloc(&q8s, (size_t)kQ8Scalars * 64 * 4));
  CK(hipMalloc(&ctr, 512));
  CK(hipMalloc(&wcount, 64));
  CK(hipMemset(ctr, 0, 512));
  CK(hipMemset(wcount, 0, 64));
  CK(hipMemset(c8 + (size_t)n * d, 0, (size_t)(r2 - n) * d));
  CK(hipMemset(sx + n, 0, (size_t)(r2 - n) * 4));
  CK(hipMemset(e8 + n, 0, (size_t)(r2 - n) * 4));
  CK(launch_f32_to_i8(tmp, n, d, c8, sx, e8, s));
  CK(launch_q8_stage(q, b, d, q8, 64, q8s, nullptr, s));
  CK(hipStreamSynchronize(s));
  SkArgs a{};
  a.corpus = (const char*)c32; a.norms = norms; a.queries = q; a.n = n; a.d = d; a.b = b; a.out = cand;
  a.eps_a = 6e-4f; a.eps_b = 4e-8f; a.sqrt_d = 32.0f;
  SkArgs v = a;
  v.vin = cand; v.nlists = cus; v.k_out = k; v.out_scores = osc; v.out_idx = oix; v.flag = flag; v.count = count;
  v.wide_verify = 1;
  v.wide_count = wcount;
  if (i8) {
    a.corpus = (const char*)c8; a.n = (n + 1) / 2; a.rows8 = n; a.q8 = q8; a.q8p2 = q8 + (size_t)64 * d; a.q8s = q8s; a.q8s_stride = 64; a.sx8 = sx; a.e8 = e8; a.ct8 = 2;
    a.eps_a = 6.0e-5f; a.eps_b = 4.0e-8f; a.sqrt_d = 32.0f * (1.0f + 0x1p-20f); a.ctr = ctr; a.dyn = 1;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> h((size_t)32 * 8);
  for (int rep = 0; rep < 6; ++rep) {
    v.seq = rep + 1;
    // (the product's instantiations, launched directly: this probe builds without the dispatch table)
    if (i8) CK((sk::launch_t<8, 2, 16, true, 2, 1, 0, 1, 0>(cus, a, s)));
    else CK((sk::launch_t<6, 4, 16, true, 2, 1, 0, 0, 0>(cus, a, s)));
    CK(hipEventRecord(e0, s));
    CK((sk::launch_t<3, 4, 16, true, 2, 1, 1, 0, 0>(32, v, s)));
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(rr::sk::probe), h.size() * 8));
    unsigned long long t0 = ~0ull;
    for (int g = 0; g < 32; ++g) t0 = std::min(t0, h[g * 8]);
    int wc = 0;
    CK(hipMemcpy(&wc, wcount, 4, hipMemcpyDeviceToHost));
    printf("{\"rows\": %lld, \"int8\": %d, \"rep\": %d, \"verify_event_us\": %.1f, \"wide_slots_total\": %d", (long long)n,
           i8, rep, ms * 1e3, wc);
    const int order[] = {0, 6, 7, 3, 1, 2, 4, 5};
    const char* nm[] = {"start", "frags_norms", "merged", "rows_known", "loop_start", "tile_done", "loop_end", "end"};
    for (int i = 0; i < 8; ++i) {
      std::vector<double> x;
      for (int g = 0; g < 32; ++g)
        if (order[i] != 5 || g < 4) x.push_back((h[g * 8 + order[i]] - t0) / 100.0);
      std::sort(x.begin(), x.end());
      printf(", \"%s_us\": [%.2f, %.2f]", nm[i], x[x.size() / 2], x.back());
    }
    std::vector<unsigned long long> h2((size_t)32 * 8);
    CK(hipMemcpyFromSymbol(h2.data(), HIP_SYMBOL(rr::sk::probe2), h2.size() * 8));
    const char* nm2[] = {"m_lists_loaded", "m_heads", "m_H", "m_cands"};
    for (int i = 0; i < 4; ++i) {
      std::vector<double> x;
      for (int g = 0; g < 32; ++g) x.push_back((h2[g * 8 + i] - t0) / 100.0);
      std::sort(x.begin(), x.end());
      printf(", \"%s_us\": [%.2f, %.2f]", nm2[i], x[x.size() / 2], x.back());
    }
    printf("}\n");
  }
  return 0;
}
