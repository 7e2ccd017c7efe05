// hbm_ceiling.hip — the streaming-read ceilings the split-K kernels are judged against: how fast MI355X
// reads an fp32 corpus of 1M x 1024 (4.1 GB) with (a) plain float4 loads, (b) non-temporal float4 loads, (c) the
// product kernels' own movement — 4-KiB slabs of 32 rows x 128 contiguous bytes per wave by `global_load_lds_dwordx4
// ... nt` into an LDS ring, one slab in flight per wave beside the one read (two slots; also three and four slots),
// one 512-thread workgroup per CU — with no arithmetic, and
// (d) a float4 copy (read + write, the number MI355X_MICROARCH.md quotes). Development tool, not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/hbm_ceiling.hip -o tools/hbm_ceiling && tools/hbm_ceiling [rows] [reps]
//
// Prints one JSON object: GB/s and the fraction of 8 TB/s per pattern (median of reps launches, HIP events).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// (a) / (b): grid-stride float4 reads, 8 in flight per lane, XOR-reduced into one word per thread (nothing dead)
template <bool NT>
__global__ __launch_bounds__(512) void read_f4(const u32x4* __restrict__ c, int64_t n16, unsigned* out) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  int64_t i = tid;
  for (; i + 7 * nth < n16; i += 8 * nth) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = NT ? __builtin_nontemporal_load(c + i + u * nth) : c[i + u * nth];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += nth) {
    const u32x4 v = c[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[tid] = acc;
}

// (d): float4 copy
__global__ __launch_bounds__(512) void copy_f4(const u32x4* __restrict__ c, u32x4* __restrict__ o, int64_t n16) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = tid; i < n16; i += nth) o[i] = c[i];
}

// (c): the split-K kernels' corpus movement without their arithmetic. Rows of `row_bytes`; wave w of the workgroup owns
// bytes [w KS, (w + 1) KS) of every row (KS = row_bytes / 8), moved as NS slabs of 32 rows x 128 B; instruction i of a
// slab covers rows 8 i + lane / 8, 16-byte column (lane % 8) ^ (lane / 8) — the swizzled LDS image. Two slab slots per
// wave, the next slab issued before waiting for the current one (vmcnt 4). Workgroup g streams rows [g per, (g+1) per).
__device__ __forceinline__ void glds16_nt(const void* src, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}
template <int SLOTS>
__global__ __launch_bounds__(512) void lds_dma_stream(const char* __restrict__ c, int64_t rows, int row_bytes,
                                                      unsigned* out) {
  // SLOTS slab slots per wave, SLOTS - 1 slabs in flight while one is read (the product kernels: 2 slots, the next
  // slab issued into the other before waiting; here also 3 and 4)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KS = row_bytes / 8, NS = KS / 128;
  const int64_t per = (rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = r0 + per < rows ? r0 + per : rows;
  const unsigned ring = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(smem + (size_t)w * SLOTS * 4096));
  const int rl = lane >> 3, cl = lane & 7;
  const char* src0 = c + (size_t)w * KS + ((cl ^ rl) << 4);
  const int64_t nslabs = (r1 - r0 + 31) / 32 * NS;   // slab s: tile s / NS, K-part s % NS
  auto issue = [&](int64_t sidx, int slot) {
    const int64_t base = r0 + sidx / NS * 32;
    const int j = (int)(sidx % NS);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t row = base + 8 * i + rl;
      row = row < r1 ? row : r1 - 1;
      glds16_nt(src0 + row * row_bytes + j * 128, ring + slot * 4096 + i * 1024);
    }
  };
  unsigned acc = 0;
  for (int p = 0; p < SLOTS - 1; ++p)
    if (p < nslabs) issue(p, p);
  for (int64_t sidx = 0; sidx < nslabs; ++sidx) {
    const int slot = (int)(sidx % SLOTS);
    const int64_t nx = sidx + SLOTS - 1;
    if (nx < nslabs) issue(nx, (int)(nx % SLOTS));
    // in flight after this slab: min(SLOTS - 1, slabs left after it), 4 instructions each
    const int64_t after = nslabs - 1 - sidx < SLOTS - 1 ? nslabs - 1 - sidx : SLOTS - 1;
    if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc ^= *(const unsigned*)(smem + (size_t)w * SLOTS * 4096 + slot * 4096 + lane * 64);   // one word per lane read
  }
  out[(size_t)blockIdx.x * 512 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 1000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int d = 1024, row_bytes = d * 4;
  const size_t bytes = (size_t)rows * row_bytes;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  char *c = nullptr, *o = nullptr;
  unsigned* out = nullptr;
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&o, bytes));
  CK(hipMalloc(&out, (size_t)64 << 20));
  CK(hipMemset(c, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_it = [&](auto&& launch) {
    std::vector<float> ms;
    for (int r = 0; r < reps + 3; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0.f;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r >= 3) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
  };
  const int64_t n16 = (int64_t)(bytes / 16);
  const int grid = cus * 8;   // 8 workgroups of 512 per CU for the register loads
  const float t_plain = time_it([&] { hipLaunchKernelGGL(read_f4<false>, dim3(grid), dim3(512), 0, 0, (const u32x4*)c, n16, out); });
  const float t_nt = time_it([&] { hipLaunchKernelGGL(read_f4<true>, dim3(grid), dim3(512), 0, 0, (const u32x4*)c, n16, out); });
  float t_dma[3];
  auto dma = [&](auto kern, int slots, float* t) {
    const int lds = 8 * slots * 4096;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    *t = time_it([&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(512), lds, 0, (const char*)c, rows, row_bytes, out); });
  };
  dma(lds_dma_stream<2>, 2, &t_dma[0]);
  dma(lds_dma_stream<3>, 3, &t_dma[1]);
  dma(lds_dma_stream<4>, 4, &t_dma[2]);
  const float t_copy = time_it([&] { hipLaunchKernelGGL(copy_f4, dim3(grid), dim3(512), 0, 0, (const u32x4*)c, (u32x4*)o, n16); });
  CK(hipGetLastError());
  auto gbs = [&](float ms, double b) { return b / (ms * 1e-3) / 1e9; };
  printf("{\"rows\": %lld, \"bytes\": %zu, \"cus\": %d, \"reps\": %d, "
         "\"read_plain_float4\": {\"us\": %.1f, \"GBps\": %.0f, \"frac_8TBps\": %.4f}, "
         "\"read_nt_float4\": {\"us\": %.1f, \"GBps\": %.0f, \"frac_8TBps\": %.4f}, "
         "\"lds_dma_nt_slabs_one_wg_per_cu\": {\"us\": %.1f, \"GBps\": %.0f, \"frac_8TBps\": %.4f}, "
         "\"lds_dma_3_slots\": {\"us\": %.1f, \"GBps\": %.0f, \"frac_8TBps\": %.4f}, "
         "\"lds_dma_4_slots\": {\"us\": %.1f, \"GBps\": %.0f, \"frac_8TBps\": %.4f}, "
         "\"copy_float4_read_plus_write\": {\"us\": %.1f, \"GBps\": %.0f, \"frac_8TBps\": %.4f}}\n",
         (long long)rows, bytes, cus, reps, t_plain * 1e3, gbs(t_plain, bytes), gbs(t_plain, bytes) / 8000.0,
         t_nt * 1e3, gbs(t_nt, bytes), gbs(t_nt, bytes) / 8000.0, t_dma[0] * 1e3, gbs(t_dma[0], bytes),
         gbs(t_dma[0], bytes) / 8000.0, t_dma[1] * 1e3, gbs(t_dma[1], bytes), gbs(t_dma[1], bytes) / 8000.0,
         t_dma[2] * 1e3, gbs(t_dma[2], bytes), gbs(t_dma[2], bytes) / 8000.0,
         t_copy * 1e3, gbs(t_copy, 2.0 * bytes), gbs(t_copy, 2.0 * bytes) / 8000.0);
  return 0;
}
