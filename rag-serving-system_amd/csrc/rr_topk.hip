// rr_topk.hip — top-k of long key segments, sorted: radix select + compaction + bitonic tiles + rank merges
// (gfx950 / MI355X). Replaces the per-row argpartition + argsort of the reference (retriever.py:118-120 and
// :750-769) on the paths that hold every key of a segment: k > 256, the exact re-run of an unproven large-k search,
// the register-streaming kernel's full-key output, and the serial exchange's merge of world x k candidates.
//
// Keys (rr_kernels.hip): uint64, ord(score) << 32 | (0xFFFFFFFF - index) — unique per segment except 0 (empty). The
// result of segment q is its k largest keys in descending order, padded with 0 when it holds fewer than k non-zero
// keys. Steps (one stream, no host round trip):
//   1. radix select (seg > k only): the k-th largest key T, one byte at a time from the top — per pass a 256-bin
//      histogram of the keys that match the bytes fixed so far (workgroup histograms in LDS, added into a per-segment
//      global one), then one workgroup per segment finds the bin holding the k-th and fixes that byte. Keys are unique,
//      so after the 8 passes T is the k-th key itself (0 when fewer than k keys are non-zero);
//   2. compaction: the non-zero keys >= T (exactly min(k, non-zero) of them) appended to out[q] in any order, the
//      rest of out[q] zero;
//   3. sort: 2048-key tiles sorted descending by a bitonic network in LDS, then merge passes doubling the run length:
//      an element's place in the merged run is its index in its own run plus its rank in the partner run (binary
//      search; ties — only the padding zeros — ordered run A first), so every pass is one independent scatter.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <utility>
#include "rr_internal.h"

namespace rr {
namespace {

constexpr int kTkThreads = 256;
constexpr int kTkPer = 16;                        // keys per thread per select / compaction block step
constexpr int kTile = 2048;                       // keys per bitonic tile (16 KiB of LDS)

struct TkState {
  uint64_t prefix, mask;   // bytes of T fixed so far, and which
  int64_t need;            // rank of T among the keys matching prefix under mask
  int64_t count;           // compaction: keys appended so far
};

// pass over one byte (shift): histogram of byte `shift` of the keys matching the fixed prefix
__global__ __launch_bounds__(kTkThreads) void tk_hist_kernel(const uint64_t* __restrict__ in, int64_t seg,
                                                              const TkState* __restrict__ st,
                                                              unsigned* __restrict__ hist, int shift) {
  const int q = blockIdx.y, tid = threadIdx.x;
  __shared__ unsigned h[256];
  h[tid] = 0;
  __syncthreads();
  const uint64_t prefix = st[q].prefix, mask = st[q].mask;
  const uint64_t* src = in + (size_t)q * seg;
  const int64_t stride = (int64_t)gridDim.x * kTkThreads;
  for (int64_t i = (int64_t)blockIdx.x * kTkThreads + tid; i < seg; i += stride) {
    const uint64_t key = src[i];
    if ((key & mask) == prefix) atomicAdd(&h[(int)(key >> shift) & 255], 1u);
  }
  __syncthreads();
  if (h[tid]) atomicAdd(&hist[(size_t)q * 256 + tid], h[tid]);
}

// one workgroup (64 lanes) per segment: the bin of byte `shift` holding the need-th largest key; clears the histogram
__global__ __launch_bounds__(64) void tk_digit_kernel(TkState* __restrict__ st, unsigned* __restrict__ hist,
                                                       int shift) {
  const int q = blockIdx.x, lane = threadIdx.x;
  unsigned* hq = hist + (size_t)q * 256;
  long long c[4], s4 = 0;   // lane L: bins 255 - 4L .. 252 - 4L, highest first
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = hq[255 - 4 * lane - j];
    s4 += c[j];
  }
  long long incl = s4;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const long long t = __shfl_up(incl, off, 64);
    if (lane >= off) incl += t;
  }
  const long long need = st[q].need;
  long long run = incl - s4;
  if (run < need && need <= incl) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (run < need && need <= run + c[j]) {
        st[q].prefix |= (uint64_t)(255 - 4 * lane - j) << shift;
        st[q].need = need - run;
      }
      run += c[j];
    }
  }
  if (lane == 0) st[q].mask |= (uint64_t)0xFF << shift;
#pragma unroll
  for (int j = 0; j < 4; ++j) hq[4 * lane + j] = 0;
}

__global__ void tk_init_kernel(TkState* __restrict__ st, unsigned* __restrict__ hist, int b, int64_t k, int select) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < b) {
    st[i].prefix = 0;
    st[i].mask = select ? 0 : ~(uint64_t)0;   // no select: T = 0 (every non-zero key)
    st[i].need = k;
    st[i].count = 0;
  }
  if (hist && i < b * 256) hist[i] = 0;
}

// the non-zero keys >= T of segment q into out[q] (any order); out[q] was zeroed
__global__ __launch_bounds__(kTkThreads) void tk_compact_kernel(const uint64_t* __restrict__ in, int64_t seg,
                                                                 TkState* __restrict__ st, uint64_t* __restrict__ out,
                                                                 int64_t k) {
  const int q = blockIdx.y, tid = threadIdx.x;
  const uint64_t t = st[q].prefix & st[q].mask;   // T (0: no select)
  const uint64_t* src = in + (size_t)q * seg;
  uint64_t* dst = out + (size_t)q * k;
  const int64_t stride = (int64_t)gridDim.x * kTkThreads;
  for (int64_t i = (int64_t)blockIdx.x * kTkThreads + tid; i < seg; i += stride) {
    const uint64_t key = src[i];
    if (key != 0 && key >= t) {
      const int64_t pos = (int64_t)atomicAdd((unsigned long long*)&st[q].count, 1ull);
      if (pos < k) dst[pos] = key;
    }
  }
}

__global__ void tk_zero_kernel(uint64_t* __restrict__ p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// bitonic sort (descending) of one 2048-key tile of out[q] in LDS; keys past the segment's end read as 0
__global__ __launch_bounds__(1024) void tk_tile_sort_kernel(uint64_t* __restrict__ keys, int64_t k) {
  const int q = blockIdx.y, tid = threadIdx.x;
  __shared__ uint64_t t[kTile];
  uint64_t* base = keys + (size_t)q * k + (size_t)blockIdx.x * kTile;
  const int64_t n = k - (int64_t)blockIdx.x * kTile;   // valid keys in this tile (> 0)
  for (int i = tid; i < kTile; i += 1024) t[i] = i < n ? base[i] : 0;
  __syncthreads();
  for (int size = 2; size <= kTile; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int i = 2 * tid - (tid & (stride - 1)), j = i + stride;   // tid < kTile / 2 = 1024
      const bool desc = (i & size) == 0;
      const uint64_t x = t[i], y = t[j];
      if ((x < y) == desc) {
        t[i] = y;
        t[j] = x;
      }
      __syncthreads();
    }
  for (int i = tid; i < kTile; i += 1024)
    if (i < n) base[i] = t[i];
}

// merge pass: runs of `run` keys (sorted descending) pairwise into runs of 2 run, src -> dst
__global__ __launch_bounds__(kTkThreads) void tk_merge_kernel(const uint64_t* __restrict__ src,
                                                               uint64_t* __restrict__ dst, int64_t k, int64_t run) {
  const int q = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * kTkThreads + threadIdx.x;
  if (i >= k) return;
  const uint64_t* s = src + (size_t)q * k;
  const int64_t pair0 = i / (2 * run) * (2 * run);
  const int64_t a0 = pair0, a1 = pair0 + run < k ? pair0 + run : k;        // run A = [a0, a1)
  const int64_t b0 = a1, b1 = pair0 + 2 * run < k ? pair0 + 2 * run : k;   // run B = [b0, b1)
  const uint64_t x = s[i];
  int64_t pos;
  if (i < a1) {   // A: B's keys strictly above x come first
    int64_t lo = b0, hi = b1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (s[mid] > x) lo = mid + 1;
      else hi = mid;
    }
    pos = pair0 + (i - a0) + (lo - b0);
  } else {        // B: A's keys at or above x come first
    int64_t lo = a0, hi = a1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (s[mid] >= x) lo = mid + 1;
      else hi = mid;
    }
    pos = pair0 + (i - b0) + (lo - a0);
  }
  dst[(size_t)q * k + pos] = x;
}

}  // namespace

size_t topk_scratch_bytes(int b, int64_t k) {
  return ((size_t)b * sizeof(TkState) + 255) / 256 * 256 + (size_t)b * 256 * 4 + 256 + (size_t)b * k * 8;
}

hipError_t preload_topk() {   // (rr_kernels.hip preload_kernels)
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, (const void*)tk_init_kernel);
}

hipError_t launch_topk_sorted(const uint64_t* in, int b, int64_t seg, int64_t k, uint64_t* out, void* scratch,
                              hipStream_t s) {
  if (b < 1 || seg < 1 || k < 1 || !in || !out || !scratch) return hipErrorInvalidValue;
  TkState* st = (TkState*)scratch;
  unsigned* hist = (unsigned*)((char*)scratch + ((size_t)b * sizeof(TkState) + 255) / 256 * 256);
  uint64_t* tmp = (uint64_t*)((char*)hist + (((size_t)b * 256 * 4 + 255) / 256 * 256));
  const bool select = seg > k;
  hipLaunchKernelGGL(tk_init_kernel, dim3((b * 256 + 255) / 256), dim3(256), 0, s, st, hist, b, k, select ? 1 : 0);
  const int64_t blocks = std::min<int64_t>(1024, (seg + (int64_t)kTkThreads * kTkPer - 1) / ((int64_t)kTkThreads * kTkPer));
  if (select) {
    for (int shift = 56; shift >= 0; shift -= 8) {
      hipLaunchKernelGGL(tk_hist_kernel, dim3((unsigned)blocks, b), dim3(kTkThreads), 0, s, in, seg, st, hist, shift);
      hipLaunchKernelGGL(tk_digit_kernel, dim3(b), dim3(64), 0, s, st, hist, shift);
    }
  }
  const int64_t total = (int64_t)b * k;
  hipLaunchKernelGGL(tk_zero_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, total);
  hipLaunchKernelGGL(tk_compact_kernel, dim3((unsigned)blocks, b), dim3(kTkThreads), 0, s, in, seg, st, out, k);
  const int64_t tiles = (k + kTile - 1) / kTile;
  hipLaunchKernelGGL(tk_tile_sort_kernel, dim3((unsigned)tiles, b), dim3(1024), 0, s, out, k);
  uint64_t* a = out;
  uint64_t* c = tmp;
  for (int64_t run = kTile; run < k; run *= 2) {
    hipLaunchKernelGGL(tk_merge_kernel, dim3((unsigned)((k + kTkThreads - 1) / kTkThreads), b), dim3(kTkThreads), 0,
                       s, a, c, k, run);
    std::swap(a, c);
  }
  if (a != out)   // an odd number of merge passes left the result in the scratch run buffer
    if (hipError_t e = hipMemcpyAsync(out, a, (size_t)total * 8, hipMemcpyDeviceToDevice, s)) return e;
  return hipGetLastError();
}

}  // namespace rr
