// api_cost.hip — host cost of the HIP calls a search block enqueues (kernel launch, event record, stream wait on an
// event, event query, set device), each timed over 2000 calls on an otherwise idle high-priority stream pair.
// Development tool: hipcc --offload-arch=gfx950 -O2 tools/api_cost.hip -o tools/api_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

// slot 0: spin `ticks` of the 100 MHz wall clock, then stamp the end; slot 1: stamp the start
__global__ void stamp_kernel(unsigned long long* ts, int slot, unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  if (ticks)
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) ts[slot] = wall_clock64();
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;
}

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
      return 2;                                                                           \
    }                                                                                     \
  } while (0)

template <class F>
double per_call_us(int n, F f) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f(i);
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t a, b;
  CK(hipStreamCreateWithPriority(&a, hipStreamNonBlocking, hi));
  CK(hipStreamCreateWithPriority(&b, hipStreamNonBlocking, hi));
  hipEvent_t ev[64];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const int n = 2000;
  // warm up
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, a, nullptr);
  CK(hipDeviceSynchronize());
  auto sync = [&]() { (void)hipStreamSynchronize(a); (void)hipStreamSynchronize(b); };
  const double t_launch = per_call_us(n, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, a, nullptr); });
  sync();
  const double t_launch_big =
      per_call_us(n, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(224), dim3(576), 0, a, nullptr); });
  sync();
  const double t_record = per_call_us(n, [&](int i) { (void)hipEventRecord(ev[i & 63], a); });
  sync();
  const double t_wait = per_call_us(n, [&](int i) { (void)hipStreamWaitEvent(b, ev[i & 63], 0); });
  sync();
  const double t_query = per_call_us(n, [&](int i) { (void)hipEventQuery(ev[i & 63]); });
  const double t_setdev = per_call_us(n, [&](int) { (void)hipSetDevice(0); });
  const double t_lasterr = per_call_us(n, [&](int) { (void)hipGetLastError(); });
  // a block's shape: record on a, wait on b, launch on b (the cross-stream hand-off)
  const double t_handoff = per_call_us(n, [&](int i) {
    (void)hipEventRecord(ev[i & 63], a);
    (void)hipStreamWaitEvent(b, ev[i & 63], 0);
    hipLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, b, nullptr);
  });
  sync();
  // device-side dependency latency: K1 (spins ~40 us, then stamps its end) -> K2 (stamps its start), on the same
  // stream vs across streams through an event; wall clock at 100 MHz
  {
    unsigned long long* ts = nullptr;
    CK(hipMalloc(&ts, 64));
    double same = 0, cross = 0;
    for (int rep = 0; rep < 20; ++rep) {
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 0, 4000ull);
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 1, 0ull);
      sync();
      unsigned long long h[2];
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      same += (double)(h[1] - h[0]) / 100.0;
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 0, 4000ull);
      (void)hipEventRecord(ev[1], a);
      (void)hipStreamWaitEvent(b, ev[1], 0);
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, b, ts, 1, 0ull);
      sync();
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      cross += (double)(h[1] - h[0]) / 100.0;
    }
    printf("{\"dep_latency_same_stream_us\": %.2f, \"dep_latency_cross_stream_event_us\": %.2f}\n", same / 20, cross / 20);
  }
  printf("{\"launch_us\": %.2f, \"launch_224x576_us\": %.2f, \"event_record_us\": %.2f, \"stream_wait_event_us\": %.2f, "
         "\"event_query_us\": %.2f, \"set_device_us\": %.2f, \"get_last_error_us\": %.3f, \"record_wait_launch_us\": %.2f}\n",
         t_launch, t_launch_big, t_record, t_wait, t_query, t_setdev, t_lasterr, t_handoff);
  return 0;
}
