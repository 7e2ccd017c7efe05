// api_cost.hip — host cost of the HIP calls a search block enqueues (kernel launch, event record, stream wait on an
// event, event query, set device), each timed over 2000 calls on an otherwise idle high-priority stream pair.
// Development tool: hipcc --offload-arch=gfx950 -O2 tools/api_cost.hip -o tools/api_cost
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

// slot 0: spin `ticks` of the 100 MHz wall clock, then stamp the end; slot 1: stamp the start
__global__ void stamp_kernel(unsigned long long* ts, int slot, unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  if (ticks)
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0 && ts) ts[slot & 1] = wall_clock64();
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
  // the record after a launch on the same stream, vs a launch whose stop event its packet records (hipExtLaunchKernelGGL)
  {
    const double t_launch_record = per_call_us(n, [&](int i) {
      hipLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, a, nullptr);
      (void)hipEventRecord(ev[i & 63], a);
    });
    sync();
    const double t_ext_stop = per_call_us(n, [&](int i) {
      hipExtLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, a, nullptr, ev[i & 63], 0, nullptr);
    });
    sync();
    // a wait on a pending event (recorded behind a 40 us kernel on the other stream), then a launch
    double t_wait_pending = 0;
    for (int rep = 0; rep < 200; ++rep) {
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, (unsigned long long*)nullptr, 2, 4000ull);
      (void)hipEventRecord(ev[rep & 63], a);
      const auto t0 = std::chrono::steady_clock::now();
      (void)hipStreamWaitEvent(b, ev[rep & 63], 0);
      const auto t1 = std::chrono::steady_clock::now();
      t_wait_pending += std::chrono::duration<double, std::micro>(t1 - t0).count();
      hipLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, b, nullptr);
      sync();
    }
    printf("{\"launch_then_record_us\": %.2f, \"ext_launch_with_stop_event_us\": %.2f, \"wait_pending_event_us\": %.2f}\n",
           t_launch_record, t_ext_stop, t_wait_pending / 200);
  }
  // stream memory operations instead of events: hipStreamWriteValue32 on a (after its kernel), hipStreamWaitValue32
  // on b, then a launch on b — host cost per hand-off and the device-side dependency latency
  {
    uint32_t* flag = nullptr;
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    unsigned long long* ts = nullptr;
    CK(hipMalloc(&ts, 64));
    double host = 0, dev = 0;
    for (int rep = 1; rep <= 200; ++rep) {
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 0, 4000ull);
      const auto t0 = std::chrono::steady_clock::now();
      (void)hipStreamWriteValue32(a, flag, (uint32_t)rep, 0);
      (void)hipStreamWaitValue32(b, flag, (uint32_t)rep, hipStreamWaitValueGte, 0xFFFFFFFFu);
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, b, ts, 1, 0ull);
      const auto t1 = std::chrono::steady_clock::now();
      host += std::chrono::duration<double, std::micro>(t1 - t0).count();
      sync();
      unsigned long long h[2];
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      dev += (double)(h[1] - h[0]) / 100.0;
    }
    // the event form of the same hand-off, same shape
    double host_e = 0, dev_e = 0;
    for (int rep = 0; rep < 200; ++rep) {
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 0, 4000ull);
      const auto t0 = std::chrono::steady_clock::now();
      (void)hipEventRecord(ev[rep & 63], a);
      (void)hipStreamWaitEvent(b, ev[rep & 63], 0);
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, b, ts, 1, 0ull);
      const auto t1 = std::chrono::steady_clock::now();
      host_e += std::chrono::duration<double, std::micro>(t1 - t0).count();
      sync();
      unsigned long long h[2];
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      dev_e += (double)(h[1] - h[0]) / 100.0;
    }
    printf("{\"handoff_write_wait_value_host_us\": %.2f, \"handoff_write_wait_value_device_us\": %.2f, "
           "\"handoff_event_host_us\": %.2f, \"handoff_event_device_us\": %.2f}\n",
           host / 200, dev / 200, host_e / 200, dev_e / 200);
  }
  // same-stream gap K1 -> K2 with packets between them: (a) nothing, (b) one event record, (c) two records, (d) a wait
  // on an event of the other stream that completed long ago, (e) a wait on an event of the other stream that completes
  // while K1 still runs (recorded behind a 10 us kernel there)
  {
    unsigned long long* ts = nullptr;
    CK(hipMalloc(&ts, 64));
    double g[5] = {0, 0, 0, 0, 0};
    const int reps = 50;
    for (int rep = 0; rep < reps; ++rep)
      for (int v = 0; v < 5; ++v) {
        if (v == 3) {   // an old event on b, complete
          hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, b, nullptr);
          (void)hipEventRecord(ev[2], b);
          sync();
        }
        hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 0, 4000ull);
        if (v == 1 || v == 2) (void)hipEventRecord(ev[3], a);
        if (v == 2) (void)hipEventRecord(ev[4], a);
        if (v == 3) (void)hipStreamWaitEvent(a, ev[2], 0);
        if (v == 4) {
          hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, b, (unsigned long long*)nullptr, 2, 1000ull);
          (void)hipEventRecord(ev[5], b);
          (void)hipStreamWaitEvent(a, ev[5], 0);
        }
        hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 1, 0ull);
        sync();
        unsigned long long h[2];
        CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
        g[v] += (double)(h[1] - h[0]) / 100.0;
      }
    // (f) K1 launched with its stop event in the launch packet (hipExtLaunchKernelGGL) instead of a separate record
    double gf = 0;
    for (int rep = 0; rep < reps; ++rep) {
      hipExtLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, nullptr, ev[6], 0, ts, 0, 4000ull);
      hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, a, ts, 1, 0ull);
      sync();
      unsigned long long h[2];
      CK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
      gf += (double)(h[1] - h[0]) / 100.0;
    }
    printf("{\"gap_ext_launch_stop_event_us\": %.2f}\n", gf / reps);
    printf("{\"gap_plain_us\": %.2f, \"gap_record_us\": %.2f, \"gap_two_records_us\": %.2f, \"gap_wait_done_event_us\": %.2f, "
           "\"gap_wait_event_done_before_k1_end_us\": %.2f}\n", g[0] / reps, g[1] / reps, g[2] / reps, g[3] / reps, g[4] / reps);
  }
  // hipDeviceSynchronize (torch.cuda.synchronize) after work that has already completed — seen through an event the
  // host polled, as rr_synchronize does — on S streams, the last command on each (0) an event record after a launch,
  // (1) a launch with its stop event in the packet; (2) a plain launch (the host sleeps 200 us instead of polling);
  // (3) as (1), but the host waits with hipEventSynchronize instead of polling hipEventQuery; (4) as (1), polled, then
  // hipEventSynchronize of the (complete) stop events; and hipStreamSynchronize of each instead
  {
    hipStream_t ss[4];
    for (auto& s : ss) CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    hipEvent_t done[4];
    for (auto& e : done) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int mode = 0; mode < 5; ++mode)
      for (int S = 1; S <= 4; S *= 2) {
        double t_dev = 0, t_str = 0;
        const int reps = 100;
        for (int rep = 0; rep < 2 * reps; ++rep) {
          for (int i = 0; i < S; ++i) {
            const bool ext = mode == 1 || mode >= 3;
            if (ext)
              hipExtLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, ss[i], nullptr, done[i], 0, nullptr);
            else
              hipLaunchKernelGGL(empty_kernel, dim3(32), dim3(64), 0, ss[i], nullptr);
            if (mode == 0) (void)hipEventRecord(done[i], ss[i]);
          }
          if (mode == 2) {
            const auto ts = std::chrono::steady_clock::now();
            while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - ts).count() < 200) {
            }
          }
          for (int i = 0; i < S; ++i) {
            if (mode == 3) (void)hipEventSynchronize(done[i]);
            if (mode == 0 || mode == 1 || mode == 4)
              while (hipEventQuery(done[i]) != hipSuccess) {
              }
            if (mode == 4) (void)hipEventSynchronize(done[i]);
          }
          const auto t0 = std::chrono::steady_clock::now();
          if (rep & 1) {
            (void)hipDeviceSynchronize();
          } else {
            for (int i = 0; i < S; ++i) (void)hipStreamSynchronize(ss[i]);
          }
          const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
          (rep & 1 ? t_dev : t_str) += us;
          CK(hipDeviceSynchronize());
        }
        printf("{\"sync_after_done_mode\": %d, \"streams\": %d, \"device_sync_us\": %.2f, \"stream_syncs_us\": %.2f}\n",
               mode, S, t_dev / reps, t_str / reps);
      }
  }
  printf("{\"launch_us\": %.2f, \"launch_224x576_us\": %.2f, \"event_record_us\": %.2f, \"stream_wait_event_us\": %.2f, "
         "\"event_query_us\": %.2f, \"set_device_us\": %.2f, \"get_last_error_us\": %.3f, \"record_wait_launch_us\": %.2f}\n",
         t_launch, t_launch_big, t_record, t_wait, t_query, t_setdev, t_lasterr, t_handoff);
  return 0;
}
