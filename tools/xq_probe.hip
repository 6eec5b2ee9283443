// xq_probe.hip -- what a cross-stream hand-off costs on this ROCm (round 6, DESIGN.md section 6: the
// strong-leg rank loses ~15 us per round between the gradient kernel's end and k_mixcs, the engine stream's
// wait for the exchange recorded on the side stream, and ~7 us between k_mixcs and the next gradient kernel,
// where an event is recorded for the side stream).
//
// Single-workgroup kernels stamp the device's constant 100 MHz clock (s_memrealtime) at their start and end
// into a device buffer, so a gap is measured on the GPU's own clock with no profiler.  Scenarios, each
// repeated REPS times after a warmup, medians printed (us):
//   same      A: K1 (long) -> K3                         gap = K3.start - K1.end (same-stream boundary)
//   rec       A: K1 -> event record -> K3                gap = K3.start - K1.end (the fork's record)
//   early     B: K2 (short) -> record; A: K1 -> wait -> K3; K2 ends long before K1: gap = K3.start - K1.end
//   late      B: K2 (longer than K1) -> record; A: K1 -> wait -> K3: gap = K3.start - K2.end
// for events created with the flags given on the command line (default, disable-timing, no system fence,
// release to device) and streams created non-blocking at normal / high priority.
//   hipcc --offload-arch=gfx950 -O2 -o tools/xq_probe tools/xq_probe.hip && tools/xq_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

// Spin for `ticks` of the 100 MHz clock, stamping start / end into st[2 * slot], st[2 * slot + 1] (lane 0 of
// wave 0 only, vector stores).  ticks = 0: a trivial kernel.
__global__ void k_spin(unsigned long long ticks, unsigned long long* st, int slot) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    __hip_atomic_store(st + 2 * slot, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(st + 2 * slot + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const unsigned long long long_ticks = 15000;  // 150 us
  CK(hipSetDevice(0));
  unsigned long long* st;
  CK(hipMalloc(&st, 4096 * sizeof(unsigned long long)));
  std::vector<unsigned long long> h(4096);
  struct EvKind {
    const char* name;
    unsigned flags;
  } evk[] = {{"default", hipEventDefault},
             {"disable_timing", hipEventDisableTiming},
             {"no_sys_fence", hipEventDisableTiming | hipEventDisableSystemFence},
             {"release_to_device", hipEventDisableTiming | hipEventReleaseToDevice}};
  struct StKind {
    const char* name;
    int prio_a, prio_b;
  } stk[] = {{"normal/normal", 0, 0}, {"high/normal", -1, 0}, {"normal/high", 0, -1}};
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  printf("# stream priority range %d..%d; reps %d; gaps in us (median over reps)\n", lo, hi, reps);
  for (const StKind& sk : stk) {
    hipStream_t A, B;
    CK(hipStreamCreateWithPriority(&A, hipStreamNonBlocking, sk.prio_a < 0 ? hi : lo));
    CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, sk.prio_b < 0 ? hi : lo));
    for (const EvKind& ek : evk) {
      hipEvent_t ev;
      CK(hipEventCreateWithFlags(&ev, ek.flags));
      std::vector<double> g_same, g_rec, g_early, g_late;
      for (int r = -3; r < reps; ++r) {
        // same: K1 -> K3 on A
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, long_ticks, st, 0);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, 0ull, st, 1);
        // rec: K1 -> record -> K3 on A
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, long_ticks, st, 2);
        CK(hipEventRecord(ev, A));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, 0ull, st, 3);
        CK(hipStreamSynchronize(A));
        // early: B: K2 short -> record; A: K1 -> wait -> K3
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, B, 1000ull, st, 4);
        CK(hipEventRecord(ev, B));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, long_ticks, st, 5);
        CK(hipStreamWaitEvent(A, ev, 0));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, 0ull, st, 6);
        CK(hipStreamSynchronize(A));
        CK(hipStreamSynchronize(B));
        // late: B: K2 longer than K1 -> record; A: K1 -> wait -> K3
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, B, long_ticks + 3000, st, 7);
        CK(hipEventRecord(ev, B));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, long_ticks, st, 8);
        CK(hipStreamWaitEvent(A, ev, 0));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, A, 0ull, st, 9);
        CK(hipStreamSynchronize(A));
        CK(hipStreamSynchronize(B));
        CK(hipMemcpy(h.data(), st, 20 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (r < 0) continue;
        auto us = [&](int a, int b) { return ((double)h[a] - (double)h[b]) / 100.0; };  // 100 MHz ticks
        g_same.push_back(us(2 * 1, 2 * 0 + 1));
        g_rec.push_back(us(2 * 3, 2 * 2 + 1));
        g_early.push_back(us(2 * 6, 2 * 5 + 1));
        g_late.push_back(us(2 * 9, 2 * 7 + 1));
      }
      printf("streams %-13s event %-17s same %6.2f  rec %6.2f  early %6.2f  late %6.2f\n", sk.name, ek.name,
             med(g_same), med(g_rec), med(g_early), med(g_late));
      CK(hipEventDestroy(ev));
    }
    CK(hipStreamDestroy(A));
    CK(hipStreamDestroy(B));
  }
  CK(hipFree(st));
  return 0;
}
