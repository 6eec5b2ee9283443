// rccl_probe.cpp -- what does one exchange cost the host when the engine calls RCCL itself?  The lagged
// schedule's exchange goes through torch's process group (`alltoall_base`: 22 us of host time per round,
// profiles/r5_host_probe.txt).  This probe times RCCL's own group call at world 1 (sends to the rank itself,
// the only form one GPU allows): ncclGroupStart, `ops` send/recv pairs over slices of the buffer,
// ncclGroupEnd, on a caller-owned stream -- host microseconds per call, and the device time of one exchange.
// Build: hipcc -O2 -o tools/rccl_probe tools/rccl_probe.cpp -I/opt/rocm/include/rccl -L/opt/rocm/lib -lrccl
#include <hip/hip_runtime.h>
#include <rccl.h>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(r_), __LINE__); exit(1); } } while (0)
#define NK(e) do { ncclResult_t r_ = (e); if (r_ != ncclSuccess) { printf("RCCL %s line %d\n", ncclGetErrorString(r_), __LINE__); exit(1); } } while (0)

static void exchange(ncclComm_t comm, hipStream_t s, const char* sb, char* rb, size_t bytes, int ops) {
  const size_t part = bytes / ops;
  NK(ncclGroupStart());
  for (int k = 0; k < ops; ++k) {
    NK(ncclSend(sb + k * part, part, ncclInt8, 0, comm, s));
    NK(ncclRecv(rb + k * part, part, ncclInt8, 0, comm, s));
  }
  NK(ncclGroupEnd());
}

int main() {
  CK(hipSetDevice(0));
  ncclUniqueId id;
  NK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NK(ncclCommInitRank(&comm, 1, id, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = 28ull << 20;
  char *sb, *rb;
  CK(hipMalloc(&sb, maxb));
  CK(hipMalloc(&rb, maxb));
  CK(hipMemset(sb, 1, maxb));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const size_t sizes[] = {64 << 10, 3538944, 27557888};  // tiny; the strong leg's 432 rows; the weak leg's 3364 rows (8 KiB each)
  for (size_t bytes : sizes)
    for (int ops : {1, 7}) {
      for (int w = 0; w < 20; ++w) exchange(comm, s, sb, rb, bytes, ops);
      CK(hipStreamSynchronize(s));
      double host = 0;
      const int reps = 400, per = 20;
      for (int r = 0; r < reps; r += per) {
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < per; ++k) exchange(comm, s, sb, rb, bytes, ops);
        host += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CK(hipStreamSynchronize(s));
      }
      float best = 1e30f, sum = 0;
      for (int r = 0; r < 50; ++r) {
        CK(hipEventRecord(a, s));
        exchange(comm, s, sb, rb, bytes, ops);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        sum += ms;
        if (ms < best) best = ms;
      }
      printf("bytes %9zu  ops %d  host %6.2f us/call  device best %7.2f us  mean %7.2f us\n", bytes, ops,
             host / reps * 1e6, best * 1e3, sum / 50 * 1e3);
    }
  NK(ncclCommDestroy(comm));
  return 0;
}
