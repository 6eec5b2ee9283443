// ipc_probe.hip -- does the pull transport's synchronisation work on this ROCm, and what does it cost?
// (round 6, DESIGN.md section 6, "A transport without RCCL's kernel").
//
// Two processes on one GPU (forked before any HIP call).  The producer owns a double-buffered device buffer
// and an interprocess event; per round k it fills slot k % 2 with the value k (a kernel), records the event
// and publishes "k records made" in host shared memory.  The consumer opens both handles once; per round it
// waits (host) until the producer has made k records, makes its stream wait on the producer's event, pulls the
// slot into a local buffer (a copy kernel reading the peer's memory, or hipMemcpyAsync), checks every word
// (a kernel counting mismatches) and publishes "round k consumed" so the producer may reuse the slot at k + 2.
// Printed: mismatches (must be 0) and microseconds per round with and without the per-round host sync.
//   hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe tools/ipc_probe.hip && tools/ipc_probe [rounds] [MB]
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      _exit(3);                                                                               \
    }                                                                                         \
  } while (0)

struct Shared {
  hipIpcMemHandle_t mh;
  hipIpcEventHandle_t eh;
  std::atomic<int64_t> ready, rec, ack, done;
};

__global__ void k_fill(uint4* p, int64_t n, unsigned v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(v, v, v, v);
}

__global__ void k_pull(uint4* dst, const uint4* src, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

__global__ void k_check(const uint4* p, int64_t n, unsigned v, unsigned* bad) {
  unsigned b = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 q = p[i];
    b += (q.x != v) + (q.y != v) + (q.z != v) + (q.w != v);
  }
  if (b) atomicAdd(bad, b);
}

static bool spin_until(const std::atomic<int64_t>& a, int64_t want, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  while (a.load(std::memory_order_acquire) < want) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return false;
    std::this_thread::yield();
  }
  return true;
}

static int producer(Shared* sh, int rounds, int64_t n) {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint4* buf;
  CK(hipMalloc(&buf, 2 * n * sizeof(uint4)));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventInterprocess | hipEventDisableTiming));
  CK(hipIpcGetMemHandle(&sh->mh, buf));
  CK(hipIpcGetEventHandle(&sh->eh, ev));
  sh->ready.store(1, std::memory_order_release);
  for (int phase = 0; phase < 2; ++phase) {
    for (int k = 1; k <= rounds; ++k) {
      const int64_t kk = (int64_t)phase * rounds + k;
      if (!spin_until(sh->ack, kk - 2, 30.0)) {
        fprintf(stderr, "producer: consumer stalled at %lld\n", (long long)kk);
        return 4;
      }
      hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, s, buf + (kk & 1) * n, n, (unsigned)kk);
      CK(hipEventRecord(ev, s));
      sh->rec.store(kk, std::memory_order_release);
    }
  }
  if (!spin_until(sh->done, 1, 60.0)) return 5;
  CK(hipStreamSynchronize(s));
  CK(hipFree(buf));
  return 0;
}

static int consumer(Shared* sh, int rounds, int64_t n) {
  if (!spin_until(sh->ready, 1, 60.0)) return 6;
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void* rp;
  CK(hipIpcOpenMemHandle(&rp, sh->mh, hipIpcMemLazyEnablePeerAccess));
  const uint4* remote = (const uint4*)rp;
  hipEvent_t rev;
  CK(hipIpcOpenEventHandle(&rev, sh->eh));
  uint4* local;
  CK(hipMalloc(&local, n * sizeof(uint4)));
  unsigned* bad;
  CK(hipMalloc(&bad, sizeof(unsigned)));
  CK(hipMemset(bad, 0, sizeof(unsigned)));
  unsigned hbad = 0;
  for (int phase = 0; phase < 2; ++phase) {  // 0: pull kernel, per-round host sync; 1: hipMemcpyAsync, no host sync
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 1; k <= rounds; ++k) {
      const int64_t kk = (int64_t)phase * rounds + k;
      if (!spin_until(sh->rec, kk, 30.0)) {
        fprintf(stderr, "consumer: producer stalled at %lld\n", (long long)kk);
        return 7;
      }
      CK(hipStreamWaitEvent(s, rev, 0));
      if (phase == 0)
        hipLaunchKernelGGL(k_pull, dim3(256), dim3(256), 0, s, local, remote + (kk & 1) * n, n);
      else
        CK(hipMemcpyAsync(local, remote + (kk & 1) * n, n * sizeof(uint4), hipMemcpyDeviceToDevice, s));
      hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, s, local, n, (unsigned)kk, bad);
      if (phase == 0 || k == rounds) CK(hipStreamSynchronize(s));
      // (phase 1: the slot may be reused once this round's copy has run; the stream order is enough here as
      // the ack is taken after the previous round's copy only -- a conservative host sync every 2 rounds)
      if (phase == 1 && (k & 1)) CK(hipStreamSynchronize(s));
      sh->ack.store(kk, std::memory_order_release);
    }
    const double us = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6 / rounds;
    CK(hipMemcpy(&hbad, bad, sizeof(unsigned), hipMemcpyDeviceToHost));
    printf("%s: %d rounds of %.2f MB, %.1f us per round, mismatching words so far %u\n",
           phase == 0 ? "pull kernel, host sync per round" : "hipMemcpyAsync, host sync every 2 rounds", rounds,
           n * 16 / 1e6, us, hbad);
  }
  sh->done.store(1, std::memory_order_release);
  CK(hipIpcCloseMemHandle(rp));
  CK(hipEventDestroy(rev));
  return hbad == 0 ? 0 : 8;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 200;
  const double mb = argc > 2 ? atof(argv[2]) : 4.0;
  const int64_t n = (int64_t)(mb * 1e6 / 16);
  void* m = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return 2;
  Shared* sh = new (m) Shared();
  const pid_t pid = fork();  // before any HIP call in either process
  if (pid < 0) return 2;
  if (pid == 0) _exit(producer(sh, rounds, n));
  const int rc = consumer(sh, rounds, n);
  int st = 0;
  waitpid(pid, &st, 0);
  const int prc = WIFEXITED(st) ? WEXITSTATUS(st) : 99;
  printf("consumer rc %d, producer rc %d\n", rc, prc);
  return rc || prc;
}
