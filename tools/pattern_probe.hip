// pattern_probe.hip -- does another wave -> row assignment read the headline's shards faster?  The round
// kernel (4096 workgroups of 4 waves, one worker's 2 MiB shard of 512 rows x 4 KiB each, two workgroups
// per CU by their ~78 KB of LDS, nontemporal 16-byte loads) has wave w stream rows w, w + 4, ... with one
// row ahead in flight; its bare read is 7.15 TB/s (bw_probe.hip).  Variants, same grid and occupancy:
//   interleaved RB rows ahead (the kernel's order), contiguous quarters (wave w: rows [128 w, 128 w + 128)),
//   and the workgroup -> shard map permuted so that the 8 XCDs' concurrent workgroups read neighbouring shards.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/pattern_probe tools/pattern_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));

// MODE 0: interleaved rows (wave w: w, w + 4, ...); 1: contiguous quarters; PERM: shard = XCD-blocked map
template <int MODE, int RB, bool PERM>
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ x, int rows, float* out) {
  extern __shared__ char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int shard = blockIdx.x;
  if (PERM) shard = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const f4* base = x + (size_t)shard * rows * 256;
  f4 acc = f4(0);
  const int q = rows / 4;
  const int r_begin = MODE == 0 ? wave : wave * q;
  const int r_end = MODE == 0 ? rows : (wave + 1) * q;
  const int step = MODE == 0 ? 4 : 1;
  for (int r0 = r_begin; r0 < r_end; r0 += step * RB) {
    f4 v[RB][4];
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = r0 + k * step;
        const f4* p = base + (size_t)(r < r_end ? r : r_end - 1) * 256 + lane + 64 * j;
        v[k][j] = __builtin_nontemporal_load(p);
      }
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += v[k][j];
  }
  if (acc.x == 1234.5f) { lds[threadIdx.x] = 1; out[0] = acc.y + acc.z + acc.w + lds[threadIdx.x ^ 1]; }
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(r_)); exit(1); } } while (0)

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

template <int MODE, int RB, bool PERM>
void arm(const char* name, const f4* x, float* out, size_t bytes, int rep) {
  const size_t lds = 78 * 1024;  // two workgroups per CU, as the round kernel
  CK(hipFuncSetAttribute((const void*)k_read<MODE, RB, PERM>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const float ms = timeit([&] { hipLaunchKernelGGL((k_read<MODE, RB, PERM>), dim3(4096), dim3(256), lds, 0, x, 512, out); }, 5);
  printf("rep %d  %-34s %.4f ms  %.0f GB/s\n", rep, name, ms, bytes / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = 8ull << 30;  // 4096 workers x 512 rows x 4 KiB
  f4* x;
  float* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(x, 0, bytes));
  for (int rep = 0; rep < 3; ++rep) {
    arm<0, 2, false>("interleaved, 2 rows in flight", x, out, bytes, rep);
    arm<0, 4, false>("interleaved, 4 rows in flight", x, out, bytes, rep);
    arm<1, 2, false>("contiguous quarters, 2 in flight", x, out, bytes, rep);
    arm<1, 4, false>("contiguous quarters, 4 in flight", x, out, bytes, rep);
    arm<0, 2, true>("interleaved, XCD-blocked shards", x, out, bytes, rep);
  }
  return 0;
}
