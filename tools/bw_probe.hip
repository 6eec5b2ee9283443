// bw_probe.hip -- HBM read-bandwidth ceiling on this MI355X for the access shape the
// D-SGD round uses (whole 4 KiB rows, 16-byte lanes, one workgroup per 2 MiB shard).
// Build: hipcc --offload-arch=gfx950 -O3 -o bw_probe bw_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int RB, bool NT>
__global__ __launch_bounds__(256) void k_shard_read(const f4* __restrict__ x, int rows_per_wg, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = x + (size_t)blockIdx.x * rows_per_wg * 256;
  f4 acc = f4(0);
  for (int r0 = wave * RB; r0 < rows_per_wg; r0 += 4 * RB) {
    f4 v[RB][4];
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f4* p = base + (size_t)(r0 + k) * 256 + lane + 64 * j;
        v[k][j] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += v[k][j];
  }
  if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}

// Occupancy / workgroup-shape sweep: W waves per workgroup, NT loads, RB rows in flight;
// the resident workgroups per CU are capped with dynamic LDS (the round kernel holds
// 4 waves per SIMD, i.e. 2 workgroups of 8 waves).
template <int W, int RB>
__global__ __launch_bounds__(W * 64) void k_shard_read_w(const f4* __restrict__ x, int rows_per_wg, float* out) {
  extern __shared__ char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = x + (size_t)blockIdx.x * rows_per_wg * 256;
  f4 acc = f4(0);
  for (int r0 = wave * RB; r0 < rows_per_wg; r0 += W * RB) {
    f4 v[RB][4];
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[k][j] = __builtin_nontemporal_load(base + (size_t)(r0 + k) * 256 + lane + 64 * j);
#pragma unroll
    for (int k = 0; k < RB; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += v[k][j];
  }
  if (acc.x == 1234.5f) { lds[threadIdx.x] = 1; out[0] = acc.y + acc.z + acc.w + lds[threadIdx.x ^ 1]; }
}

// C5's stream shape: every workgroup reads 17 rows' segments per 1 KiB column block and (WR)
// writes one 1 KiB segment -- 94 % reads, 6 % writes interleaved -- vs the same reads alone.
// x: [n_wg][17][cols] f4 rows, y: [n_wg][cols] f4.
// WR = 2: the written segments are gathered in LDS and leave in 16 KiB bursts (16 blocks).
template <int WR>
__global__ __launch_bounds__(256) void k_c5_stream(const f4* __restrict__ x, f4* __restrict__ y, int cols,
                                                   float* out) {
  __shared__ f4 wbuf[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4* base = x + (size_t)blockIdx.x * 17 * cols;
  f4 acc = f4(0);
  for (int cb = 0; cb < cols; cb += 64) {
    f4 v[5];
#pragma unroll
    for (int r = 0; r < 5; ++r) {  // waves 0..3 read rows wave, wave+4, ... (17 rows; wave 0 the 17th)
      const int row = wave + 4 * r;
      const f4* p = base + (size_t)row * cols + cb + lane;
      v[r] = row < 17 ? (WR >= 3 ? *p : __builtin_nontemporal_load(p)) : f4(0);
    }
#pragma unroll
    for (int r = 0; r < 5; ++r) acc += v[r];
    if ((WR == 1 || WR == 4) && wave == 0) y[(size_t)blockIdx.x * cols + cb + lane] = acc;
    if (WR == 5 && wave == 0) __builtin_nontemporal_store(acc, y + (size_t)blockIdx.x * cols + cb + lane);
    if (WR == 2 && wave == 0) {
      const int k = (cb >> 6) & 15;
      wbuf[k][lane] = acc;
      if (k == 15 || cb + 64 >= cols) {
        const int cb0 = cb - 64 * k;
        for (int q = 0; q <= k; ++q) y[(size_t)blockIdx.x * cols + cb0 + 64 * q + lane] = wbuf[q][lane];
      }
    }
  }
  if (acc.x == 1234.5f) out[0] = acc.y + acc.z + acc.w;
}

__global__ __launch_bounds__(256) void k_grid_read(const f4* __restrict__ x, size_t n, float* out) {
  f4 acc = f4(0);
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    f4 a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
    acc += a + b + c + d;
  }
  for (; i < n; i += stride) acc += x[i];
  if (acc.x == 1234.5f) out[0] = acc.y;
}

__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ x, f4* __restrict__ y, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) y[i] = x[i];
}

#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("HIP %s\n", hipGetErrorString(r)); exit(1); } } while (0)

template <typename F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
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

int main() {
  const size_t bytes = 8ull << 30;  // 8 GiB = 4096 workers x 512 rows x 4 KiB
  const size_t n4 = bytes / 16;
  f4 *x, *y;
  float* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes / 4));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(x, 0, bytes));
  const int wg = 4096, rpw = 512;
  auto gbs = [&](double ms, size_t b) { return b / (ms * 1e-3) / 1e9; };
  double ms;
  ms = timeit([&] { hipLaunchKernelGGL((k_shard_read<2, false>), dim3(wg), dim3(256), 0, 0, x, rpw, out); }, 5);
  printf("shard_read RB=2        %.3f ms  %.0f GB/s\n", ms, gbs(ms, bytes));
  ms = timeit([&] { hipLaunchKernelGGL((k_shard_read<2, true>), dim3(wg), dim3(256), 0, 0, x, rpw, out); }, 5);
  printf("shard_read RB=2 nt     %.3f ms  %.0f GB/s\n", ms, gbs(ms, bytes));
  ms = timeit([&] { hipLaunchKernelGGL((k_shard_read<4, false>), dim3(wg), dim3(256), 0, 0, x, rpw, out); }, 5);
  printf("shard_read RB=4        %.3f ms  %.0f GB/s\n", ms, gbs(ms, bytes));
  ms = timeit([&] { hipLaunchKernelGGL((k_shard_read<1, false>), dim3(wg), dim3(256), 0, 0, x, rpw, out); }, 5);
  printf("shard_read RB=1        %.3f ms  %.0f GB/s\n", ms, gbs(ms, bytes));
  // finer shards: same bytes, 8192 workgroups of 256 rows
  ms = timeit([&] { hipLaunchKernelGGL((k_shard_read<2, false>), dim3(wg * 2), dim3(256), 0, 0, x, rpw / 2, out); }, 5);
  printf("shard_read RB=2 x2 WGs %.3f ms  %.0f GB/s\n", ms, gbs(ms, bytes));
  for (int g : {1024, 2048, 4096, 8192}) {
    ms = timeit([&] { hipLaunchKernelGGL(k_grid_read, dim3(g), dim3(256), 0, 0, x, n4, out); }, 5);
    printf("grid_read %5d WGs     %.3f ms  %.0f GB/s\n", g, ms, gbs(ms, bytes));
  }
  CK(hipFuncSetAttribute((const void*)k_shard_read_w<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_shard_read_w<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  for (int per_cu : {1, 2, 3, 4, 8}) {  // resident workgroups per CU, capped by LDS
    const size_t l = (160 * 1024) / per_cu - 1024;
    ms = timeit([&] { hipLaunchKernelGGL((k_shard_read_w<8, 2>), dim3(wg), dim3(512), l, 0, x, rpw, out); }, 5);
    printf("8 waves, %d WG/CU       %.3f ms  %.0f GB/s\n", per_cu, ms, gbs(ms, bytes));
    ms = timeit([&] { hipLaunchKernelGGL((k_shard_read_w<4, 2>), dim3(wg), dim3(256), l, 0, x, rpw, out); }, 5);
    printf("4 waves, %d WG/CU       %.3f ms  %.0f GB/s\n", per_cu, ms, gbs(ms, bytes));
  }
  ms = timeit([&] { hipLaunchKernelGGL((k_shard_read_w<8, 2>), dim3(wg / 2), dim3(512), 0, 0, x, rpw * 2, out); }, 5);
  printf("8 waves, 2048 WGs x 1024 rows %.3f ms  %.0f GB/s\n", ms, gbs(ms, bytes));
  ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, x, y, n4 / 4); }, 5);
  printf("copy 2 GiB             %.3f ms  %.0f GB/s (read+write)\n", ms, gbs(ms, bytes / 2));
  {  // C5's shape scaled to the 8 GiB buffer: 1024 workgroups x 17 rows x 480 KiB (+ 1 row written)
    const int cols = (int)(bytes / 16 / 1024 / 17) / 64 * 64;
    const size_t rbytes = (size_t)1024 * 17 * cols * 16, wbytes = (size_t)1024 * cols * 16;
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<0>), dim3(1024), dim3(256), 0, 0, x, y, cols, out); }, 5);
    printf("C5 shape, reads only   %.3f ms  %.0f GB/s\n", ms, gbs(ms, rbytes));
    const double ms_r = ms;
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<1>), dim3(1024), dim3(256), 0, 0, x, y, cols, out); }, 5);
    printf("C5 shape, + 6%% writes  %.3f ms  %.0f GB/s (read+write); the writes cost %.3f ms = %.0f GB/s\n", ms,
           gbs(ms, rbytes + wbytes), ms - ms_r, gbs(ms - ms_r, wbytes));
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<2>), dim3(1024), dim3(256), 0, 0, x, y, cols, out); }, 5);
    printf("  ... writes in 16 KiB bursts %.3f ms; the writes cost %.3f ms = %.0f GB/s\n", ms, ms - ms_r,
           gbs(ms - ms_r, wbytes));
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<3>), dim3(1024), dim3(256), 0, 0, x, y, cols, out); }, 5);
    printf("  default-policy reads only %.3f ms\n", ms);
    const double ms_d = ms;
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<4>), dim3(1024), dim3(256), 0, 0, x, y, cols, out); }, 5);
    printf("  default-policy reads + writes %.3f ms; the writes cost %.3f ms\n", ms, ms - ms_d);
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<5>), dim3(1024), dim3(256), 0, 0, x, y, cols, out); }, 5);
    printf("  default-policy reads + nt writes %.3f ms; the writes cost %.3f ms\n", ms, ms - ms_d);
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<0>), dim3(4096), dim3(256), 0, 0, x, y, cols / 4, out); }, 5);
    printf("  4096 WGs, reads only %.3f ms\n", ms);
    const double ms_r4 = ms;
    ms = timeit([&] { hipLaunchKernelGGL((k_c5_stream<1>), dim3(4096), dim3(256), 0, 0, x, y, cols / 4, out); }, 5);
    printf("  4096 WGs, + writes   %.3f ms; the writes cost %.3f ms\n", ms, ms - ms_r4);
  }
  return 0;
}
