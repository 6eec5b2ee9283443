// rs_probe.hip -- the access pattern of the C5 row-space pass (rowspace.hip k_rs_pass) alone, to
// separate what the pattern itself reads at from what the pass's arithmetic costs.
//   grid (nblk column blocks, wg row groups), 256 threads; wave w of workgroup (blk, g) streams a
//   contiguous quarter of row group g's rows; per row it reads CB 16-byte chunks per lane of column
//   block blk (64 * CB * 16 bytes), NBUF rows in flight (rotating buffers, as the pass).
// COMP 0: a float sum per lane (loads used, nothing else); COMP 1: the x32 pass's arithmetic per
// element (widen to double, dot with a double xbar chunk, coefficient FMA into double column sums)
// plus the per-row 64-lane DPP butterfly of the dot.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rs_probe.hip -o tools/rs_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("HIP %s\n", hipGetErrorString(r)); exit(1); } } while (0)

template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_add(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, RM, BM, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, RM, BM, false);
  return v + __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v = dpp_add<0xb1, 0xf, 0xf>(v);
  v = dpp_add<0x4e, 0xf, 0xf>(v);
  v = dpp_add<0x114, 0xf, 0xe>(v);
  v = dpp_add<0x118, 0xf, 0xc>(v);
  v = dpp_add<0x142, 0xa, 0xf>(v);
  v = dpp_add<0x143, 0xc, 0xf>(v);
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

template <int CB, int NBUF, int COMP>
__global__ __launch_bounds__(256) void k_probe(const float* __restrict__ X, int64_t ld, int64_t rows, int wg,
                                               const double* __restrict__ xbar, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int blk = blockIdx.x, g = blockIdx.y;
  const int64_t r0 = rows * g / wg, r1 = rows * (g + 1) / wg;
  const int64_t per = (r1 - r0 + 3) / 4;
  const int64_t wr0 = r0 + wave * per < r1 ? r0 + wave * per : r1;
  const int64_t wr1 = wr0 + per < r1 ? wr0 + per : r1;
  int64_t cc[CB];
  double xb[CB][4], acc[CB][4];
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    cc[j] = (int64_t)(blk * 64 * CB + j * 64 + lane) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xb[j][e] = xbar[(cc[j] + e) & 1023];
      acc[j][e] = 0.0;
    }
  }
  float fs = 0.f;
  double stash = 0.0;
  // COMP 2 / 3: the same blocks in a column-block-tiled layout (tile blk = every row's block blk,
  // rows contiguous: X[blk][row][64 * CB * 4 floats]), so a wave streams contiguous memory
  // COMP 4 / 5: 1 KiB tiles (the engine's layout, kcommon.h XAddr): a block of CB = 2 chunks per
  // lane reads two tiles, i.e. two contiguous streams per wave
  constexpr bool TILED = COMP >= 2;
  constexpr bool T1K = COMP >= 4;
  constexpr int64_t TW = 64 * CB * 4;  // floats per row of a tile (COMP 2 / 3)
  auto load = [&](int64_t r, f4 (&dst)[CB]) {
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const float* p = T1K     ? X + (((int64_t)blk * CB + j) * rows + r) * 256 + lane * 4
                       : TILED ? X + ((int64_t)blk * rows + r) * TW + (j * 64 + lane) * 4
                               : X + r * ld + cc[j];
      dst[j] = __builtin_nontemporal_load((const f4*)p);
    }
  };
  auto process = [&](const f4 (&rv)[CB], int64_t r) {
    if constexpr (COMP == 0 || COMP == 2 || COMP == 4) {
#pragma unroll
      for (int j = 0; j < CB; ++j) fs += (rv[j][0] + rv[j][1]) + (rv[j][2] + rv[j][3]);
    } else {
      double p = 0.0;
      const double cf = 1.0 + 1e-9 * (double)(r & 7);
#pragma unroll
      for (int j = 0; j < CB; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double v = (double)rv[j][e];
          p += v * xb[j][e];
          acc[j][e] += cf * v;
        }
      const double dot = wave_sum_dpp(p);
      if (lane == (int)(r & 63)) stash += dot;
    }
  };
  if (wr0 < wr1) {
    const int64_t last = wr1 - 1;
    f4 buf[NBUF][CB];
#pragma unroll
    for (int k = 0; k < NBUF; ++k) load(wr0 + k < last ? wr0 + k : last, buf[k]);
    int64_t r = wr0;
    for (; r + NBUF <= wr1; r += NBUF) {
#pragma unroll
      for (int k = 0; k < NBUF; ++k) {
        process(buf[k], r + k);
        load(r + k + NBUF < last ? r + k + NBUF : last, buf[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NBUF; ++k)
      if (r + k < wr1) process(buf[k], r + k);
  }
  double s = (double)fs + stash;
#pragma unroll
  for (int j = 0; j < CB; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s += acc[j][e];
  if (lane == 0) out[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave] = s;  // keeps the work
}

template <int CB, int NBUF, int COMP>
static void run(const float* X, int64_t ld, int64_t rows, int wg, const double* xbar, double* out, const char* tag) {
  const int nblk = (int)(ld / 4 / (64 * CB));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f, tot = 0.f;
  const int reps = 6;
  for (int it = 0; it < reps + 1; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_probe<CB, NBUF, COMP>), dim3(nblk, wg), dim3(256), 0, 0, X, ld, rows, wg, xbar, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it > 0) {
      tot += ms;
      if (ms < best) best = ms;
    }
  }
  const double bytes = (double)rows * ld * 4;
  printf("%-28s CB=%d NBUF=%-2d wg=%d  avg %.3f ms  best %.3f ms  %.0f GB/s (avg)\n", tag, CB, NBUF, wg, tot / reps,
         best, bytes / (tot / reps * 1e-3) / 1e9);
  fflush(stdout);
}

int main() {
  const int64_t ld = 1 << 20, rows = 1024 * 16;  // C5: 1024 workers x 16 rows x 2^20 float32 = 64 GiB
  float* X;
  double *xbar, *out;
  CK(hipMalloc(&X, (size_t)rows * ld * sizeof(float)));
  CK(hipMemset(X, 0, (size_t)rows * ld * sizeof(float)));
  CK(hipMalloc(&xbar, 1024 * sizeof(double)));
  CK(hipMemset(xbar, 0, 1024 * sizeof(double)));
  CK(hipMalloc(&out, 1 << 20));
  run<2, 6, 4>(X, ld, rows, 2, xbar, out, "1K tiles, pattern only");
  run<2, 6, 5>(X, ld, rows, 2, xbar, out, "1K tiles, x32 arithmetic");
  run<2, 12, 5>(X, ld, rows, 2, xbar, out, "1K tiles, x32 arithmetic");
  run<1, 8, 5>(X, ld, rows, 2, xbar, out, "1K tiles, x32 arithmetic");
  run<1, 12, 5>(X, ld, rows, 2, xbar, out, "1K tiles, x32 arithmetic");
  run<2, 6, 3>(X, ld, rows, 2, xbar, out, "2K tiles, x32 arithmetic");
  run<2, 6, 0>(X, ld, rows, 2, xbar, out, "pattern only");
  run<2, 6, 1>(X, ld, rows, 2, xbar, out, "x32 arithmetic");
  run<2, 6, 0>(X, ld, rows, 4, xbar, out, "pattern only");
  run<2, 6, 0>(X, ld, rows, 1, xbar, out, "pattern only");
  run<2, 12, 0>(X, ld, rows, 2, xbar, out, "pattern only");
  run<2, 3, 0>(X, ld, rows, 2, xbar, out, "pattern only");
  run<4, 6, 0>(X, ld, rows, 2, xbar, out, "pattern only");
  run<1, 12, 0>(X, ld, rows, 2, xbar, out, "pattern only");
  run<2, 3, 1>(X, ld, rows, 2, xbar, out, "x32 arithmetic");
  run<2, 6, 1>(X, ld, rows, 4, xbar, out, "x32 arithmetic");
  run<1, 8, 1>(X, ld, rows, 2, xbar, out, "x32 arithmetic");
  run<2, 6, 1>(X, ld, rows, 2, xbar, out, "x32 arithmetic (again)");
  run<2, 6, 0>(X, ld, rows, 2, xbar, out, "pattern only (again)");
  run<2, 6, 2>(X, ld, rows, 2, xbar, out, "tiled, pattern only");
  run<2, 6, 3>(X, ld, rows, 2, xbar, out, "tiled, x32 arithmetic");
  run<2, 12, 2>(X, ld, rows, 2, xbar, out, "tiled, pattern only");
  run<2, 3, 3>(X, ld, rows, 2, xbar, out, "tiled, x32 arithmetic");
  run<2, 6, 3>(X, ld, rows, 4, xbar, out, "tiled, x32 arithmetic");
  run<2, 6, 3>(X, ld, rows, 1, xbar, out, "tiled, x32 arithmetic");
  run<4, 6, 3>(X, ld, rows, 2, xbar, out, "tiled, x32 arithmetic");
  run<1, 8, 3>(X, ld, rows, 2, xbar, out, "tiled, x32 arithmetic");
  run<2, 6, 3>(X, ld, rows, 2, xbar, out, "tiled, x32 arithmetic (again)");
  run<2, 6, 1>(X, ld, rows, 2, xbar, out, "x32 arithmetic (again)");
  CK(hipFree(X));
  return 0;
}
