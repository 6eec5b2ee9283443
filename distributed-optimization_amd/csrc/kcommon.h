// kcommon.h -- device helpers shared by the gfx950 kernel translation units
// (kernels.hip, round_*.hip): element / chunk types, wave reductions, the Philox
// minibatch draw, the objective row terms and the mix of one chunk.
#pragma once
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include <type_traits>

#include "engine.h"

namespace dopt {

template <typename T>
struct VT;
template <>
struct VT<float> {
  static constexpr int n = 4;
  typedef float v __attribute__((ext_vector_type(4)));
};
template <>
struct VT<double> {
  static constexpr int n = 2;
  typedef double v __attribute__((ext_vector_type(2)));
};

// Data (S) and state (T) element types of a context.  A 16-byte DATA chunk holds
// VN = 16 / sizeof(S) elements of a shard row; the STATE chunk at the same columns (the
// iterate, xbar, the gradient) is VN elements of T: 16 bytes when S = T, 32 bytes for
// float64 iterates and arithmetic over float32-stored rows (dopt_set_data_dtype).
template <typename E, int N>
struct VecOf {
  typedef E v __attribute__((ext_vector_type(N)));
};
template <typename T, typename S>
struct KV {
  static constexpr int VN = 16 / sizeof(S);
  using V = typename VecOf<T, VN>::v;   // state chunk
  using VX = typename VecOf<S, VN>::v;  // data chunk (one 16-byte load)
};

// Shard rows of column-blocked contexts (rows longer than the row-resident kernel) are stored
// column-block TILED: tile t holds the 16-byte chunks [64 t, 64 t + 64) of every row of the array,
// rows contiguous (1 KiB per row per tile), so a workgroup walking one column block over many
// rows streams contiguous memory instead of 1-2 KiB pieces 4 MB apart (C5: 6.85-6.97 vs
// 6.35-6.55 TB/s for the bare access pattern, tools/rs_probe.hip).  XAddr<VN> maps (row, data
// chunk c) to an element offset: xrows = rows of the array (0: row-major with stride ld).
constexpr int kTileChunks = 64;
template <int VN>
struct XAddr {
  int64_t rs;  // elements from one row to the next (at a fixed column)
  int64_t ts;  // elements from one tile to the next (0: row-major)
  __device__ __forceinline__ XAddr(int64_t xrows, int64_t ld)
      : rs(xrows ? (int64_t)kTileChunks * VN : ld), ts(xrows * kTileChunks * VN) {}
  __device__ __forceinline__ int64_t col(int64_t c) const {  // element offset of data chunk c in row 0
    return ts ? (c >> 6) * ts + (c & (kTileChunks - 1)) * VN : c * VN;
  }
  __device__ __forceinline__ int64_t at(int64_t row, int64_t c) const { return row * rs + col(c); }
};

constexpr int NW = 4;         // waves per workgroup
constexpr int NT = NW * 64;   // threads per workgroup
constexpr int MAX_CPL = 16;   // 16-byte chunks per lane: d <= 4096 (fp32) / 2048 (fp64)
static_assert(NW == 4, "k_cons folds four wave sums");

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave-wide sum by DPP: quad swaps, row_shr 4/8, row_bcast 15/31 (GFX9-family DPP), then
// one v_readlane of lane 63 -- the result lands in an SGPR (the coefficient is wave-uniform).
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, BM, false);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __builtin_bit_cast(float, dpp_i<CTRL, RM, BM>(__builtin_bit_cast(int, v)));
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_add(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = dpp_i<CTRL, RM, BM>((int)(b & 0xffffffffll));
  const int hi = dpp_i<CTRL, RM, BM>((int)(b >> 32));
  return v + __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
template <typename T>
__device__ __forceinline__ T wave_sum_dpp(T v) {
  v = dpp_add<0xb1, 0xf, 0xf>(v);   // quad_perm [1,0,3,2]
  v = dpp_add<0x4e, 0xf, 0xf>(v);   // quad_perm [2,3,0,1]
  v = dpp_add<0x114, 0xf, 0xe>(v);  // row_shr:4
  v = dpp_add<0x118, 0xf, 0xc>(v);  // row_shr:8
  v = dpp_add<0x142, 0xa, 0xf>(v);  // row_bcast:15
  v = dpp_add<0x143, 0xc, 0xf>(v);  // row_bcast:31  -> lane 63 holds the sum
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
  } else {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned int)lo);
  }
}

// Two wave-wide sums in one butterfly: the first step splits the values by lane parity
// (even lanes carry a, odd lanes b), the remaining five steps reduce both at once.  Every
// step is unmasked -- quad_perm, row_ror inside a row of 16 lanes, then the gfx950 row /
// half-wave swaps (v_permlane16_swap, v_permlane32_swap) -- so no lane needs a zeroed
// destination, and the totals end up in every lane of their parity (read from lanes 0 / 1).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
// x + (the same register of the partner lane l ^ 16 (W = 16) or l ^ 32 (W = 32)); both lanes of
// a pair get the sum in the same order, so the result is lane-independent
template <int W>
__device__ __forceinline__ float swap_add(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = W == 16 ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                         : __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
template <int W>
__device__ __forceinline__ double swap_add(double x) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  const auto rl = W == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                          : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto rh = W == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                          : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const double r0 = __builtin_bit_cast(double, ((unsigned long long)(unsigned)rh[0] << 32) | (unsigned)rl[0]);
  const double r1 = __builtin_bit_cast(double, ((unsigned long long)(unsigned)rh[1] << 32) | (unsigned)rl[1]);
  return r0 + r1;
}
template <typename T>
__device__ __forceinline__ T readlane_t(T v, int lane) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
  } else {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned int)lo);
  }
}
template <typename T>
__device__ __forceinline__ void wave_sum_pair(T a, T b, T& sa, T& sb) {
  const bool odd = (threadIdx.x & 1) != 0;
  T x = odd ? b : a;
  const T y = odd ? a : b;
  x += dpp_mov<0xb1>(y);   // quad_perm [1,0,3,2]: lane l pairs with l ^ 1 (same parity sums)
  x += dpp_mov<0x4e>(x);   // quad_perm [2,3,0,1]
  x += dpp_mov<0x124>(x);  // row_ror:4
  x += dpp_mov<0x128>(x);  // row_ror:8 -> the row's (16 lanes) sum of this parity's value
  x = swap_add<16>(x);     // rows 0+1, 2+3
  x = swap_add<32>(x);     // halves
  sa = readlane_t(x, 0);
  sb = readlane_t(x, 1);
}

// A row chunk in the state type: the identity when rows are stored in the arithmetic type, the
// exact float -> double widening for float32 rows under float64 arithmetic.
template <typename V, typename VX>
__device__ __forceinline__ V widen(VX x) {
  if constexpr (std::is_same<V, VX>::value) return x;
  else return __builtin_convertvector(x, V);
}

template <typename T, typename V>
__device__ __forceinline__ T hsum(V v) {
  T s = v[0];
#pragma unroll
  for (int e = 1; e < VT<T>::n; ++e) s += v[e];
  return s;
}
template <typename T, int N, typename V>
__device__ __forceinline__ T hsumn(V v) {  // the same left-to-right sum over N elements
  T s = v[0];
#pragma unroll
  for (int e = 1; e < N; ++e) s += v[e];
  return s;
}

// Philox4x32-10 (Salmon et al., SC'11): counter-based, so a worker's minibatch of a round
// is a pure function of (seed, round, worker) -- no generator state anywhere.
struct U4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ U4 philox4x32(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Device minibatch (sampling = 'device', the non-parity throughput mode of SURVEY section 7):
// Floyd's algorithm marks a uniform nb-subset of [0, m) in the LDS byte map; draw k is word
// k % 4 of philox(counter = (k / 4, worker, round lo, round hi), key = seed), mapped to
// [0, j] by a 32x32 multiply-high (bias <= m / 2^32).  oracle/device_sampler.py restates it.
__device__ inline void floyd_sample(unsigned char* bmask, int64_t m, int64_t nb, uint64_t seed, int64_t round,
                             int64_t worker) {
  U4 r = {0, 0, 0, 0};
  int64_t k = 0;
  for (int64_t j = m - nb; j < m; ++j, ++k) {
    if ((k & 3) == 0)
      r = philox4x32(U4{(uint32_t)(k >> 2), (uint32_t)worker, (uint32_t)round, (uint32_t)((uint64_t)round >> 32)},
                     (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t u = (k & 3) == 0 ? r.x : (k & 3) == 1 ? r.y : (k & 3) == 2 ? r.z : r.w;
    const int64_t t = (int64_t)(((uint64_t)u * (uint64_t)(j + 1)) >> 32);
    if (bmask[t]) bmask[j] = 1;
    else bmask[t] = 1;
  }
}

// scipy.special.expit(x) = 1 / (1 + exp(-x)); the gradient needs expit(-y z).
template <typename T>
__device__ __forceinline__ T sigmoid_neg(T yz) {
  return T(1) / (T(1) + exp(yz));
}

// Hardware transcendentals for float (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp): the
// library expf / logf / division add range reduction and Newton steps per row.
__device__ __forceinline__ float sigmoid_neg_fast(float yz) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(yz));
}
__device__ __forceinline__ double row_loss_fast(float yv, float u) {
  const float t = yv * u;
  const float a = t < 0.f ? -t : t;
  return (double)((t < 0.f ? -t : 0.f) + __logf(1.0f + __expf(-a)));
}

// obj_problems.py:5-7 (logistic, np.log(1 + exp(-|t|)) as written, not log1p)
// and obj_problems.py:41-42 (quadratic, the 0.5 is applied once at the end).
template <typename T, int PROB>
__device__ __forceinline__ double row_loss(T yv, T u) {
  if (PROB == 0) {
    const T t = yv * u;
    const T a = t < T(0) ? -t : t;
    return (double)((t < T(0) ? -t : T(0)) + log(T(1) + exp(-a)));
  } else {
    const T e = u - yv;
    return (double)(e * e);
  }
}

// sum_j W_ij x_j for the 16-byte chunk c of worker i: CSR over local / halo rows, or, for the
// complete graph (F_MEAN), w_off (S - x_i) + W_ii x_i from the column sums S (trainer.py:173).
template <typename T, typename S>
__device__ __forceinline__ typename KV<T, S>::V mix_chunk(const RoundArgs& a, int i, int c,
                                                          typename KV<T, S>::V own) {
  using V = typename KV<T, S>::V;
  constexpr int VN = KV<T, S>::VN;
  V acc = V(0);
  if (a.flags & F_MEAN) {
    const double wii = (double)((const T*)a.wdiag)[i];
    if (a.colsum_t) {  // sums rounded to T: one 16-byte load per chunk instead of VN doubles
      const V sv = *(const V*)((const T*)a.colsum_t + (int64_t)c * VN);
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        const double x = (double)own[e];
        acc[e] = (T)(a.w_off * ((double)sv[e] - x) + wii * x);
      }
      return acc;
    }
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      const double x = (double)own[e];
      acc[e] = (T)(a.w_off * (a.colsum[(int64_t)c * VN + e] - x) + wii * x);
    }
    return acc;
  }
  for (int64_t e = a.rp[i]; e < a.rp[i + 1]; ++e) {
    const T wt = ((const T*)a.cw)[e];
    const int col = a.ci[e];
    const T* src = col < a.n_local ? (const T*)a.x_old + (int64_t)col * a.ld
                                   : (const T*)a.halo + (int64_t)(col - a.n_local) * a.ld;
    acc += wt * *(const V*)(src + (int64_t)c * VN);
  }
  return acc;
}

}  // namespace dopt
