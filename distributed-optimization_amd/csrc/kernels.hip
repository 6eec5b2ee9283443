// kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the D-SGD round.
//
// The round of the reference (trainer.py:161-193) per worker i:
//   g_i   = (1/b) sum_k c_k(x_i . a_k) a_k + lam x_i      obj_problems.py:13-20 / :46-53
//   x_i'  = sum_j W_ij x_j - eta_t g_i                     trainer.py:173-175
// then xbar = mean_i x_i' (trainer.py:182), the consensus error (trainer.py:185)
// and the objective at xbar over all data (trainer.py:188-191).
//
// Everything here is HBM-bound (two GEMVs per worker, ~1 FLOP/B at fp32), so the
// design goal is ONE pass over the shard bytes per round:
//
//  k_round   one 256-thread workgroup (4 waves) per worker.  Each wave streams whole
//            rows (16-byte loads, lane l holds columns [16B chunk l + 64j]), forms the
//            row dot(s) by a 64-lane butterfly, turns them into the sigmoid / residual
//            coefficient in registers and accumulates coef*row from the SAME registers
//            (no second read of the row).  The waves' partial gradients meet in LDS;
//            the epilogue applies 1/b and lam, reads the <= deg+1 neighbour iterates
//            (L2 / Infinity-Cache resident) and writes x_i' -- grad, mix and step in
//            one launch.  With metrics fused (full-shard batches) the same row pass
//            also dots each row with xbar_t and accumulates the objective of the
//            previous round, so logging every round costs no extra HBM bytes.
//  k_colsum_part / k_colsum_final
//            deterministic two-stage column mean (fp64 partials, fixed order): xbar,
//            or the centralized gradient average + update.
//  k_history one workgroup folds the per-worker partials into history[t].
//
// No atomics anywhere: every reduction has a fixed order, so runs are bitwise
// reproducible.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

#include "kcommon.h"

namespace dopt {

// ---------------------------------------------------------------------------- k_round
// The fused round kernel lives in k_round.inc (one translation unit per element-type pair).
hipError_t launch_round(int dtype, int xdtype, int problem, int cpl, bool grad, bool met, const RoundArgs& a,
                        int n_groups, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  if (dtype == 0) return launch_round_f32(problem, cpl, grad, met, a, n_groups, s);
  if (xdtype == 0) return launch_round_x32(problem, cpl, grad, met, a, n_groups, s);
  return launch_round_f64(problem, cpl, grad, met, a, n_groups, s);
}

int max_chunks_per_lane(int dtype, int xdtype) { return (dtype == 1 && xdtype == 0) ? 8 : MAX_CPL; }



// ---------------------------------------------------------------------------- large d
// Column-blocked round for rows too long to hold in registers (config C5: d = 2^20).
// Workgroup (i, g) walks column blocks cb = g, g + G, ... of 64 16-byte chunks.  The
// mix is column-local for every topology, so per block: rows' segments -> gradient
// block -> x_i' block (waves meet in LDS) -> the next round's partial dots x_k . x_i'
// from the SAME row registers.  Per-row partial dots go to fp64 slabs [n][bcap][G]
// that k_split_coef folds in a fixed order.  One pass over the shard per round.
template <typename T>
__device__ __forceinline__ typename VT<T>::v ld_nt(const T* p) {
  return __builtin_nontemporal_load((const typename VT<T>::v*)p);
}

// RPW = rows per wave held in registers (4 for <= 16 rows per worker, 16 for <= 64);
// CPB = 16-byte chunks per lane per column block (a block is 64 * CPB chunks of every row).
// One barrier per block: the waves' gradient partials go to a double-buffered LDS
// slot, every wave folds them and forms the new block itself (wave 0 stores it).
// Round 2 (C5, float32, interleaved A/B build): the block's mix before its
// barrier 14.93 -> 14.60 ms; all of the next block's loads in flight through the barrier
// (PF, unrolled by two over fixed register sets, branch-free loads so the compiler's waits
// stay partial) 14.60 -> 14.24; 1/16 as a multiply 14.24 -> ~14.0 (5.5 TB/s, 69 %).
// Little's law says why it stops there: 4 waves / SIMD x 4 KB ahead per wave = 64 KB in
// flight per CU, where ~90 KB are needed at the loaded latency (the dots-only kernel, 32
// VGPRs, 8 waves / SIMD, streams the same rows at 85 %).  Not kept: 2 chunks per lane with
// PF (166 VGPRs, 13.90 vs 13.99), a column-per-wave kernel without barriers that re-reads
// the rows from L2 for the dots (k_split_colwave: 17.6 ms).
// CPB > 1 keeps 2-4x the bytes in flight per wave between two barriers but costs
// occupancy (C5: CPB 1 / 2 / 4 = 85 / 115 / 169 VGPRs, 15.1 / 15.5 / 16.7 ms): 1.  Not kept either: own / xbar / column sums
// loaded once per workgroup and shared through LDS instead of by every wave (15.22 vs
// 15.14 ms).  The kernel waits on memory 78 % of its wave cycles (SQ_WAIT_ANY) at 42 %
// VALU issue per SIMD.
// Where the rest goes (round 2, C5, timing-only builds interleaved with this one, same box):
// WITHOUT the x' store the kernel runs 11.3-11.7 ms instead of 13.3-14.5 (reads alone at
// 6.4-6.6 TB/s) -- the 4.2 GB of writes cost 1.8-2.8 ms, ~2x what a copy kernel's write share
// predicts.  Unchanged by: which wave stores (one wave / round robin), nt / sc1 / sc0 sc1
// stores, a block-major x' layout (each generation writing one contiguous region), a
// rotated block walk per worker, removing the block barrier (13.8), and more bytes in flight
// (k_split_glds: 2-3 blocks per wave by LDS-DMA, 15.0-15.2; the no-prefetch kernel capped at
// 6 / 8 waves per SIMD: 15.3 / 24.8 with spills).  So this kernel is bound by HBM write
// turnaround, not by latency.
// LDS-only workgroup barrier: waits for this wave's LDS traffic, not for its global loads
// (__syncthreads() also drains vmcnt, which would cancel the next block's prefetch).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Blocks of column-block group grp: a contiguous range (a.contig: each row of a workgroup
// streams forward through memory) or every G-th block.
struct BlockWalk {
  int b0, b1, st;
  __device__ BlockWalk(const RoundArgs& a, int grp, int G, int nblk) {
    if (a.contig) {
      const int per = (nblk + G - 1) / G;
      b0 = grp * per;
      b1 = min(nblk, b0 + per);
      st = 1;
    } else {
      b0 = grp;
      b1 = nblk;
      st = G;
    }
  }
};

// T = iterates and arithmetic, XT = row storage (XT = T, or float32 rows under float64 arithmetic:
// a 16-byte row chunk is 4 floats, the state chunk at the same columns 4 doubles; every product
// and sum is then the float64 one).
template <typename T, typename XT, int RPW, bool ZNEXT, bool MET, bool PF, int CPB = 1>
__global__ __launch_bounds__(NT) void k_split_step(const RoundArgs a) {
  using V = typename KV<T, XT>::V;    // state chunk
  using VX = typename KV<T, XT>::VX;  // row chunk (one 16-byte load)
  constexpr int VN = KV<T, XT>::VN;
  constexpr int BC = 64 * CPB;  // chunks per column block
  __shared__ V gred[2][NW][BC];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.x, grp = blockIdx.y, G = gridDim.y;
  const int nch = a.nchunks, nblk = (nch + BC - 1) / BC;
  const BlockWalk bw(a, grp, G, nblk);
  const int64_t ld = a.ld;
  const int64_t row0 = a.off[i], m = a.off[i + 1] - row0;
  const int64_t nb = a.idx ? (a.b < m ? a.b : m) : m;  // <= NW * RPW (host-checked)
  const XT* __restrict__ X = (const XT*)a.X;
  const XAddr<VN> xa(a.xrows, ld);  // row-major or column-block tiled rows
  const bool shared = (a.flags & F_SHARED) != 0;  // centralized: every worker at w_shared
  const bool gout = (a.flags & F_GOUT) != 0;
  const T* own_p = shared ? (const T*)a.w_shared : (const T*)a.x_old + (int64_t)i * ld;
  int64_t rowp[RPW];
  T coef[RPW];
  double zacc[RPW], uacc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int k = wave + NW * r;
    const bool ok = k < nb;
    const int64_t lr = ok ? (a.idx ? (int64_t)a.idx[(int64_t)i * a.b + k] : (int64_t)k) : 0;
    rowp[r] = ok ? (row0 + lr) * xa.rs : -1;
    coef[r] = ok ? ((const T*)a.coef)[(int64_t)i * a.bcap + k] : T(0);
    zacc[r] = 0.0;
    uacc[r] = 0.0;
  }
  double cacc = 0.0;
  const T inv_eta = (T)a.eta, lam = (T)a.lam;
  // 1 / nb when nb is a power of two (C5: 16): a multiply instead of an IEEE division per element
  const bool pow2 = nb > 0 && (nb & (nb - 1)) == 0;
  const T inv_nb = nb > 0 ? T(1) / (T)nb : T(0);
  // PF: everything block cb + st needs -- its column sums (complete-graph mix), own and xbar
  // chunks, then its row segments -- is loaded while block cb is processed.  The loop is
  // unrolled by two over register sets A / B with fixed roles (stage B, process A, stage A,
  // process B), so no loaded register is copied: a copy needs its load complete, and the
  // compiler's wait for it would drain the whole next group (vmcnt counts in issue order).
  // The block's barrier is LDS-only.  Mixes other than the column-sum one read their
  // neighbour rows inside the block, as without PF.
  const bool mean = (a.flags & F_MEAN) != 0;
  const T* sums = (sizeof(T) == 8 && !a.colsum_t) ? (const T*)(const void*)a.colsum : (const T*)a.colsum_t;
  // PF launches are complete-graph D-SGD steps with the sums in T (launch_split_step checks):
  // the mix is formed from prefetched column sums, never from neighbour rows
  constexpr bool pf_mix = PF;
  (void)mean;
  (void)pf_mix;
  double wii = mean ? (double)((const T*)a.wdiag)[i] : 0.0;
  asm volatile("" : "+v"(wii));  // loaded here, once: a load sunk into the block loop would wait for the prefetch
  const bool early = (a.flags & F_EARLYMIX) != 0 && !gout;
  struct Set {
    VX rw[RPW][CPB];
    V own[CPB], xb[CPB], sv[CPB];
  };
  auto stage = [&](Set& S, int cbn) {  // small loads first, then the rows
    if (PF) {
      // branch-free: every load is issued (a block past the walk re-reads its last block, lanes
      // past the row its last chunk, absent rows the worker's first row -- all unused), so the
      // compiler's count of loads in flight is exact and the waits for the older set stay partial
      const int cbc = cbn < bw.b1 ? cbn : bw.b1 - 1;
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const int c0 = cbc * BC + j * 64 + lane;
        const int c = c0 < nch ? c0 : nch - 1;
        S.sv[j] = *(const V*)(sums + (int64_t)c * VN);
        S.own[j] = *(const V*)(own_p + (int64_t)c * VN);
        if (MET) S.xb[j] = *(const V*)((const T*)a.xbar + (int64_t)c * VN);
      }
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const int c0 = cbc * BC + j * 64 + lane;
        const int c = c0 < nch ? c0 : nch - 1;
#pragma unroll
        for (int r = 0; r < RPW; ++r) S.rw[r][j] = ld_nt<XT>(X + (rowp[r] >= 0 ? rowp[r] : row0 * xa.rs) + xa.col(c));
      }
      return;
    }
    const bool blk = cbn < bw.b1;
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int c = cbn * BC + j * 64 + lane;
      const bool in = blk && c < nch;
      S.own[j] = in ? *(const V*)(own_p + (int64_t)c * VN) : V(0);
      S.xb[j] = (MET && in) ? *(const V*)((const T*)a.xbar + (int64_t)c * VN) : V(0);
    }
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int c = cbn * BC + j * 64 + lane;
      const bool in = blk && c < nch;
#pragma unroll
      for (int r = 0; r < RPW; ++r) S.rw[r][j] = (in && rowp[r] >= 0) ? ld_nt<XT>(X + rowp[r] + xa.col(c)) : VX(0);
    }
  };
  auto process = [&](Set& S, int cb, int buf) {
    V mixv[CPB];
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int c = cb * BC + j * 64 + lane;
      const bool in = c < nch;
      if constexpr (PF) {  // mix_chunk's column-sum form, from the prefetched sums (same arithmetic)
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          const double x = (double)S.own[j][e];
          mixv[j][e] = (T)(a.w_off * ((double)S.sv[j][e] - x) + wii * x);
        }
      } else {
        // the mix does not depend on the gradient: with F_EARLYMIX its loads (column sums or the
        // neighbour rows) are issued before the block's barrier instead of after it
        mixv[j] = (early && in) ? mix_chunk<T, XT>(a, i, c, S.own[j]) : V(0);
      }
      V gp = V(0);
#pragma unroll
      for (int r = 0; r < RPW; ++r) gp += coef[r] * widen<V>(S.rw[r][j]);  // absent rows: coef 0
      gred[buf][wave][j * 64 + lane] = gp;
    }
    if (PF)
      lds_barrier();
    else
      __syncthreads();
#pragma unroll
    for (int j = 0; j < CPB; ++j) {
      const int c = cb * BC + j * 64 + lane;
      const bool in = c < nch;
      const int q = j * 64 + lane;
      V g = V(0);
      if (nb > 0) {
        const V gs = gred[buf][0][q] + gred[buf][1][q] + gred[buf][2][q] + gred[buf][3][q];
        g = (pow2 ? gs * inv_nb : gs / (T)nb) + lam * S.own[j];  // x * 2^-k == x / 2^k exactly
      }
      V xn = V(0);
      if (gout) {
        if (wave == 0 && in) *(V*)((T*)a.g_out + (int64_t)i * ld + (int64_t)c * VN) = g;
      } else if (in) {
        if constexpr (PF) xn = mixv[j] - inv_eta * g;
        else xn = (early ? mixv[j] : mix_chunk<T, XT>(a, i, c, S.own[j])) - inv_eta * g;
        if (wave == 0) *(V*)((T*)a.x_new + (int64_t)i * ld + (int64_t)c * VN) = xn;
      }
      if (ZNEXT) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) zacc[r] += (double)hsumn<T, VN>(widen<V>(S.rw[r][j]) * xn);
      }
      if (MET && in) {  // (PF: lanes past the row hold re-read chunks)
#pragma unroll
        for (int r = 0; r < RPW; ++r) uacc[r] += (double)hsumn<T, VN>(widen<V>(S.rw[r][j]) * S.xb[j]);
        if (wave == 0) {
          const V dv = S.own[j] - S.xb[j];
          cacc += (double)hsumn<T, VN>(dv * dv);
        }
      }
    }
  };
  if (PF) {
    Set A, B;
    stage(A, bw.b0);
    for (int cb = bw.b0; cb < bw.b1; cb += 2 * bw.st) {
      stage(B, cb + bw.st);
      process(A, cb, 0);
      if (cb + bw.st >= bw.b1) break;
      stage(A, cb + 2 * bw.st);
      process(B, cb + bw.st, 1);
    }
  } else {
    Set A;
    int buf = 0;
    for (int cb = bw.b0; cb < bw.b1; cb += bw.st, buf ^= 1) {
      stage(A, cb);
      process(A, cb, buf);
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int k = wave + NW * r;
    const int64_t slot = ((int64_t)i * a.bcap + k) * G + grp;
    if (ZNEXT) {
      const double z = wave_sum_dpp(zacc[r]);
      if (lane == 0 && k < nb) a.zpart[slot] = z;
    }
    if (MET) {
      const double u = wave_sum_dpp(uacc[r]);
      if (lane == 0 && k < nb) a.upart[slot] = u;
    }
  }
  if (MET && wave == 0) {
    const double cs = wave_sum_dpp(cacc);
    if (lane == 0) a.cpart[(int64_t)i * G + grp] = cs;
  }
}


template <typename T, typename S, int MODE, int RPW>
__global__ __launch_bounds__(NT) void k_split_dots(const RoundArgs a) {
  using V = typename KV<T, S>::V;
  constexpr int VN = KV<T, S>::VN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.x, grp = blockIdx.y, G = gridDim.y;
  const int nch = a.nchunks, nblk = (nch + 63) / 64;
  const BlockWalk bw(a, grp, G, nblk);
  const int64_t ld = a.ld;
  const int64_t row0 = a.off[i], m = a.off[i + 1] - row0;
  const int64_t nb = (MODE == 0 && a.idx) ? (a.b < m ? a.b : m) : m;
  const S* __restrict__ X = (const S*)a.X;
  const XAddr<VN> xa(a.xrows, ld);  // row-major or column-block tiled rows
  const T* own_p = (a.flags & F_SHARED) ? (const T*)a.w_shared : (const T*)a.x_old + (int64_t)i * ld;
  const T* pt = MODE == 0 ? own_p : (const T*)a.xbar;
  double* out = MODE == 0 ? a.zpart : a.upart;
  if (MODE == 1 && wave == 0 && (a.flags & F_CONS)) {  // ||x_i - xbar||^2 partial over this group's blocks
    double cacc = 0.0;
    for (int cb = bw.b0; cb < bw.b1; cb += bw.st) {
      const int c = cb * 64 + lane;
      if (c < nch) {
        const V dv = *(const V*)(own_p + (int64_t)c * VN) - *(const V*)(pt + (int64_t)c * VN);
        cacc += (double)hsumn<T, VN>(dv * dv);
      }
    }
    cacc = wave_sum(cacc);
    if (lane == 0) a.cpart[(int64_t)i * G + grp] = cacc;
  }
  if (MODE == 1 && !(a.flags & F_LOSS)) return;
  for (int64_t rc = 0; rc < nb; rc += NW * RPW) {
    int64_t rowp[RPW];
    double acc[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int64_t k = rc + wave + NW * r;
      const bool ok = k < nb;
      const int64_t lr = ok ? ((MODE == 0 && a.idx) ? (int64_t)a.idx[(int64_t)i * a.b + k] : k) : 0;
      rowp[r] = ok ? (row0 + lr) * xa.rs : -1;
      acc[r] = 0.0;
    }
    for (int cb = bw.b0; cb < bw.b1; cb += bw.st) {
      const int c = cb * 64 + lane;
      if (c >= nch) continue;
      const V pv = *(const V*)(pt + (int64_t)c * VN);
      const int64_t co = xa.col(c);
#pragma unroll
      for (int r = 0; r < RPW; ++r)
        if (rowp[r] >= 0) acc[r] += (double)hsumn<T, VN>(widen<V>(ld_nt<S>(X + rowp[r] + co)) * pv);
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int64_t k = rc + wave + NW * r;
      const double z = wave_sum(acc[r]);
      if (lane == 0 && k < nb) out[((int64_t)i * a.bcap + k) * G + grp] = z;
    }
  }
}

template <typename T, typename S, int PROB>
__global__ __launch_bounds__(NT) void k_split_coef(const RoundArgs a, int mode) {
  __shared__ double red[NW];
  const int i = blockIdx.x, G = a.groups;
  const int64_t row0 = a.off[i], m = a.off[i + 1] - row0;
  const S* Y = (const S*)a.y;  // labels / targets in the rows' storage type
  if (mode & 1) {  // next coefficients from the partial dots (obj_problems.py:16-17 / :49-50)
    const int64_t nb = a.idx ? (a.b < m ? a.b : m) : m;
    for (int64_t k = threadIdx.x; k < nb; k += NT) {
      double z = 0.0;
      for (int q = 0; q < G; ++q) z += a.zpart[((int64_t)i * a.bcap + k) * G + q];
      const int64_t lr = a.idx ? (int64_t)a.idx[(int64_t)i * a.b + k] : k;
      const double yv = (double)Y[row0 + lr];
      const double cf = (PROB == 0) ? -yv * (1.0 / (1.0 + exp(yv * z))) : z - yv;
      ((T*)a.coef)[(int64_t)i * a.bcap + k] = (T)cf;
    }
  }
  if (mode & 2) {  // objective partial over ALL rows of the worker, consensus partial
    double l = 0.0;
    for (int64_t k = threadIdx.x; k < m; k += NT) {
      double u = 0.0;
      for (int q = 0; q < G; ++q) u += a.upart[((int64_t)i * a.bcap + k) * G + q];
      l += row_loss<double, PROB>((double)Y[row0 + k], u);
    }
    l = wave_sum(l);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0, cs = 0.0;
      for (int q = 0; q < NW; ++q) s += red[q];
      for (int q = 0; q < G; ++q) cs += a.cpart[(int64_t)i * G + q];
      if (a.flags & F_LOSS) a.slab_loss[i] = s;
      if (a.flags & F_CONS) a.slab_cons[i] = cs;
    }
  }
}


static void note_split(const char* kernel, int dtype, int xdtype, const char* params) {
  char buf[160];
  if (dtype == 1 && xdtype == 0)
    snprintf(buf, sizeof(buf), "void dopt::%s<double, float, %s>(dopt::RoundArgs)", kernel, params);
  else
    snprintf(buf, sizeof(buf), "void dopt::%s<%s, %s, %s>(dopt::RoundArgs)", kernel, dtype == 0 ? "float" : "double",
             dtype == 0 ? "float" : "double", params);
  note_round_kernel(buf);
}
static const char* tf(bool b) { return b ? "true" : "false"; }

// element types of a launch: (0, 0) float, (1, 1) double, (1, 0) float64 over float32 rows
static bool split_types_ok(int dtype, int xdtype) { return dtype == xdtype || (dtype == 1 && xdtype == 0); }

template <typename T, typename S>
static void split_step_t(bool znext, bool met, bool small, bool pf, dim3 grid, const RoundArgs& a2,
                         hipStream_t s) {
#define SPLIT_STEP2(R_, P_, C_)                                                                                    \
  if (znext && met) hipLaunchKernelGGL((k_split_step<T, S, R_, true, true, P_, C_>), grid, dim3(NT), 0, s, a2);     \
  else if (znext) hipLaunchKernelGGL((k_split_step<T, S, R_, true, false, P_, C_>), grid, dim3(NT), 0, s, a2);      \
  else if (met) hipLaunchKernelGGL((k_split_step<T, S, R_, false, true, P_, C_>), grid, dim3(NT), 0, s, a2);        \
  else hipLaunchKernelGGL((k_split_step<T, S, R_, false, false, P_, C_>), grid, dim3(NT), 0, s, a2);
  if (small) {
    if (pf) { SPLIT_STEP2(4, true, 1) } else { SPLIT_STEP2(4, false, 1) }
  } else {
    if (pf) { SPLIT_STEP2(16, true, 1) } else { SPLIT_STEP2(16, false, 1) }
  }
#undef SPLIT_STEP2
}

hipError_t launch_split_step(int dtype, int xdtype, bool znext, bool met, const RoundArgs& a, int n_workers,
                             hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  if (!split_types_ok(dtype, xdtype)) return hipErrorInvalidValue;
  char params[96];
  const dim3 grid(n_workers, a.groups);
  const bool small = a.b_rows <= 4 * NW;  // rows per worker this step touches
  RoundArgs a2 = a;
  // every G-th column block per group (contiguous ranges measured 13.91 vs 14.02 ms at C5, round 2)
  a2.contig = 0;
  // the block's mix before its barrier
  a2.flags |= F_EARLYMIX;
  // the next block's loads in flight through the block's barrier: complete-graph D-SGD steps with
  // the column sums in T (C5 14.60 -> 14.24 ms, and 13.99 with the exact 1/16, interleaved A/B)
  const bool pf = (a.flags & F_MEAN) && !(a.flags & F_GOUT) && (dtype == 1 ? a.colsum != nullptr : a.colsum_t != nullptr);
  // one 16-byte chunk per lane per block (2 / 4 were measured slower, round 3)
  snprintf(params, sizeof(params), "%d, %s, %s, %s, 1", small ? 4 : 16, tf(znext), tf(met), tf(pf));
  note_split("k_split_step", dtype, xdtype, params);
  if (dtype == 0) split_step_t<float, float>(znext, met, small, pf, grid, a2, s);
  else if (xdtype == 0) split_step_t<double, float>(znext, met, small, pf, grid, a2, s);
  else split_step_t<double, double>(znext, met, small, pf, grid, a2, s);
  return hipGetLastError();
}

template <typename T, typename S>
static void split_dots_t(int mode, bool small, dim3 grid, const RoundArgs& a2, hipStream_t s) {
#define SPLIT_DOTS(R_)                                                                        \
  if (mode == 0) hipLaunchKernelGGL((k_split_dots<T, S, 0, R_>), grid, dim3(NT), 0, s, a2);   \
  else hipLaunchKernelGGL((k_split_dots<T, S, 1, R_>), grid, dim3(NT), 0, s, a2);
  if (small) { SPLIT_DOTS(4) } else { SPLIT_DOTS(16) }
#undef SPLIT_DOTS
}

hipError_t launch_split_dots(int dtype, int xdtype, int mode, const RoundArgs& a, int n_workers, hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  if (!split_types_ok(dtype, xdtype)) return hipErrorInvalidValue;
  const dim3 grid(n_workers, a.groups);
  const bool small = a.b_rows <= 4 * NW;  // <= 16 rows: one 4-row chunk per wave, high occupancy
  RoundArgs a2 = a;
  a2.contig = 0;  // every G-th column block per group, as in launch_split_step
  if (dtype == 0) split_dots_t<float, float>(mode, small, grid, a2, s);
  else if (xdtype == 0) split_dots_t<double, float>(mode, small, grid, a2, s);
  else split_dots_t<double, double>(mode, small, grid, a2, s);
  return hipGetLastError();
}

hipError_t launch_split_coef(int dtype, int xdtype, int problem, int mode, const RoundArgs& a, int n_workers,
                             hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  if (!split_types_ok(dtype, xdtype)) return hipErrorInvalidValue;
  const dim3 grid(n_workers);
#define COEF(T_, S_)                                                                                  \
  if (problem == 0) hipLaunchKernelGGL((k_split_coef<T_, S_, 0>), grid, dim3(NT), 0, s, a, mode);   \
  else hipLaunchKernelGGL((k_split_coef<T_, S_, 1>), grid, dim3(NT), 0, s, a, mode);
  if (dtype == 0) { COEF(float, float) } else if (xdtype == 0) { COEF(double, float) } else { COEF(double, double) }
#undef COEF
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- wide single evaluations
// The obj_problems.py API (dopt_eval_gradient / dopt_eval_objective) for rows too long for
// the row-resident kernel, float64: k_wide_dots -> per-row partial dots over column ranges,
// k_wide_rows -> per row z = sum of partials (fixed order) -> gradient coefficient
// (obj_problems.py:16-17 / :49-50) or loss term (:5-7 / :41-42), k_wide_colsum -> g_c =
// sum_k coef_k x_kc in row order (fixed), / b + reg w_c (:18-19 / :51-52).  Not a hot path.
__global__ __launch_bounds__(NT) void k_wide_dots(const double* __restrict__ X, const double* __restrict__ w,
                                                  int64_t ld, int64_t d, int G, double* __restrict__ part) {
  __shared__ double red[NW];
  const int64_t r = blockIdx.x;
  const int g = blockIdx.y;
  const int64_t per = (d + G - 1) / G, c0 = g * per, c1 = c0 + per < d ? c0 + per : d;
  double acc = 0.0;
  for (int64_t c = c0 + threadIdx.x; c < c1; c += NT) acc += X[r * ld + c] * w[c];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[r * G + g] = ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(NT) void k_wide_rows(const double* __restrict__ part, int G, const double* __restrict__ y,
                                                  int64_t rows, int problem, int grad, double* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (r >= rows) return;
  double z = 0.0;
  for (int g = 0; g < G; ++g) z += part[r * G + g];
  const double yv = y[r];
  if (grad) out[r] = problem == 0 ? -yv * sigmoid_neg(yv * z) : z - yv;
  else out[r] = problem == 0 ? row_loss<double, 0>(yv, z) : row_loss<double, 1>(yv, z);
}

__global__ __launch_bounds__(NT) void k_wide_colsum(const double* __restrict__ X, const double* __restrict__ coef,
                                                    int64_t ld, int64_t d, int64_t rows, const double* __restrict__ w,
                                                    double reg, double* __restrict__ g) {
  const int64_t c = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (c >= d) return;
  double acc = 0.0;
  for (int64_t r = 0; r < rows; ++r) acc += coef[r] * X[r * ld + c];
  g[c] = rows > 0 ? acc / (double)rows + reg * w[c] : 0.0;
}

hipError_t launch_wide_eval(const double* X, const double* y, const double* w, int64_t rows, int64_t d, int64_t ld,
                            int problem, bool grad, double reg, double* part, int G, double* rowbuf, double* g_out,
                            hipStream_t s) {
  if (rows > 0) {
    hipLaunchKernelGGL(k_wide_dots, dim3((unsigned)rows, G), dim3(NT), 0, s, X, w, ld, d, G, part);
    hipLaunchKernelGGL(k_wide_rows, dim3((unsigned)((rows + NT - 1) / NT)), dim3(NT), 0, s, part, G, y, rows,
                       problem, grad ? 1 : 0, rowbuf);
  }
  if (grad)
    hipLaunchKernelGGL(k_wide_colsum, dim3((unsigned)((d + NT - 1) / NT)), dim3(NT), 0, s, X, rowbuf, ld, d, rows, w,
                       reg, g_out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- column sums
// Stage 1: workgroup (g, cb) sums rows [g*rpg, (g+1)*rpg) of the 64-chunk column block cb;
// lane = chunk in the block, the 4 waves split the rows and meet in LDS (fixed order).
// Stage 2: workgroup cb sums the G partials of its block, waves split the groups.
// Both stages are coalesced 1 KiB row segments per wave-instruction.
template <typename T>
__global__ __launch_bounds__(NT) void k_colsum_part(const T* __restrict__ x, int64_t n, int64_t ld,
                                                    int nch, int rpg, double* __restrict__ part,
                                                    uint64_t* stamp) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  __shared__ double red[NW][64 * VN];
  if (stamp && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *stamp = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.x * rpg;
  const int64_t r1 = (r0 + rpg < n) ? r0 + rpg : n;
  double acc[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) acc[e] = 0.0;
  if (c < nch) {
    int64_t r = r0 + wave;
    for (; r + 3 * NW < r1; r += 4 * NW) {  // 4 rows in flight per wave
      V v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = *(const V*)(x + (r + k * NW) * ld + (int64_t)c * VN);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < VN; ++e) acc[e] += (double)v[k][e];
    }
    for (; r < r1; r += NW) {
      const V v = *(const V*)(x + r * ld + (int64_t)c * VN);
#pragma unroll
      for (int e = 0; e < VN; ++e) acc[e] += (double)v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) red[wave][lane * VN + e] = acc[e];
  __syncthreads();
  if (wave == 0 && c < nch) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      double s = red[0][lane * VN + e];
#pragma unroll
      for (int q = 1; q < NW; ++q) s += red[q][lane * VN + e];
      part[(int64_t)blockIdx.x * ld + (int64_t)c * VN + e] = s;
    }
  }
}

// sum_{k = threadIdx.x + j NT < cnt} v[k] in fold_block's order -- four accumulators s0..s3 taking
// k, k + NT, k + 2 NT, k + 3 NT per step of 4 NT, the rest into s0, then (s0 + s1) + (s2 + s3) -- with
// two steps' loads (and the tail's up to three) issued before their adds: fewer dependent memory
// round trips in the one-workgroup folds, the same sums bit for bit.
__device__ __forceinline__ double fold_sum4(const double* v, int64_t cnt) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int64_t k = threadIdx.x;
  for (; k + 7 * NT < cnt; k += 8 * NT) {
    double a[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] = v[k + q * NT];
    s0 += a[0];
    s1 += a[1];
    s2 += a[2];
    s3 += a[3];
    s0 += a[4];
    s1 += a[5];
    s2 += a[6];
    s3 += a[7];
  }
  for (; k + 3 * NT < cnt; k += 4 * NT) {
    double a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = v[k + q * NT];
    s0 += a[0];
    s1 += a[1];
    s2 += a[2];
    s3 += a[3];
  }
  double t[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) t[q] = k + q * NT < cnt ? v[k + q * NT] : 0.0;
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (k + q * NT < cnt) s0 += t[q];
  return (s0 + s1) + (s2 + s3);
}

// ||xbar||^2 over nch chunks of vn elements, thread-strided by chunk, in that order; up to four
// chunks' loads in flight per thread.
template <typename T>
__device__ __forceinline__ double fold_xnorm(const T* x, int nch, int vn) {
  double q = 0.0;
  for (int c0 = threadIdx.x; c0 < nch; c0 += 4 * NT) {
    double v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + u * NT;
        v[u][e] = (c < nch && e < vn) ? (double)x[(int64_t)c * vn + e] : 0.0;
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c0 + u * NT < nch)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < vn) q += v[u][e] * v[u][e];
  }
  return q;
}

// The history fold of k_history by one NT-thread block (fixed order): *out_c = sum sc[0:nc],
// *out_l = sum sl[0:nl], *out_q = ||xbar||^2; null outputs are skipped.
template <typename T>
__device__ void fold_block(const FoldArgs& f, int nch, double (*red)[64 * VT<T>::n]) {
  constexpr int VN = VT<T>::n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double a = 0.0, b = 0.0, q = 0.0;
  if (f.sc && f.out_c) a = fold_sum4(f.sc, f.nc);
  if (f.sl && f.out_l) b = fold_sum4(f.sl, f.nl);
  if (f.xbar && f.out_q) q = fold_xnorm<T>((const T*)f.xbar, nch, VN);
  a = wave_sum(a);
  b = wave_sum(b);
  q = wave_sum(q);
  if (lane == 0) {
    red[wave][0] = a;
    red[wave][1] = b;
    red[wave][2] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0, sq = 0.0;
    for (int k = 0; k < NW; ++k) {
      sa += red[k][0];
      sb += red[k][1];
      sq += red[k][2];
    }
    if (f.out_c) *f.out_c = sa;
    if (f.out_l) *f.out_l = sb;
    if (f.out_q) *f.out_q = sq;
  }
}

// Stage 2 (+ optionally, in one extra block, the history fold of the previous round's slabs:
// it rides this launch instead of a k_history launch of its own).
template <typename T>
__global__ __launch_bounds__(NT) void k_colsum_final(const double* __restrict__ part, int groups,
                                                     int64_t n, int64_t ld, int nch, T* out,
                                                     const T* base, double eta, int mode, double* raw,
                                                     const FoldArgs fold) {
  constexpr int VN = VT<T>::n;
  __shared__ double red[NW][64 * VN];
  if ((int)blockIdx.x == (nch + 63) / 64) {  // the fold block
    fold_block<T>(fold, nch, red);
    return;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double acc[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) acc[e] = 0.0;
  if (c < nch) {
    int q = wave;
    for (; q + 3 * NW < groups; q += 4 * NW) {
      double v[4][VN];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < VN; ++e) v[k][e] = part[(int64_t)(q + k * NW) * ld + (int64_t)c * VN + e];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < VN; ++e) acc[e] += v[k][e];
    }
    for (; q < groups; q += NW)
#pragma unroll
      for (int e = 0; e < VN; ++e) acc[e] += part[(int64_t)q * ld + (int64_t)c * VN + e];
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) red[wave][lane * VN + e] = acc[e];
  __syncthreads();
  if (wave == 0 && c < nch) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      const int64_t col = (int64_t)c * VN + e;
      double s = red[0][lane * VN + e];
#pragma unroll
      for (int q = 1; q < NW; ++q) s += red[q][lane * VN + e];
      if (raw) {  // column sums (cross-rank all-reduce input, or S for complete-graph mixing)
        raw[col] = s;
        if (!out) continue;
      }
      const double mean = s / (double)n;  // np.mean: sum / count
      if (mode == 0)
        out[col] = (T)mean;
      else
        out[col] = base[col] - (T)eta * (T)mean;  // trainer.py:57
    }
  }
}

// Both stages in one launch when the rows form a single group (n <= rpg: the small configs,
// C1 / C2 / main.py's N = 25, where a round is launch-bound): workgroup cb sums all n rows
// of its column block exactly as stage 1 does, then applies stage 2's epilogue to the one
// partial (stage 2 adds it to 0.0 and three empty wave sums, repeated here, so the output
// is bitwise the two-launch path's).  One extra block folds the history, as in stage 2.
template <typename T>
__global__ __launch_bounds__(NT) void k_colsum_one(const T* __restrict__ x, int64_t rows, int64_t ld, int nch,
                                                   uint64_t* stamp, int64_t n, T* out, const T* base,
                                                   double eta, int mode, double* raw, const FoldArgs fold,
                                                   double* cons_out) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  __shared__ double red[NW][64 * VN];
  __shared__ T xm[64 * VN];  // (T) xbar of this column block (cons_out)
  __shared__ double cred[NW];
  if ((int)blockIdx.x == (nch + 63) / 64) {  // the fold block
    fold_block<T>(fold, nch, red);
    return;
  }
  if (stamp && blockIdx.x == 0 && threadIdx.x == 0) *stamp = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double acc[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) acc[e] = 0.0;
  if (c < nch) {
    int64_t r = wave;
    for (; r + 3 * NW < rows; r += 4 * NW) {
      V v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = *(const V*)(x + (r + k * NW) * ld + (int64_t)c * VN);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < VN; ++e) acc[e] += (double)v[k][e];
    }
    for (; r < rows; r += NW) {
      const V v = *(const V*)(x + r * ld + (int64_t)c * VN);
#pragma unroll
      for (int e = 0; e < VN; ++e) acc[e] += (double)v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) red[wave][lane * VN + e] = acc[e];
  __syncthreads();
  if (wave == 0 && c < nch) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      const int64_t col = (int64_t)c * VN + e;
      double p = red[0][lane * VN + e];
#pragma unroll
      for (int q = 1; q < NW; ++q) p += red[q][lane * VN + e];
      double s = 0.0;  // stage 2 over one group
      s += p;
      s = ((s + 0.0) + 0.0) + 0.0;
      const double mean = s / (double)n;
      if (cons_out) xm[lane * VN + e] = (T)mean;
      if (raw) {
        raw[col] = s;
        if (!out) continue;
      }
      if (mode == 0)
        out[col] = (T)mean;
      else
        out[col] = base[col] - (T)eta * (T)mean;
    }
  }
  if (cons_out) {  // this block's share of sum_i ||x_i - xbar||^2 (trainer.py:183-186), xbar in T
    __syncthreads();
    double q = 0.0;
    if (c < nch) {
      V xv;
#pragma unroll
      for (int e = 0; e < VN; ++e) xv[e] = xm[lane * VN + e];
      for (int64_t r = wave; r < rows; r += NW) {
        const V dv = *(const V*)(x + r * ld + (int64_t)c * VN) - xv;
        q += (double)hsum<T>(dv * dv);
      }
    }
    q = wave_sum(q);
    if (lane == 0) cred[wave] = q;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int w = 0; w < NW; ++w) t += cred[w];
      cons_out[blockIdx.x] = t;
    }
  }
}

hipError_t launch_colsum(int dtype, const void* x, int64_t rows, int64_t ld, int32_t nchunks, int32_t rpg,
                         double* part, uint64_t* stamp, int64_t n, void* out, const void* base, double eta,
                         int mode, hipStream_t s, double* raw, const FoldArgs* fold, double* cons_out) {
  const int groups = (int)((rows + rpg - 1) / rpg);
  static const bool two = [] {  // A/B knob DOPT_COLSUM_TWO=1: always the two-launch path
    const char* v = getenv("DOPT_COLSUM_TWO");
    return v && atoi(v) != 0;
  }();
  if (groups > 1 || two) {
    if (cons_out) return hipErrorInvalidValue;  // one-launch path only (caller checks)
    hipError_t e = launch_colsum_partial(dtype, x, rows, ld, nchunks, rpg, part, stamp, s);
    if (e != hipSuccess) return e;
    return launch_colsum_final(dtype, part, groups > 0 ? groups : 1, n, ld, nchunks, out, base, eta, mode, s,
                               raw, fold);
  }
  FoldArgs f;
  memset(&f, 0, sizeof(f));
  if (fold) f = *fold;
  const dim3 grid((nchunks + 63) / 64 + (fold ? 1 : 0));
  if (dtype == 0)
    hipLaunchKernelGGL(k_colsum_one<float>, grid, dim3(NT), 0, s, (const float*)x, rows, ld, nchunks, stamp, n,
                       (float*)out, (const float*)base, eta, mode, raw, f, cons_out);
  else
    hipLaunchKernelGGL(k_colsum_one<double>, grid, dim3(NT), 0, s, (const double*)x, rows, ld, nchunks, stamp,
                       n, (double*)out, (const double*)base, eta, mode, raw, f, cons_out);
  return hipGetLastError();
}

hipError_t launch_colsum_partial(int dtype, const void* x, int64_t n, int64_t ld, int32_t nchunks,
                                 int32_t rpg, double* part, uint64_t* stamp, hipStream_t s) {
  const int groups = (int)((n + rpg - 1) / rpg);
  const dim3 grid(groups > 0 ? groups : 1, (nchunks + 63) / 64);
  if (dtype == 0)
    hipLaunchKernelGGL(k_colsum_part<float>, grid, dim3(NT), 0, s, (const float*)x, n, ld, nchunks,
                       rpg, part, stamp);
  else
    hipLaunchKernelGGL(k_colsum_part<double>, grid, dim3(NT), 0, s, (const double*)x, n, ld, nchunks,
                       rpg, part, stamp);
  return hipGetLastError();
}

hipError_t launch_colsum_final(int dtype, const double* part, int32_t groups, int64_t n, int64_t ld,
                               int32_t nchunks, void* out, const void* base, double eta, int mode,
                               hipStream_t s, double* raw, const FoldArgs* fold) {
  FoldArgs f;
  memset(&f, 0, sizeof(f));
  if (fold) f = *fold;
  const dim3 grid((nchunks + 63) / 64 + (fold ? 1 : 0));
  if (dtype == 0)
    hipLaunchKernelGGL(k_colsum_final<float>, grid, dim3(NT), 0, s, part, groups, n, ld, nchunks,
                       (float*)out, (const float*)base, eta, mode, raw, f);
  else
    hipLaunchKernelGGL(k_colsum_final<double>, grid, dim3(NT), 0, s, part, groups, n, ld, nchunks,
                       (double*)out, (const double*)base, eta, mode, raw, f);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- history
constexpr int NTH = 1024;  // k_history: 16 waves, so each thread folds only a few slabs
// Folds slabs into history sums: *out_c = sum sc[0:nc], *out_l = sum sl[0:nl],
// *out_q = ||xbar||^2.  A null input contributes 0; a null output is not written, so the
// consensus of one round and the objective of another can be folded by one launch.
template <typename T>
__global__ __launch_bounds__(NTH) void k_history(const double* sc, int64_t nc, const double* sl, int64_t nl,
                                                 const T* xbar, int64_t ld, int nch, double* out_c,
                                                 double* out_l, double* out_q) {
  constexpr int VN = VT<T>::n;
  constexpr int NWH = NTH / 64;
  __shared__ double part[3][NWH];
  double a = 0.0, b = 0.0, q = 0.0;
  if (sc && out_c)
    for (int64_t k = threadIdx.x; k < nc; k += NTH) a += sc[k];
  if (sl && out_l)
    for (int64_t k = threadIdx.x; k < nl; k += NTH) b += sl[k];
  if (xbar && out_q)
    for (int c = threadIdx.x; c < nch; c += NTH)
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        const double v = (double)xbar[(int64_t)c * VN + e];
        q += v * v;
      }
  a = wave_sum(a);
  b = wave_sum(b);
  q = wave_sum(q);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][wave] = a;
    part[1][wave] = b;
    part[2][wave] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0, sq = 0.0;
    for (int k = 0; k < NWH; ++k) {
      sa += part[0][k];
      sb += part[1][k];
      sq += part[2][k];
    }
    if (out_c) *out_c = sa;
    if (out_l) *out_l = sb;
    if (out_q) *out_q = sq;
  }
}

hipError_t launch_fold(int dtype, const double* sc, int64_t nc, const double* sl, int64_t nl, const void* xbar,
                       int64_t ld, int32_t nchunks, double* out_c, double* out_l, double* out_q, hipStream_t s) {
  if (dtype == 0)
    hipLaunchKernelGGL(k_history<float>, dim3(1), dim3(NTH), 0, s, sc, nc, sl, nl, (const float*)xbar, ld,
                       nchunks, out_c, out_l, out_q);
  else
    hipLaunchKernelGGL(k_history<double>, dim3(1), dim3(NTH), 0, s, sc, nc, sl, nl, (const double*)xbar, ld,
                       nchunks, out_c, out_l, out_q);
  return hipGetLastError();
}

hipError_t launch_history(int dtype, const double* slab_cons, const double* slab_loss, int64_t n,
                          int64_t ng, const void* xbar, int64_t ld, int32_t nchunks, bool xnorm,
                          double* out, hipStream_t s) {
  return launch_fold(dtype, slab_cons, n, slab_loss, ng, xnorm ? xbar : nullptr, ld, nchunks, out, out + 1,
                     out + 2, s);
}

// ---------------------------------------------------------------------------- consensus
// slab[g] = sum over workers i in [64 g, 64 g + 64) of ||x_i - xbar||^2 (trainer.py:185),
// fp64, fixed order: wave w takes workers 64 g + w + 4 k, the 4 wave sums meet in LDS.
// Per-worker terms are formed exactly as the fused k_round pass forms them.
template <typename T>
__global__ __launch_bounds__(NT) void k_cons(const T* __restrict__ x, const T* __restrict__ xbar, int64_t n,
                                             int64_t ld, int nch, double* __restrict__ slab) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  __shared__ double red[NW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * 64;
  const int64_t i1 = (i0 + 64 < n) ? i0 + 64 : n;
  double acc = 0.0;
  for (int64_t i = i0 + wave; i < i1; i += NW) {
    V dv = V(0);
    for (int c = lane; c < nch; c += 64) {
      const V t = *(const V*)(x + i * ld + (int64_t)c * VN) - *(const V*)(xbar + (int64_t)c * VN);
      dv += t * t;
    }
    acc += wave_sum((double)hsum<T>(dv));
  }
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) slab[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

hipError_t launch_cons(int dtype, const void* x, const void* xbar, int64_t n, int64_t ld, int32_t nchunks,
                       double* slab, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 63) / 64));
  if (dtype == 0)
    hipLaunchKernelGGL(k_cons<float>, grid, dim3(NT), 0, s, (const float*)x, (const float*)xbar, n, ld, nchunks,
                       slab);
  else
    hipLaunchKernelGGL(k_cons<double>, grid, dim3(NT), 0, s, (const double*)x, (const double*)xbar, n, ld,
                       nchunks, slab);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- mix (multi-GPU)
// One wave per worker: lane l owns 16-byte chunks l, l+64, ... (CPL per lane, as k_round).
// The neighbour rows are local iterates or halo rows received from other ranks; same CSR
// order and arithmetic as the fused kernel, so the result is bitwise the single-GPU one.
// All loads of the worker (own row, gradient, up to MAXE neighbour rows) are issued before
// the first use, so a wave has ~30 16-byte loads in flight instead of one dependent chain
// per chunk.
// k_mix: the multi-GPU phase path's mix + step (and the lagged schedule's xbar, consensus and
// send rows).  WPW waves per worker, each holding CPL 16-byte chunks per lane of its slice
// of the row: rows of 8-16 chunks per lane run as 2-4 waves of 4, so every CSR entry's loads
// of a wave are in flight at once (one latency per wave instead of one per entry; C3 float64
// rows, 4 neighbours: 37.3 us per round with one wave of 8 chunks per worker).
template <typename T, int CPL, int WPW = 1>
__global__ __launch_bounds__(NT) void k_mix(const RoundArgs a, const T* __restrict__ G, int n) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  constexpr int MAXE = CPL <= 4 ? 6 : 0;  // CSR entries held in registers (deg + 1 <= 5 for ring / torus / 4-regular)
  static_assert(NW % WPW == 0, "a worker's waves share one workgroup");
  __shared__ double cred[NW];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = (blockIdx.x * NW + wave) / WPW;
  const int c0 = (wave % WPW) * 64 * CPL;  // first chunk of this wave's slice
  const bool live = i < n;
  const int64_t ld = a.ld;
  const int nch = a.nchunks;
  const T eta = (T)a.eta;
  V dv = V(0);  // consensus term of x_old[i] (a.xsum): formed as k_round's F_CONS forms it
  // a.interior[i]: the gradient kernel mixed and stepped this worker already (no halo row, no
  // send row): only its consensus term (and xbar) here
  const bool skip = live && a.interior && a.interior[i];
  if (live) {
  const T* xo = (const T*)a.x_old + (int64_t)i * ld;
  V own[CPL], gc[CPL], acc[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = c0 + lane + 64 * j;
    const bool in = c < nch;
    own[j] = in ? *(const V*)(xo + (int64_t)c * VN) : V(0);
    gc[j] = (in && !skip) ? *(const V*)(G + (int64_t)i * ld + (int64_t)c * VN) : V(0);
    acc[j] = V(0);
  }
  if (skip) {
  } else if (a.flags & F_MEAN) {
#pragma unroll
    for (int j = 0; j < CPL; ++j)
      if (c0 + lane + 64 * j < nch) acc[j] = mix_chunk<T, T>(a, i, c0 + lane + 64 * j, own[j]);
  } else {
    const int64_t e0 = a.rp[i], e1 = a.rp[i + 1];
    auto row_of = [&](int64_t e) {
      const int col = a.ci[e];
      return col < a.n_local ? (const T*)a.x_old + (int64_t)col * ld
                             : (const T*)a.halo + (int64_t)(col - a.n_local) * ld;
    };
    if (e1 - e0 <= MAXE) {
      V r[MAXE > 0 ? MAXE : 1][CPL];
#pragma unroll
      for (int k = 0; k < MAXE; ++k) {
        if (e0 + k < e1) {
          const T* src = row_of(e0 + k);
#pragma unroll
          for (int j = 0; j < CPL; ++j) {
            const int c = c0 + lane + 64 * j;
            r[k][j] = c < nch ? *(const V*)(src + (int64_t)c * VN) : V(0);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < MAXE; ++k) {
        if (e0 + k < e1) {
          const T wt = ((const T*)a.cw)[e0 + k];
#pragma unroll
          for (int j = 0; j < CPL; ++j) acc[j] += wt * r[k][j];
        }
      }
    } else {
      for (int64_t e = e0; e < e1; ++e) {
        const T wt = ((const T*)a.cw)[e];
        const T* src = row_of(e);
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
          const int c = c0 + lane + 64 * j;
          if (c < nch) acc[j] += wt * *(const V*)(src + (int64_t)c * VN);
        }
      }
    }
  }
  const int64_t s0 = a.sptr ? a.sptr[i] : 0, s1 = a.sptr ? a.sptr[i + 1] : 0;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c = c0 + lane + 64 * j;
    if (c >= nch) continue;
    if (a.xsum) {  // xbar = (T)(column sum / n) of the iterates being mixed, as k_colsum_final rounds it
      V xb;
#pragma unroll
      for (int e = 0; e < VN; ++e) xb[e] = (T)(a.xsum[(int64_t)c * VN + e] / a.xsum_n);
      if (i == 0) *(V*)((T*)a.xbar_out + (int64_t)c * VN) = xb;
      const V t = own[j] - xb;
      dv += t * t;
    }
    if (skip) continue;
    const V xn = acc[j] - eta * gc[j];
    *(V*)((T*)a.x_new + (int64_t)i * ld + (int64_t)c * VN) = xn;
    for (int64_t q = s0; q < s1; ++q)  // rows peers read next round: the send buffer is refreshed here
      *(V*)((T*)a.send + (int64_t)a.sslot[q] * ld + (int64_t)c * VN) = xn;
  }
  }
  if (a.xsum && a.slab_cons) {
    const double cs = wave_sum((double)hsum<T>(dv));
    if constexpr (WPW == 1) {
      if (live && lane == 0) a.slab_cons[i] = cs;
    } else {  // the worker's waves meet in LDS, summed in slice order
      if (lane == 0) cred[wave] = cs;
      __syncthreads();
      if (live && lane == 0 && wave % WPW == 0) {
        double t = cred[wave];
#pragma unroll
        for (int q = 1; q < WPW; ++q) t += cred[wave + q];
        a.slab_cons[i] = t;
      }
    }
  }
}

template <typename T>
static hipError_t launch_mix_t(int cpl, const RoundArgs& a, const T* G, int n, hipStream_t s) {
  const dim3 grid((n + NW - 1) / NW);
  if (cpl == 8 || cpl == 16) {  // rows of 8 / 16 chunks per lane: several waves per worker
    const int wpw = cpl / 4;
    const dim3 g2(((int64_t)n * wpw + NW - 1) / NW);
    if (wpw == 2) hipLaunchKernelGGL((k_mix<T, 4, 2>), g2, dim3(NT), 0, s, a, G, n);
    else hipLaunchKernelGGL((k_mix<T, 4, 4>), g2, dim3(NT), 0, s, a, G, n);
    return hipGetLastError();
  }
  switch (cpl) {
    case 1: hipLaunchKernelGGL((k_mix<T, 1>), grid, dim3(NT), 0, s, a, G, n); break;
    case 2: hipLaunchKernelGGL((k_mix<T, 2>), grid, dim3(NT), 0, s, a, G, n); break;
    case 4: hipLaunchKernelGGL((k_mix<T, 4>), grid, dim3(NT), 0, s, a, G, n); break;
    case 8: hipLaunchKernelGGL((k_mix<T, 8>), grid, dim3(NT), 0, s, a, G, n); break;
    case 16: hipLaunchKernelGGL((k_mix<T, 16>), grid, dim3(NT), 0, s, a, G, n); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_mix(int dtype, int cpl, const RoundArgs& a, const void* G, int n_workers, hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  return dtype == 0 ? launch_mix_t<float>(cpl, a, (const float*)G, n_workers, s)
                    : launch_mix_t<double>(cpl, a, (const double*)G, n_workers, s);
}

// ---------------------------------------------------------------------------- lagged mix + column sums
// k_mixcs (round 4): the lagged schedule's mix (k_mix with a.xsum) with the column sums of the new
// iterates fused in, so a multi-GPU round is the gradient pass, this and k_mixcs_final, and the
// next round's exchange carries the column sums beside the halo rows (no all-reduce; every rank
// sums the ranks' vectors in rank order, so all ranks hold the same bits).
//   block 0: the history fold of McsArgs' caller (FoldArgs; nothing when no output is set);
//   block 1 + g * ncb + cb: workers [g R, g R + R) x state chunks [64 CPB cb, 64 CPB (cb + 1)).
// A wave takes workers g R + w, g R + w + 4, ..., two at a time (every load of both in flight at
// once); per worker: xbar of x_old from the rank-ordered sums, the consensus partial of this column
// block, the mix + step (CSR order and arithmetic of k_mix / k_round: bitwise the same iterates) or,
// for an interior worker the gradient kernel stepped, its new row read back; the new rows' column
// sums accumulate per lane in float64 in worker order, meet in LDS in wave order, and go to part[g];
// k_mixcs_final (the next launch) sums part[0..ng) of each column block in group order and writes
// the sums to own_out and to every peer's sum rows in the send buffer.  (Round 4 measured a one-launch
// form -- the last arriving workgroup of a column block summing write-through partials after an
// agent-scope ticket -- at ~9 us more per round at 512 workers than the second launch)
template <int RW>
__device__ void fold_block_rw(const FoldArgs& f, int nch, int vn, double (*red)[RW]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double a = 0.0, b = 0.0, q = 0.0;
  if (f.sc && f.out_c) a = fold_sum4(f.sc, f.nc);
  if (f.sl && f.out_l) b = fold_sum4(f.sl, f.nl);
  if (f.xbar && f.out_q)
    q = vn == 2 ? fold_xnorm<double>((const double*)f.xbar, nch, 2) : fold_xnorm<float>((const float*)f.xbar, nch, 4);
  a = wave_sum(a);
  b = wave_sum(b);
  q = wave_sum(q);
  if (lane == 0) {
    red[wave][0] = a;
    red[wave][1] = b;
    red[wave][2] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0, sq = 0.0;
    for (int k = 0; k < NW; ++k) {
      sa += red[k][0];
      sb += red[k][1];
      sq += red[k][2];
    }
    if (f.out_c) *f.out_c = sa;
    if (f.out_l) *f.out_l = sb;
    if (f.out_q) *f.out_q = sq;
  }
}

// Column sum of global column `col` over every rank's vector, in rank order (k_mixcs, k_xbar_ranks);
// eight ranks' loads in flight at a time (one memory latency for a node of 8 GPUs, not eight).
template <typename T>
__device__ __forceinline__ double ranks_sum(const McsArgs& m, const T* halo, int64_t ld, int64_t col) {
  double s = 0.0;
  for (int p0 = 0; p0 < m.world; p0 += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int p = p0 + k;
      // p's sums: the halo row they arrived in, or -- this rank, unless its own sums travel through the
      // exchange too (a self block: RCCL world 1 with the collectives forced) -- own_in
      const int64_t row = p >= m.world ? -1 : p < kMcsKargRanks ? (int64_t)m.kin[p] : m.sum_in[p];
      v[k] = p >= m.world ? 0.0 : row < 0 ? m.own_in[col] : ((const double*)(halo + row * ld))[col];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (p0 + k < m.world) s += v[k];
  }
  return s;
}

constexpr int kMixcsBatch = 16;        // group partials loaded per batch (all in flight; few VGPRs, so
                                       // k_mixcs_final fits beside two round-kernel workgroups per CU)
constexpr int kMixcsMaxGroups = 1024;  // mixcs_shape keeps ng <= this

// The group partials by plain stores; k_mixcs_final, a second launch after a stream hand-off, sums them.
// (Round 5 also tried a form in which the launch's last workgroup released a sequence number for the side
// stream to wait on, so that no event sat on the engine stream: the agent-scope release of every
// workgroup took k_mixcs from 6 to 35 us and the side stream's spinning wait slowed the gradient kernel
// beside it; profiles/r5_sync_ab.txt.)
template <typename T, int CPB>
__global__ __launch_bounds__(NT) void k_mixcs(const RoundArgs a, const T* __restrict__ G, int n, const McsArgs m,
                                              const FoldArgs fold) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  constexpr int MAXE = 6;            // CSR entries held in registers (the rest of a longer row: loaded at use)
  constexpr int MAXS = 2;            // send slots of a row held in registers (the rest: loaded at use)
  constexpr int BC = 64 * CPB * VN;  // columns of a column block
  constexpr int XR = 2 * NW;         // ranks' sums staged through LDS per pass (two per wave)
  constexpr int XT = BC / 64;        // columns per lane in the staging
  __shared__ double red[NW][BC];
  __shared__ double xsum[XR][BC];
  if (blockIdx.x == 0) {
    fold_block_rw<BC>(fold, a.nchunks, VN, red);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = (int)blockIdx.x - 1;
  const int cb = b % m.ncb, g = b / m.ncb;
  const int64_t ld = a.ld;
  const int nch = a.nchunks;
  const int cbase = cb * 64 * CPB;
  const int64_t colbase = (int64_t)cbase * VN, ncol = (int64_t)nch * VN;
  const T eta = (T)a.eta;
  const T* halo = (const T*)a.halo;
  const int i_end = (g + 1) * m.r < n ? (g + 1) * m.r : n;

  // Every load of a wave's two workers is issued before any of them is used: (A) the CSR range,
  // interior flag, send range and own row, (B) the CSR columns, the send slots and the gradient
  // (or, for an interior worker, the row the gradient kernel stepped), (C) the neighbour rows.
  V own[2][CPB], gv[2][CPB], r[2][MAXE][CPB];
  int64_t e0[2], e1[2], s0[2], s1[2];
  int32_t sl[2][MAXS];
  bool live[2], skip[2];
  auto issue = [&](int i0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * NW;
      live[u] = i < i_end;
      e0[u] = live[u] ? a.rp[i] : 0;
      e1[u] = live[u] ? a.rp[i + 1] : 0;
      skip[u] = live[u] && a.interior && a.interior[i];
      s0[u] = (live[u] && a.sptr) ? a.sptr[i] : 0;
      s1[u] = (live[u] && a.sptr) ? a.sptr[i + 1] : 0;
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const int c = cbase + lane + 64 * j;
        own[u][j] = (live[u] && c < nch) ? *(const V*)((const T*)a.x_old + (int64_t)i * ld + (int64_t)c * VN) : V(0);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * NW;
#pragma unroll
      for (int q = 0; q < MAXS; ++q) sl[u][q] = (!skip[u] && s0[u] + q < s1[u]) ? a.sslot[s0[u] + q] : -1;
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const int c = cbase + lane + 64 * j;
        const bool in = live[u] && c < nch;
        // an interior worker's new row (written by the gradient kernel) comes back in gv
        gv[u][j] = !in ? V(0) : skip[u] ? *(const V*)((const T*)a.x_new + (int64_t)i * ld + (int64_t)c * VN)
                                        : *(const V*)(G + (int64_t)i * ld + (int64_t)c * VN);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int k = 0; k < MAXE; ++k) {
        if (!skip[u] && e0[u] + k < e1[u]) {
          const int col = a.ci[e0[u] + k];
          const T* src = col < a.n_local ? (const T*)a.x_old + (int64_t)col * ld : halo + (int64_t)(col - a.n_local) * ld;
#pragma unroll
          for (int j = 0; j < CPB; ++j) {
            const int c = cbase + lane + 64 * j;
            r[u][k][j] = c < nch ? *(const V*)(src + (int64_t)c * VN) : V(0);
          }
        }
      }
    }
  };

  // xbar of x_old at this lane's chunks, (T)(sum / n) of the ranks' column sums added in rank order
  // (as k_xbar_ranks / k_colsum_final round it).  The ranks' sums of this column block come through
  // LDS, XR ranks per pass, wave w loading ranks w and w + NW of the pass: a rank's row is read by
  // one wave, and the first pass's loads are in flight with the first workers' rows.
  double xv[2][XT];
  auto xload = [&](int p0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = p0 + wave + k * NW;
      const double* src = nullptr;
      if (p < m.world) {
        const int64_t row = p < kMcsKargRanks ? (int64_t)m.kin[p] : m.sum_in[p];
        src = row < 0 ? m.own_in : (const double*)(halo + row * ld);  // (row < 0: this rank, no self block)
      }
#pragma unroll
      for (int t = 0; t < XT; ++t) {
        const int64_t col = colbase + lane + 64 * t;
        xv[k][t] = (src && col < ncol) ? src[col] : 0.0;
      }
    }
  };
  double xs[CPB][VN];
#pragma unroll
  for (int j = 0; j < CPB; ++j)
#pragma unroll
    for (int e = 0; e < VN; ++e) xs[j][e] = 0.0;
  auto xfold = [&](int p0) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int t = 0; t < XT; ++t) xsum[wave + k * NW][lane + 64 * t] = xv[k][t];
    __syncthreads();
    for (int q = 0; q < XR && p0 + q < m.world; ++q)
#pragma unroll
      for (int j = 0; j < CPB; ++j)
#pragma unroll
        for (int e = 0; e < VN; ++e) xs[j][e] += xsum[q][(lane + 64 * j) * VN + e];
    __syncthreads();
  };
  xload(0);
  int i0 = g * m.r + wave;
  issue(i0);
  xfold(0);
  for (int p0 = XR; p0 < m.world; p0 += XR) {  // more than XR ranks: further passes
    xload(p0);
    xfold(p0);
  }
  V xb[CPB];
#pragma unroll
  for (int j = 0; j < CPB; ++j) {
    const int c = cbase + lane + 64 * j;
#pragma unroll
    for (int e = 0; e < VN; ++e) xb[j][e] = c < nch ? (T)(xs[j][e] / m.n_div) : T(0);
    if (c < nch && g == 0 && wave == 0 && a.xbar_out) *(V*)((T*)a.xbar_out + (int64_t)c * VN) = xb[j];
  }

  double cs[CPB][VN];
#pragma unroll
  for (int j = 0; j < CPB; ++j)
#pragma unroll
    for (int e = 0; e < VN; ++e) cs[j][e] = 0.0;
  for (bool first = true; i0 < i_end; i0 += 2 * NW, first = false) {
    if (!first) issue(i0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!live[u]) continue;
      const int i = i0 + u * NW;
      V dv = V(0);
      V xn[CPB];
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const V t = own[u][j] - xb[j];  // consensus term of x_old[i] (zero past the row: both 0)
        dv += t * t;
        if (skip[u]) {
          xn[j] = gv[u][j];
        } else {
          V acc = V(0);
#pragma unroll
          for (int k = 0; k < MAXE; ++k)
            if (e0[u] + k < e1[u]) acc += ((const T*)a.cw)[e0[u] + k] * r[u][k][j];
          for (int64_t e = e0[u] + MAXE; e < e1[u]; ++e) {  // longer rows (dense graphs): CSR order
            const int col = a.ci[e];
            const T* src = col < a.n_local ? (const T*)a.x_old + (int64_t)col * ld : halo + (int64_t)(col - a.n_local) * ld;
            const int c = cbase + lane + 64 * j;
            acc += ((const T*)a.cw)[e] * (c < nch ? *(const V*)(src + (int64_t)c * VN) : V(0));
          }
          xn[j] = acc - eta * gv[u][j];
        }
      }
      if (m.cons_part) {
        const double t = wave_sum((double)hsum<T>(dv));
        if (lane == 0) m.cons_part[(int64_t)cb * n + i] = t;
      }
#pragma unroll
      for (int j = 0; j < CPB; ++j) {
        const int c = cbase + lane + 64 * j;
        if (c >= nch) continue;
#pragma unroll
        for (int e = 0; e < VN; ++e) cs[j][e] += (double)xn[j][e];
        if (skip[u]) continue;
        *(V*)((T*)a.x_new + (int64_t)i * ld + (int64_t)c * VN) = xn[j];
#pragma unroll
        for (int q = 0; q < MAXS; ++q)  // rows peers read next round
          if (sl[u][q] >= 0) *(V*)((T*)a.send + (int64_t)sl[u][q] * ld + (int64_t)c * VN) = xn[j];
        for (int64_t q = s0[u] + MAXS; q < s1[u]; ++q)
          *(V*)((T*)a.send + (int64_t)a.sslot[q] * ld + (int64_t)c * VN) = xn[j];
      }
    }
  }
  // this group's partial of the column block: waves in order
#pragma unroll
  for (int j = 0; j < CPB; ++j)
#pragma unroll
    for (int e = 0; e < VN; ++e) red[wave][(lane + 64 * j) * VN + e] = cs[j][e];
  __syncthreads();
  for (int t = threadIdx.x; t < BC; t += NT) {
    if (colbase + t >= ncol) break;
    m.part[(int64_t)g * ld + colbase + t] = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
  }
}

// The second launch of k_mixcs: the ng group partials of every column,
// summed per column block -- workgroup (64 columns), wave w summing groups [w ng / 4, (w + 1) ng / 4)
// in group order with 64 loads in flight, the four waves' sums added in wave order through LDS --
// to own_out and to every peer's sum rows.  The kernel boundary is the hand-off: the single-launch
// form's write-through stores, agent-scope ticket and acquire cost ~9 us of dependent latency per
// round at 512 workers (timing-only cuts, profiles/r4_mixcs_cut.txt), the boundary a few.
template <typename T>
__global__ __launch_bounds__(NT) void k_mixcs_final(const McsArgs m, int64_t ld, int nch, T* send) {
  constexpr int VN = VT<T>::n;
  __shared__ double red[NW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + lane, ncol = (int64_t)nch * VN;
  const int q0 = (int)((int64_t)m.ng * wave / NW), q1 = (int)((int64_t)m.ng * (wave + 1) / NW);
  double s = 0.0;
  if (col < ncol) {
    for (int qb = q0; qb < q1; qb += kMixcsBatch) {
      double v[kMixcsBatch];
#pragma unroll
      for (int q = 0; q < kMixcsBatch; ++q) v[q] = qb + q < q1 ? m.part[(int64_t)(qb + q) * ld + col] : 0.0;
#pragma unroll
      for (int q = 0; q < kMixcsBatch; ++q)
        if (qb + q < q1) s += v[q];
    }
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && col < ncol) {
    const double t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    m.own_out[col] = t;
    for (int p = 0; p < m.world; ++p) {
      const int64_t row = p < kMcsKargRanks ? (int64_t)m.kout[p] : m.sum_out[p];
      if (row >= 0) ((double*)(send + row * ld))[col] = t;
    }
  }
}

// One 16-byte chunk per lane of a k_mixcs column block: twice the column blocks of two chunks, 105 VGPRs
// (four waves per SIMD instead of two at 192), and, with every worker mixed there, 40.0 vs 48.5 us at 4096
// workers and 11.0 vs 13.6 at 512 (profiles/r4_mixcs_cpb.txt)
constexpr int kMixcsCpb = 1;

void mixcs_shape(int dtype, int64_t n, int32_t nch, int32_t* ncb, int32_t* r, int32_t* ng) {
  constexpr int CPB = kMixcsCpb;
  (void)dtype;
  *ncb = (nch + 64 * CPB - 1) / (64 * CPB);
  // groups of 8 workers (one iteration of the two-worker loop per wave), up to kMixcsMaxGroups groups:
  // many short workgroups rather than few long ones -- a wave's workers run one after the other, each
  // a few dependent memory round trips (profiles/r4_mixcs_groups.txt)
  int64_t rr = 8;
  while ((n + rr - 1) / rr > kMixcsMaxGroups) rr += 8;
  *r = (int32_t)rr;
  *ng = (int32_t)std::max<int64_t>(1, (n + rr - 1) / rr);
}

hipError_t launch_mixcs(int dtype, const RoundArgs& a, const void* G, int n_workers, const McsArgs& m,
                        const FoldArgs* fold, hipStream_t s, hipStream_t side, hipEvent_t ev) {
  FoldArgs f;
  memset(&f, 0, sizeof(f));
  if (fold) f = *fold;
  const McsArgs& mm = m;
  const dim3 grid(1 + (unsigned)m.ng * (unsigned)m.ncb);
  if (dtype == 0)
    hipLaunchKernelGGL((k_mixcs<float, kMixcsCpb>), grid, dim3(NT), 0, s, a, (const float*)G, n_workers, mm, f);
  else
    hipLaunchKernelGGL((k_mixcs<double, kMixcsCpb>), grid, dim3(NT), 0, s, a, (const double*)G, n_workers, mm, f);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipStream_t fs = s;
  if (side && ev) {  // k_mixcs_final on the side stream, after an event on the engine stream
    if ((e = hipEventRecord(ev, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(side, ev, 0)) != hipSuccess) return e;
    fs = side;
  }
  const int vn = dtype == 0 ? 4 : 2;
  const dim3 g2((unsigned)(((int64_t)a.nchunks * vn + 63) / 64));
  if (dtype == 0)
    hipLaunchKernelGGL(k_mixcs_final<float>, g2, dim3(NT), 0, fs, mm, a.ld, a.nchunks, (float*)a.send);
  else
    hipLaunchKernelGGL(k_mixcs_final<double>, g2, dim3(NT), 0, fs, mm, a.ld, a.nchunks, (double*)a.send);
  return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(NT) void k_xbar_ranks(const McsArgs m, const T* __restrict__ halo, int64_t ld, int nch,
                                                   T* xbar_out, T* send) {
  constexpr int VN = VT<T>::n;
  const int64_t col = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (col >= (int64_t)nch * VN) return;
  if (xbar_out) xbar_out[col] = (T)(ranks_sum<T>(m, halo, ld, col) / m.n_div);
  if (send)
    for (int p = 0; p < m.world; ++p)
      if (m.sum_out[p] >= 0) ((double*)(send + m.sum_out[p] * ld))[col] = m.own_in[col];
}

hipError_t launch_xbar_ranks(int dtype, const McsArgs& m, const void* halo, int64_t ld, int32_t nch, void* xbar_out,
                             void* send, hipStream_t s) {
  const int vn = dtype == 0 ? 4 : 2;
  const dim3 grid((unsigned)(((int64_t)nch * vn + NT - 1) / NT));
  if (dtype == 0)
    hipLaunchKernelGGL(k_xbar_ranks<float>, grid, dim3(NT), 0, s, m, (const float*)halo, ld, nch, (float*)xbar_out,
                       (float*)send);
  else
    hipLaunchKernelGGL(k_xbar_ranks<double>, grid, dim3(NT), 0, s, m, (const double*)halo, ld, nch,
                       (double*)xbar_out, (double*)send);
  return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(NT) void k_gather_rows(const T* __restrict__ x, const int32_t* ids, int64_t n,
                                                    int64_t ld, int nch, T* __restrict__ dst) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * NW + (threadIdx.x >> 6);
  if (k >= n) return;
  const int64_t r = ids[k];
  if (r < 0) return;  // not a worker's row (a column-sum row of the lagged exchange)
  for (int c = lane; c < nch; c += 64)
    *(V*)(dst + k * ld + (int64_t)c * VN) = *(const V*)(x + r * ld + (int64_t)c * VN);
}

hipError_t launch_gather_rows(int dtype, const void* x, const int32_t* ids, int64_t n, int64_t ld,
                              int32_t nchunks, void* dst, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + NW - 1) / NW));
  if (dtype == 0)
    hipLaunchKernelGGL(k_gather_rows<float>, grid, dim3(NT), 0, s, (const float*)x, ids, n, ld, nchunks,
                       (float*)dst);
  else
    hipLaunchKernelGGL(k_gather_rows<double>, grid, dim3(NT), 0, s, (const double*)x, ids, n, ld, nchunks,
                       (double*)dst);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- the pull transport
// One launch pulls every peer's block of this round (DOPT_TRANSPORT=ipc, runtime.cpp "pull transport"): block b
// of the grid's y dimension copies the 16-byte chunks of peer block b from the peer's send slot (a pointer into
// the peer's allocation, opened through its IPC handle) into this rank's halo.  The ordering against the peer's
// writes is the peer's interprocess event, waited for before the launch; the slots are uncached allocations
// (written through to memory by the peer's kernels) and the loads are system-scope (sc0 sc1: no L2 line of an
// earlier round of the same slot can answer them), so the copy sees the peer's round on another GPU too.
// Vector loads and stores only.
__global__ __launch_bounds__(NT) void k_pull(const PullArgs a, int slot) {
  const int b = blockIdx.y;
  const uint64_t* __restrict__ src = (const uint64_t*)a.src[2 * b + slot];
  uint4* __restrict__ dst = (uint4*)(a.dst + a.dst_off[b]);
  const int64_t n = a.n16[b];
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const uint64_t lo = __hip_atomic_load(src + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t hi = __hip_atomic_load(src + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    dst[i] = make_uint4((unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32));
  }
}

hipError_t launch_pull(const PullArgs& a, int slot, hipStream_t s) {
  if (a.nb <= 0) return hipSuccess;
  // enough workgroups for the largest block at 4 chunks per thread, at most 64 per block (a few MB per
  // peer per round: the copy is latency-bound over xGMI, not a full-chip stream)
  const int64_t gx = std::min<int64_t>(64, std::max<int64_t>(1, (a.max16 + 4 * NT - 1) / (4 * NT)));
  hipLaunchKernelGGL(k_pull, dim3((unsigned)gx, (unsigned)a.nb), dim3(NT), 0, s, a, slot);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- synthetic data
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double unif01(uint64_t h) {  // (0, 1]
  return ((double)(h >> 11) + 1.0) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double normal_at(uint64_t seed, uint64_t a, uint64_t b) {
  const uint64_t h = mix64(seed ^ mix64(a * 0xD1B54A32D192ED03ull + b));
  const double u1 = unif01(h), u2 = unif01(mix64(h));
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

// The planted w* of the synthetic labels, once per data set (k_generate reads it per element).
__global__ __launch_bounds__(NT) void k_wstar(double* w, int64_t d, uint64_t seed) {
  for (int64_t c = (int64_t)blockIdx.x * NT + threadIdx.x; c < d; c += (int64_t)gridDim.x * NT)
    w[c] = normal_at(seed ^ 0x5DEECE66Dull, 0, (uint64_t)c);
}

// Two standard normals from one 64-bit hash: Box-Muller on two 24-bit uniforms, in float with
// the hardware log / sqrt / sin / cos (both outputs of the transform are used).  The values are
// float32 numbers, so float32 and float64 contexts hold exactly the same data.
__device__ __forceinline__ void normal_pair(uint64_t key, uint64_t j, float& a, float& b) {
  const uint64_t h = mix64(key ^ (j * 0xD1B54A32D192ED03ull));
  const float u1 = ((float)(uint32_t)(h >> 40) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  const float u2 = (float)(uint32_t)(h & 0xFFFFFFu) * (1.0f / 16777216.0f);     // [0, 1)
  const float r = __builtin_sqrtf(-2.0f * __logf(u1));
  float s, c;
  __sincosf(6.28318530717958647f * u2, &s, &c);
  a = r * c;
  b = r * s;
}

// Workgroup = GR consecutive rows; thread t writes element quads t, t + NT, ... of each of them
// (16-byte float stores / two 16-byte double stores), so w* is read once per GR rows and the
// labels' dots (float64, the row's values times w*) fold over the threads in a fixed order.
// xrows > 0: X in the column-block tiled layout of column-blocked contexts (kcommon.h XAddr;
// ld = the padded row length, whole tiles), else row-major with stride ld.
constexpr int kGenRows = 8;
template <typename T>
__global__ __launch_bounds__(NT) void k_generate(T* X, T* y, int64_t rows, int64_t d, int64_t ld, int64_t xrows,
                                                 const double* __restrict__ wstar, uint64_t seed, double flip,
                                                 double noise, int problem, int64_t row_base) {
  constexpr int GR = kGenRows;
  constexpr int64_t TE = kTileChunks * (16 / sizeof(T));  // elements of a row in one tile
  __shared__ double sdot[NW][GR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t rl0 = (int64_t)blockIdx.x * GR;
  const int nr = (int)min((int64_t)GR, rows - rl0);
  uint64_t key[GR];
  double dot[GR];
#pragma unroll
  for (int k = 0; k < GR; ++k) {
    // values depend on the GLOBAL row: a rank's slice equals the same rows of the single-GPU set
    key[k] = mix64(seed ^ mix64((uint64_t)(row_base + rl0 + k) + 1));
    dot[k] = 0.0;
  }
  for (int64_t q = threadIdx.x; 4 * q < ld; q += NT) {
    const int64_t c0 = 4 * q;
    double ws[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) ws[e] = c0 + e < d ? wstar[c0 + e] : 0.0;
#pragma unroll
    for (int k = 0; k < GR; ++k) {
      if (k < nr) {
        float v[4];
        normal_pair(key[k], 2 * q, v[0], v[1]);
        normal_pair(key[k], 2 * q + 1, v[2], v[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t c = c0 + e;
          if (c >= d - 1) v[e] = c == d - 1 ? 1.0f : 0.0f;  // bias column (utils.py:28), then padding
          dot[k] += (double)v[e] * ws[e];                   // planted w*
        }
        const int64_t rl = rl0 + k;
        T* dst = X + (xrows ? ((c0 / TE) * xrows + rl) * TE + c0 % TE : rl * ld + c0);
        if constexpr (sizeof(T) == 4) {
          *(typename VT<float>::v*)dst = typename VT<float>::v{v[0], v[1], v[2], v[3]};
        } else {
          *(typename VT<double>::v*)dst = typename VT<double>::v{(double)v[0], (double)v[1]};
          if (c0 + 2 < ld) *(typename VT<double>::v*)(dst + 2) = typename VT<double>::v{(double)v[2], (double)v[3]};
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < GR; ++k) {
    const double s = wave_sum(dot[k]);
    if (lane == 0) sdot[wave][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < nr) {
    const int k = threadIdx.x;
    const int64_t r = row_base + rl0 + k;
    double dt = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) dt += sdot[w][k];
    if (problem == 0) {
      T lab = dt >= 0.0 ? T(1) : T(-1);
      if (unif01(mix64(seed ^ mix64(~(uint64_t)r))) <= flip) lab = -lab;
      y[rl0 + k] = lab;
    } else {
      y[rl0 + k] = (T)(dt + noise * normal_at(seed ^ 0xA5A5A5A5ull, (uint64_t)r, 0xFFFFFFFFull));
    }
  }
}

hipError_t launch_generate(int dtype, int problem, void* X, void* y, int64_t rows, int64_t d,
                           int64_t ld, int64_t xrows, double* wstar, uint64_t seed, double flip, double noise,
                           int64_t row_base, hipStream_t s) {
  hipLaunchKernelGGL(k_wstar, dim3((unsigned)std::min<int64_t>(1024, (d + NT - 1) / NT)), dim3(NT), 0, s, wstar, d,
                     seed);
  if (rows <= 0) return hipGetLastError();
  if (ld % (dtype == 0 ? 4 : 2) != 0) return hipErrorInvalidValue;  // rows are whole 16-byte chunks
  const dim3 grid((unsigned)((rows + kGenRows - 1) / kGenRows));
  if (dtype == 0)
    hipLaunchKernelGGL(k_generate<float>, grid, dim3(NT), 0, s, (float*)X, (float*)y, rows, d, ld, xrows,
                       (const double*)wstar, seed, flip, noise, problem, row_base);
  else
    hipLaunchKernelGGL(k_generate<double>, grid, dim3(NT), 0, s, (double*)X, (double*)y, rows, d, ld, xrows,
                       (const double*)wstar, seed, flip, noise, problem, row_base);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- clock stamp
__global__ void k_stamp(uint64_t* out) { *out = wall_clock64(); }

hipError_t launch_stamp(uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, s, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- conversion
template <typename T, typename S>
__global__ __launch_bounds__(NT) void k_convert(const S* __restrict__ src, T* __restrict__ dst,
                                                int64_t rows, int64_t d, int64_t ld) {
  const int64_t total = rows * ld;
  for (int64_t k = (int64_t)blockIdx.x * NT + threadIdx.x; k < total; k += (int64_t)gridDim.x * NT) {
    const int64_t r = k / ld, c = k - r * ld;
    dst[k] = c < d ? (T)src[r * d + c] : T(0);
  }
}

// Host rows [nr x d] -> rows r0 .. r0 + nr of a column-block tiled array of xrows rows (row length
// ld, whole tiles), zero padded.
template <typename T, typename S>
__global__ __launch_bounds__(NT) void k_convert_tiled(const S* __restrict__ src, T* __restrict__ dst, int64_t r0,
                                                      int64_t nr, int64_t d, int64_t ld, int64_t xrows) {
  constexpr int64_t TE = kTileChunks * (16 / sizeof(T));
  const int64_t total = nr * ld;
  for (int64_t k = (int64_t)blockIdx.x * NT + threadIdx.x; k < total; k += (int64_t)gridDim.x * NT) {
    const int64_t r = k / ld, c = k - r * ld;
    dst[((c / TE) * xrows + r0 + r) * TE + c % TE] = c < d ? (T)src[r * d + c] : T(0);
  }
}

// Rows r0 .. r0 + nr of a tiled array -> row-major dst [nr x ld] (downloads, parity checks).
template <typename T>
__global__ __launch_bounds__(NT) void k_untile(const T* __restrict__ X, int64_t xrows, int64_t r0, int64_t nr,
                                               int64_t ld, T* __restrict__ dst) {
  constexpr int64_t TE = kTileChunks * (16 / sizeof(T));
  const int64_t total = nr * ld;
  for (int64_t k = (int64_t)blockIdx.x * NT + threadIdx.x; k < total; k += (int64_t)gridDim.x * NT) {
    const int64_t r = k / ld, c = k - r * ld;
    dst[k] = X[((c / TE) * xrows + r0 + r) * TE + c % TE];
  }
}

static dim3 grid_for(int64_t total) {
  int64_t blocks = (total + NT - 1) / NT;
  return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(blocks, 8192)));
}

hipError_t launch_convert_tiled(int dtype, const void* src, int src_f32, void* dst, int64_t r0, int64_t nr, int64_t d,
                                int64_t ld, int64_t xrows, hipStream_t s) {
  const dim3 grid = grid_for(nr * ld);
  if (dtype == 0) {
    if (src_f32) hipLaunchKernelGGL((k_convert_tiled<float, float>), grid, dim3(NT), 0, s, (const float*)src, (float*)dst, r0, nr, d, ld, xrows);
    else hipLaunchKernelGGL((k_convert_tiled<float, double>), grid, dim3(NT), 0, s, (const double*)src, (float*)dst, r0, nr, d, ld, xrows);
  } else {
    if (src_f32) hipLaunchKernelGGL((k_convert_tiled<double, float>), grid, dim3(NT), 0, s, (const float*)src, (double*)dst, r0, nr, d, ld, xrows);
    else hipLaunchKernelGGL((k_convert_tiled<double, double>), grid, dim3(NT), 0, s, (const double*)src, (double*)dst, r0, nr, d, ld, xrows);
  }
  return hipGetLastError();
}

hipError_t launch_untile(int dtype, const void* X, int64_t xrows, int64_t r0, int64_t nr, int64_t ld, void* dst,
                         hipStream_t s) {
  const dim3 grid = grid_for(nr * ld);
  if (dtype == 0) hipLaunchKernelGGL(k_untile<float>, grid, dim3(NT), 0, s, (const float*)X, xrows, r0, nr, ld, (float*)dst);
  else hipLaunchKernelGGL(k_untile<double>, grid, dim3(NT), 0, s, (const double*)X, xrows, r0, nr, ld, (double*)dst);
  return hipGetLastError();
}

hipError_t launch_convert(int dtype, const void* src, int src_f32, void* dst, int64_t rows, int64_t d,
                          int64_t ld, hipStream_t s) {
  const int64_t total = rows * ld;
  int64_t blocks = (total + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  const dim3 grid((unsigned)blocks);
  if (dtype == 0) {
    if (src_f32)
      hipLaunchKernelGGL((k_convert<float, float>), grid, dim3(NT), 0, s, (const float*)src,
                         (float*)dst, rows, d, ld);
    else
      hipLaunchKernelGGL((k_convert<float, double>), grid, dim3(NT), 0, s, (const double*)src,
                         (float*)dst, rows, d, ld);
  } else {
    if (src_f32)
      hipLaunchKernelGGL((k_convert<double, float>), grid, dim3(NT), 0, s, (const float*)src,
                         (double*)dst, rows, d, ld);
    else
      hipLaunchKernelGGL((k_convert<double, double>), grid, dim3(NT), 0, s, (const double*)src,
                         (double*)dst, rows, d, ld);
  }
  return hipGetLastError();
}

}  // namespace dopt
