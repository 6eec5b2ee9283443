// rowspace.hip -- row-space D-SGD rounds for the complete graph (config C5: quadratic, N = 1024
// workers, d = 2^20, m = b = 16; the logistic objective works the same way).
//
// The reference round (trainer.py:173-175, obj_problems.py:46-53) with the complete-graph MH
// matrix (w_off off the diagonal, W_ii on it, the same for every worker) is
//   x_i' = w_off S + (W_ii - w_off) x_i - eta (X_i^T r_i / m_i + mu x_i),   r_ik = x_i . X_ik - y_ik
//        = a1 xbar + q x_i - eta X_i^T (r_i / m_i),      a1 = w_off N, q = W_ii - w_off - eta mu.
// (logistic, obj_problems.py:13-20: r_ik -> c(z_ik) = -y_ik expit(-y_ik z_ik), still one weight per
// row.)  Every term but q x_i lies in span{xbar} + rowspace(X_i), so iterates that start equal
// (Worker.x = zeros, worker.py:13) stay of the form
//   x_i = Z + X_i^T beta_i       (Z shared: Z' = a1 xbar + q Z;  beta_i' = q beta_i - eta r_i / m_i)
// and the row dots follow without touching x_i:
//   z_ik' = X_ik . x_i' = a1 u_ik + q z_ik - eta sum_l Gram_i[k][l] r_il / m_i,   u_ik = X_ik . xbar
//   xbar' = (a1 + q) xbar - (eta / N) C,   C = sum_ik (r_ik / m_i) X_ik.
// So a round is ONE read-only pass over the shard rows (k_rs_pass: u and C together), a
// per-worker scalar update (k_rs_rows) and an O(d) update (k_rs_cols) -- the 4 GB iterate
// read and the 4 GB iterate write of the direct column-blocked step (k_split_step) are gone.
// The metrics of x_t come out of the same pass:
//   objective at xbar_t: (u_ik - y_ik)^2 over every row  (obj_problems.py:39-44)
//   ||x_i - xbar||^2 = ||D||^2 + sum_k beta_ik (2 X_ik . D + (Gram_i beta_i)_k),  D = Z - xbar,
//   X_ik . D = v_ik - u_ik with v_ik = X_ik . Z carried by v' = a1 u + q v     (trainer.py:185)
// x_i is formed only when asked for (k_rs_materialise: dopt_get_models, other run kinds).
// All sums have a fixed order: runs are bitwise reproducible and chains equal one run.
#include <algorithm>

#include "kcommon.h"

namespace dopt {

template <typename T>
__device__ __forceinline__ typename VT<T>::v rs_ld_nt(const T* p) {
  return __builtin_nontemporal_load((const typename VT<T>::v*)p);
}

// k_rs_pass<T, COLS, CB, NBUF>: workgroup (blk, g) = column block blk (64 * CB 16-byte chunks
// of every row) over the rows of row group g.  Wave w streams a contiguous quarter of the
// group's rows through NBUF rotating row buffers: the loads of rows r+1 .. r+NBUF-1 are in
// flight while row r is processed, and a buffer is refilled right after its row is done (no
// register copies, so the compiler's wait before a row covers that row only; loads past the
// wave's rows re-read its last row).  Per row: the partial dot with xbar over the block
// (64-lane DPP butterfly, stashed one row per lane, stored 64 rows at a time into
// upart[blk][row], in T) and, with COLS, coef_row * row summed into float64 registers (float32
// contexts: in float over each 64-row window, then flushed); the four waves' column sums meet in
// LDS (fixed order) -> cpart[g][columns of blk].  Row weights come 64 rows per vector load, read
// with v_readlane.
//
// rs_pass_body<T, XT, ...>: T = arithmetic and state, XT = storage of the rows.  k_rs_pass<T, ...>
// (XT = T) and k_rs_pass_x32<...> (float64 arithmetic over float32-stored rows, the C3 headline's
// layout: the 16-byte chunk is 4 floats, xbar's 4 doubles stay in registers, every product and
// sum in float64).
// LDOT (round 4): each row's per-lane partial dot goes to LDS instead of a six-step DPP butterfly and
// its dependency chain per row (a wave per SIMD has nothing else to issue while the chain drains);
// after the window, lane k sums row k's partials.  LDOT 1: pdot [64 rows][64 lanes] per wave, lane
// l's value of row k at slot (l + k) % 64, summed in lane order (32 KiB per wave: 147 KiB per
// workgroup, one workgroup per CU; the default).  LDOT 2 (measured in an A/B build): adjacent lanes'
// partials are first added by one DPP quad swap, and the even lanes store [64 rows][32 pairs] (slot
// (l/2 + k) % 32), summed in pair order -- 16 KiB per wave, 80 KiB per workgroup with the column-sum
// LDS, so two workgroups (two waves per SIMD at <= 256 VGPRs) share a CU: 1 % slower than LDOT 1
// (profiles/r4_c5_ldot2.txt) -- the pass does not want more waves, as no shape A/B has shown.
template <typename T, typename XT, bool COLS, int CB, int NBUF, int LDOT = 0>
__device__ __forceinline__ void rs_pass_body(const RsArgs& a, double* red, double* pdot = nullptr) {
  using V = typename VT<XT>::v;
  constexpr int VN = VT<XT>::n;
  constexpr bool SAME = std::is_same<T, XT>::value;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int blk = blockIdx.x + a.blk0, g = blockIdx.y;
  const int nch = a.nch;
  const int64_t ld = a.ld;
  const XT* __restrict__ X = (const XT*)a.X;
  const XAddr<VN> xa(a.tiled ? a.rows : 0, ld);  // column-block tiled rows: each block streams contiguously
  const int64_t r0 = a.grow[g], r1 = a.grow[g + 1];
  const int64_t per = (r1 - r0 + NW - 1) / NW;
  const int64_t wr0 = min(r1, r0 + wave * per), wr1 = min(r1, wr0 + per);
  int cc[CB];
  int64_t co[CB];                   // element offset of chunk cc[j] in row 0
  V xb[SAME ? CB : 1];              // xbar chunks in the row type (XT = T)
  T xbs[SAME ? 1 : CB][SAME ? 1 : VN];  // xbar elements in T (float32 rows, float64 arithmetic)
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const int c = blk * 64 * CB + j * 64 + lane;
    const bool in = c < nch;
    cc[j] = in ? c : nch - 1;  // lanes past the row re-read its last chunk (xbar is 0 there)
    co[j] = xa.col(cc[j]);
    if constexpr (SAME) {
      xb[j] = in ? *(const V*)((const T*)a.xbar + (int64_t)c * VN) : V(0);
    } else {
#pragma unroll
      for (int e = 0; e < VN; ++e) xbs[j][e] = in ? ((const T*)a.xbar)[(int64_t)c * VN + e] : T(0);
    }
  }
  // column sums: T products accumulated over each 64-row window in T, flushed into float64 (a
  // float32 context trades the per-element float64 convert + FMA for one float FMA; float64
  // contexts accumulate in float64 directly)
  constexpr bool TACC = std::is_same<T, float>::value;
  double acc[CB][VN];
  T acct[TACC ? CB : 1][VN];
#pragma unroll
  for (int j = 0; j < CB; ++j)
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      acc[j][e] = 0.0;
      if constexpr (TACC) acct[j][e] = T(0);
    }
  auto flush = [&]() {
    if constexpr (TACC) {
#pragma unroll
      for (int j = 0; j < CB; ++j)
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          acc[j][e] += (double)acct[j][e];
          acct[j][e] = T(0);
        }
    }
  };
  // partial dots: T (a float32 context's 256-1024-element partial dots keep float precision;
  // half the bytes of this launch's only large writes)
  T* __restrict__ up = (T*)a.upart + (int64_t)blk * a.rows;
  double stash = 0.0;
  // the rows' column-sum weights, 64 rows per vector load (lane k: row base + k), one window
  // ahead; row r reads its weight with v_readlane (no scalar load and wait per row)
  const double* __restrict__ cw = a.coef_row;
  auto cwin_load = [&](int64_t base) { return (COLS && base + lane < wr1) ? cw[base + lane] : 0.0; };
  double cw_cur = cwin_load(wr0), cw_nxt = cwin_load(wr0 + 64);
  auto load = [&](int64_t row, V (&dst)[CB]) {
    const XT* p = X + row * xa.rs;
#pragma unroll
    for (int j = 0; j < CB; ++j) dst[j] = rs_ld_nt<XT>(p + co[j]);
  };
  auto process = [&](const V (&rv)[CB], int64_t r) {
    double p = 0.0;
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      if constexpr (SAME) {
        p += (double)hsum<T>(rv[j] * xb[j]);
      } else {
#pragma unroll
        for (int e = 0; e < VN; ++e) p += (double)rv[j][e] * xbs[j][e];
      }
    }
    const double dot = wave_sum_dpp(p);
    const int k = (int)((r - wr0) & 63);
    if constexpr (COLS) {
      const double cf = readlane_t(cw_cur, k);  // wave-uniform
      if constexpr (TACC) {
        const T cft = (T)cf;
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
          for (int e = 0; e < VN; ++e) acct[j][e] += cft * rv[j][e];
      } else {
#pragma unroll
        for (int j = 0; j < CB; ++j)
#pragma unroll
          for (int e = 0; e < VN; ++e) acc[j][e] += cf * (double)rv[j][e];
      }
      if (k == 63) {  // next window
        flush();
        cw_cur = cw_nxt;
        cw_nxt = cwin_load(r + 65);
      }
    }
    if (lane == k) stash = dot;
    if (k == 63 || r + 1 == wr1) {
      if (lane <= k) up[r - k + lane] = (T)stash;
    }
  };
  if constexpr (64 % NBUF == 0) {
    // Windows of 64 rows (NBUF divides 64): a window's weights come in one vector load, its partial
    // dots leave in one store, and no branch sits inside the unrolled row groups of a full window
    // (the buffers rotate in step with the windows).  Partial windows (the wave's last) take the
    // same groups with every row predicated.
    if (wr0 < wr1) {
      const int64_t last = wr1 - 1;
      V buf[NBUF][CB];
#pragma unroll
      for (int k = 0; k < NBUF; ++k) load(min(wr0 + k, last), buf[k]);
      for (int64_t w0 = wr0; w0 < wr1; w0 += 64) {
        const double cwv = cw_cur;
        cw_cur = cw_nxt;
        cw_nxt = cwin_load(w0 + 128);
        const int nw = (int)min((int64_t)64, wr1 - w0);
        double st = 0.0;
        auto row = [&](const V (&rv)[CB], int kk) {
          double p = 0.0;
#pragma unroll
          for (int j = 0; j < CB; ++j) {
            if constexpr (SAME) {
              p += (double)hsum<T>(rv[j] * xb[j]);
            } else {
#pragma unroll
              for (int e = 0; e < VN; ++e) p += (double)rv[j][e] * xbs[j][e];
            }
          }
          double dot = 0.0;
          if constexpr (LDOT == 1) {
            pdot[kk * 64 + ((lane + kk) & 63)] = p;
          } else if constexpr (LDOT == 2) {
            const double pp = dpp_add<0xb1, 0xf, 0xf>(p);  // p[l] + p[l ^ 1] (quad_perm [1,0,3,2])
            if (!(lane & 1)) pdot[kk * 32 + (((lane >> 1) + kk) & 31)] = pp;
          } else {
            dot = wave_sum_dpp(p);
          }
          if constexpr (COLS) {
            const double cf = readlane_t(cwv, kk);  // wave-uniform
            if constexpr (TACC) {
              const T cft = (T)cf;
#pragma unroll
              for (int j = 0; j < CB; ++j)
#pragma unroll
                for (int e = 0; e < VN; ++e) acct[j][e] += cft * rv[j][e];
            } else {
#pragma unroll
              for (int j = 0; j < CB; ++j)
#pragma unroll
                for (int e = 0; e < VN; ++e) acc[j][e] += cf * (double)rv[j][e];
            }
          }
          if constexpr (LDOT == 0) st = lane == kk ? dot : st;
        };
        if (nw == 64) {
          for (int g0 = 0; g0 < 64; g0 += NBUF) {
#pragma unroll
            for (int k = 0; k < NBUF; ++k) {
              row(buf[k], g0 + k);
              load(min(w0 + g0 + k + NBUF, last), buf[k]);
            }
          }
        } else {
          for (int g0 = 0; g0 < nw; g0 += NBUF) {
#pragma unroll
            for (int k = 0; k < NBUF; ++k) {
              if (g0 + k < nw) {
                row(buf[k], g0 + k);
                load(min(w0 + g0 + k + NBUF, last), buf[k]);
              }
            }
          }
        }
        flush();
        if constexpr (LDOT != 0) {  // row `lane` of the window: its partials in lane (pair) order
          constexpr int PW = LDOT == 1 ? 64 : 32;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          double s0 = 0.0;
#pragma unroll 8
          for (int j = 0; j < PW; ++j) s0 += pdot[lane * PW + ((j + lane) & (PW - 1))];
          st = s0;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the next window's stores
        }
        if (lane < nw) up[w0 + lane] = (T)st;
      }
    }
  } else if (wr0 < wr1) {
    const int64_t last = wr1 - 1;
    V buf[NBUF][CB];
#pragma unroll
    for (int k = 0; k < NBUF; ++k) load(min(wr0 + k, last), buf[k]);
    int64_t r = wr0;
    for (; r + NBUF <= wr1; r += NBUF) {
#pragma unroll
      for (int k = 0; k < NBUF; ++k) {
        process(buf[k], r + k);
        load(min(r + k + NBUF, last), buf[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NBUF; ++k)
      if (r + k < wr1) process(buf[k], r + k);
  }
  if constexpr (COLS) {
    flush();
#pragma unroll
    for (int j = 0; j < CB; ++j)
#pragma unroll
      for (int e = 0; e < VN; ++e) red[wave * 64 * CB * VN + (j * 64 + lane) * VN + e] = acc[j][e];
    __syncthreads();
    const int64_t col0 = (int64_t)blk * 64 * CB * VN;
    double* __restrict__ out = a.cpart + (int64_t)g * ld + col0;
    constexpr int W = 64 * CB * VN;
    for (int q = threadIdx.x; q < W; q += NT) {
      if (col0 + q < ld) out[q] = ((red[q] + red[W + q]) + red[2 * W + q]) + red[3 * W + q];
    }
  }
}

template <typename T, bool COLS, int CB, int NBUF, int LDOT = 0>
__global__ __launch_bounds__(NT, LDOT == 2 ? 2 : 1) void k_rs_pass(const RsArgs a) {
  constexpr int PWV = LDOT == 1 ? 64 * 64 : LDOT == 2 ? 64 * 32 : 0;  // pdot doubles per wave
  __shared__ double red[COLS ? NW * 64 * CB * VT<T>::n : 1];
  __shared__ double pdot[LDOT ? NW * PWV : 1];
  rs_pass_body<T, T, COLS, CB, NBUF, LDOT>(a, red, pdot + (threadIdx.x >> 6) * PWV);
}

template <bool COLS, int CB, int NBUF, int LDOT = 0>
__global__ __launch_bounds__(NT, LDOT == 2 ? 2 : 1) void k_rs_pass_x32(const RsArgs a) {  // (LDOT 2: <= 256 VGPRs)
  constexpr int PWV = LDOT == 1 ? 64 * 64 : LDOT == 2 ? 64 * 32 : 0;
  __shared__ double red[COLS ? NW * 64 * CB * VT<float>::n : 1];
  __shared__ double pdot[LDOT ? NW * PWV : 1];
  rs_pass_body<double, float, COLS, CB, NBUF, LDOT>(a, red, pdot + (threadIdx.x >> 6) * PWV);
}

// k_rs_rows: one workgroup per worker (m_i <= 64 rows, lane k = row k).  u_k = sum over the
// pass's column blocks (4 waves x a quarter each, then in wave order); then the metric partials
// of the iterate the pass read (mode & 1), the next round's row state (mode & 2), the initial
// state z = v = u, beta = 0 (mode & 4), or that of unequal starts, z = p0, v = 0, beta = 0 (mode 16).
// With unequal starts (x_i = c x_i(0) + Z + X_i^T beta_i, a.p0 set) the consensus partial of a
// worker is c^2 ||x_i(0) - xbar0||^2 + ||D||^2 + beta . (2 (c p0 + v - u) + G beta), D = c xbar0 +
// Z - xbar: the cross terms 2 c (x_i(0) - xbar0) . D sum to zero over the workers.
template <typename T>
__global__ __launch_bounds__(NT) void k_rs_rows(const RsArgs a, int mode) {
  __shared__ double ured[16][64];
  __shared__ double sb[64], sr[64];
  __shared__ double dred[NW];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = blockIdx.x;
  const int64_t row0 = a.off[i];
  const int m = (int)(a.off[i + 1] - row0);
  const int nb = a.nblk;
  // u_k: the partial dots over the pass's column blocks, in slices of blocks (lane = (slice, row):
  // R lanes per row set, 64 / R slices per wave), four accumulators per lane, slices in order
  const int R = m <= 16 ? 16 : m <= 32 ? 32 : 64;
  const int S = 64 / R, slices = NW * S;
  {
    const int sub = lane / R, k = lane % R, sl = wave * S + sub;
    const int b0 = (int)((int64_t)nb * sl / slices), b1 = (int)((int64_t)nb * (sl + 1) / slices);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if (k < m && !(mode & 8)) {
      const T* u = (const T*)a.upart + row0 + k;
      int b = b0;
      for (; b + 3 < b1; b += 4) {
        s0 += (double)u[(int64_t)b * a.rows];
        s1 += (double)u[(int64_t)(b + 1) * a.rows];
        s2 += (double)u[(int64_t)(b + 2) * a.rows];
        s3 += (double)u[(int64_t)(b + 3) * a.rows];
      }
      for (; b < b1; ++b) s0 += (double)u[(int64_t)b * a.rows];
    }
    ured[sl][k] = (s0 + s1) + (s2 + s3);
  }
  // ||D||^2 = ||Z - xbar||^2 of the iterate the pass read: the block partials of k_rs_cols /
  // k_rs_init, in one fixed order (every workgroup forms the same value)
  double dn = 0.0;
  if (mode & 1) {
    for (int q = threadIdx.x; q < a.nd; q += NT) dn += a.dpart[q];
    dn = wave_sum(dn);
    if (lane == 0) dred[wave] = dn;
  }
  const int64_t s0 = (int64_t)i * a.bcap;
  if (wave == 0) {
    sb[lane] = (lane < m && !(mode & 4)) ? a.beta[s0 + lane] : 0.0;
    sr[lane] = lane < m ? a.coef_row[row0 + lane] : 0.0;
  }
  __syncthreads();
  if (wave != 0) return;
  if (mode & 1) dn = ((dred[0] + dred[1]) + dred[2]) + dred[3];
  const bool live = lane < m;
  double u = 0.0;
  if (live)
    for (int q = 0; q < slices; ++q) u += ured[q][lane];
  const double yv = live ? (a.y_is_f32 ? (double)((const float*)a.y)[row0 + lane] : ((const double*)a.y)[row0 + lane])
                         : 0.0;
  // the gradient's row weight c(z) (obj_problems.py:16-17 logistic / :49-50 quadratic), / m_i
  auto weight = [&](double z) { return (a.problem == 0 ? -yv / (1.0 + exp(yv * z)) : z - yv) / (double)m; };
  if (mode & 4) {  // initial state of iterates that all equal xbar: z = v = X . xbar, beta = 0
    if (live) {
      a.z[s0 + lane] = u;
      a.v[s0 + lane] = u;
      a.beta[s0 + lane] = 0.0;
      a.coef_row[row0 + lane] = weight(u);
    }
    return;
  }
  if (mode & 16) {  // unequal starts: z = X_i . x_i(0), v = X . Z = 0, beta = 0
    if (live) {
      const double z0 = a.p0[s0 + lane];
      a.z[s0 + lane] = z0;
      a.v[s0 + lane] = 0.0;
      a.beta[s0 + lane] = 0.0;
      a.coef_row[row0 + lane] = weight(z0);
    }
    return;
  }
  const double zv = live ? a.z[s0 + lane] : 0.0;
  const double vv = live ? a.v[s0 + lane] : 0.0;
  const double bk = sb[lane];
  double gb = 0.0, gr = 0.0;
  const double* gi = a.gram + ((int64_t)i * a.bcap + lane) * a.bcap;
  if (live) {
    for (int l = 0; l < m; ++l) {
      const double gkl = gi[l];
      gb += gkl * sb[l];
      gr += gkl * sr[l];
    }
  }
  if (mode & 1) {
    const double ls = wave_sum(live ? (a.problem == 0 ? row_loss<double, 0>(yv, u) : row_loss<double, 1>(yv, u)) : 0.0);
    const double xd = a.p0 && live ? a.c * a.p0[s0 + lane] : 0.0;  // X_ik . c x_i(0)
    const double cs = wave_sum(live ? bk * (2.0 * (xd + vv - u) + gb) : 0.0);
    if (lane == 0) {
      if (a.slab_loss) a.slab_loss[i] = ls;
      if (a.slab_cons) a.slab_cons[i] = dn + cs + (a.d0 ? a.c * a.c * a.d0[i] : 0.0);
    }
  }
  if ((mode & 2) && live) {
    const double zn = a.a1 * u + a.q * zv - a.eta * gr;
    a.z[s0 + lane] = zn;
    a.v[s0 + lane] = a.a1 * u + a.q * vv;
    a.beta[s0 + lane] = a.q * bk - a.eta * sr[lane];
    a.coef_row[row0 + lane] = weight(zn);
  }
}

// k_rs_cols: C = sum_g cpart[g] (fixed order; or the all-reduced sums a.csum), then
// xbar' = (a1 + q) xbar - (eta / N) C, Z' = a1 xbar + q Z, the T copy of xbar' for the next
// pass and the metrics, and per-block partials of ||D'||^2, D' = Z' - xbar' (+ q c xbar0 for
// unequal starts).  Columns [e0, e1) (e0 a multiple of NT: block b of the launch is block
// e0 / NT + b of the whole vector), so a column-chunked round updates each chunk as soon as its
// all-reduced sums arrive (distributed.py, dopt_rs_phase_cols_range).
template <typename T>
__global__ __launch_bounds__(NT) void k_rs_cols(const RsArgs a, int64_t e0, int64_t e1) {
  __shared__ double red[2 * NW];
  const int64_t e = e0 + (int64_t)blockIdx.x * NT + threadIdx.x;
  double dd = 0.0, xx = 0.0;
  if (e < e1) {
    double C;
    if (a.csum) {
      C = a.csum[e];
    } else {
      C = 0.0;
      for (int g = 0; g < a.wg; ++g) C += a.cpart[(int64_t)g * a.ld + e];
    }
    const double xo = a.rxbar[e], zo = a.rZ[e];
    const double xn = (a.a1 + a.q) * xo - a.eta_n * C;
    const double zn = a.a1 * xo + a.q * zo;
    a.rxbar[e] = xn;
    a.rZ[e] = zn;
    const T xt = (T)xn;
    ((T*)a.xbar_out)[e] = xt;
    const double dn = a.xbar0 ? (a.q * a.c) * a.xbar0[e] + (zn - xn) : zn - xn;  // D' = c' xbar0 + Z' - xbar'
    dd = dn * dn;
    xx = (double)xt * (double)xt;
  }
  dd = wave_sum(dd);
  xx = wave_sum(xx);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = dd;
    red[NW + (threadIdx.x >> 6)] = xx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t b = e0 / NT + blockIdx.x;
    a.dpart[b] = ((red[0] + red[1]) + red[2]) + red[3];
    a.dpart[a.nd + b] = ((red[NW] + red[NW + 1]) + red[NW + 2]) + red[NW + 3];  // ||xbar'||^2 (as T)
  }
}

// Local column sums C_rank = sum_g cpart[g] into csum, columns [c0, c1) (multi-GPU: all-reduced
// before k_rs_cols; a column-chunked pass reduces each chunk's columns as soon as they are done).
__global__ __launch_bounds__(NT) void k_rs_csum(const RsArgs a, double* out, int64_t c0, int64_t c1) {
  const int64_t e = c0 + (int64_t)blockIdx.x * NT + threadIdx.x;
  if (e >= c1) return;
  double C = 0.0;
  for (int g = 0; g < a.wg; ++g) C += a.cpart[(int64_t)g * a.ld + e];
  out[e] = C;
}

// Z = xbar = row 0 of x (iterates that all equal it), the T copy of xbar, ||D||^2 partials 0.
template <typename T>
__global__ __launch_bounds__(NT) void k_rs_init(const RsArgs a, const T* x0) {
  __shared__ double red[NW];
  const int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x;
  double xx = 0.0;
  if (e < a.ld) {
    const T v = x0[e];
    a.rxbar[e] = (double)v;
    a.rZ[e] = (double)v;
    ((T*)a.xbar_out)[e] = v;
    xx = (double)v * (double)v;
  }
  xx = wave_sum(xx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = xx;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.dpart[blockIdx.x] = 0.0;
    a.dpart[a.nd + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
  }
}

// History row of the row-space rounds (one workgroup, fixed order): out[0] = sum slab_cons[0:n],
// out[1] = sum slab_loss[0:n], out[2] = ||xbar||^2 from k_rs_cols' / k_rs_init's partials.
__global__ __launch_bounds__(NT) void k_rs_hist(const RsArgs a, int n, double* out) {
  __shared__ double red[3][NW];
  auto sum4 = [&](const double* v, int64_t cnt) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int64_t k = threadIdx.x;
    for (; k + 3 * NT < cnt; k += 4 * NT) {
      s0 += v[k];
      s1 += v[k + NT];
      s2 += v[k + 2 * NT];
      s3 += v[k + 3 * NT];
    }
    for (; k < cnt; k += NT) s0 += v[k];
    return wave_sum((s0 + s1) + (s2 + s3));
  };
  const double c = a.slab_cons ? sum4(a.slab_cons, n) : 0.0;
  const double l = a.slab_loss ? sum4(a.slab_loss, n) : 0.0;
  const double q = a.slab_loss ? sum4(a.dpart + a.nd, a.nd) : 0.0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = c;
    red[1][w] = l;
    red[2][w] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 0; k < 3; ++k) out[k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
}

// The history fold of a rank's row-space rounds (dopt_phase_fold while row-space mode is live): k_rs_hist
// with each output optional, the consensus and loss slabs given -- a rank contributes ||xbar||^2 to the
// all-reduced history row only once across the ranks.  The norm is the sum of k_rs_cols' / k_rs_init's
// per-block partials, not a one-workgroup pass over the d-vector (launch_fold: 155 us per round at
// d = 2^20, profiles/r5_rs_chunks.txt).
__global__ __launch_bounds__(NT) void k_rs_fold(const RsArgs a, const double* sc, int64_t nc, const double* sl,
                                                int64_t nl, double* out_c, double* out_l, double* out_q) {
  __shared__ double red[3][NW];
  auto sum4 = [&](const double* v, int64_t cnt) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int64_t k = threadIdx.x;
    for (; k + 3 * NT < cnt; k += 4 * NT) {
      s0 += v[k];
      s1 += v[k + NT];
      s2 += v[k + 2 * NT];
      s3 += v[k + 3 * NT];
    }
    for (; k < cnt; k += NT) s0 += v[k];
    return wave_sum((s0 + s1) + (s2 + s3));
  };
  const double c = (sc && out_c) ? sum4(sc, nc) : 0.0;
  const double l = (sl && out_l) ? sum4(sl, nl) : 0.0;
  const double q = out_q ? sum4(a.dpart + a.nd, a.nd) : 0.0;
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = c;
    red[1][w] = l;
    red[2][w] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* out[3] = {out_c, out_l, out_q};
    for (int k = 0; k < 3; ++k)
      if (out[k]) *out[k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
}

// flags[i * G + g] = 1 when row i of x differs from row 0 on the chunks of group g; zflag[g] = 1
// when row 0 is nonzero there.
template <typename T>
__global__ __launch_bounds__(NT) void k_rs_check(const T* x, int64_t ld, int32_t nch, int32_t* flags,
                                                 int32_t* zflag) {
  using V = typename VT<T>::v;
  constexpr int VN = VT<T>::n;
  const int i = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  int diff = 0, nz = 0;
  for (int c = g * NT + threadIdx.x; c < nch; c += G * NT) {
    const V r0 = *(const V*)(x + (int64_t)c * VN);
    const V ri = *(const V*)(x + (int64_t)i * ld + (int64_t)c * VN);
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      diff |= __builtin_bit_cast(typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type, ri[e]) !=
              __builtin_bit_cast(typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type, r0[e]);
      nz |= r0[e] != T(0);
    }
  }
  diff = __syncthreads_or(diff);
  nz = __syncthreads_or(nz);
  if (threadIdx.x == 0) {
    flags[(int64_t)i * G + g] = diff;
    if (i == 0) zflag[g] = nz;
  }
}

// Gram matrices Gram_i[k][l] = X_ik . X_il (float64) on the float64 matrix cores, partial over
// the column range of workgroup (i, g).  v_mfma_f64_16x16x4_f64 with A = a 16-row block of the
// worker's rows over 4 columns and B = the same (or another 16-row block) transposed: lane l holds
// X[16 b + (l & 15)][col (l >> 4)] for both operands (A[l & 15][l >> 4], B[l >> 4][l & 15]), so one
// 16-byte row chunk per lane feeds VN of them and a Gram block is a single register per operand.
// Lane (i, k) of a wave loads chunk 4 s + k of row i at step s: every load instruction reads 64
// contiguous bytes of each of 16 rows (1 KiB rows of the tiled layout), U steps in flight; the
// waves of a workgroup take groups of U steps round-robin, their accumulators (two per block,
// alternating when there is one block, for two independent dependency chains) fold in LDS in a fixed order.  Products of
// float32 rows are exact in float64; the sums are float64 (the order is the MFMA's).  C/D: lane l,
// register r = Gram block [(l >> 4) + 4 r][l & 15].  gpart[(i * G + g) * P + p], p = the pair
// (k <= l) packed over this worker's m rows.  MB = 16-row blocks (1..4: up to kRsMaxRows rows).
typedef double rs_d4 __attribute__((ext_vector_type(4)));
template <typename XT, int MB>
__global__ __launch_bounds__(NT) void k_rs_gram(const RsArgs a, double* gpart, int P) {
  using V = typename VT<XT>::v;
  constexpr int VN = VT<XT>::n;
  constexpr int NB = MB * (MB + 1) / 2;  // blocks bi <= bj
  constexpr int U = MB >= 3 ? 2 : 4;      // 4-chunk steps in flight per wave
  constexpr int H = NB == 1 ? 2 : 1;      // accumulator sets (one block: two chains)
  __shared__ rs_d4 red[NW - 1][NB][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  const int64_t row0 = a.off[i];
  const int m = (int)(a.off[i + 1] - row0);
  const int ri = lane & 15, kq = lane >> 4;
  const XAddr<VN> xa(a.tiled ? a.rows : 0, a.ld);
  const int64_t nstep = ((int64_t)a.nch + 3) / 4;
  const int64_t s0 = nstep * g / G, s1 = nstep * (g + 1) / G;
  bool rok[MB];
  int64_t rbase[MB];
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    rok[b] = b * 16 + ri < m;
    rbase[b] = (rok[b] ? row0 + b * 16 + ri : row0) * xa.rs;
  }
  rs_d4 acc[H][NB];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int p = 0; p < NB; ++p) acc[h][p] = rs_d4(0.0);
  for (int64_t s = s0 + (int64_t)wave * U; s < s1; s += NW * U) {
    V x[U][MB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = 4 * (s + u) + kq;
      const bool ok = s + u < s1 && c < a.nch;
#pragma unroll
      for (int b = 0; b < MB; ++b) x[u][b] = (ok && rok[b]) ? rs_ld_nt<XT>((const XT*)a.X + rbase[b] + xa.col(c)) : V(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        double xd[MB];
#pragma unroll
        for (int b = 0; b < MB; ++b) xd[b] = (double)x[u][b][e];
        int p = 0;
#pragma unroll
        for (int bi = 0; bi < MB; ++bi)
#pragma unroll
          for (int bj = bi; bj < MB; ++bj, ++p)
            acc[e % H][p] = __builtin_amdgcn_mfma_f64_16x16x4f64(xd[bi], xd[bj], acc[e % H][p], 0, 0, 0);
      }
  }
  if constexpr (H == 2) {
#pragma unroll
    for (int p = 0; p < NB; ++p) acc[0][p] += acc[1][p];
  }
  if (wave > 0) {
#pragma unroll
    for (int p = 0; p < NB; ++p) red[wave - 1][p][lane] = acc[0][p];
  }
  __syncthreads();
  if (wave == 0) {
    double* out = gpart + ((int64_t)i * G + g) * P;
    int p = 0;
#pragma unroll
    for (int bi = 0; bi < MB; ++bi)
#pragma unroll
      for (int bj = bi; bj < MB; ++bj, ++p) {
        rs_d4 t = acc[0][p];
#pragma unroll
        for (int w = 0; w < NW - 1; ++w) t += red[w][p][lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = bi * 16 + (lane >> 4) + 4 * r, l = bj * 16 + (lane & 15);
          if (k <= l && l < m) out[k * m - k * (k - 1) / 2 + (l - k)] = t[r];
        }
      }
  }
}

// Fold the partial Gram matrices over the column ranges (fixed order), symmetric fill.
__global__ __launch_bounds__(NT) void k_rs_gram_fold(const RsArgs a, const double* gpart, int G, int P) {
  const int i = blockIdx.x;
  const int m = (int)(a.off[i + 1] - a.off[i]);
  for (int p = threadIdx.x; p < m * (m + 1) / 2; p += NT) {
    int q = p, k = 0;
    while (q >= m - k) {
      q -= m - k;
      ++k;
    }
    const int l = k + q;
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += gpart[((int64_t)i * G + g) * P + p];
    double* gi = a.gram_w + (int64_t)i * a.bcap * a.bcap;
    gi[k * a.bcap + l] = s;
    gi[l * a.bcap + k] = s;
  }
}

// x_i = Z + X_i^T beta_i (+ c x_i(0): unequal starts) for every worker (T; rows stored as XT),
// chunk-strided over column groups.
template <typename T, typename XT>
__device__ __forceinline__ void rs_materialise_body(const RsArgs& a, T* xout) {
  using V = typename VT<XT>::v;
  constexpr int VN = VT<XT>::n;
  __shared__ double sb[64];
  const int i = blockIdx.x, g = blockIdx.y, G = gridDim.y;
  const int64_t row0 = a.off[i];
  const int m = (int)(a.off[i + 1] - row0);
  const XAddr<VN> xa(a.tiled ? a.rows : 0, a.ld);
  if (threadIdx.x < 64) sb[threadIdx.x] = threadIdx.x < m ? a.beta[(int64_t)i * a.bcap + threadIdx.x] : 0.0;
  __syncthreads();
  for (int c = g * NT + threadIdx.x; c < a.nch; c += G * NT) {
    double s[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) s[e] = a.rZ[(int64_t)c * VN + e];
    if (a.x0) {  // unequal starts: + c x_i(0)
#pragma unroll
      for (int e = 0; e < VN; ++e) s[e] += a.c * (double)((const T*)a.x0)[(int64_t)i * a.ld + (int64_t)c * VN + e];
    }
    for (int k = 0; k < m; ++k) {
      const V r = rs_ld_nt<XT>((const XT*)a.X + xa.at(row0 + k, c));
#pragma unroll
      for (int e = 0; e < VN; ++e) s[e] += sb[k] * (double)r[e];
    }
    if constexpr (std::is_same<T, XT>::value) {
      V o;
#pragma unroll
      for (int e = 0; e < VN; ++e) o[e] = (T)s[e];
      *(V*)(xout + (int64_t)i * a.ld + (int64_t)c * VN) = o;
    } else {
      using W2 = typename VT<T>::v;  // 16-byte stores of T
      constexpr int WN = VT<T>::n;
#pragma unroll
      for (int h = 0; h < VN / WN; ++h) {
        W2 o;
#pragma unroll
        for (int e = 0; e < WN; ++e) o[e] = (T)s[h * WN + e];
        *(W2*)(xout + (int64_t)i * a.ld + (int64_t)c * VN + h * WN) = o;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void k_rs_materialise(const RsArgs a, T* xout) {
  rs_materialise_body<T, T>(a, xout);
}

__global__ __launch_bounds__(NT) void k_rs_materialise_x32(const RsArgs a, double* xout) {
  rs_materialise_body<double, float>(a, xout);
}

// ---------------------------------------------------------------------------- minibatches
// The pass's row weights for a round whose gradients take a minibatch (b < m_i rows, or host
// indices): coef_k = c(z_k) / nb_i on the batch rows, 0 elsewhere (obj_problems.py:16-17 / 49-50
// over X_b; nb_i = min(b, m_i), worker.py:21).  The batch is the round's host indices (idx: local
// row ids, [n x b]) or the device sampler's Floyd subset of (seed, round, wid0 + i) -- the same
// draw the direct kernels take.  One 64-lane workgroup per worker (m_i <= 64).
__global__ __launch_bounds__(64) void k_rs_coef(const RsArgs a, const int32_t* idx, int64_t b, uint64_t seed,
                                                int64_t round, int64_t wid0) {
  __shared__ unsigned char mk[64];
  const int i = blockIdx.x, k = threadIdx.x;
  const int64_t row0 = a.off[i];
  const int m = (int)(a.off[i + 1] - row0);
  const int64_t nb = b < m ? b : m;
  mk[k] = 0;
  __syncthreads();
  if (idx) {
    if (k < nb) mk[idx[(int64_t)i * b + k]] = 1;
  } else if (k == 0 && nb > 0) {
    floyd_sample(mk, m, nb, seed, round, wid0 + i);
  }
  __syncthreads();
  if (k >= m) return;
  double w = 0.0;
  if (mk[k]) {
    const double z = a.z[(int64_t)i * a.bcap + k];
    const double yv = a.y_is_f32 ? (double)((const float*)a.y)[row0 + k] : ((const double*)a.y)[row0 + k];
    w = (a.problem == 0 ? -yv / (1.0 + exp(yv * z)) : z - yv) / (double)nb;
  }
  a.coef_row[row0 + k] = w;
}

// ---------------------------------------------------------------------------- unequal starts
// xbar0 = mean_i x_i (float64, workers in order; its T copy), Z = 0, xbar = xbar0, ||D||^2
// partials 0 and ||xbar||^2 partials (as T) -- the state of k_rs_init for starts that differ.
template <typename T>
__global__ __launch_bounds__(NT) void k_rs_x0_mean(const RsArgs a, const T* __restrict__ x, int n, double* xbar0) {
  __shared__ double red[NW];
  const int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x;
  double xx = 0.0;
  if (e < a.ld) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += (double)x[(int64_t)i * a.ld + e];
    const double xb = s / (double)n;
    xbar0[e] = xb;
    a.rxbar[e] = xb;
    a.rZ[e] = 0.0;
    const T xt = (T)xb;
    ((T*)a.xbar_out)[e] = xt;
    xx = (double)xt * (double)xt;
  }
  xx = wave_sum(xx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = xx;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.dpart[blockIdx.x] = 0.0;
    a.dpart[a.nd + blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
  }
}

// d0[i] = ||x_i - xbar0||^2 (thread-strided, then waves in order)
template <typename T>
__global__ __launch_bounds__(NT) void k_rs_x0_dev(const RsArgs a, const T* __restrict__ x, const double* xbar0,
                                                   double* d0) {
  __shared__ double red[NW];
  const int i = blockIdx.x;
  double s = 0.0;
  for (int64_t e = threadIdx.x; e < a.ld; e += NT) {
    const double t = (double)x[(int64_t)i * a.ld + e] - xbar0[e];
    s += t * t;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) d0[i] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Partial row dots X_ik . x_i over column range g of G (16-byte data chunks strided over the
// workgroup's threads, each row's partial reduced in wave then wave order): gpart[(i * bcap + k)
// * G + g].  XT: row storage, T: iterate type.
template <typename T, typename XT>
__global__ __launch_bounds__(NT) void k_rs_x0_dots(const RsArgs a, const T* __restrict__ x, double* gpart, int G) {
  using VX = typename VT<XT>::v;
  constexpr int VN = VT<XT>::n;
  __shared__ double red[NW];
  const int i = blockIdx.x, g = blockIdx.y;
  const int64_t row0 = a.off[i];
  const int m = (int)(a.off[i + 1] - row0);
  const XAddr<VN> xa(a.tiled ? a.rows : 0, a.ld);
  const int64_t c0 = (int64_t)a.nch * g / G, c1 = (int64_t)a.nch * (g + 1) / G;
  const T* xi = x + (int64_t)i * a.ld;
  for (int k = 0; k < m; ++k) {
    double s = 0.0;
    for (int64_t c = c0 + threadIdx.x; c < c1; c += NT) {
      const VX r = rs_ld_nt<XT>((const XT*)a.X + xa.at(row0 + k, c));
#pragma unroll
      for (int e = 0; e < VN; ++e) s += (double)r[e] * (double)xi[c * VN + e];
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) gpart[((int64_t)i * a.bcap + k) * G + g] = ((red[0] + red[1]) + red[2]) + red[3];
    __syncthreads();
  }
}

__global__ __launch_bounds__(64) void k_rs_x0_fold(const RsArgs a, const double* gpart, int G, double* p0) {
  const int i = blockIdx.x, k = threadIdx.x;
  const int m = (int)(a.off[i + 1] - a.off[i]);
  if (k >= a.bcap) return;
  double s = 0.0;
  if (k < m)
    for (int g = 0; g < G; ++g) s += gpart[((int64_t)i * a.bcap + k) * G + g];
  p0[(int64_t)i * a.bcap + k] = s;
}

// ---------------------------------------------------------------------------- launchers
static const char* rs_tn(int dtype) { return dtype == 0 ? "float" : "double"; }

// The pass shape the runtime picks (RsArgs.cb / nbuf / ldot: 2 / 8 / 1; the other shapes
// were measured in round 3-4 A/B builds, removed in round 6).  X32: float64 arithmetic over float32-stored
// rows (k_rs_pass_x32).
template <typename T, bool X32, bool COLS>
static hipError_t rs_pass_shape(const RsArgs& a, dim3 grid, hipStream_t s) {
  if (a.ldot == 1 && a.cb == 2 && a.nbuf == 8) {  // every lane's partial through LDS
    if constexpr (X32) hipLaunchKernelGGL((k_rs_pass_x32<COLS, 2, 8, 1>), grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((k_rs_pass<T, COLS, 2, 8, 1>), grid, dim3(NT), 0, s, a);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

void rs_block_cols(const RsArgs& a, int xdtype, int b0, int b1, int64_t* c0, int64_t* c1) {
  const int64_t per = (int64_t)64 * a.cb * (xdtype == 0 ? 4 : 2);  // elements of one column block
  *c0 = std::min<int64_t>(a.ld, b0 * per);
  *c1 = std::min<int64_t>(a.ld, b1 * per);
}

hipError_t launch_rs_pass(int dtype, int xdtype, bool cols, const RsArgs& a, hipStream_t s, int nblk) {
  if (nblk <= 0) {
    if (a.blk0 != 0) return hipErrorInvalidValue;
    nblk = a.nblk;
  }
  if (a.blk0 < 0 || a.blk0 + nblk > a.nblk) return hipErrorInvalidValue;
  const dim3 grid(nblk, a.wg);
  const bool x32 = dtype == 1 && xdtype == 0;
  if (dtype != xdtype && !x32) return hipErrorInvalidValue;
  char buf[112];
  const int ld = ((a.cb == 2 && (a.nbuf == 8 || (a.nbuf == 16 && a.ldot == 1))) || (a.cb == 4 && a.nbuf == 4 && a.ldot == 1))
                     ? a.ldot : 0;
  char lds[8] = "";
  if (ld) snprintf(lds, sizeof(lds), ", %d", ld);
  if (x32)
    snprintf(buf, sizeof(buf), "void dopt::k_rs_pass_x32<%s, %d, %d%s>(dopt::RsArgs)", cols ? "true" : "false", a.cb,
             a.nbuf, lds);
  else
    snprintf(buf, sizeof(buf), "void dopt::k_rs_pass<%s, %s, %d, %d%s>(dopt::RsArgs)", rs_tn(dtype),
             cols ? "true" : "false", a.cb, a.nbuf, lds);
  if (cols) note_round_kernel(buf);
  if (x32) return cols ? rs_pass_shape<double, true, true>(a, grid, s) : rs_pass_shape<double, true, false>(a, grid, s);
  if (dtype == 0)
    return cols ? rs_pass_shape<float, false, true>(a, grid, s) : rs_pass_shape<float, false, false>(a, grid, s);
  return cols ? rs_pass_shape<double, false, true>(a, grid, s) : rs_pass_shape<double, false, false>(a, grid, s);
}

hipError_t launch_rs_rows(int dtype, const RsArgs& a, int n_workers, int mode, hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  if (dtype == 0) hipLaunchKernelGGL((k_rs_rows<float>), dim3(n_workers), dim3(NT), 0, s, a, mode);
  else hipLaunchKernelGGL((k_rs_rows<double>), dim3(n_workers), dim3(NT), 0, s, a, mode);
  return hipGetLastError();
}

int rs_col_blocks(int64_t ld) { return (int)((ld + NT - 1) / NT); }

hipError_t launch_rs_cols(int dtype, const RsArgs& a, hipStream_t s, int64_t c0, int64_t c1) {
  if (c1 < 0) c1 = a.ld;
  if (c0 < 0 || c1 > a.ld || c0 % NT != 0 || (c1 != a.ld && c1 % NT != 0)) return hipErrorInvalidValue;
  if (c1 <= c0) return hipSuccess;
  const dim3 grid(rs_col_blocks(c1 - c0));
  if (dtype == 0) hipLaunchKernelGGL((k_rs_cols<float>), grid, dim3(NT), 0, s, a, c0, c1);
  else hipLaunchKernelGGL((k_rs_cols<double>), grid, dim3(NT), 0, s, a, c0, c1);
  return hipGetLastError();
}

hipError_t launch_rs_hist(const RsArgs& a, int n_workers, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_rs_hist, dim3(1), dim3(NT), 0, s, a, n_workers, out);
  return hipGetLastError();
}

hipError_t launch_rs_fold(const RsArgs& a, const double* sc, int64_t nc, const double* sl, int64_t nl, double* out_c,
                          double* out_l, double* out_q, hipStream_t s) {
  hipLaunchKernelGGL(k_rs_fold, dim3(1), dim3(NT), 0, s, a, sc, nc, sl, nl, out_c, out_l, out_q);
  return hipGetLastError();
}

hipError_t launch_rs_csum(const RsArgs& a, double* out, hipStream_t s, int64_t c0, int64_t c1) {
  if (c1 < 0) c1 = a.ld;
  if (c1 <= c0) return hipSuccess;
  hipLaunchKernelGGL(k_rs_csum, dim3(rs_col_blocks(c1 - c0)), dim3(NT), 0, s, a, out, c0, c1);
  return hipGetLastError();
}

hipError_t launch_rs_init(int dtype, const RsArgs& a, const void* x0, hipStream_t s) {
  const dim3 grid(rs_col_blocks(a.ld));
  if (dtype == 0) hipLaunchKernelGGL((k_rs_init<float>), grid, dim3(NT), 0, s, a, (const float*)x0);
  else hipLaunchKernelGGL((k_rs_init<double>), grid, dim3(NT), 0, s, a, (const double*)x0);
  return hipGetLastError();
}

hipError_t launch_rs_check(int dtype, const void* x, int64_t n, int64_t ld, int32_t nch, int G, int32_t* flags,
                           int32_t* zflag, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)n, G);
  if (dtype == 0) hipLaunchKernelGGL((k_rs_check<float>), grid, dim3(NT), 0, s, (const float*)x, ld, nch, flags, zflag);
  else hipLaunchKernelGGL((k_rs_check<double>), grid, dim3(NT), 0, s, (const double*)x, ld, nch, flags, zflag);
  return hipGetLastError();
}

hipError_t launch_rs_gram(int xdtype, const RsArgs& a, int n_workers, int max_m, double* gpart, int G, hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  if (max_m < 1 || max_m > kRsMaxRows) return hipErrorInvalidValue;
  const int P = max_m * (max_m + 1) / 2;
  const dim3 grid(n_workers, G);
  const int mb = (max_m + 15) / 16;
#define RS_GRAM(XT_)                                                                        \
  switch (mb) {                                                                             \
    case 1: hipLaunchKernelGGL((k_rs_gram<XT_, 1>), grid, dim3(NT), 0, s, a, gpart, P); break; \
    case 2: hipLaunchKernelGGL((k_rs_gram<XT_, 2>), grid, dim3(NT), 0, s, a, gpart, P); break; \
    case 3: hipLaunchKernelGGL((k_rs_gram<XT_, 3>), grid, dim3(NT), 0, s, a, gpart, P); break; \
    default: hipLaunchKernelGGL((k_rs_gram<XT_, 4>), grid, dim3(NT), 0, s, a, gpart, P); break; \
  }
  if (xdtype == 0) {  // the Gram matrices read the rows only: their storage type
    RS_GRAM(float)
  } else {
    RS_GRAM(double)
  }
#undef RS_GRAM
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_rs_gram_fold, dim3(n_workers), dim3(NT), 0, s, a, (const double*)gpart, G, P);
  return hipGetLastError();
}

hipError_t launch_rs_coef(const RsArgs& a, int n_workers, const int32_t* idx, int64_t b, uint64_t seed, int64_t round,
                          int64_t wid0, hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  if (a.bcap > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rs_coef, dim3(n_workers), dim3(64), 0, s, a, idx, b, seed, round, wid0);
  return hipGetLastError();
}

hipError_t launch_rs_x0(int dtype, int xdtype, const RsArgs& a, int n_workers, const void* x, double* xbar0,
                        double* d0, double* p0, double* gpart, int G, hipStream_t s) {
  if (n_workers <= 0 || a.bcap > 64) return hipErrorInvalidValue;
  const dim3 gc(rs_col_blocks(a.ld)), gd(n_workers, G);
  if (dtype == 0 && xdtype == 0) {
    hipLaunchKernelGGL((k_rs_x0_mean<float>), gc, dim3(NT), 0, s, a, (const float*)x, n_workers, xbar0);
    hipLaunchKernelGGL((k_rs_x0_dev<float>), dim3(n_workers), dim3(NT), 0, s, a, (const float*)x, (const double*)xbar0, d0);
    hipLaunchKernelGGL((k_rs_x0_dots<float, float>), gd, dim3(NT), 0, s, a, (const float*)x, gpart, G);
  } else if (dtype == 1 && xdtype == 0) {
    hipLaunchKernelGGL((k_rs_x0_mean<double>), gc, dim3(NT), 0, s, a, (const double*)x, n_workers, xbar0);
    hipLaunchKernelGGL((k_rs_x0_dev<double>), dim3(n_workers), dim3(NT), 0, s, a, (const double*)x, (const double*)xbar0, d0);
    hipLaunchKernelGGL((k_rs_x0_dots<double, float>), gd, dim3(NT), 0, s, a, (const double*)x, gpart, G);
  } else if (dtype == 1 && xdtype == 1) {
    hipLaunchKernelGGL((k_rs_x0_mean<double>), gc, dim3(NT), 0, s, a, (const double*)x, n_workers, xbar0);
    hipLaunchKernelGGL((k_rs_x0_dev<double>), dim3(n_workers), dim3(NT), 0, s, a, (const double*)x, (const double*)xbar0, d0);
    hipLaunchKernelGGL((k_rs_x0_dots<double, double>), gd, dim3(NT), 0, s, a, (const double*)x, gpart, G);
  } else {
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(k_rs_x0_fold, dim3(n_workers), dim3(64), 0, s, a, (const double*)gpart, G, p0);
  return hipGetLastError();
}

hipError_t launch_rs_materialise(int dtype, int xdtype, const RsArgs& a, int n_workers, void* xout, hipStream_t s) {
  if (n_workers <= 0) return hipSuccess;
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>((a.nch + NT - 1) / NT, (8192 + n_workers - 1) / n_workers));
  const dim3 grid(n_workers, G);
  if (dtype == 1 && xdtype == 0) hipLaunchKernelGGL(k_rs_materialise_x32, grid, dim3(NT), 0, s, a, (double*)xout);
  else if (dtype != xdtype) return hipErrorInvalidValue;
  else if (dtype == 0) hipLaunchKernelGGL((k_rs_materialise<float>), grid, dim3(NT), 0, s, a, (float*)xout);
  else hipLaunchKernelGGL((k_rs_materialise<double>), grid, dim3(NT), 0, s, a, (double*)xout);
  return hipGetLastError();
}

}  // namespace dopt
