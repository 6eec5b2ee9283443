// engine.h -- internal interface between the C-ABI runtime (runtime.cpp) and
// the gfx950 kernels (kernels.hip).  Not part of the public ABI (include/dopt.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

struct dopt_comm;  // transport.cpp: an RCCL communicator (include/dopt.h)

namespace dopt {

// Error text for dopt_last_error from the library's other translation units (runtime.cpp).
int fail_code(int code, const char* fmt, ...);

// One point-to-point transfer of a round's exchange: `bytes` at byte offset `off` of the send buffer
// (recv = 0) or of the halo buffer (recv = 1), with rank `peer`.
struct XpOp {
  int64_t off, bytes;
  int32_t peer, recv;
};
// The ops as one RCCL group on stream s (transport.cpp).
int comm_exchange(dopt_comm* c, const XpOp* ops, size_t n_ops, const void* send, void* recv, hipStream_t s);
int32_t comm_world(const dopt_comm* c);
int32_t comm_rank(const dopt_comm* c);
int32_t comm_device(const dopt_comm* c);

// RoundArgs.flags
enum : int32_t {
  F_STEP = 1,          // fused mix + step: x_new = sum_j W_ij x_old[j] - eta * g  (trainer.py:173-175)
  F_GOUT = 2,          // store per-worker gradient rows instead (centralized, trainer.py:47-53)
  F_SHARED = 4,        // every worker evaluates at w_shared (centralized, trainer.py:43,48)
  F_CONS = 8,          // consensus partial ||x_i - xbar||^2 (trainer.py:185)
  F_LOSS = 16,         // objective partial at xbar over this workgroup's rows (trainer.py:189)
  F_LOSS_FROM_Z = 32,  // the objective point IS the gradient point: reuse z = x.w
  F_MEAN = 64,         // complete graph: sum_j W_ij x_j = w_off (S - x_i) + W_ii x_i, S = column sums
  F_GSUM = 128,        // with F_GOUT: store the raw sum of coef * row (no 1/b, no lam) -- full gradients
  F_LOSS2 = 256,       // metrics-only pass: also the objective at w_shared (from z) into slab_loss2
  F_BIP = 512,         // minibatch gradient inside the metrics pass over all rows (k_round VAR bit 6)
  F_DEVSAMPLE = 1024,  // with F_BIP: the minibatch is drawn on the device (Philox + Floyd), not from idx
  F_EARLYMIX = 2048,   // k_split_step: sum_j W_ij x_j of a block before the block's barrier (set by the launcher)
};
constexpr int64_t kMaxBipRows = 65536;  // shard rows the F_BIP byte map holds in LDS

// One workgroup per worker (or per objective-row chunk).  All pointers are
// device pointers; T-typed arrays are float or double per the launch.
struct RoundArgs {
  const void* X;          // [rows x ld] shard rows, back to back (column-blocked contexts: tiled, kcommon.h XAddr)
  int64_t xrows;          // tiled layout of X: rows of the X array (the tile stride); 0 = row-major, stride ld
  const void* y;          // [rows]
  const int64_t* off;     // [n+1] first row of every worker's rows
  const int32_t* idx;     // [n x b] local row ids of this round's minibatch, or null (all rows)
  int64_t b;              // minibatch size when idx != null
  const void* x_old;      // [n x ld] iterates before the round (read only during the round)
  void* x_new;            // [n x ld] iterates after the round
  void* g_out;            // [n x ld] gradients (F_GOUT)
  const void* w_shared;   // [ld] shared iterate (F_SHARED)
  const void* xbar;       // [ld] metric point (F_CONS / F_LOSS)
  const int64_t* rp;      // CSR mixing matrix, diagonal included
  const int32_t* ci;
  const void* cw;         // T-typed weights
  double* slab_cons;      // [n] per-workgroup partial sums (deterministic two-stage reduction)
  double* slab_loss;      // [n]
  double* slab_loss2;     // [n] second objective point (F_LOSS2)
  double eta;             // eta0 / sqrt(t+1)  (trainer.py:138-140)
  double lam;             // gradient regulariser (worker.py:36-42)
  const void* halo;       // [n_halo x ld] remote iterates (multi-GPU); CSR columns >= n_local index it
  int64_t ld;             // padded row stride in elements (multiple of the 16-byte vector)
  int32_t nchunks;        // ld / elements-per-16B
  int32_t flags;
  int32_t n_local;        // rows of x_old owned by this rank (columns below it are local)
  // complete-graph mixing (F_MEAN)
  const double* colsum;   // [ld] column sums of x_old (all workers, all ranks)
  const void* colsum_t;   // the same sums rounded to T (fp32 contexts: half the bytes every worker re-reads), or null
  const void* wdiag;      // [n] T diagonal weights W_ii
  double w_off;           // the uniform off-diagonal weight
  // column-blocked (large d) rounds
  const void* coef;       // [n x bcap] T per-row coefficients c(z_k) of the current round
  double* zpart;          // [n x bcap x groups] partial dots for the next coefficients
  double* upart;          // [n x bcap x groups] partial dots with xbar (objective)
  double* cpart;          // [n x groups] partial ||x_i - xbar||^2
  int32_t bcap;           // row capacity per worker in coef / partials
  int32_t b_rows;         // max rows per worker a column-blocked step touches (picks the kernel)
  int32_t pre_rows;       // CSR rows per worker prefetched to LDS by the fused kernel (0: off)
  int32_t groups;         // column-block groups = gridDim.y
  int32_t contig;         // column-blocked kernels: contiguous block range per group (set by the launcher)
  int32_t bip_rows;       // F_BIP: the largest shard (LDS byte map size)
  int32_t defer_rows;     // k_round VAR bit 14: >= the rows of every workgroup of this launch (loss terms
                          // buffered in LDS), or 0 when they do not all fit (the launch keeps them inline)
  // F_DEVSAMPLE: the minibatch of worker i in this round is a function of (seed, round, wid0 + i)
  uint64_t seed;
  int64_t round;
  int64_t wid0;
  // multi-GPU send rows written by k_mix: worker i's new row also goes to send rows
  // sslot[sptr[i] .. sptr[i+1]) (null sptr: no halo plan)
  const int64_t* sptr;
  const int32_t* sslot;
  // multi-GPU phase path: workers whose CSR row is all local (and who send no row) are mixed and
  // stepped by the gradient kernel itself (F_STEP per worker; k_mix then skips them), or null
  const int32_t* interior;
  void* send;
  // lagged multi-GPU mix: xbar of x_old from the all-reduced column sums xsum / xsum_n, written
  // to xbar_out, and the per-worker consensus ||x_old[i] - xbar||^2 into slab_cons (if non-null)
  const double* xsum;
  double xsum_n;
  void* xbar_out;
};

// History fold riding a k_colsum_final launch (one extra block): *out_c = sum sc[0:nc],
// *out_l = sum sl[0:nl], *out_q = ||xbar||^2 (T-typed xbar); null outputs are skipped.
struct FoldArgs {
  const double* sc;
  int64_t nc;
  const double* sl;
  int64_t nl;
  const void* xbar;
  double* out_c;
  double* out_l;
  double* out_q;
};

// The lagged multi-GPU mix with the column sums fused in (k_mixcs, kernels.hip).  Workgroup
// (group g of R workers, column block cb of 64 * CPB state chunks) mixes and steps its workers'
// slices (interior workers: stepped by the gradient kernel, read back), takes their consensus
// partials at xbar = (rank-ordered sum of every rank's column sums of x_old) / n, and writes the
// column-block partial of the column sums of x_new to part[g].  A second launch, k_mixcs_final (on
// the side stream when the caller gave one), sums the NG partials in group order into own_out and
// into the send buffer's sum rows of every peer.
// Block 0 folds a history row (FoldArgs).
constexpr int kMcsKargRanks = 16;  // sum rows of the first ranks passed as kernel arguments
struct McsArgs {
  double* part;            // [ng x ld] group partials of the column sums of x_new
  int32_t ng, ncb, r;      // worker groups, column blocks, workers per group
  int32_t world, rank;     // the rank-ordered global sums: rank p's halo rows, or own_in (row -1)
  const double* own_in;    // [ld] this rank's column sums of x_old
  double* own_out;         // [ld] this rank's column sums of x_new
  // [world] halo-buffer row of rank p's column sums of x_old; -1 for this rank (own_in) unless its
  // sums travel through the exchange to itself (a self block: RCCL world 1, collectives forced)
  const int64_t* sum_in;
  const int64_t* sum_out;  // [world] send-buffer row of the sums of x_new for rank p (-1: none)
  double* cons_part;       // [ncb x n] consensus partial of (column block, worker), or null
  double n_div;            // the mean's divisor (workers on all ranks)
  int32_t kin[kMcsKargRanks], kout[kMcsKargRanks];  // sum_in / sum_out of ranks < kMcsKargRanks
};

// Row-space rounds (rowspace.hip): complete graph (uniform W_ii), either objective, full
// shards of 1..kRsMaxRows rows, iterates that start equal.  x_i = Z + X_i^T beta_i.
constexpr int kRsMaxRows = 64;  // rows per worker (one lane each in k_rs_rows; Gram pairs in k_rs_gram)
struct RsArgs {
  const void* X;           // [rows x ld] T shard rows
  const void* y;           // [rows] T labels / targets
  int32_t y_is_f32;
  int32_t tiled;           // X in the column-block-tiled layout (tile stride: rows)
  int32_t problem;         // 0 logistic, 1 quadratic
  const int64_t* off;      // [n+1] first row of every worker
  int64_t rows;            // all rows (upart stride)
  int64_t ld;              // row stride in elements
  int32_t nch;             // 16-byte chunks of a row
  const int64_t* grow;     // [wg+1] row bounds of the pass's row groups
  int32_t wg;              // row groups (cpart rows)
  int32_t nblk;            // column blocks of the pass (64 * cb chunks each)
  int32_t cb, nbuf;        // pass shape: 16-byte chunks per lane per block, rows in flight per wave
  const void* xbar;        // [ld] T point of the pass's dots (xbar of the iterates)
  double* coef_row;        // [rows] r_k / m_i of the current iterates (the pass's column-sum weights)
  double* upart;           // [nblk x rows] partial dots X_k . xbar per column block (stored as T)
  double* cpart;           // [wg x ld] partial column sums sum_k coef_k X_k per row group
  int32_t bcap;            // row capacity per worker of z / v / beta / gram
  double* z;               // [n x bcap] X_ik . x_i
  double* v;               // [n x bcap] X_ik . Z
  double* beta;            // [n x bcap]
  const double* gram;      // [n x bcap x bcap] X_ik . X_il
  double* gram_w;          // the same, written by the Gram fold
  double* slab_cons;       // [n] ||x_i - xbar||^2 (k_rs_rows mode 1), or null
  double* slab_loss;       // [n] sum_k (u_k - y_k)^2, or null
  double* dpart;           // [2 nd] partials of ||Z - xbar||^2, then of ||xbar||^2 (k_rs_cols / k_rs_init)
  int32_t nd;
  double* rZ;              // [ld] Z
  double* rxbar;           // [ld] xbar (float64 master)
  void* xbar_out;          // [ld] T copy of the updated xbar
  const double* csum;      // [ld] all-reduced column sums C (multi-GPU), or null: sum cpart
  double a1, q, eta, eta_n;  // w_off N, W_ii - w_off - eta mu, eta, eta / N
  int32_t blk0;            // first column block of this pass launch (column-chunked passes)
  int32_t ldot;            // k_rs_pass: row dots through LDS per 64-row window, every lane's partial (1) or lane
                           // pairs first (2, A/B), or by DPP per row (0)
  // iterates that did not start equal: x_i = c x_i(0) + Z + X_i^T beta_i (else c = 0, pointers null)
  double c;                // the x_i(0) coefficient of the iterates the pass reads (prod of q so far)
  const double* xbar0;     // [ld] mean of the starting iterates
  const double* p0;        // [n x bcap] X_ik . x_i(0)
  const double* d0;        // [n] ||x_i(0) - xbar0||^2
  const void* x0;          // [n x ld] T the starting iterates (materialisation)
};
// dtype: arithmetic; xdtype: row storage (float32 rows under float64 arithmetic: k_rs_pass_x32).
// Column blocks [a.blk0, a.blk0 + nblk) of the pass (nblk <= 0: all of a.nblk from a.blk0 = 0).
hipError_t launch_rs_pass(int dtype, int xdtype, bool cols, const RsArgs& a, hipStream_t s, int nblk = 0);
// Elements [c0, c1) of one pass's column blocks [b0, b1) (clipped to the row stride).
void rs_block_cols(const RsArgs& a, int xdtype, int b0, int b1, int64_t* c0, int64_t* c1);
// mode bits: 1 metric partials of the iterate the pass read, 2 next round's row state,
// 4 initial state (z = v = u, beta = 0), 8 u = 0 without reading upart (zero start)
hipError_t launch_rs_rows(int dtype, const RsArgs& a, int n_workers, int mode, hipStream_t s);
int rs_col_blocks(int64_t ld);  // blocks of k_rs_cols / k_rs_init (= RsArgs.nd)
hipError_t launch_rs_cols(int dtype, const RsArgs& a, hipStream_t s, int64_t c0 = 0, int64_t c1 = -1);
// out[c0:c1) = sum_g cpart[g][c0:c1) (this rank's column sums of those columns).
hipError_t launch_rs_csum(const RsArgs& a, double* out, hipStream_t s, int64_t c0 = 0, int64_t c1 = -1);
// History row (cons, loss, ||xbar||^2) of the row-space rounds from the slabs and partials.
hipError_t launch_rs_hist(const RsArgs& a, int n_workers, double* out, hipStream_t s);
hipError_t launch_rs_fold(const RsArgs& a, const double* sc, int64_t nc, const double* sl, int64_t nl, double* out_c,
                          double* out_l, double* out_q, hipStream_t s);
hipError_t launch_rs_init(int dtype, const RsArgs& a, const void* x0, hipStream_t s);
hipError_t launch_rs_check(int dtype, const void* x, int64_t n, int64_t ld, int32_t nch, int G, int32_t* flags,
                           int32_t* zflag, hipStream_t s);
hipError_t launch_rs_gram(int xdtype, const RsArgs& a, int n_workers, int max_m, double* gpart, int G,
                          hipStream_t s);
hipError_t launch_rs_materialise(int dtype, int xdtype, const RsArgs& a, int n_workers, void* xout, hipStream_t s);
// Minibatch row weights of a round: the host indices idx ([n x b] local rows) or, idx == null,
// the device sampler's draw (seed, round, wid0 + i); coef = c(z) / min(b, m_i) on the batch rows.
hipError_t launch_rs_coef(const RsArgs& a, int n_workers, const int32_t* idx, int64_t b, uint64_t seed, int64_t round,
                          int64_t wid0, hipStream_t s);
// Unequal starting iterates x (T, [n x ld]): xbar0 = their mean (float64; xbar_out its T copy),
// d0[i] = ||x_i - xbar0||^2, p0[i][k] = X_ik . x_i (partials over G column ranges in gpart, folded in
// order), then the row-space state of such a start: Z = 0, xbar = xbar0, ||D||^2 partials 0.
hipError_t launch_rs_x0(int dtype, int xdtype, const RsArgs& a, int n_workers, const void* x, double* xbar0,
                        double* d0, double* p0, double* gpart, int G, hipStream_t s);

// Kernel launchers (kernels.hip).  dtype: 0 = float, 1 = double.
// k_round: dtype = iterates and arithmetic, xdtype = shard storage (equal, or float32 rows
// under float64 arithmetic); cpl = 16-byte DATA chunks per lane (1, 2, 4, 8, 16); a.nchunks
// counts data chunks.  The state-only kernels below take STATE chunks (nchunks, cpl).
// grad / met select the variant.
hipError_t launch_round(int dtype, int xdtype, int problem, int cpl, bool grad, bool met, const RoundArgs& a,
                        int n_groups, hipStream_t s);
// The instance name (rocprofv3's spelling) of the last gradient-round kernel launched --
// k_round or the column-blocked step -- for reports (dopt_last_round_kernel).
void note_round_kernel(const char* name);
int max_chunks_per_lane(int dtype, int xdtype);
// per element-type pair (round_f32.hip / round_f64.hip / round_x32.hip)
hipError_t launch_round_f32(int problem, int cpl, bool grad, bool met, const RoundArgs& a, int n_groups,
                            hipStream_t s);
hipError_t launch_round_f64(int problem, int cpl, bool grad, bool met, const RoundArgs& a, int n_groups,
                            hipStream_t s);
hipError_t launch_round_x32(int problem, int cpl, bool grad, bool met, const RoundArgs& a, int n_groups,
                            hipStream_t s);

// ---- large d (column-blocked): one workgroup per (worker, group of 64-chunk column blocks)
constexpr int kSplitMaxRows = 64;  // rows held in registers by a step workgroup (16 per wave)
// Step: g_i = (1/nb) sum_k coef_k x_k + lam x_i, x_i' = mix - eta g_i (block by block); with
// znext also the partial dots x_k . x_i' for the next round's coefficients (rows still in
// registers); with met the metric partials of x_i at xbar.  nb <= kSplitMaxRows.
// dtype = arithmetic / state, xdtype = row storage (equal, or float32 rows under float64 arithmetic).
hipError_t launch_split_step(int dtype, int xdtype, bool znext, bool met, const RoundArgs& a, int n_workers,
                             hipStream_t s);
// Dots only: mode 0 -> zpart = x_k . x_i (minibatch rows via idx, or all rows);
// mode 1 -> upart = x_k . xbar over all rows, cpart = ||x_i - xbar||^2 partials.
hipError_t launch_split_dots(int dtype, int xdtype, int mode, const RoundArgs& a, int n_workers, hipStream_t s);
// Per worker: z_k = sum_g zpart -> coef (mode bit 1), sum_k loss(u_k) -> slab_loss and
// sum_g cpart -> slab_cons (mode bit 2).  Fixed reduction order.
hipError_t launch_split_coef(int dtype, int xdtype, int problem, int mode, const RoundArgs& a, int n_workers,
                             hipStream_t s);

// Column sums of rows x[0:rows] in one launch when rows <= rpg (k_colsum_one), else the two
// stages below; arguments as theirs (n = the mean's divisor).  cons_out (one-launch path
// only, mode 0): per column block b, cons_out[b] = sum_i sum_{c in b} (x_ic - (T)xbar_c)^2.
hipError_t launch_colsum(int dtype, const void* x, int64_t rows, int64_t ld, int32_t nchunks, int32_t rpg,
                         double* part, uint64_t* stamp, int64_t n, void* out, const void* base, double eta,
                         int mode, hipStream_t s, double* raw, const FoldArgs* fold,
                         double* cons_out = nullptr);
// Column sums of an [n x ld] matrix into fp64 partials [G x ld], G = ceil(n / rpg).
hipError_t launch_colsum_partial(int dtype, const void* x, int64_t n, int64_t ld, int32_t nchunks,
                                 int32_t rpg, double* part, uint64_t* stamp, hipStream_t s);
// out = sum_g part / n (mode 0, the average model, trainer.py:182), or
// out = base - eta * (sum_g part / n) (mode 1, centralized update, trainer.py:53-57);
// with raw != null the column sums themselves go to raw[ld] (float64) instead.
// With fold != null one extra block also folds the history slabs (FoldArgs).
hipError_t launch_colsum_final(int dtype, const double* part, int32_t groups, int64_t n, int64_t ld,
                               int32_t nchunks, void* out, const void* base, double eta, int mode,
                               hipStream_t s, double* raw = nullptr, const FoldArgs* fold = nullptr);
// Raw metric sums of one round (one workgroup, fixed reduction order):
// out[0] = sum(slab_cons[0:n]), out[1] = sum(slab_loss[0:ng]), out[2] = ||xbar||^2 (0 if !xnorm).
// The host turns them into history values (runtime.cpp: finish_metrics) after any
// cross-rank sum.
hipError_t launch_history(int dtype, const double* slab_cons, const double* slab_loss, int64_t n,
                          int64_t ng, const void* xbar, int64_t ld, int32_t nchunks, bool xnorm,
                          double* out, hipStream_t s);
// The same fold with separate (nullable) outputs: *out_c = sum sc[0:nc], *out_l = sum sl[0:nl],
// *out_q = ||xbar||^2; null outputs are left alone (the lagged multi-GPU schedule folds the
// consensus of one round and the objective of another in one launch).
hipError_t launch_fold(int dtype, const double* sc, int64_t nc, const double* sl, int64_t nl, const void* xbar,
                       int64_t ld, int32_t nchunks, double* out_c, double* out_l, double* out_q, hipStream_t s);
// slab[g] = sum_{i in [64g, 64g+64)} ||x_i - xbar||^2, g < ceil(n / 64) (trainer.py:185).
hipError_t launch_cons(int dtype, const void* x, const void* xbar, int64_t n, int64_t ld, int32_t nchunks,
                       double* slab, hipStream_t s);
// x_next[i] = sum_e cw[e] * src(ci[e]) - eta * G[i]  (trainer.py:173-175), src = x_old or halo.
hipError_t launch_mix(int dtype, int cpl, const RoundArgs& a, const void* G, int n_workers, hipStream_t s);
// The lagged mix with fused column sums (McsArgs); fold: the history row folded by block 0
// (null: none).  xsum / xsum_n of `a` are unused (the rank-ordered sums of m replace them).
// side != null: k_mixcs_final goes to `side` after a wait for k_mixcs on s, so the next gradient kernel
// on s need not wait for it (the exchange, issued on `side`, does): an event `ev` recorded on s and
// waited for on side.
hipError_t launch_mixcs(int dtype, const RoundArgs& a, const void* G, int n_workers, const McsArgs& m,
                        const FoldArgs* fold, hipStream_t s, hipStream_t side = nullptr, hipEvent_t ev = nullptr);
// Column-block count / workers per group / groups of k_mixcs for n workers and nch state chunks.
void mixcs_shape(int dtype, int64_t n, int32_t nch, int32_t* ncb, int32_t* r, int32_t* ng);
// xbar_out = (T)(rank-ordered sum of the column sums, as k_mixcs forms it / n_div); with send != null
// also own -> the send buffer's sum rows (the chain's first exchange of x_0's sums).
hipError_t launch_xbar_ranks(int dtype, const McsArgs& m, const void* halo, int64_t ld, int32_t nch,
                             void* xbar_out, void* send, hipStream_t s);
// dst[k] = x[ids[k]] rows (halo send buffer); ids[k] < 0: row k left alone.
// The pull transport's copies (kernels.hip k_pull): nb peer blocks; block b's source in send slot k is
// src[2 b + k] (device array of pointers into the peers' allocations), its destination dst + dst_off[b] (bytes,
// device array), n16[b] 16-byte chunks (device array); max16 the largest block (host value, grid size).
struct PullArgs {
  const void* const* src;
  char* dst;
  const int64_t* dst_off;
  const int64_t* n16;
  int32_t nb;
  int64_t max16;
};
hipError_t launch_pull(const PullArgs& a, int slot, hipStream_t s);
hipError_t launch_gather_rows(int dtype, const void* x, const int32_t* ids, int64_t n, int64_t ld,
                              int32_t nchunks, void* dst, hipStream_t s);
// Synthetic shards (rows_per_worker rows per worker), X ~ N(0,1) + bias column; xrows > 0: X in
// the tiled layout of column-blocked contexts (ld = the padded row length, whole tiles);
// wstar = d doubles of scratch (the planted w*).
hipError_t launch_generate(int dtype, int problem, void* X, void* y, int64_t rows, int64_t d,
                           int64_t ld, int64_t xrows, double* wstar, uint64_t seed, double flip, double noise,
                           int64_t row_base, hipStream_t s);
// Host rows -> rows [r0, r0 + nr) of a tiled array of xrows rows (row length ld); and back
// (rows of a tiled array -> row-major [nr x ld]).
hipError_t launch_convert_tiled(int dtype, const void* src, int src_f32, void* dst, int64_t r0, int64_t nr, int64_t d,
                                int64_t ld, int64_t xrows, hipStream_t s);
hipError_t launch_untile(int dtype, const void* X, int64_t xrows, int64_t r0, int64_t nr, int64_t ld, void* dst,
                         hipStream_t s);
// Single float64 evaluation for rows too long for the row-resident kernel (obj_problems.py
// API): part[rows x G] partial dots, rowbuf[rows] coefficients (grad) or loss terms
// (objective), g_out[d] the gradient (grad).  Fixed reduction orders.
hipError_t launch_wide_eval(const double* X, const double* y, const double* w, int64_t rows, int64_t d, int64_t ld,
                            int problem, bool grad, double reg, double* part, int G, double* rowbuf, double* g_out,
                            hipStream_t s);
// One thread writes the constant-rate wall clock (trainer.py:181 timestamps).
hipError_t launch_stamp(uint64_t* out, hipStream_t s);
// float64 host data -> T rows padded to ld (zero padding).
hipError_t launch_convert(int dtype, const void* src, int src_f32, void* dst, int64_t rows, int64_t d,
                          int64_t ld, hipStream_t s);

}  // namespace dopt
