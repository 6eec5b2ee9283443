// runtime.cpp -- the C ABI of libdopt.so (include/dopt.h): device context, data
// layout in HBM, and the per-round launch schedule of the D-SGD / centralized
// trainers (trainer.py:33-74, :154-197).
//
// HBM layout (one context = one GPU):
//   X      [rows x ld]  T   shard rows back to back, worker i = rows [off[i], off[i+1]);
//                           ld = d rounded up to a 16-byte multiple, zero padded
//   y      [rows]       T
//   xs[2]  [N x ld]     T   iterate ping-pong: round t reads xs[cur], writes xs[cur^1]
//   xbar[2][ld]         T   average model ping-pong (xbar_t and xbar_{t+1} live together)
//   part   [G x ld]   f64   column-sum partials, G = ceil(N / rows_per_group)
//   slabs  [N]        f64   per-worker consensus / objective partials
//   rp/ci/cw                CSR mixing matrix (diagonal included), cw in T
//   G      [N x ld]     T   per-worker gradients (centralized trainer, multi-GPU phases)
//
// Launch schedule of one D-SGD round t (metrics every round):
//   k_round(t)       grad + mix + step for every worker, and the consensus /
//                    objective partials of x_t at xbar_t from the same row pass over
//                    every shard row (minibatch rows feed the gradient: F_BIP)
//   k_colsum_part(t) + k_colsum_final(t)   xbar_{t+1}; one extra block folds history[t-1]
// plus one metrics-only pass after the last round.  Only a separate objective dataset
// (X_full that is not the shards) takes a metrics-only pass every round.
// The multi-GPU phase functions (dopt_phase_*) split the same round at its
// communication points; distributed.py drives them.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <string>
#include <vector>

#include "dopt.h"
#include "engine.h"

using namespace dopt;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace

int dopt::fail_code(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

namespace {

#define HIPOK(expr)                                                                      \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail(DOPT_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

constexpr int64_t kRsColsBlock = 256;  // columns per k_rs_cols workgroup (kcommon.h NT)
constexpr int64_t kTileRowChunks = 64;  // 16-byte data chunks of a row per tile (kcommon.h kTileChunks)

#define CHECK_ARG(cond, ...)                          \
  do {                                                \
    if (!(cond)) return fail(DOPT_ERR_INVALID, __VA_ARGS__); \
  } while (0)

constexpr size_t kStaging = 64ull << 20;  // host->device staging chunk
constexpr int kRowsPerGroup = 64;         // column-sum partial group height (16 rows per wave)
constexpr int64_t kLossChunk = 64;        // objective rows per workgroup in a separate metrics pass
constexpr int64_t kDeferRows = 1024;      // rows per workgroup whose loss terms k_round may defer (LDS)

}  // namespace

struct dopt_ctx {
  int device = 0;
  int dtype = DOPT_F64;   // iterates and arithmetic
  size_t esz = 8;
  int xdtype = DOPT_F64;  // shard storage (dopt_set_data_dtype): float32 rows under float64 arithmetic
  size_t xesz = 8;
  int vn = 2;  // data elements per 16-byte vector (a "chunk"; the state chunk has as many elements)
  hipStream_t stream = nullptr;      // the stream every launch goes to
  hipStream_t own_stream = nullptr;  // created by dopt_create; dopt_set_stream may override
  double clock_hz = 1e8;

  // problem
  bool have_data = false;
  int problem = DOPT_LOGISTIC;
  int64_t n = 0, d = 0, ld = 0, nch = 0, rows = 0, max_m = 0;
  int cpl = 1;
  int64_t nchs = 0;  // 16-byte chunks of a STATE row (= nch unless float32 data under float64 state)
  int cpls = 1;      // ... and per lane (k_mix)
  bool split = false;  // d too long for the row-resident kernel: column-blocked rounds
  int split_groups = 1;
  // column-blocked contexts store X (and Xo) column-block TILED (kcommon.h XAddr): tile t = data
  // chunks [64 t, 64 t + 64) of every row, rows contiguous; ldx = the row length in elements padded
  // to whole tiles (row-major contexts: ldx = ld)
  bool tiled = false;
  int64_t ldx = 0;
  // dopt_run_dsgd_pipelined: the metrics of the current iterate (at xbar[xb]) are still owed
  // by the last pipelined run and ride the next pipelined run's first pass
  bool carry_pending = false;
  uint32_t carry_flags = 0;
  void* X = nullptr;
  void* y = nullptr;
  int64_t* off = nullptr;
  std::vector<int64_t> off_h;
  // global divisors when this context holds one rank's slice (dopt_set_partition)
  int64_t n_global = 0, rows_global = 0;

  // separate objective dataset (X_full that is not the union of the shards)
  bool obj_sep = false;
  void* Xo = nullptr;
  void* yo = nullptr;
  int64_t* offo = nullptr;
  int64_t rows_o = 0;

  // state
  void* xs[2] = {nullptr, nullptr};
  int cur = 0;
  void* xg[2] = {nullptr, nullptr};
  int gcur = 0;
  void* G = nullptr;
  void* xbar[2] = {nullptr, nullptr};
  int xb = 0;  // xbar[xb] = average of the current iterates
  double* S = nullptr;             // [ld] column sums of the current iterates (complete-graph mixing)
  const double* S_ext = nullptr;   // all-reduced sums (multi-GPU), used by the mix when set
  void* S_t = nullptr;             // [ld] T copy of the sums the mix reads (fp32 complete-graph mixing)
  // complete-graph mixing: sum_j W_ij x_j = w_off (S - x_i) + W_ii x_i
  bool mean_mix = false;
  double w_off = 0.0;
  void* wdiag = nullptr;
  // column-blocked buffers
  void* coef = nullptr;
  double* zpart = nullptr;
  double* upart = nullptr;
  double* cpart = nullptr;
  int64_t bcap = 0;
  size_t split_cap = 0;
  // phase API bookkeeping (column-blocked mode defers the step to dopt_phase_mix)
  int64_t ph_batch = 0;
  double ph_lam = 0.0;
  uint32_t ph_flags = 0;
  bool ph_have_idx = false;
  double* part = nullptr;
  int groups = 0;
  double* slab_cons = nullptr;
  double* slab_loss = nullptr;      // per worker (fused) or per 64-row chunk (metrics pass)
  double* slab_loss_b = nullptr;    // second loss slab (lagged multi-GPU schedule, two-point pass)
  int64_t slab_n[2] = {0, 0};       // valid entries of slab_loss / slab_loss_b (lagged schedule)
  int64_t cons_n = 0;               // valid entries of slab_cons (per worker, or per 64 workers)
  int64_t slab_cap = 0;
  int64_t loss_groups = 0;          // valid entries of slab_loss from the last producer
  int64_t* choff = nullptr;         // 64-row chunk offsets of the shard rows
  int64_t n_chunks = 0;
  int64_t* choff_o = nullptr;       // ... and of the separate objective dataset
  int64_t n_chunks_o = 0;

  // topology
  bool have_topo = false;
  int64_t* rp = nullptr;
  int32_t* ci = nullptr;
  void* cw = nullptr;
  int32_t max_row_nnz = 0;  // largest CSR row (mix prefetch sizing)

  // halo plan (multi-GPU): remote iterates land in `halo` (caller-owned device memory),
  // rows send_ids of the current iterates are gathered into `send` (caller-owned)
  int64_t n_halo = 0, n_send = 0;
  void* halo = nullptr;
  void* send = nullptr;
  int32_t* send_ids = nullptr;
  int64_t* sptr = nullptr;   // send rows by worker: worker i's row goes to send rows sslot[sptr[i]..sptr[i+1])
  int32_t* sslot = nullptr;
  std::vector<uint8_t> is_send;  // host: local workers whose row some peer reads
  int32_t* interior = nullptr;   // [n] CSR row all local and no send row (phase path: stepped in the gradient kernel);
                                 // int32 so the kernels read it with one scalar load
  int64_t n_interior = 0;
  double ph_eta = 0.0;           // dopt_phase_set_step: the step size of the next dopt_phase_grad
  bool ph_eta_set = false;
  bool ph_interior = false;      // the last dopt_phase_grad stepped the interior workers
  bool send_fresh = false;   // the last dopt_phase_mix already wrote the current iterates' send rows
  // lagged schedule with the column sums in the exchange (dopt_lagged_*, k_mixcs): every rank's
  // sums of x_g travel beside the halo rows; the send / halo buffers hold one block of sum rows per
  // peer at the rows dopt_lagged_exchange_layout names
  int32_t lg_world = 1, lg_rank = 0;
  bool lg_self = false;  // a self block in the exchange layout (RCCL world 1, collectives forced)
  std::vector<int64_t> lg_in_h, lg_out_h;  // host copies of the sum rows (-1: self)
  hipStream_t lg_side = nullptr;  // dopt_lagged_side_stream: k_mixcs_final and the exchange go there
  hipEvent_t lg_side_ev = nullptr;
  bool lg_xwait = false;  // the next mix / tail waits for the exchange (lg_xev)
  hipEvent_t lg_xev = nullptr;  // recorded on the side stream behind an exchange issued there
  // dopt_lagged_transport: the exchange through an RCCL communicator of the caller's (transport.cpp), one
  // send / receive per non-empty block of the layout, issued by dopt_lagged_exchange
  dopt_comm* xp = nullptr;
  std::vector<XpOp> xp_ops;
  // dopt_lagged_ipc_*: the pull transport (DOPT_TRANSPORT=ipc).  The send rows live in two slots (round
  // parity) of this rank's own allocation, exported through an IPC handle; each round every rank pulls its
  // blocks out of the peers' slots with one k_pull launch, after the peers' interprocess events (section
  // "pull transport" below)
  bool ipc = false;
  char* ipc_send = nullptr;             // [2 x ipc_slot bytes]
  int64_t ipc_slot = 0;
  hipEvent_t ipc_ev = nullptr;          // interprocess: recorded behind each slot's rows and sums
  std::vector<void*> ipc_open;          // the peers' allocations opened here
  std::vector<hipEvent_t> ipc_pev;      // the peers' events, opened here
  std::vector<int32_t> ipc_peers;       // ranks pulled from (not this one)
  int64_t* ipc_cnt = nullptr;           // [world] host shared memory of the caller's: events recorded per rank
  int64_t ipc_rec = 0;                  // events this rank recorded
  double ipc_timeout = 0.0;
  PullArgs ipc_pa{};
  void** ipc_src_d = nullptr;           // device copies of the pull's arrays
  int64_t* ipc_off_d = nullptr;
  int64_t* ipc_n16_d = nullptr;
  int64_t* lg_sum_in = nullptr;            // [world] halo row of peer p's sums
  int64_t* lg_sum_out = nullptr;           // [world] send row of the sums for peer p
  double* lg_own[2] = {nullptr, nullptr};  // [ld] this rank's column sums of x_g (g parity)
  double* lg_cons[2] = {nullptr, nullptr}; // [ncb x n] consensus partials of x_g (g parity)
  double* lg_part = nullptr;               // [ng x ld] group partials of k_mixcs
  int32_t lg_ncb = 0, lg_r = 0, lg_ng = 0;
  int64_t lg_alloc_n = -1, lg_alloc_ld = -1;
  int64_t lg = 0;                          // rounds of the current lagged chain

  // per-run buffers
  int32_t* idx = nullptr;
  size_t idx_cap = 0;
  void* idx_pin[2] = {nullptr, nullptr};  // pinned staging of the phase calls' indices (upload_idx_chunk)
  size_t idx_pin_cap[2] = {0, 0};
  hipEvent_t idx_ev[2] = {nullptr, nullptr};
  int idx_slot = 0;
  double* hraw = nullptr;  // [T x 3] raw metric sums per round (cons, loss, ||xbar||^2)
  uint64_t* stamps = nullptr;
  size_t hcap = 0;
  void* staging = nullptr;

  // scratch for the single-evaluation API (float64)
  void* sx = nullptr;
  size_t sx_cap = 0;

  // minibatch sampling for rounds run with idx == NULL and batch < shard (dopt_set_sampler)
  int sampler = DOPT_SAMPLE_HOST;
  uint64_t sample_seed = 0;
  int64_t sample_wid0 = 0;
  int64_t ph_round = 0;  // round index of the next dopt_phase_grad (device sampler counter)

  // row-space rounds (rowspace.hip; complete graph, quadratic, full shards): while rs_live the
  // iterates are x_i = rs_Z + X_i^T beta_i and xs[cur] holds them only when rs_xs_valid
  bool rs_live = false;
  bool rs_xs_valid = false;
  bool rs_gram_ok = false;
  // a column-chunked average update in progress (dopt_rs_phase_cols_range): chunks already updated
  // hold the next average in xbar[xb ^ 1], which the passes of those chunks read
  bool rs_sweep = false;
  // unequal starting iterates: x_i = rs_c x_i(0) + Z + X_i^T beta_i, x(0) kept in rs_x0buf and
  // its mean / deviations / row dots in rs_x0d (rs_x0 false: starts that were all equal, rs_c = 0)
  bool rs_x0 = false;
  double rs_c = 0.0;
  void* rs_x0buf = nullptr;
  size_t rs_x0buf_bytes = 0;
  double* rs_x0d = nullptr;
  bool wdiag_uniform = false;  // complete-graph mixing with one W_ii for every worker
  double wdiag_u = 0.0;
  int64_t min_m = 0;           // smallest shard
  int rs_wg = 0, rs_nblk = 0, rs_nd = 0, rs_cb = 4, rs_nbuf = 3, rs_ldot = 1;
  int64_t rs_bcap = 0;
  double* rs_coef = nullptr;   // [rows]
  double* rs_up = nullptr;     // [nblk x rows]
  double* rs_cp = nullptr;     // [wg x ld]
  double* rs_z = nullptr;      // [n x bcap] (z, v, beta back to back)
  double* rs_gram = nullptr;   // [n x bcap x bcap]
  double* rs_dpart = nullptr;  // [nd]
  double* rs_Z = nullptr;      // [ld] (Z, xbar back to back)
  int64_t* rs_grow = nullptr;  // [wg + 1]
  int32_t* rs_flags = nullptr;

  // profiling of k_round
  bool prof = false;
  int64_t prof_every = 1;      // bracket every k-th gradient-kernel launch (events cost ~30 us per pair)
  int64_t prof_seq = 0;        // gradient-kernel launches seen while profiling
  bool prof_skip = false;      // the current launch is not sampled
  std::vector<hipEvent_t> ev;  // (start, stop) pairs around the sampled gradient-kernel launches
  int64_t prof_n = 0;          // pairs recorded since the last dopt_kernel_stats
};

namespace {

void dfree(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
template <typename P>
void dfree_t(P*& p) {
  void* v = (void*)p;
  dfree(v);
  p = nullptr;
}

int dalloc(void** p, size_t bytes) {
  dfree(*p);
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(DOPT_ERR_HIP, "hipMalloc(%zu bytes): %s", bytes, hipGetErrorString(e));
  }
  return DOPT_OK;
}
int ipc_publish(dopt_ctx* c);
int ipc_pull(dopt_ctx* c);

// The pull transport's peer side: handles opened by dopt_lagged_ipc_import closed, its arrays freed.
void ipc_close(dopt_ctx* c) {
  // (no pull of this context may still read a peer's allocation when its mapping goes: teardown and setup only)
  if (!c->ipc_open.empty()) (void)hipDeviceSynchronize();
  for (void* q : c->ipc_open)
    if (q) (void)hipIpcCloseMemHandle(q);
  for (hipEvent_t e : c->ipc_pev)
    if (e) (void)hipEventDestroy(e);
  c->ipc_open.clear();
  c->ipc_pev.clear();
  c->ipc_peers.clear();
  dfree_t(c->ipc_src_d);
  dfree_t(c->ipc_off_d);
  dfree_t(c->ipc_n16_d);
  c->ipc_pa = PullArgs{};
  c->ipc_cnt = nullptr;
  c->ipc = false;
}

template <typename P>
int dalloc_t(P** p, size_t bytes) {
  void* v = (void*)*p;
  int rc = dalloc(&v, bytes);
  *p = (P*)v;
  return rc;
}

int cpl_for(int64_t nch) {
  int c = 1;
  while ((int64_t)c * 64 < nch) c *= 2;
  return c;
}

int set_device(dopt_ctx* c) {
  HIPOK(hipSetDevice(c->device));
  return DOPT_OK;
}

// Upload rows x d host values (float64 or float32) into a T-typed [rows x ld]
// device array through the staging buffer and the convert kernel.  tile_rows > 0: dst is a
// column-block tiled array of that many rows (row length ld, whole tiles).
int upload_rows(dopt_ctx* c, int dtype, const void* src, int src_f32, void* dst, int64_t rows,
                int64_t d, int64_t ld, int64_t tile_rows = 0) {
  if (rows == 0) return DOPT_OK;
  const size_t src_esz = src_f32 ? 4 : 8;
  const size_t dst_esz = dtype == DOPT_F32 ? 4 : 8;
  if (!c->staging) {
    int rc = dalloc(&c->staging, kStaging);
    if (rc) return rc;
  }
  const int64_t row_bytes = d * (int64_t)src_esz;
  int64_t chunk = std::max<int64_t>(1, (int64_t)kStaging / std::max<int64_t>(1, row_bytes));
  if (row_bytes > (int64_t)kStaging) return fail(DOPT_ERR_UNSUPPORTED, "row of %lld bytes exceeds staging", (long long)row_bytes);
  for (int64_t r0 = 0; r0 < rows; r0 += chunk) {
    const int64_t nr = std::min(chunk, rows - r0);
    HIPOK(hipMemcpyAsync(c->staging, (const char*)src + r0 * row_bytes, (size_t)(nr * row_bytes),
                         hipMemcpyHostToDevice, c->stream));
    if (tile_rows > 0)
      HIPOK(launch_convert_tiled(dtype, c->staging, src_f32, dst, r0, nr, d, ld, tile_rows, c->stream));
    else
      HIPOK(launch_convert(dtype, c->staging, src_f32, (char*)dst + r0 * ld * (int64_t)dst_esz, nr, d, ld,
                           c->stream));
  }
  HIPOK(hipStreamSynchronize(c->stream));
  return DOPT_OK;
}

// Device T [rows x ld] -> host float64 [rows x d].
int download_rows(dopt_ctx* c, int edtype, const void* src, double* dst, int64_t rows, int64_t d, int64_t ld) {
  if (rows == 0) return DOPT_OK;
  const size_t esz = edtype == DOPT_F32 ? 4 : 8;
  std::vector<char> tmp((size_t)(rows * ld) * esz);
  HIPOK(hipMemcpyAsync(tmp.data(), src, tmp.size(), hipMemcpyDeviceToHost, c->stream));
  HIPOK(hipStreamSynchronize(c->stream));
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t k = 0; k < d; ++k) {
      const int64_t s = r * ld + k;
      dst[r * d + k] = edtype == DOPT_F32 ? (double)((const float*)tmp.data())[s]
                                          : ((const double*)tmp.data())[s];
    }
  return DOPT_OK;
}

// Offsets of consecutive kLossChunk-row chunks of `rows` rows (device array).
int make_chunks(dopt_ctx* c, int64_t rows, int64_t** dst, int64_t* count) {
  const int64_t nc = (rows + kLossChunk - 1) / kLossChunk;
  std::vector<int64_t> o((size_t)nc + 1);
  for (int64_t k = 0; k <= nc; ++k) o[(size_t)k] = std::min(rows, k * kLossChunk);
  int rc;
  if ((rc = dalloc_t(dst, o.size() * sizeof(int64_t)))) return rc;
  HIPOK(hipMemcpy(*dst, o.data(), o.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  *count = nc;
  return DOPT_OK;
}

int ensure_slabs(dopt_ctx* c, int64_t need) {
  need = std::max<int64_t>(need, 1);
  if (need <= c->slab_cap && c->slab_loss) return DOPT_OK;
  int rc;
  if ((rc = dalloc_t(&c->slab_cons, (size_t)need * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->slab_loss, (size_t)need * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->slab_loss_b, (size_t)need * sizeof(double)))) return rc;
  c->slab_cap = need;
  return DOPT_OK;
}

int alloc_state(dopt_ctx* c) {
  const size_t st = (size_t)std::max<int64_t>(1, c->n) * c->ld * c->esz;
  int rc;
  for (int k = 0; k < 2; ++k) {
    if ((rc = dalloc(&c->xs[k], st))) return rc;
    HIPOK(hipMemsetAsync(c->xs[k], 0, st, c->stream));  // Worker.x = zeros (worker.py:13)
    if ((rc = dalloc(&c->xg[k], c->ld * c->esz))) return rc;
    HIPOK(hipMemsetAsync(c->xg[k], 0, c->ld * c->esz, c->stream));  // trainer.py:11
    if ((rc = dalloc(&c->xbar[k], c->ld * c->esz))) return rc;
    HIPOK(hipMemsetAsync(c->xbar[k], 0, c->ld * c->esz, c->stream));
  }
  dfree(c->G);  // allocated on first centralized run
  c->cur = 0;
  c->gcur = 0;
  c->xb = 0;
  c->groups = (int)((std::max<int64_t>(1, c->n) + kRowsPerGroup - 1) / kRowsPerGroup);
  if ((rc = dalloc_t(&c->part, (size_t)c->groups * c->ld * sizeof(double)))) return rc;
  if ((rc = make_chunks(c, c->rows, &c->choff, &c->n_chunks))) return rc;
  c->slab_cap = 0;
  if ((rc = ensure_slabs(c, std::max(c->n, c->n_chunks)))) return rc;
  if ((rc = dalloc_t(&c->S, (size_t)c->ld * sizeof(double)))) return rc;
  HIPOK(hipMemsetAsync(c->S, 0, (size_t)c->ld * sizeof(double), c->stream));
  if ((rc = dalloc(&c->S_t, (size_t)c->ld * c->esz))) return rc;
  HIPOK(hipStreamSynchronize(c->stream));
  return DOPT_OK;
}

int set_layout(dopt_ctx* c, int problem, int64_t n, int64_t d) {
  c->carry_pending = false;
  c->rs_live = c->rs_gram_ok = false;  // new data: the row-space state and the Gram matrices are gone
  c->rs_wg = 0;
  if (problem != DOPT_LOGISTIC && problem != DOPT_QUADRATIC)
    return fail(DOPT_ERR_UNSUPPORTED, "unknown problem %d", problem);
  CHECK_ARG(n >= 1 && d >= 1, "n_workers (%lld) and d (%lld) must be >= 1", (long long)n, (long long)d);
  CHECK_ARG(n < (1LL << 31), "n_workers too large");
  const int64_t ld = (d + c->vn - 1) / c->vn * c->vn;
  const int64_t nch = ld / c->vn;
  const int cpl = cpl_for(nch);
  c->split = cpl > max_chunks_per_lane(c->dtype, c->xdtype);
  // float32 rows under float64 arithmetic past the row-resident kernel: the row-space rounds
  // (k_rs_pass_x32) or the direct column-blocked kernels (k_split_*<double, float, ...>)
  if (c->split) {  // enough workgroups to fill 256 CUs several times over
    const int64_t nblk = (nch + 63) / 64;
    const int64_t target = std::max<int64_t>(1, 4096);  // workgroups per launch
    c->split_groups = (int)std::max<int64_t>(1, std::min<int64_t>(nblk, (target + n - 1) / n));
  }
  c->problem = problem;
  c->mean_mix = false;
  c->S_ext = nullptr;
  c->n = n;
  c->d = d;
  c->ld = ld;
  c->nch = nch;
  c->tiled = c->split;
  c->ldx = c->tiled ? (nch + kTileRowChunks - 1) / kTileRowChunks * kTileRowChunks * c->vn : ld;
  c->cpl = cpl;
  c->nchs = ld * (int64_t)c->esz / 16;
  c->cpls = cpl_for(c->nchs);
  c->have_topo = false;
  c->obj_sep = false;
  c->n_global = c->rows_global = 0;
  c->n_halo = c->n_send = 0;
  c->halo = c->send = nullptr;
  c->send_fresh = false;
  c->lg_world = 1;
  c->lg_rank = 0;
  c->lg_self = false;
  c->lg_in_h.clear();
  c->lg_out_h.clear();
  return DOPT_OK;
}

int ensure_hist(dopt_ctx* c, int64_t T) {
  if ((size_t)T <= c->hcap && c->hraw) return DOPT_OK;
  const size_t cap = (size_t)std::max<int64_t>(T, 16);
  int rc;
  if ((rc = dalloc_t(&c->hraw, 3 * cap * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->stamps, (cap + 1) * sizeof(uint64_t)))) return rc;
  c->hcap = cap;
  return DOPT_OK;
}

// fp32 complete-graph mixing reads the column sums as T (measured faster than reading them as float64)
bool sums_t_enabled(dopt_ctx* c) { return c->dtype == DOPT_F32; }

// The T copy of the sums the next mix reads (after every producer of S / S_ext).
int refresh_sums_t(dopt_ctx* c) {
  if (!c->mean_mix || !sums_t_enabled(c)) return DOPT_OK;
  HIPOK(launch_convert(c->dtype, c->S_ext ? c->S_ext : c->S, 0, c->S_t, 1, c->ld, c->ld, c->stream));
  return DOPT_OK;
}

RoundArgs base_args(dopt_ctx* c) {
  RoundArgs a;
  memset(&a, 0, sizeof(a));
  a.X = c->X;
  a.y = c->y;
  a.off = c->off;
  a.ld = c->ld;
  a.xrows = c->tiled ? c->rows : 0;
  a.nchunks = (int32_t)c->nch;
  a.slab_cons = c->slab_cons;
  a.slab_loss = c->slab_loss;
  a.slab_loss2 = c->slab_loss_b;
  a.halo = c->halo;
  a.n_local = (int32_t)c->n;
  a.rp = c->rp;
  a.ci = c->ci;
  a.cw = c->cw;
  if (c->mean_mix) {
    a.flags |= F_MEAN;
    a.colsum = c->S_ext ? c->S_ext : c->S;
    a.colsum_t = sums_t_enabled(c) ? c->S_t : nullptr;
    a.wdiag = c->wdiag;
    a.w_off = c->w_off;
  }
  a.coef = c->coef;
  a.zpart = c->zpart;
  a.upart = c->upart;
  a.cpart = c->cpart;
  a.bcap = (int32_t)c->bcap;
  a.b_rows = (int32_t)std::min<int64_t>(c->max_m, kSplitMaxRows);
  a.pre_rows = (c->max_row_nnz <= 6 && !c->mean_mix) ? c->max_row_nnz : 0;
  a.groups = c->split_groups;
  a.bip_rows = (int32_t)std::min<int64_t>(c->max_m, kMaxBipRows);
  // worker launches: every workgroup holds one shard (launches over 64-row chunks set kLossChunk)
  a.defer_rows = (c->max_m > 0 && c->max_m <= kDeferRows) ? (int32_t)c->max_m : 0;
  return a;
}

// Metrics-only pass over the objective rows (shards or the separate dataset).
// Metrics-only pass at `point` (xbar, or the shared iterate): the objective over the
// objective rows in 64-row chunks (many workgroups even when there are few workers),
// and ||x_i - point||^2 per worker.  (`shared` only says the point is the centralized
// iterate; the loss is x . point either way.)
int metrics_pass(dopt_ctx* c, const void* x_state, const void* point, bool shared, bool cons,
                 bool loss) {
  (void)shared;
  if (loss) {
    RoundArgs a = base_args(c);
    a.X = c->obj_sep ? c->Xo : c->X;
    a.y = c->obj_sep ? c->yo : c->y;
    a.off = c->obj_sep ? c->choff_o : c->choff;
    a.w_shared = point;
    a.flags |= F_LOSS | F_SHARED | F_LOSS_FROM_Z;
    a.defer_rows = (int32_t)kLossChunk;  // 64-row chunks
    const int64_t nc = c->obj_sep ? c->n_chunks_o : c->n_chunks;
    HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, false, true, a, (int)nc, c->stream));
    c->loss_groups = nc;
  }
  if (cons) {
    RoundArgs a = base_args(c);
    a.x_old = x_state;
    a.xbar = point;
    a.flags |= F_CONS;
    HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, false, true, a, (int)c->n, c->stream));
  }
  return DOPT_OK;
}

int64_t obj_rows(dopt_ctx* c) {  // objective divisor: all ranks' objective rows when partitioned
  if (c->rows_global) return c->rows_global;
  return c->obj_sep ? c->rows_o : c->rows;
}
int64_t n_div(dopt_ctx* c) { return c->n_global ? c->n_global : c->n; }

// Raw sums of round h -> history values (trainer.py:185, :189-190, obj_problems.py:3-11/:39-44).
void finalize_metrics(const double* raw, int64_t T, int problem, int64_t n, int64_t m_obj, double lam_obj,
                      double f_opt, double* obj_out, double* cons_out) {
  for (int64_t h = 0; h < T; ++h) {
    const double* r = raw + 3 * h;
    if (cons_out) cons_out[h] = r[0] / (double)n;
    if (obj_out) {
      double obj = 0.0;  // empty data -> 0.0, no regulariser (obj_problems.py:4,40)
      if (m_obj > 0) {
        const double data = (problem == DOPT_LOGISTIC) ? r[1] / (double)m_obj : 0.5 * (r[1] / (double)m_obj);
        obj = data + (lam_obj / 2.0) * r[2];
      }
      obj_out[h] = obj - f_opt;
    }
  }
}

// nc: valid consensus slab entries (c->n per-worker partials, or per column block)
int history(dopt_ctx* c, int64_t h, const void* point, bool cons, bool loss, int64_t nc) {
  HIPOK(launch_history(c->dtype, cons ? c->slab_cons : nullptr, loss ? c->slab_loss : nullptr, nc,
                       c->loss_groups, point, c->ld, (int32_t)c->nchs, loss, c->hraw + 3 * h, c->stream));
  return DOPT_OK;
}

// Minibatch indices of rounds [h0, h0 + nr) -> c->idx (stream-ordered).  stage: the call returns
// before the stream runs (the phase API), so the host array may be gone by the time the copy runs
// -- the indices go through one of two pinned staging buffers (the one whose previous copy has
// completed) first; the ABI borrows host pointers only for the duration of a call (dopt.h).  Runs
// (dopt_run_*) copy straight from the caller's array: they synchronise before returning.
int upload_idx_chunk(dopt_ctx* c, const int32_t* idx, int64_t h0, int64_t nr, int64_t b, bool stage = false) {
  const size_t bytes = (size_t)(nr * c->n * b) * sizeof(int32_t);
  if (bytes > c->idx_cap * sizeof(int32_t) || !c->idx) {
    int rc = dalloc_t(&c->idx, bytes);
    if (rc) return rc;
    c->idx_cap = bytes / sizeof(int32_t);
  }
  const int32_t* src = idx + h0 * c->n * b;
  if (stage && bytes > 0) {
    const int k = c->idx_slot;
    c->idx_slot ^= 1;
    if (!c->idx_ev[k]) HIPOK(hipEventCreateWithFlags(&c->idx_ev[k], hipEventDisableTiming));
    else HIPOK(hipEventSynchronize(c->idx_ev[k]));  // this buffer's previous copy has run
    if (bytes > c->idx_pin_cap[k]) {
      if (c->idx_pin[k]) (void)hipHostFree(c->idx_pin[k]);
      c->idx_pin[k] = nullptr;
      c->idx_pin_cap[k] = 0;
      HIPOK(hipHostMalloc(&c->idx_pin[k], bytes, hipHostMallocDefault));
      c->idx_pin_cap[k] = bytes;
    }
    memcpy(c->idx_pin[k], src, bytes);
    HIPOK(hipMemcpyAsync(c->idx, c->idx_pin[k], bytes, hipMemcpyHostToDevice, c->stream));
    HIPOK(hipEventRecord(c->idx_ev[k], c->stream));
    return DOPT_OK;
  }
  HIPOK(hipMemcpyAsync(c->idx, src, bytes, hipMemcpyHostToDevice, c->stream));
  return DOPT_OK;
}

// Events that only order this device's streams (or only time them) skip the system-scope fence of an event
// record: the kernels before them release their writes at their own end, exactly as for a consumer later on
// the same stream.  tools/xq_probe.hip (profiles/r6_xq_probe.txt, one-workgroup kernels on the device clock):
// a record between two kernels of a stream costs 3.8 us with the fence and 2.4 without (1.0 with no record);
// a kernel waiting on another stream's event that completes just before it could run starts 11.4 us after
// that event's kernel with the fence and 8.2 without (4.0 when the event completed long before); a
// device-scope release (hipEventReleaseToDevice) is no cheaper than the system-scope one.  The lagged
// schedule's fork (the side stream waits for k_mixcs) and join (the engine stream waits for the exchange)
// are such events.
constexpr unsigned kOrderEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;
// The sampled profiling events (timing only)
constexpr unsigned kProfEventFlags = hipEventDefault | hipEventDisableSystemFence;

int prof_event(dopt_ctx* c, bool stop) {
  if (!stop) c->prof_skip = (c->prof_seq++ % c->prof_every) != 0;
  if (c->prof_skip) return DOPT_OK;
  const size_t k = (size_t)(2 * c->prof_n + (stop ? 1 : 0));
  while (c->ev.size() <= k) {
    hipEvent_t e;
    HIPOK(hipEventCreateWithFlags(&e, kProfEventFlags));
    c->ev.push_back(e);
  }
  HIPOK(hipEventRecord(c->ev[k], c->stream));
  if (stop) c->prof_n++;
  return DOPT_OK;
}

// T history entries (metrics) and `rounds` end-of-round time stamps (they differ only for
// pipelined runs).
int finish_run(dopt_ctx* c, int64_t T, int64_t rounds, double lam_obj, double f_opt, double* obj_out,
               double* cons_out, double* time_out) {
  HIPOK(hipStreamSynchronize(c->stream));
  if ((obj_out || cons_out) && T > 0) {
    std::vector<double> raw((size_t)(3 * T));
    HIPOK(hipMemcpy(raw.data(), c->hraw, raw.size() * sizeof(double), hipMemcpyDeviceToHost));
    finalize_metrics(raw.data(), T, c->problem, n_div(c), obj_rows(c), lam_obj, f_opt, obj_out, cons_out);
  }
  if (time_out && rounds > 0) {
    std::vector<uint64_t> st((size_t)rounds + 1);
    HIPOK(hipMemcpy(st.data(), c->stamps, st.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (int64_t h = 0; h < rounds; ++h) time_out[h] = (double)(st[(size_t)h + 1] - st[0]) / c->clock_hz;
  }
  return DOPT_OK;
}

int64_t idx_chunk_rounds(dopt_ctx* c, int64_t T, int64_t b) {
  const int64_t per = std::max<int64_t>(1, c->n * b * (int64_t)sizeof(int32_t));
  return std::max<int64_t>(1, std::min<int64_t>(T, (int64_t)(256ll << 20) / per));
}

// xbar[xb] and S of the current iterates (run prologue).
int colsum_current(dopt_ctx* c) {
  HIPOK(launch_colsum(c->dtype, c->xs[c->cur], c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part, nullptr,
                      n_div(c), c->xbar[c->xb], nullptr, 0.0, 0, c->stream, c->S, nullptr));
  return refresh_sums_t(c);
}

// The direct column-blocked kernels read the rows in their storage type (float32 rows under
// float64 arithmetic: every product and sum the float64 one).
hipError_t split_dots(dopt_ctx* c, int mode, const RoundArgs& a) {
  return launch_split_dots(c->dtype, c->xdtype, mode, a, (int)c->n, c->stream);
}

hipError_t split_step(dopt_ctx* c, bool znext, bool met, const RoundArgs& a) {
  return launch_split_step(c->dtype, c->xdtype, znext, met, a, (int)c->n, c->stream);
}

// Column-blocked buffers: coefficients [n x bcap] and fp64 partial slabs.
int ensure_split(dopt_ctx* c) {
  int64_t bcap = std::max<int64_t>(1, c->max_m);
  if (c->obj_sep) bcap = std::max<int64_t>(bcap, (c->rows_o + c->n - 1) / c->n);
  const size_t need = (size_t)(c->n * bcap * c->split_groups);
  if (c->coef && bcap <= c->bcap && need <= c->split_cap) return DOPT_OK;
  int rc;
  if ((rc = dalloc(&c->coef, (size_t)(c->n * bcap) * c->esz))) return rc;
  if ((rc = dalloc_t(&c->zpart, need * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->upart, need * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->cpart, (size_t)(c->n * c->split_groups) * sizeof(double)))) return rc;
  c->bcap = bcap;
  c->split_cap = need;
  return DOPT_OK;
}

// Metrics of the current iterates at `point` over the objective rows, column-blocked:
// partial dots -> per-worker loss / consensus slabs.
int split_metrics(dopt_ctx* c, const void* x_state, const void* point, bool shared, bool cons, bool loss) {
  RoundArgs a = base_args(c);
  if (c->obj_sep) {
    a.X = c->Xo;
    a.xrows = c->tiled ? c->rows_o : 0;
    a.y = c->yo;
    a.off = c->offo;
  }
  a.x_old = x_state;
  a.w_shared = point;
  a.xbar = point;
  a.flags = (cons ? F_CONS : 0) | (loss ? F_LOSS : 0) | (shared ? F_SHARED : 0);
  if (a.flags & F_LOSS) c->loss_groups = c->n;  // per-worker loss slabs
  HIPOK(split_dots(c, 1, a));
  HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 2, a, (int)c->n, c->stream));
  return DOPT_OK;
}

// D-SGD rounds for rows longer than the row-resident kernel takes (config C5).
// lag = 1: a pipelined run that owes the metrics of the current iterate (computed by this
// call's first step; coefficients, S and xbar of that iterate are current); carry_out: leave
// the metrics of the last iterate owed.  *nh = history entries written.
int run_dsgd_split(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch, const int32_t* idx,
                   double lam_grad, double lam_obj, double f_opt, uint32_t flags, double* obj_out,
                   double* cons_out, double* time_out, int64_t lag, bool carry_out, int64_t* nh_out) {
  int rc;
  const bool want_obj = flags & DOPT_RUN_OBJECTIVE, want_cons = flags & DOPT_RUN_CONSENSUS;
  const bool metrics = want_obj || want_cons;
  const bool full = batch >= c->max_m;
  const int64_t nb_max = std::min(batch, c->max_m);
  if (nb_max > kSplitMaxRows)
    return fail(DOPT_ERR_UNSUPPORTED, "d = %lld with %lld rows per minibatch: the column-blocked kernel holds "
                "at most %d rows", (long long)c->d, (long long)nb_max, kSplitMaxRows);
  const bool fused_met = full && !c->obj_sep;
  if ((rc = ensure_split(c))) return rc;
  const int64_t CH = idx ? idx_chunk_rounds(c, T, batch) : 1;
  int& xb = c->xb;
  if (!lag && (rc = colsum_current(c))) return rc;
  RoundArgs p = base_args(c);
  p.x_old = c->xs[c->cur];
  if (full && !lag) {  // prologue: coefficients of the starting iterates (carried: the last step made them)
    HIPOK(split_dots(c, 0, p));
    HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 1, p, (int)c->n, c->stream));
  }
  HIPOK(launch_stamp(c->stamps, c->stream));
  for (int64_t h = 0; h < T; ++h) {
    const int64_t t = t0 + h;
    RoundArgs a = base_args(c);
    if (!full) {
      if (h % CH == 0 && (rc = upload_idx_chunk(c, idx, h, std::min(CH, T - h), batch))) return rc;
      a.idx = c->idx + (h % CH) * c->n * batch;
      a.b = batch;
      a.b_rows = (int32_t)std::min<int64_t>(a.b_rows, batch);
    }
    a.x_old = c->xs[c->cur];
    a.x_new = c->xs[c->cur ^ 1];
    a.xbar = c->xbar[xb];
    a.eta = eta0 / sqrt((double)(t + 1));  // trainer.py:138-140
    a.lam = lam_grad;
    if (!full) {  // this round's minibatch coefficients
      HIPOK(split_dots(c, 0, a));
      HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 1, a, (int)c->n, c->stream));
    }
    const bool met = fused_met && metrics && (h > 0 || lag);
    a.flags |= (met && want_cons ? F_CONS : 0) | (met && want_obj ? F_LOSS : 0);
    if (a.flags & F_LOSS) c->loss_groups = c->n;  // per-worker loss slabs
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(split_step(c, full, met, a));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    if (full || met) {  // next coefficients (rows of the full shard) and the metric slabs
      RoundArgs q = a;
      q.idx = nullptr;
      HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, (full ? 1 : 0) | (met ? 2 : 0), q, (int)c->n, c->stream));
    }
    HIPOK(launch_colsum_partial(c->dtype, c->xs[c->cur ^ 1], c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup,
                                c->part, c->stamps + h + 1, c->stream));
    HIPOK(launch_colsum_final(c->dtype, c->part, c->groups, n_div(c), c->ld, (int32_t)c->nchs, c->xbar[xb ^ 1],
                              nullptr, 0.0, 0, c->stream, c->S));
    if ((rc = refresh_sums_t(c))) return rc;
    if (met) {
      if ((rc = history(c, h - 1 + lag, c->xbar[xb], want_cons, want_obj, c->n))) return rc;
    } else if (!fused_met && metrics) {
      if ((rc = split_metrics(c, c->xs[c->cur ^ 1], c->xbar[xb ^ 1], false, want_cons, want_obj))) return rc;
      if ((rc = history(c, h, c->xbar[xb ^ 1], want_cons, want_obj, c->n))) return rc;
    }
    c->cur ^= 1;
    xb ^= 1;
  }
  int64_t nh = T + lag;
  if (carry_out && T > 0) {
    nh -= 1;  // the metrics of x_T: owed to the next pipelined run
  } else if (fused_met && metrics && (T > 0 || lag)) {
    if ((rc = split_metrics(c, c->xs[c->cur], c->xbar[xb], false, want_cons, want_obj))) return rc;
    if ((rc = history(c, nh - 1, c->xbar[xb], want_cons, want_obj, c->n))) return rc;
  }
  if (nh_out) *nh_out = nh;
  return finish_run(c, nh, T, lam_obj, f_opt, want_obj ? obj_out : nullptr, want_cons ? cons_out : nullptr,
                    time_out);
}

// Centralized rounds, column-blocked: dots at the shared iterate -> coefficients ->
// per-worker gradients -> deterministic mean -> step (trainer.py:41-71).
int run_centralized_split(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch, const int32_t* idx,
                          double lam_grad, double lam_obj, double f_opt, bool want_obj, double* obj_out,
                          double* time_out) {
  int rc;
  if (std::min(batch, c->max_m) > kSplitMaxRows)
    return fail(DOPT_ERR_UNSUPPORTED, "d = %lld with more than %d rows per minibatch", (long long)c->d,
                kSplitMaxRows);
  if ((rc = ensure_split(c))) return rc;
  if (!c->G && (rc = dalloc(&c->G, (size_t)c->n * c->ld * c->esz))) return rc;
  const int64_t CH = idx ? idx_chunk_rounds(c, T, batch) : 1;
  HIPOK(launch_stamp(c->stamps, c->stream));
  for (int64_t h = 0; h < T; ++h) {
    const int64_t t = t0 + h;
    RoundArgs a = base_args(c);
    if (idx) {
      if (h % CH == 0 && (rc = upload_idx_chunk(c, idx, h, std::min(CH, T - h), batch))) return rc;
      a.idx = c->idx + (h % CH) * c->n * batch;
      a.b = batch;
      a.b_rows = (int32_t)std::min<int64_t>(a.b_rows, batch);
    }
    a.w_shared = c->xg[c->gcur];
    a.g_out = c->G;
    a.lam = lam_grad;
    a.flags = F_SHARED | F_GOUT;  // no mixing here
    HIPOK(split_dots(c, 0, a));
    HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 1, a, (int)c->n, c->stream));
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(split_step(c, false, false, a));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    HIPOK(launch_colsum_partial(c->dtype, c->G, c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part,
                                c->stamps + h + 1, c->stream));
    HIPOK(launch_colsum_final(c->dtype, c->part, c->groups, c->n, c->ld, (int32_t)c->nchs, c->xg[c->gcur ^ 1],
                              c->xg[c->gcur], eta0 / sqrt((double)(t + 1)), 1, c->stream));
    if (want_obj) {
      if ((rc = split_metrics(c, nullptr, c->xg[c->gcur ^ 1], true, false, true))) return rc;
      if ((rc = history(c, h, c->xg[c->gcur ^ 1], false, true, c->n))) return rc;
    }
    c->gcur ^= 1;
  }
  return finish_run(c, T, T, lam_obj, f_opt, want_obj ? obj_out : nullptr, nullptr, time_out);
}

// ---------------------------------------------------------------------------- row-space rounds
// (rowspace.hip).  Complete graph with one W_ii, either objective, full-shard batches of
// 1..kRsMaxRows rows, one context (no rank slices), iterates that start equal: then
// x_i = Z + X_i^T beta_i for the whole run and a round is one read-only pass over the rows.
// DOPT_ROWSPACE=0 keeps the direct column-blocked rounds (A/B runs, tests).
bool rs_enabled() {
  const char* v = getenv("DOPT_ROWSPACE");
  return !(v && v[0] == '0');
}

// Minibatches (round 3): host indices, or batch < m with the device sampler -- the pass's row
// weights come from k_rs_coef each round (zero off the batch).
bool rs_eligible(dopt_ctx* c, int64_t batch, const int32_t* idx) {
  const bool batch_ok = idx || batch >= c->max_m || c->sampler == DOPT_SAMPLE_DEVICE;
  return rs_enabled() && c->split && c->mean_mix && c->wdiag_uniform && batch_ok && !c->obj_sep && c->min_m >= 1 &&
         c->max_m <= kRsMaxRows && c->n_global == 0 && !c->S_ext;
}

// Row storage for the row-space launchers (0 float32, 1 float64).
int rs_xdt(dopt_ctx* c) { return c->xdtype == DOPT_F32 ? 0 : 1; }

RsArgs rs_args(dopt_ctx* c) {
  RsArgs a;
  memset(&a, 0, sizeof(a));
  a.X = c->X;
  a.y = c->y;
  a.y_is_f32 = c->xdtype == DOPT_F32;
  a.tiled = c->tiled ? 1 : 0;
  a.problem = c->problem == DOPT_LOGISTIC ? 0 : 1;
  a.off = c->off;
  a.rows = c->rows;
  a.ld = c->ld;
  a.nch = (int32_t)c->nch;
  a.grow = c->rs_grow;
  a.wg = c->rs_wg;
  a.nblk = c->rs_nblk;
  a.cb = c->rs_cb;
  a.nbuf = c->rs_nbuf;
  a.ldot = c->rs_ldot;
  a.coef_row = c->rs_coef;
  a.upart = c->rs_up;
  a.cpart = c->rs_cp;
  a.bcap = (int32_t)c->rs_bcap;
  a.z = c->rs_z;
  a.v = c->rs_z ? c->rs_z + c->n * c->rs_bcap : nullptr;
  a.beta = c->rs_z ? c->rs_z + 2 * c->n * c->rs_bcap : nullptr;
  a.gram = c->rs_gram;
  a.gram_w = c->rs_gram;
  a.dpart = c->rs_dpart;
  a.nd = c->rs_nd;
  a.rZ = c->rs_Z;
  a.rxbar = c->rs_Z ? c->rs_Z + c->ld : nullptr;
  if (c->rs_x0) {
    a.c = c->rs_c;
    a.xbar0 = c->rs_x0d;
    a.d0 = c->rs_x0d + c->ld;
    a.p0 = c->rs_x0d + c->ld + c->n;
    a.x0 = c->rs_x0buf;
  }
  return a;
}

constexpr int kRsCheckGroups = 16;  // column groups of the equal-start check

int ensure_rs(dopt_ctx* c) {
  if (c->rs_wg > 0) return DOPT_OK;
  // pass shape, measured in A/B builds:
  // C5 float32 (round-3 A/B build, interleaved on one box, round ms): CB / NBUF / row groups
  // 2 / 6 / 2 11.22, 2 / 4 / 2 11.50, 1 / 8 / 4 11.46-11.84, 2 / 6 / 4 11.33-11.57, 4 / 2 / 4 12.36,
  // 1 / 8 / 16 12.36, 4 / 2 / 16 13.1-13.2: the partial sums' writes (dots nblk x rows, column
  // sums groups x ld) and long row visits matter more than the tail of ~4k 16 MiB workgroups.
  // Round 3 (tiled rows, C5 x32, alternated twice on one box, scripts/r3_rs_shape.sh): the windowed
  // row loop (NBUF dividing 64) at 2 / 8 10.66-10.83 ms, 2 / 4 10.79-10.81, 1 / 16 10.76-10.77,
  // 1 / 8 10.93-11.41, the 2 / 6 row loop 10.87-11.12.  Round 4 (row dots through LDS, LDOT 1, one
  // workgroup per CU; profiles/r4_c5_shapes.txt, 3 reps interleaved): 1 row group of 16k rows
  // 10.757-10.762 ms, 2 groups 10.867-10.909, 4 groups 10.924-10.963, 16 rows in flight 10.874-10.895
  c->rs_cb = 2;
  c->rs_nbuf = 8;
  c->rs_ldot = 1;
  const int64_t nblk = (c->nch + 64 * c->rs_cb - 1) / (64 * c->rs_cb);
  int64_t wg = (c->rows + 16383) / 16384;  // ~16k rows per row group
  wg = std::max<int64_t>(1, std::min<int64_t>(wg, (c->rows + 255) / 256));
  int rc;
  c->rs_nblk = (int)nblk;
  c->rs_nd = rs_col_blocks(c->ld);
  c->rs_bcap = std::max<int64_t>(1, c->max_m);
  const size_t nb = (size_t)c->n * c->rs_bcap;
  if ((rc = dalloc_t(&c->rs_coef, (size_t)c->rows * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_up, (size_t)nblk * c->rows * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_cp, (size_t)wg * c->ld * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_z, 3 * nb * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_gram, nb * c->rs_bcap * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_dpart, 2 * (size_t)c->rs_nd * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_Z, 2 * (size_t)c->ld * sizeof(double)))) return rc;
  if ((rc = dalloc_t(&c->rs_flags, ((size_t)c->n + 1) * kRsCheckGroups * sizeof(int32_t)))) return rc;
  std::vector<int64_t> gr((size_t)wg + 1);
  for (int64_t g = 0; g <= wg; ++g) gr[(size_t)g] = c->rows * g / wg;
  if ((rc = dalloc_t(&c->rs_grow, gr.size() * sizeof(int64_t)))) return rc;
  HIPOK(hipMemcpy(c->rs_grow, gr.data(), gr.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  c->rs_wg = (int)wg;
  c->rs_gram_ok = false;
  return DOPT_OK;
}

// xs[cur] = the iterates the row-space state holds (the state stays live).
int rs_sync(dopt_ctx* c) {
  if (!c->rs_live || c->rs_xs_valid) return DOPT_OK;
  HIPOK(launch_rs_materialise(c->dtype == DOPT_F32 ? 0 : 1, rs_xdt(c), rs_args(c), (int)c->n, c->xs[c->cur], c->stream));
  c->rs_xs_valid = true;
  return DOPT_OK;
}

static int rs_sweep_closed(dopt_ctx* c) {
  return c->rs_sweep ? fail(DOPT_ERR_STATE, "a column-chunked average update is open: finish it "
                                            "(dopt_rs_phase_cols_range with last = 1)")
                     : DOPT_OK;
}

// Leave row-space mode: xs[cur] holds the iterates, xbar[xb] their average.  An owed metrics
// entry of a row-space chain is dropped (the direct rounds carry other state).
int rs_end(dopt_ctx* c) {
  int rc;
  if ((rc = rs_sweep_closed(c))) return rc;
  if ((rc = rs_sync(c))) return rc;
  if (c->rs_live) c->carry_pending = false;
  c->rs_live = false;
  c->rs_x0 = false;
  return DOPT_OK;
}

enum { RS_FALLBACK = 1 };

// 64-bit content hash of a byte range (8-byte words through a multiply-rotate mix, a
// SplitMix64-style finaliser): multi-rank callers compare the iterates ranks start from.
uint64_t content_hash(const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, b + i, 8);
    h ^= w * 0xBF58476D1CE4E5B9ull;
    h = ((h << 27) | (h >> 37)) * 0x94D049BB133111EBull;
  }
  for (; i < n; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
  h ^= h >> 31;
  h *= 0x9E3779B97F4A7C15ull;
  return h ^ (h >> 29);
}

// Are the iterates xs[cur] all equal (*equal), and is that iterate zero (*zero)?  With hash != null
// also the content hash of the first iterate's bytes (multi-rank callers compare it across ranks).
int rs_check(dopt_ctx* c, bool* equal, bool* zero, uint64_t* hash) {
  int rc;
  if ((rc = ensure_rs(c))) return rc;
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  const int G = kRsCheckGroups;
  HIPOK(launch_rs_check(dt, c->xs[c->cur], c->n, c->ld, (int32_t)c->nchs, G, c->rs_flags, c->rs_flags + c->n * G,
                        c->stream));
  std::vector<int32_t> fl((size_t)(c->n + 1) * G);
  HIPOK(hipMemcpyAsync(fl.data(), c->rs_flags, fl.size() * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  std::vector<char> row(hash ? (size_t)c->d * c->esz : 0);
  if (hash) HIPOK(hipMemcpyAsync(row.data(), c->xs[c->cur], row.size(), hipMemcpyDeviceToHost, c->stream));
  HIPOK(hipStreamSynchronize(c->stream));
  *equal = true;
  *zero = true;
  for (int64_t k = 0; k < c->n * G; ++k)
    if (fl[(size_t)k]) *equal = false;
  for (int g = 0; g < G; ++g)
    if (fl[(size_t)(c->n * G + g)]) *zero = false;
  if (hash) *hash = content_hash(row.data(), row.size());
  return DOPT_OK;
}

// Round t's scalars: a1 = w_off N, q = W_ii - w_off - eta lam, eta, eta / N (N: all ranks' workers).
void rs_round_args(dopt_ctx* c, RsArgs& a, int64_t t, double eta0, double lam_grad) {
  const double N = (double)n_div(c), eta = eta0 / sqrt((double)(t + 1));  // trainer.py:138-140
  a.a1 = c->w_off * N;
  a.q = c->wdiag_u - c->w_off - eta * lam_grad;
  a.eta = eta;
  a.eta_n = eta / N;
}

// Start row-space mode from xs[cur].  Iterates that are not all equal (allow_unequal: one
// context) are kept as x(0) with x_i = c x_i(0) + Z + X_i^T beta_i, c = 1 now and q times itself
// every round; RS_FALLBACK when they differ and that is not allowed.
int rs_begin(dopt_ctx* c, bool allow_unequal) {
  int rc;
  bool equal = false, zero = false;
  if ((rc = rs_check(c, &equal, &zero, nullptr))) return rc;
  if (!equal && !allow_unequal) return RS_FALLBACK;
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  c->rs_x0 = false;
  c->rs_c = 0.0;
  RsArgs a = rs_args(c);
  if (!c->rs_gram_ok) {
    const int64_t P = c->rs_bcap * (c->rs_bcap + 1) / 2;
    // column ranges per worker: ~16k workgroups in all, each at least 64 four-chunk steps
    const int64_t nstep = ((int64_t)a.nch + 3) / 4;
    const int Gg = (int)std::max<int64_t>(1, std::min<int64_t>((nstep + 63) / 64, (16384 + c->n - 1) / c->n));
    double* gpart = nullptr;
    if ((rc = dalloc_t(&gpart, (size_t)c->n * Gg * P * sizeof(double)))) return rc;
    hipError_t e = launch_rs_gram(rs_xdt(c), a, (int)c->n, (int)c->rs_bcap, gpart, Gg, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree_t(gpart);
    if (e != hipSuccess) return fail(DOPT_ERR_HIP, "Gram matrices: %s", hipGetErrorString(e));
    c->rs_gram_ok = true;
  }
  a.xbar_out = c->xbar[c->xb];
  if (!equal) {  // keep x(0); its mean, deviations and row dots; Z = 0, xbar = xbar0
    const size_t xb = (size_t)c->n * c->ld * c->esz;
    if (c->rs_x0buf_bytes < xb) {  // (dalloc frees the previous buffer)
      c->rs_x0buf_bytes = 0;
      if ((rc = dalloc(&c->rs_x0buf, xb))) return rc;
      c->rs_x0buf_bytes = xb;
    }
    if ((rc = dalloc_t(&c->rs_x0d, ((size_t)c->ld + c->n + (size_t)c->n * c->rs_bcap) * sizeof(double)))) return rc;
    HIPOK(hipMemcpyAsync(c->rs_x0buf, c->xs[c->cur], xb, hipMemcpyDeviceToDevice, c->stream));
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>((c->nch + 1023) / 1024, (16384 + c->n - 1) / c->n));
    double* gpart = nullptr;
    if ((rc = dalloc_t(&gpart, (size_t)c->n * c->rs_bcap * G * sizeof(double)))) return rc;
    hipError_t e = launch_rs_x0(dt, rs_xdt(c), a, (int)c->n, c->xs[c->cur], c->rs_x0d, c->rs_x0d + c->ld,
                                c->rs_x0d + c->ld + c->n, gpart, G, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree_t(gpart);
    if (e != hipSuccess) return fail(DOPT_ERR_HIP, "row-space start from unequal iterates: %s", hipGetErrorString(e));
    c->rs_x0 = true;
    c->rs_c = 1.0;
    a = rs_args(c);
    HIPOK(launch_rs_rows(dt, a, (int)c->n, 16 | 8, c->stream));  // z = X_i . x_i(0), v = beta = 0
    c->rs_live = true;
    c->rs_xs_valid = true;  // xs[cur] is x(0) itself
    return DOPT_OK;
  }
  HIPOK(launch_rs_init(dt, a, c->xs[c->cur], c->stream));  // Z = xbar = x_0, ||D||^2 = 0
  if (zero) {
    HIPOK(launch_rs_rows(dt, a, (int)c->n, 4 | 8, c->stream));  // z = v = 0
  } else {
    a.xbar = c->xbar[c->xb];
    HIPOK(launch_rs_pass(dt, rs_xdt(c), false, a, c->stream));  // z = v = X . x_0
    HIPOK(launch_rs_rows(dt, a, (int)c->n, 4, c->stream));
  }
  c->rs_live = true;
  c->rs_xs_valid = true;  // xs[cur] is x_0 itself
  return DOPT_OK;
}

// D-SGD rounds in row-space mode; the history / carry contract of run_dsgd_split.
// RS_FALLBACK: not applicable here (unequal starting iterates, or a direct chain is open).
int run_dsgd_rs(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch, const int32_t* idx, int64_t CH,
                double lam_grad, double lam_obj, double f_opt, uint32_t flags, double* obj_out, double* cons_out,
                double* time_out, bool carry_in, bool pipelined, int64_t* nh_out) {
  int rc;
  const bool want_obj = flags & DOPT_RUN_OBJECTIVE, want_cons = flags & DOPT_RUN_CONSENSUS;
  const bool metrics = want_obj || want_cons;
  if (!c->rs_live) {
    if (carry_in) return RS_FALLBACK;
    if ((rc = rs_begin(c, true))) return rc;
  }
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  const int64_t lag = carry_in ? 1 : 0;
  const bool minibatch = idx || batch < c->max_m;
  int& xb = c->xb;
  HIPOK(launch_stamp(c->stamps, c->stream));
  for (int64_t h = 0; h < T; ++h) {
    RsArgs a = rs_args(c);
    rs_round_args(c, a, t0 + h, eta0, lam_grad);
    a.xbar = c->xbar[xb];
    const bool met = metrics && (h > 0 || lag);
    a.slab_cons = want_cons ? c->slab_cons : nullptr;
    a.slab_loss = want_obj ? c->slab_loss : nullptr;
    if (minibatch) {  // this round's row weights: c(z) / nb on its batch rows
      if (idx && h % CH == 0 && (rc = upload_idx_chunk(c, idx, h, std::min(CH, T - h), batch))) return rc;
      HIPOK(launch_rs_coef(a, (int)c->n, idx ? c->idx + (h % CH) * c->n * batch : nullptr, batch, c->sample_seed,
                           t0 + h, c->sample_wid0, c->stream));
    }
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(launch_rs_pass(dt, rs_xdt(c), true, a, c->stream));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    HIPOK(launch_rs_rows(dt, a, (int)c->n, 2 | (met ? 1 : 0), c->stream));
    if (met) HIPOK(launch_rs_hist(a, (int)c->n, c->hraw + 3 * (h - 1 + lag), c->stream));
    a.xbar_out = c->xbar[xb ^ 1];
    HIPOK(launch_rs_cols(dt, a, c->stream));
    HIPOK(launch_stamp(c->stamps + h + 1, c->stream));
    xb ^= 1;
    c->rs_c *= a.q;  // the x(0) coefficient of x_{t+1} (0 stays 0)
    c->rs_xs_valid = false;
  }
  int64_t nh = T + lag;
  if (pipelined && metrics && T > 0) {
    nh -= 1;  // the metrics of x_T: owed to the next pipelined run
    c->carry_pending = true;
    c->carry_flags = flags & (DOPT_RUN_OBJECTIVE | DOPT_RUN_CONSENSUS);
  } else if (metrics && (T > 0 || lag)) {  // one dots pass at xbar_T
    RsArgs a = rs_args(c);
    a.xbar = c->xbar[xb];
    a.slab_cons = want_cons ? c->slab_cons : nullptr;
    a.slab_loss = want_obj ? c->slab_loss : nullptr;
    HIPOK(launch_rs_pass(dt, rs_xdt(c), false, a, c->stream));
    HIPOK(launch_rs_rows(dt, a, (int)c->n, 1, c->stream));
    HIPOK(launch_rs_hist(a, (int)c->n, c->hraw + 3 * (nh - 1), c->stream));
  }
  if (nh_out) *nh_out = nh;
  return finish_run(c, nh, T, lam_obj, f_opt, want_obj ? obj_out : nullptr, want_cons ? cons_out : nullptr,
                    time_out);
}

// Minibatch rounds whose metrics need a pass over every shard row anyway take the gradient
// inside that pass (k_round F_BIP).  DOPT_BIP=0: a separate metrics pass (A/B runs).
static_assert(kMaxBipRows == DOPT_MAX_BIP_ROWS, "dopt.h and engine.h disagree");
static_assert(HIP_IPC_HANDLE_SIZE == DOPT_IPC_HANDLE_BYTES, "dopt.h and HIP disagree on IPC handle bytes");
bool bip_possible(dopt_ctx* c, int64_t batch, const int32_t* idx) {
  const char* v = getenv("DOPT_BIP");
  if (v && v[0] == '0') return false;
  return idx && batch < c->max_m && c->max_m <= kMaxBipRows && !c->obj_sep && !c->split;
}

// Separate metrics pass for few logistic workers (dopt_run_dsgd).  DOPT_FEW_SPLIT=0 / 1
// forces it off / on (A/B runs, tests).
bool split_few_metrics(dopt_ctx* c) {
  const char* v = getenv("DOPT_FEW_SPLIT");
  if (v) return v[0] == '1' && !c->split && !c->obj_sep;
  return c->n < 256 && c->problem == DOPT_LOGISTIC && !c->split && !c->obj_sep;
}

int check_run(dopt_ctx* c, int64_t T, int64_t batch, const int32_t* idx, bool need_topo) {
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  if (need_topo && !c->have_topo) return fail(DOPT_ERR_STATE, "no topology set");
  CHECK_ARG(T >= 0, "T must be >= 0");
  CHECK_ARG(batch >= 0, "batch must be >= 0");
  if (!idx && batch < c->max_m) {
    if (c->sampler != DOPT_SAMPLE_DEVICE)
      return fail(DOPT_ERR_INVALID, "idx == NULL needs full-shard batches (batch %lld < shard %lld) or the "
                  "device sampler", (long long)batch, (long long)c->max_m);
    if ((c->split || c->max_m > kMaxBipRows) && !(c->split && rs_eligible(c, batch, nullptr)))
      return fail(DOPT_ERR_UNSUPPORTED, "device sampling: row-resident contexts with shards of at most %lld rows, "
                  "or the complete graph's row-space rounds", (long long)kMaxBipRows);
  }
  return DOPT_OK;
}


}  // namespace

static std::string g_round_kernel;
void dopt::note_round_kernel(const char* name) { g_round_kernel = name; }

// ============================================================================ C ABI
extern "C" {

int dopt_abi_version(void) { return DOPT_ABI_VERSION; }
const char* dopt_last_error(void) { return g_err.c_str(); }
const char* dopt_last_round_kernel(void) { return g_round_kernel.c_str(); }

int dopt_device_count(int* count) {
  CHECK_ARG(count, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return DOPT_OK;
}

int dopt_create(int device, int dtype, dopt_ctx** out) {
  CHECK_ARG(out, "out is NULL");
  CHECK_ARG(dtype == DOPT_F32 || dtype == DOPT_F64, "dtype must be DOPT_F32 or DOPT_F64");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(DOPT_ERR_HIP, "no HIP device visible");
  CHECK_ARG(device >= 0 && device < n, "device %d out of range (%d visible)", device, n);
  dopt_ctx* c = new dopt_ctx();
  c->device = device;
  c->dtype = dtype;
  c->esz = dtype == DOPT_F32 ? 4 : 8;
  c->xdtype = dtype;
  c->xesz = c->esz;
  c->vn = dtype == DOPT_F32 ? 4 : 2;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  c->stream = c->own_stream;
  if (e != hipSuccess) {
    delete c;
    return fail(DOPT_ERR_HIP, "context init: %s", hipGetErrorString(e));
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    c->clock_hz = (double)khz * 1e3;
  *out = c;
  return DOPT_OK;
}

int dopt_set_data_dtype(dopt_ctx* c, int xdtype) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(xdtype == c->dtype || (c->dtype == DOPT_F64 && xdtype == DOPT_F32),
            "data dtype %d with compute dtype %d: the shards are stored in the compute dtype, or as float32 "
            "under float64 arithmetic", xdtype, c->dtype);
  c->xdtype = xdtype;
  c->xesz = xdtype == DOPT_F32 ? 4 : 8;
  c->vn = (int)(16 / c->xesz);
  c->have_data = false;  // the layout changes: load / generate the shards again
  c->have_topo = false;
  return DOPT_OK;
}

int dopt_get_data_dtype(dopt_ctx* c, int* xdtype) {
  CHECK_ARG(c && xdtype, "NULL argument");
  *xdtype = c->xdtype;
  return DOPT_OK;
}

int dopt_destroy(dopt_ctx* c) {
  if (!c) return DOPT_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
  for (void** p : {&c->X, &c->y, &c->Xo, &c->yo, &c->xs[0], &c->xs[1], &c->xg[0], &c->xg[1], &c->G,
                   &c->xbar[0], &c->xbar[1], &c->cw, &c->staging, &c->sx, &c->wdiag, &c->coef})
    dfree(*p);
  dfree_t(c->off);
  dfree_t(c->offo);
  dfree_t(c->choff);
  dfree_t(c->choff_o);
  dfree_t(c->part);
  dfree_t(c->slab_cons);
  dfree_t(c->slab_loss);
  dfree_t(c->slab_loss_b);
  dfree_t(c->sptr);
  dfree_t(c->sslot);
  dfree_t(c->interior);
  dfree_t(c->rp);
  dfree_t(c->ci);
  dfree_t(c->idx);
  dfree_t(c->hraw);
  dfree_t(c->S);
  dfree(c->S_t);
  dfree_t(c->zpart);
  dfree_t(c->upart);
  dfree_t(c->cpart);
  dfree_t(c->send_ids);
  dfree_t(c->stamps);
  for (double** p : {&c->rs_coef, &c->rs_up, &c->rs_cp, &c->rs_z, &c->rs_gram, &c->rs_dpart, &c->rs_Z, &c->rs_x0d})
    dfree_t(*p);
  dfree(c->rs_x0buf);
  dfree_t(c->rs_grow);
  dfree_t(c->rs_flags);
  for (double** p : {&c->lg_own[0], &c->lg_own[1], &c->lg_cons[0], &c->lg_cons[1], &c->lg_part}) dfree_t(*p);
  dfree_t(c->lg_sum_in);
  dfree_t(c->lg_sum_out);
  ipc_close(c);
  if (c->ipc_send) (void)hipFree(c->ipc_send);
  if (c->ipc_ev) (void)hipEventDestroy(c->ipc_ev);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->lg_side_ev) (void)hipEventDestroy(c->lg_side_ev);
  if (c->lg_xev) (void)hipEventDestroy(c->lg_xev);
  for (int k = 0; k < 2; ++k) {
    if (c->idx_ev[k]) (void)hipEventDestroy(c->idx_ev[k]);
    if (c->idx_pin[k]) (void)hipHostFree(c->idx_pin[k]);
  }
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return DOPT_OK;
}

int dopt_load_shards(dopt_ctx* c, int problem, int64_t n_workers, int64_t d, const int64_t* off,
                     const void* X, const void* y, int src_f32) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(off, "shard_offsets is NULL");
  int rc;
  if ((rc = set_device(c))) return rc;
  c->have_data = false;
  if ((rc = set_layout(c, problem, n_workers, d))) return rc;
  CHECK_ARG(off[0] == 0, "shard_offsets[0] must be 0");
  int64_t max_m = 0, min_m = n_workers > 0 ? off[1] - off[0] : 0;
  for (int64_t i = 0; i < n_workers; ++i) {
    CHECK_ARG(off[i + 1] >= off[i], "shard_offsets must be non-decreasing");
    max_m = std::max(max_m, off[i + 1] - off[i]);
    min_m = std::min(min_m, off[i + 1] - off[i]);
  }
  const int64_t rows = off[n_workers];
  CHECK_ARG(rows == 0 || (X && y), "X / y are NULL");
  c->rows = rows;
  c->max_m = max_m;
  c->min_m = min_m;
  c->off_h.assign(off, off + n_workers + 1);
  if ((rc = dalloc(&c->X, (size_t)rows * c->ldx * c->xesz))) return rc;
  if ((rc = dalloc(&c->y, (size_t)rows * c->xesz))) return rc;
  if ((rc = dalloc_t(&c->off, (size_t)(n_workers + 1) * sizeof(int64_t)))) return rc;
  HIPOK(hipMemcpy(c->off, off, (size_t)(n_workers + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if ((rc = upload_rows(c, c->xdtype, X, src_f32, c->X, rows, d, c->ldx, c->tiled ? rows : 0))) return rc;
  if ((rc = upload_rows(c, c->xdtype, y, src_f32, c->y, rows, 1, 1))) return rc;
  if ((rc = alloc_state(c))) return rc;
  c->have_data = true;
  return DOPT_OK;
}

int dopt_generate_shards(dopt_ctx* c, int problem, int64_t n_workers, int64_t d, int64_t rpw,
                         uint64_t seed, double flip, double noise, int64_t first_worker) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = set_device(c))) return rc;
  c->have_data = false;
  if ((rc = set_layout(c, problem, n_workers, d))) return rc;
  CHECK_ARG(rpw >= 1, "rows_per_worker must be >= 1");
  const int64_t rows = n_workers * rpw;
  c->rows = rows;
  c->max_m = rpw;
  c->min_m = rpw;
  c->off_h.resize((size_t)n_workers + 1);
  for (int64_t i = 0; i <= n_workers; ++i) c->off_h[(size_t)i] = i * rpw;
  if ((rc = dalloc(&c->X, (size_t)rows * c->ldx * c->xesz))) return rc;
  if ((rc = dalloc(&c->y, (size_t)rows * c->xesz))) return rc;
  if ((rc = dalloc_t(&c->off, (size_t)(n_workers + 1) * sizeof(int64_t)))) return rc;
  HIPOK(hipMemcpy(c->off, c->off_h.data(), (size_t)(n_workers + 1) * sizeof(int64_t),
                  hipMemcpyHostToDevice));
  CHECK_ARG(first_worker >= 0, "first_worker must be >= 0");
  double* wstar = nullptr;
  if ((rc = dalloc_t(&wstar, (size_t)d * sizeof(double)))) return rc;
  hipError_t e = launch_generate(c->xdtype, problem, c->X, c->y, rows, d, c->ldx, c->tiled ? rows : 0, wstar, seed,
                                 flip, noise, first_worker * rpw, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree_t(wstar);
  if (e != hipSuccess) return fail(DOPT_ERR_HIP, "dopt_generate_shards: %s", hipGetErrorString(e));
  if ((rc = alloc_state(c))) return rc;
  c->have_data = true;
  return DOPT_OK;
}

int dopt_load_objective_data(dopt_ctx* c, int64_t n_rows, const void* X, const void* y, int src_f32) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  CHECK_ARG(n_rows >= 0, "n_rows must be >= 0");
  CHECK_ARG(n_rows == 0 || (X && y), "X / y are NULL");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = dalloc(&c->Xo, (size_t)n_rows * c->ldx * c->xesz))) return rc;
  if ((rc = dalloc(&c->yo, (size_t)n_rows * c->xesz))) return rc;
  if ((rc = upload_rows(c, c->xdtype, X, src_f32, c->Xo, n_rows, c->d, c->ldx, c->tiled ? n_rows : 0))) return rc;
  if ((rc = upload_rows(c, c->xdtype, y, src_f32, c->yo, n_rows, 1, 1))) return rc;
  // split the objective rows over the N metric workgroups (array_split sizes)
  std::vector<int64_t> o((size_t)c->n + 1);
  const int64_t q = n_rows / c->n, r = n_rows % c->n;
  o[0] = 0;
  for (int64_t i = 0; i < c->n; ++i) o[(size_t)i + 1] = o[(size_t)i] + q + (i < r ? 1 : 0);
  if ((rc = dalloc_t(&c->offo, o.size() * sizeof(int64_t)))) return rc;
  HIPOK(hipMemcpy(c->offo, o.data(), o.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  c->rows_o = n_rows;
  if ((rc = make_chunks(c, n_rows, &c->choff_o, &c->n_chunks_o))) return rc;
  if ((rc = ensure_slabs(c, std::max(c->n, c->n_chunks_o)))) return rc;
  c->obj_sep = true;
  return DOPT_OK;
}

int dopt_clear_objective_data(dopt_ctx* c) {
  CHECK_ARG(c, "ctx is NULL");
  c->obj_sep = false;
  c->rows_o = 0;
  return DOPT_OK;
}

int dopt_get_shard(dopt_ctx* c, int64_t worker, double* X_out, double* y_out) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  CHECK_ARG(worker >= 0 && worker < c->n, "worker %lld out of range", (long long)worker);
  int rc;
  if ((rc = set_device(c))) return rc;
  const int64_t r0 = c->off_h[(size_t)worker], nr = c->off_h[(size_t)worker + 1] - r0;
  if (X_out && c->tiled && nr > 0) {  // the worker's rows out of the tiles, row-major, then down
    void* tmp = nullptr;
    if ((rc = dalloc_t(&tmp, (size_t)(nr * c->ldx) * c->xesz))) return rc;
    hipError_t e = launch_untile(c->xdtype == DOPT_F32 ? 0 : 1, c->X, c->rows, r0, nr, c->ldx, tmp, c->stream);
    rc = e == hipSuccess ? download_rows(c, c->xdtype, tmp, X_out, nr, c->d, c->ldx)
                         : fail(DOPT_ERR_HIP, "dopt_get_shard: %s", hipGetErrorString(e));
    dfree_t(tmp);
    if (rc) return rc;
  } else if (X_out && (rc = download_rows(c, c->xdtype, (const char*)c->X + r0 * c->ld * (int64_t)c->xesz, X_out, nr,
                                          c->d, c->ld))) {
    return rc;
  }
  if (y_out && (rc = download_rows(c, c->xdtype, (const char*)c->y + r0 * (int64_t)c->xesz, y_out, nr, 1, 1))) return rc;
  return DOPT_OK;
}

int dopt_set_topology(dopt_ctx* c, int64_t n_workers, const int64_t* row_ptr, const int32_t* col,
                      const double* w) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  CHECK_ARG(n_workers == c->n, "topology has %lld workers, data has %lld", (long long)n_workers,
            (long long)c->n);
  CHECK_ARG(row_ptr && row_ptr[0] == 0, "row_ptr[0] must be 0");
  for (int64_t i = 0; i < n_workers; ++i) CHECK_ARG(row_ptr[i + 1] >= row_ptr[i], "row_ptr not monotone");
  const int64_t nnz = row_ptr[n_workers];
  CHECK_ARG(nnz == 0 || (col && w), "col / w are NULL");
  for (int64_t e = 0; e < nnz; ++e)
    CHECK_ARG(col[e] >= 0 && col[e] < n_workers + c->n_halo, "col %d out of range (%lld local + %lld halo rows)",
              col[e], (long long)n_workers, (long long)c->n_halo);
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = rs_end(c))) return rc;
  if ((rc = dalloc_t(&c->rp, (size_t)(n_workers + 1) * sizeof(int64_t)))) return rc;
  if ((rc = dalloc_t(&c->ci, (size_t)nnz * sizeof(int32_t)))) return rc;
  if ((rc = dalloc(&c->cw, (size_t)nnz * c->esz))) return rc;
  HIPOK(hipMemcpy(c->rp, row_ptr, (size_t)(n_workers + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (nnz) {
    HIPOK(hipMemcpy(c->ci, col, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice));
    if (c->dtype == DOPT_F64) {
      HIPOK(hipMemcpy(c->cw, w, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice));
    } else {
      std::vector<float> wf((size_t)nnz);
      for (int64_t e = 0; e < nnz; ++e) wf[(size_t)e] = (float)w[e];
      HIPOK(hipMemcpy(c->cw, wf.data(), (size_t)nnz * sizeof(float), hipMemcpyHostToDevice));
    }
  }
  int64_t mx = 0;
  for (int64_t i = 0; i < n_workers; ++i) mx = std::max(mx, row_ptr[i + 1] - row_ptr[i]);
  c->max_row_nnz = (int32_t)std::min<int64_t>(mx, 1 << 30);
  // rank slices (a halo plan is set): the workers the gradient kernel can mix and step itself
  c->n_interior = 0;
  if (c->n_halo > 0 || !c->is_send.empty()) {
    std::vector<int32_t> in((size_t)n_workers, 0);
    for (int64_t i = 0; i < n_workers; ++i) {
      bool local = (size_t)i >= c->is_send.size() || !c->is_send[(size_t)i];
      for (int64_t e = row_ptr[i]; e < row_ptr[i + 1] && local; ++e) local = col[e] < n_workers;
      in[(size_t)i] = local;
      c->n_interior += local;
    }
    if ((rc = dalloc_t(&c->interior, in.size() * sizeof(int32_t)))) return rc;
    HIPOK(hipMemcpy(c->interior, in.data(), in.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  c->have_topo = true;
  c->mean_mix = false;
  return DOPT_OK;
}

int dopt_set_mixing_mean(dopt_ctx* c, int64_t n_workers, double w_off, const double* w_diag) {
  CHECK_ARG(c && w_diag, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  CHECK_ARG(n_workers == c->n, "mixing has %lld workers, data has %lld", (long long)n_workers, (long long)c->n);
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = rs_end(c))) return rc;
  c->rs_wg = 0;  // the row-space pass is planned again (shape knobs re-read, Gram recomputed)
  if ((rc = dalloc(&c->wdiag, (size_t)n_workers * c->esz))) return rc;
  if (c->dtype == DOPT_F64) {
    HIPOK(hipMemcpy(c->wdiag, w_diag, (size_t)n_workers * sizeof(double), hipMemcpyHostToDevice));
  } else {
    std::vector<float> wf(w_diag, w_diag + n_workers);
    HIPOK(hipMemcpy(c->wdiag, wf.data(), (size_t)n_workers * sizeof(float), hipMemcpyHostToDevice));
  }
  c->w_off = w_off;
  c->mean_mix = true;
  c->have_topo = true;
  // the row-space rounds need one W_ii for every worker (as the kernels read it: in T)
  const double w0 = c->dtype == DOPT_F64 ? w_diag[0] : (double)(float)w_diag[0];
  c->wdiag_uniform = true;
  for (int64_t i = 1; i < n_workers; ++i) {
    const double wi = c->dtype == DOPT_F64 ? w_diag[i] : (double)(float)w_diag[i];
    if (wi != w0) c->wdiag_uniform = false;
  }
  c->wdiag_u = w0;
  return DOPT_OK;
}

int dopt_set_models(dopt_ctx* c, const double* x) {
  if (c) c->send_fresh = c->carry_pending = c->rs_live = false;
  CHECK_ARG(c && x, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  int rc;
  if ((rc = set_device(c))) return rc;
  return upload_rows(c, c->dtype, x, 0, c->xs[c->cur], c->n, c->d, c->ld);
}

int dopt_zero_models(dopt_ctx* c) {
  if (c) c->send_fresh = c->carry_pending = c->rs_live = false;
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  int rc;
  if ((rc = set_device(c))) return rc;
  HIPOK(hipMemsetAsync(c->xs[c->cur], 0, (size_t)c->n * c->ld * c->esz, c->stream));  // worker.py:13
  return DOPT_OK;
}

int dopt_get_models(dopt_ctx* c, double* x) {
  CHECK_ARG(c && x, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = rs_sync(c))) return rc;
  return download_rows(c, c->dtype, c->xs[c->cur], x, c->n, c->d, c->ld);
}

int dopt_set_global(dopt_ctx* c, const double* x) {
  CHECK_ARG(c && x, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  int rc;
  if ((rc = set_device(c))) return rc;
  return upload_rows(c, c->dtype, x, 0, c->xg[c->gcur], 1, c->d, c->ld);
}

int dopt_get_global(dopt_ctx* c, double* x) {
  CHECK_ARG(c && x, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  int rc;
  if ((rc = set_device(c))) return rc;
  return download_rows(c, c->dtype, c->xg[c->gcur], x, 1, c->d, c->ld);
}

static int run_dsgd(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch, const int32_t* idx,
                    double lam_grad, double lam_obj, double f_opt, uint32_t flags, double* obj_out,
                    double* cons_out, double* time_out, bool pipelined, int64_t* n_out) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if (T == 0) {  // no round: at most the owed metrics pass, which does not depend on the batch
    batch = c->max_m;
    idx = nullptr;
  }
  if ((rc = check_run(c, T, batch, idx, true))) return rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = ensure_hist(c, T + 1))) return rc;
  const bool carry_in = pipelined && c->carry_pending && c->carry_flags != 0;
  c->carry_pending = false;
  if (carry_in && c->carry_flags != (flags & (DOPT_RUN_OBJECTIVE | DOPT_RUN_CONSENSUS)))
    return fail(DOPT_ERR_INVALID, "pipelined run: metrics flags %u differ from the pending metrics' %u", flags,
                c->carry_flags);
  if (T == 0 && !carry_in) {  // nothing to run, nothing owed
    if (n_out) *n_out = 0;
    return DOPT_OK;
  }
  c->send_fresh = false;
  const bool want_obj = flags & DOPT_RUN_OBJECTIVE, want_cons = flags & DOPT_RUN_CONSENSUS;
  const bool metrics = want_obj || want_cons;
  const bool dev = !idx && batch < c->max_m;  // device sampler (check_run)
  // Few logistic workers (C2: 10-25): one workgroup per worker puts a round on <= 25 CUs, and
  // the fused objective (a second dot + exp / log per row) makes those CUs VALU-bound
  // (fp64 C2: 55-62 us per round kernel vs 17 us without metrics and 7 us for the
  // separate metrics pass over 64-row chunks on many CUs): take the metrics pass apart.
  // With the device sampler the round kernel still walks every row (the draw marks the
  // batch rows in that pass) but computes only the batch rows: no metric work in it.
  const bool few_split = split_few_metrics(c);
  const bool bip = metrics && !few_split && (dev ? !c->obj_sep : bip_possible(c, batch, idx));
  const bool fused = !few_split && (batch >= c->max_m || bip) && !c->obj_sep;
  // separate metrics with <= 64 workers: the consensus rides the one-launch column sums
  // (per column block partials; one metrics launch less per round)
  const int64_t cs_blocks = (c->nchs + 63) / 64;
  const char* two = getenv("DOPT_COLSUM_TWO");  // the two-stage column sums carry no consensus
  const char* ccs = getenv("DOPT_CONS_CS");     // A/B knob: 0 = consensus from the metrics pass instead
  const bool cons_cs = !fused && want_cons && c->n <= kRowsPerGroup && cs_blocks <= c->slab_cap && !c->split &&
                       !(two && atoi(two) != 0) && !(ccs && ccs[0] == '0');
  const int64_t CH = idx ? idx_chunk_rounds(c, T, batch) : 1;
  int& xb = c->xb;
  if (c->split) {  // the column-blocked rounds pipeline the same way (full-shard batches)
    if (rs_eligible(c, batch, idx)) {  // complete graph, quadratic: row-space rounds
      int64_t nh = 0;
      rc = run_dsgd_rs(c, t0, T, eta0, batch, idx, CH, lam_grad, lam_obj, f_opt, flags, obj_out, cons_out, time_out,
                       carry_in, pipelined, &nh);
      if (rc != RS_FALLBACK) {
        if (rc) return rc;
        if (n_out) *n_out = nh;
        return DOPT_OK;
      }
    } else {
      if (carry_in && c->rs_live)
        return fail(DOPT_ERR_INVALID, "pipelined run: the pending metrics belong to a row-space chain");
      if ((rc = rs_end(c))) return rc;
    }
    if (!idx && batch < c->max_m)  // (the device sampler reaches here only past the row-space rounds)
      return fail(DOPT_ERR_UNSUPPORTED, "device sampling on long rows: the complete graph's row-space rounds only");
    const bool sfused = batch >= c->max_m && !c->obj_sep && metrics;
    if (carry_in && !sfused) return fail(DOPT_ERR_INVALID, "pipelined run: the pending metrics need a fused run");
    int64_t nh = 0;
    if ((rc = run_dsgd_split(c, t0, T, eta0, batch, idx, lam_grad, lam_obj, f_opt, flags, obj_out, cons_out,
                             time_out, carry_in ? 1 : 0, pipelined && sfused, &nh)))
      return rc;
    if (pipelined && sfused && T > 0) {
      c->carry_pending = true;
      c->carry_flags = flags & (DOPT_RUN_OBJECTIVE | DOPT_RUN_CONSENSUS);
    }
    if (n_out) *n_out = nh;
    return DOPT_OK;
  }
  // pipelined: the last round's metrics stay owed (its pass would be the only unfused one)
  const bool carry_out = pipelined && fused && metrics;
  const int64_t lag = (carry_in && fused && metrics) ? 1 : 0;  // output entry of round h's fused metrics: h - 1 + lag
  if (carry_in && !lag) return fail(DOPT_ERR_INVALID, "pipelined run: the pending metrics need a fused run");
  if (!carry_in && (rc = colsum_current(c))) return rc;  // xbar and S of the starting iterates (carried: current)
  HIPOK(launch_stamp(c->stamps, c->stream));

  for (int64_t h = 0; h < T; ++h) {
    const int64_t t = t0 + h;
    if (idx && h % CH == 0) {
      if ((rc = upload_idx_chunk(c, idx, h, std::min(CH, T - h), batch))) return rc;
    }
    RoundArgs a = base_args(c);
    a.idx = idx ? c->idx + (h % CH) * c->n * batch : nullptr;
    a.b = batch;
    a.x_old = c->xs[c->cur];
    a.x_new = c->xs[c->cur ^ 1];
    a.xbar = c->xbar[xb];
    a.eta = eta0 / sqrt((double)(t + 1));  // trainer.py:138-140
    a.lam = lam_grad;
    const bool met = fused && metrics && (h > 0 || lag);
    a.flags |= F_STEP | (met && want_cons ? F_CONS : 0) | (met && want_obj ? F_LOSS : 0) |
               ((met && bip) || dev ? F_BIP : 0) | (dev ? F_DEVSAMPLE : 0);
    a.seed = c->sample_seed;
    a.round = t;
    a.wid0 = c->sample_wid0;
    if (a.flags & F_LOSS) c->loss_groups = c->n;  // per-worker loss slabs
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, true, met || dev, a, (int)c->n, c->stream));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    // xbar_{t+1} (trainer.py:182); the stamp marks the end of round t's update (trainer.py:181)
    // history[h-1] (this round's fused partials of x_h at xbar_h) rides the same launch
    double* hr = met ? c->hraw + 3 * (h - 1 + lag) : c->hraw;
    const FoldArgs fold = {want_cons ? c->slab_cons : nullptr, c->n, want_obj ? c->slab_loss : nullptr,
                           c->loss_groups, want_obj ? c->xbar[xb] : nullptr, hr, hr + 1, hr + 2};
    HIPOK(launch_colsum(c->dtype, c->xs[c->cur ^ 1], c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part,
                        c->stamps + h + 1, n_div(c), c->xbar[xb ^ 1], nullptr, 0.0, 0, c->stream, c->S,
                        met ? &fold : nullptr, cons_cs ? c->slab_cons : nullptr));
    if ((rc = refresh_sums_t(c))) return rc;
    if (!met && !fused && metrics) {
      if ((rc = metrics_pass(c, c->xs[c->cur ^ 1], c->xbar[xb ^ 1], false, want_cons && !cons_cs, want_obj)))
        return rc;
      if ((rc = history(c, h, c->xbar[xb ^ 1], want_cons, want_obj, cons_cs ? cs_blocks : c->n))) return rc;
    }
    c->cur ^= 1;
    xb ^= 1;
  }
  int64_t nh = T + lag;  // history entries this call produces
  if (carry_out && T > 0) {
    nh -= 1;  // history of x_T: owed to the next pipelined run
    c->carry_pending = true;
    c->carry_flags = flags & (DOPT_RUN_OBJECTIVE | DOPT_RUN_CONSENSUS);
  } else if (fused && metrics && (T > 0 || lag)) {  // one metrics pass over x_T
    if ((rc = metrics_pass(c, c->xs[c->cur], c->xbar[xb], false, want_cons, want_obj))) return rc;
    if ((rc = history(c, nh - 1, c->xbar[xb], want_cons, want_obj, c->n))) return rc;
  }
  if (n_out) *n_out = nh;
  return finish_run(c, nh, T, lam_obj, f_opt, want_obj ? obj_out : nullptr, want_cons ? cons_out : nullptr,
                    time_out);
}

int dopt_run_dsgd(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch, const int32_t* idx,
                  double lam_grad, double lam_obj, double f_opt, uint32_t flags, double* obj_out,
                  double* cons_out, double* time_out) {
  return run_dsgd(c, t0, T, eta0, batch, idx, lam_grad, lam_obj, f_opt, flags, obj_out, cons_out, time_out, false,
                  nullptr);
}

int dopt_run_dsgd_pipelined(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch, const int32_t* idx,
                            double lam_grad, double lam_obj, double f_opt, uint32_t flags, double* obj_out,
                            double* cons_out, double* time_out, int64_t* n_out) {
  CHECK_ARG(n_out, "n_out is NULL");
  return run_dsgd(c, t0, T, eta0, batch, idx, lam_grad, lam_obj, f_opt, flags, obj_out, cons_out, time_out, true,
                  n_out);
}

int dopt_run_centralized(dopt_ctx* c, int64_t t0, int64_t T, double eta0, int64_t batch,
                         const int32_t* idx, double lam_grad, double lam_obj, double f_opt,
                         uint32_t flags, double* obj_out, double* time_out) {
  CHECK_ARG(c, "ctx is NULL");
  c->carry_pending = false;
  int rc;
  if ((rc = check_run(c, T, batch, idx, false))) return rc;
  if (!idx && batch < c->max_m) return fail(DOPT_ERR_UNSUPPORTED, "device sampling: D-SGD rounds only");
  if ((rc = set_device(c))) return rc;
  if ((rc = ensure_hist(c, T))) return rc;
  if (!c->G && (rc = dalloc(&c->G, (size_t)c->n * c->ld * c->esz))) return rc;
  const bool want_obj = flags & DOPT_RUN_OBJECTIVE;
  if (c->split) return run_centralized_split(c, t0, T, eta0, batch, idx, lam_grad, lam_obj, f_opt, want_obj,
                                             obj_out, time_out);
  const bool fused = batch >= c->max_m && !c->obj_sep;
  const int64_t CH = idx ? idx_chunk_rounds(c, T, batch) : 1;
  HIPOK(launch_stamp(c->stamps, c->stream));

  for (int64_t h = 0; h < T; ++h) {
    const int64_t t = t0 + h;
    if (idx && h % CH == 0) {
      if ((rc = upload_idx_chunk(c, idx, h, std::min(CH, T - h), batch))) return rc;
    }
    RoundArgs a = base_args(c);
    a.idx = idx ? c->idx + (h % CH) * c->n * batch : nullptr;
    a.b = batch;
    a.w_shared = c->xg[c->gcur];
    a.g_out = c->G;
    a.lam = lam_grad;
    const bool met = fused && want_obj && h > 0;
    a.flags |= F_GOUT | F_SHARED | (met ? (F_LOSS | F_LOSS_FROM_Z) : 0);
    if (a.flags & F_LOSS) c->loss_groups = c->n;  // per-worker loss slabs
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, true, met, a, (int)c->n, c->stream));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    // mean of the worker gradients and the step (trainer.py:53-57)
    HIPOK(launch_colsum(c->dtype, c->G, c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part, c->stamps + h + 1,
                        c->n, c->xg[c->gcur ^ 1], c->xg[c->gcur], eta0 / sqrt((double)(t + 1)), 1, c->stream,
                        nullptr, nullptr));
    if (met) {
      if ((rc = history(c, h - 1, c->xg[c->gcur], false, true, c->n))) return rc;
    } else if (!fused && want_obj) {
      if ((rc = metrics_pass(c, nullptr, c->xg[c->gcur ^ 1], true, false, true))) return rc;
      if ((rc = history(c, h, c->xg[c->gcur ^ 1], false, true, c->n))) return rc;
    }
    c->gcur ^= 1;
  }
  if (fused && want_obj && T > 0) {
    if ((rc = metrics_pass(c, nullptr, c->xg[c->gcur], true, false, true))) return rc;
    if ((rc = history(c, T - 1, c->xg[c->gcur], false, true, c->n))) return rc;
  }
  return finish_run(c, T, T, lam_obj, f_opt, want_obj ? obj_out : nullptr, nullptr, time_out);
}

// ---------------------------------------------------------------------------- single evaluations
namespace {
// Rows longer than the row-resident kernel holds (d > 2048 in float64): dots over column
// ranges, per-row coefficient / loss, column sums of coef * row (kernels.hip k_wide_*).
int eval_wide(dopt_ctx* c, int problem, int64_t rows, int64_t d, const double* w, const double* X, const double* y,
              bool grad, double reg, double* out) {
  const int64_t ld = (d + 1) / 2 * 2, nch = ld / 2;
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(64, d / 8192));
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bX = al((size_t)rows * ld * 8), by = al((size_t)rows * 8 + 8), bw = al((size_t)ld * 8),
               bp = al((size_t)rows * G * 8 + 8), br = al((size_t)rows * 8 + 8), bg = al((size_t)ld * 8),
               bout = al(3 * 8);
  const size_t need = bX + by + bw + bp + br + bg + bout;
  int rc;
  if (need > c->sx_cap) {
    if ((rc = dalloc(&c->sx, need))) return rc;
    c->sx_cap = need;
  }
  char* base = (char*)c->sx;
  double* dX = (double*)base;
  double* dy = (double*)(base + bX);
  double* dw = (double*)(base + bX + by);
  double* dpart = (double*)(base + bX + by + bw);
  double* drow = (double*)(base + bX + by + bw + bp);
  double* dg = (double*)(base + bX + by + bw + bp + br);
  double* dout = (double*)(base + bX + by + bw + bp + br + bg);
  if ((rc = upload_rows(c, DOPT_F64, X, 0, dX, rows, d, ld))) return rc;
  if ((rc = upload_rows(c, DOPT_F64, y, 0, dy, rows, 1, 1))) return rc;
  if ((rc = upload_rows(c, DOPT_F64, w, 0, dw, 1, d, ld))) return rc;
  HIPOK(launch_wide_eval(dX, dy, dw, rows, d, ld, problem, grad, reg, dpart, G, drow, dg, c->stream));
  if (grad) {
    std::vector<double> g((size_t)d);
    HIPOK(hipMemcpyAsync(g.data(), dg, (size_t)d * 8, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    memcpy(out, g.data(), (size_t)d * sizeof(double));
    return DOPT_OK;
  }
  HIPOK(launch_fold(DOPT_F64, nullptr, 0, drow, rows, dw, ld, (int32_t)nch, nullptr, dout + 1, dout + 2, c->stream));
  double raw[3] = {0.0, 0.0, 0.0};
  HIPOK(hipMemcpyAsync(raw + 1, dout + 1, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPOK(hipStreamSynchronize(c->stream));
  finalize_metrics(raw, 1, problem, 1, rows, reg, 0.0, out, nullptr);
  return DOPT_OK;
}

int eval_common(dopt_ctx* c, int problem, int64_t rows, int64_t d, const double* w, const double* X,
                const double* y, bool grad, double reg, double* out) {
  CHECK_ARG(c, "ctx is NULL");
  if (problem != DOPT_LOGISTIC && problem != DOPT_QUADRATIC)
    return fail(DOPT_ERR_UNSUPPORTED, "unknown problem %d", problem);
  CHECK_ARG(rows >= 0 && d >= 1, "bad shape");
  CHECK_ARG(w && out && (rows == 0 || (X && y)), "NULL argument");
  int rc;
  if ((rc = set_device(c))) return rc;
  const int vn = 2;  // float64
  const int64_t ld = (d + vn - 1) / vn * vn, nch = ld / vn;
  const int cpl = cpl_for(nch);
  if (cpl > max_chunks_per_lane(DOPT_F64, DOPT_F64)) return eval_wide(c, problem, rows, d, w, X, y, grad, reg, out);
  // objective: split rows over workgroups; gradient: one workgroup (one worker)
  const int64_t groups = grad ? 1 : std::max<int64_t>(1, std::min<int64_t>(4096, (rows + 255) / 256));
  // scratch layout (bytes, 16-aligned): X | y | w | g | off | slab | out
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bX = al((size_t)rows * ld * 8), by = al((size_t)rows * 8), bw = al((size_t)ld * 8),
               bg = al((size_t)ld * 8), bo = al((size_t)(groups + 1) * 8), bs = al((size_t)groups * 8),
               bout = al(3 * 8);
  const size_t need = bX + by + bw + bg + bo + bs + bout;
  if (need > c->sx_cap) {
    if ((rc = dalloc(&c->sx, need))) return rc;
    c->sx_cap = need;
  }
  char* base = (char*)c->sx;
  void* dX = base;
  void* dy = base + bX;
  void* dw = base + bX + by;
  void* dg = base + bX + by + bw;
  int64_t* doff = (int64_t*)(base + bX + by + bw + bg);
  double* dslab = (double*)(base + bX + by + bw + bg + bo);
  double* dout = (double*)(base + bX + by + bw + bg + bo + bs);
  if ((rc = upload_rows(c, DOPT_F64, X, 0, dX, rows, d, ld))) return rc;
  if ((rc = upload_rows(c, DOPT_F64, y, 0, dy, rows, 1, 1))) return rc;
  if ((rc = upload_rows(c, DOPT_F64, w, 0, dw, 1, d, ld))) return rc;
  std::vector<int64_t> o((size_t)groups + 1);
  for (int64_t k = 0; k <= groups; ++k) o[(size_t)k] = rows * k / groups;
  HIPOK(hipMemcpy(doff, o.data(), o.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  RoundArgs a;
  memset(&a, 0, sizeof(a));
  a.X = dX;
  a.y = dy;
  a.off = doff;
  a.w_shared = dw;
  a.g_out = dg;
  a.lam = reg;
  a.ld = ld;
  a.nchunks = (int32_t)nch;
  a.n_local = 1;
  a.slab_loss = dslab;
  if (grad) {
    a.flags = F_GOUT | F_SHARED;
    HIPOK(launch_round(DOPT_F64, DOPT_F64, problem, cpl, true, false, a, 1, c->stream));
    std::vector<double> g((size_t)ld);
    HIPOK(hipMemcpyAsync(g.data(), dg, (size_t)ld * 8, hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    memcpy(out, g.data(), (size_t)d * sizeof(double));
  } else {
    a.flags = F_SHARED | F_LOSS | F_LOSS_FROM_Z;
    HIPOK(launch_round(DOPT_F64, DOPT_F64, problem, cpl, false, true, a, (int)groups, c->stream));
    HIPOK(launch_history(DOPT_F64, nullptr, dslab, 1, groups, dw, ld, (int32_t)nch, true, dout, c->stream));
    double raw[3];
    HIPOK(hipMemcpyAsync(raw, dout, sizeof(raw), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    finalize_metrics(raw, 1, problem, 1, rows, reg, 0.0, out, nullptr);
  }
  return DOPT_OK;
}
}  // namespace

int dopt_eval_gradient(dopt_ctx* c, int problem, int64_t b, int64_t d, const double* w, const double* X,
                       const double* y, double reg, double* g_out) {
  return eval_common(c, problem, b, d, w, X, y, true, reg, g_out);
}

int dopt_eval_objective(dopt_ctx* c, int problem, int64_t n, int64_t d, const double* w, const double* X,
                        const double* y, double reg, double* out) {
  return eval_common(c, problem, n, d, w, X, y, false, reg, out);
}

int dopt_eval_full(dopt_ctx* c, const double* w, double reg, double* f_out, double* g_out) {
  CHECK_ARG(c && w && f_out, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  int rc;
  if ((rc = set_device(c))) return rc;
  if (c->split) {
    // column-blocked rows (large d): the objective only, by the direct kernels' dots pass at the
    // shared point (k_split_dots mode 1 -> k_split_coef mode 2), independent of the round kernels
    if (g_out) return fail(DOPT_ERR_UNSUPPORTED, "full-data gradient of column-blocked rows (pass g_out = NULL)");
    if ((rc = ensure_split(c))) return rc;
    if ((rc = ensure_hist(c, 1))) return rc;
    if ((rc = upload_rows(c, c->dtype, w, 0, c->xg[c->gcur ^ 1], 1, c->d, c->ld))) return rc;
    if ((rc = split_metrics(c, nullptr, c->xg[c->gcur ^ 1], true, false, true))) return rc;
    if ((rc = history(c, 0, c->xg[c->gcur ^ 1], false, true, c->n))) return rc;
    double raw[3];
    HIPOK(hipMemcpyAsync(raw, c->hraw, sizeof(raw), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    finalize_metrics(raw, 1, c->problem, 1, obj_rows(c), reg, 0.0, f_out, nullptr);
    return DOPT_OK;
  }
  CHECK_ARG(g_out, "NULL argument");
  if (!c->G && (rc = dalloc(&c->G, (size_t)c->n * c->ld * c->esz))) return rc;
  if ((rc = ensure_hist(c, 1))) return rc;
  if ((rc = upload_rows(c, c->dtype, w, 0, c->xg[c->gcur ^ 1], 1, c->d, c->ld))) return rc;
  RoundArgs a = base_args(c);
  if (c->obj_sep) {
    a.X = c->Xo;
    a.y = c->yo;
    a.off = c->offo;
    a.defer_rows = 0;  // rows per workgroup of the objective split, not of the shards
  }
  a.w_shared = c->xg[c->gcur ^ 1];
  a.g_out = c->G;
  a.flags = F_GOUT | F_GSUM | F_SHARED | F_LOSS | F_LOSS_FROM_Z;
  HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, true, true, a, (int)c->n, c->stream));
  c->loss_groups = c->n;  // per-worker loss slabs
  HIPOK(launch_colsum_partial(c->dtype, c->G, c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part, nullptr,
                              c->stream));
  if ((rc = history(c, 0, a.w_shared, false, true, c->n))) return rc;
  std::vector<double> colsum((size_t)c->ld), raw(3);
  double* dsum = nullptr;
  if ((rc = dalloc_t(&dsum, (size_t)c->ld * sizeof(double)))) return rc;
  hipError_t e = launch_colsum_final(c->dtype, c->part, c->groups, c->n, c->ld, (int32_t)c->nchs, nullptr, nullptr,
                                     0.0, 0, c->stream, dsum);
  if (e == hipSuccess) e = hipMemcpyAsync(colsum.data(), dsum, (size_t)c->ld * sizeof(double), hipMemcpyDeviceToHost,
                                          c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(raw.data(), c->hraw, 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree_t(dsum);
  if (e != hipSuccess) return fail(DOPT_ERR_HIP, "dopt_eval_full: %s", hipGetErrorString(e));
  const int64_t M = obj_rows(c);
  // full-data mean over every row (obj_problems.py:22-36 / :55-69), objective (:3-11 / :39-44)
  for (int64_t k = 0; k < c->d; ++k) g_out[k] = (M > 0 ? colsum[(size_t)k] / (double)M : 0.0) + reg * w[k];
  finalize_metrics(raw.data(), 1, c->problem, 1, M, reg, 0.0, f_out, nullptr);
  return DOPT_OK;
}

int dopt_set_sampler(dopt_ctx* c, int mode, uint64_t seed, int64_t first_worker) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(mode == DOPT_SAMPLE_HOST || mode == DOPT_SAMPLE_DEVICE, "unknown sampler %d", mode);
  CHECK_ARG(first_worker >= 0, "first_worker must be >= 0");
  c->sampler = mode;
  c->sample_seed = seed;
  c->sample_wid0 = first_worker;
  return DOPT_OK;
}

int dopt_phase_set_round(dopt_ctx* c, int64_t t) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(t >= 0, "round must be >= 0");
  c->ph_round = t;
  return DOPT_OK;
}

int dopt_phase_set_step(dopt_ctx* c, int64_t t, double eta0) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(t >= 0, "round must be >= 0");
  c->ph_round = t;
  c->ph_eta = eta0 / sqrt((double)(t + 1));  // trainer.py:138-140
  c->ph_eta_set = true;
  return DOPT_OK;
}

int dopt_set_profiling(dopt_ctx* c, int enable) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(enable >= 0, "enable must be >= 0");
  c->prof = enable != 0;
  c->prof_every = enable > 0 ? enable : 1;
  c->prof_seq = 0;
  return DOPT_OK;
}

int dopt_kernel_stats(dopt_ctx* c, int64_t* launches, double* total_ms) {
  CHECK_ARG(c && launches && total_ms, "NULL argument");
  int rc;
  if ((rc = set_device(c))) return rc;
  HIPOK(hipStreamSynchronize(c->stream));
  double ms_sum = 0.0;
  for (int64_t k = 0; k < c->prof_n; ++k) {
    float ms = 0.f;
    HIPOK(hipEventElapsedTime(&ms, c->ev[(size_t)(2 * k)], c->ev[(size_t)(2 * k + 1)]));
    ms_sum += ms;
  }
  *launches = c->prof_n;
  *total_ms = ms_sum;
  c->prof_n = 0;  // the next statistics window starts here
  return DOPT_OK;
}

// ---------------------------------------------------------------------------- multi-GPU phases
int dopt_set_stream(dopt_ctx* c, void* stream) {
  CHECK_ARG(c, "ctx is NULL");
  c->stream = stream ? (hipStream_t)stream : c->own_stream;
  return DOPT_OK;
}

int dopt_get_layout(dopt_ctx* c, int64_t* ld, int64_t* elem_bytes) {
  CHECK_ARG(c && ld && elem_bytes, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  *ld = c->ld;
  *elem_bytes = (int64_t)c->esz;
  return DOPT_OK;
}

int dopt_set_partition(dopt_ctx* c, int64_t n_global, int64_t rows_global) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  CHECK_ARG(n_global >= c->n && rows_global >= 0, "global sizes smaller than the local slice");
  int rc;
  if ((rc = rs_end(c))) return rc;  // rank slices run the phase API (xs[cur] is the state)
  c->n_global = n_global;
  c->rows_global = rows_global;
  return DOPT_OK;
}

int dopt_set_halo(dopt_ctx* c, int64_t n_halo, void* halo_dev, int64_t n_send, void* send_dev,
                  const int32_t* send_ids) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  CHECK_ARG(n_halo >= 0 && n_send >= 0, "negative sizes");
  CHECK_ARG(n_halo == 0 || halo_dev, "halo buffer is NULL");
  CHECK_ARG(n_send == 0 || (send_dev && send_ids), "send buffer / ids are NULL");
  for (int64_t k = 0; k < n_send; ++k)  // -1: a row that carries no worker (column sums, dopt_lagged_*)
    CHECK_ARG(send_ids[k] >= -1 && send_ids[k] < c->n, "send id out of range");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = rs_end(c))) return rc;
  if ((rc = dalloc_t(&c->send_ids, (size_t)std::max<int64_t>(1, n_send) * sizeof(int32_t)))) return rc;
  if (n_send) HIPOK(hipMemcpy(c->send_ids, send_ids, (size_t)n_send * sizeof(int32_t), hipMemcpyHostToDevice));
  c->n_halo = n_halo;
  c->halo = halo_dev;
  c->n_send = n_send;
  c->send = send_dev;
  c->ipc = false;  // (a pull transport is set up again after the buffers: dopt_lagged_ipc_export)
  c->send_fresh = false;
  // inverse map for dopt_phase_mix: worker -> the send rows that carry it (one row per peer)
  std::vector<int64_t> sp((size_t)c->n + 1, 0);
  for (int64_t k = 0; k < n_send; ++k)
    if (send_ids[k] >= 0) sp[(size_t)send_ids[k] + 1]++;
  for (int64_t i = 0; i < c->n; ++i) sp[(size_t)i + 1] += sp[(size_t)i];
  std::vector<int32_t> slot((size_t)std::max<int64_t>(1, n_send));
  std::vector<int64_t> fill(sp.begin(), sp.end() - 1);
  for (int64_t k = 0; k < n_send; ++k)
    if (send_ids[k] >= 0) slot[(size_t)fill[(size_t)send_ids[k]]++] = (int32_t)k;
  c->is_send.assign((size_t)c->n, 0);
  for (int64_t k = 0; k < n_send; ++k)
    if (send_ids[k] >= 0) c->is_send[(size_t)send_ids[k]] = 1;
  if ((rc = dalloc_t(&c->sptr, sp.size() * sizeof(int64_t)))) return rc;
  if ((rc = dalloc_t(&c->sslot, slot.size() * sizeof(int32_t)))) return rc;
  HIPOK(hipMemcpy(c->sptr, sp.data(), sp.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(c->sslot, slot.data(), slot.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  c->have_topo = false;  // the CSR must be re-set in the local+halo index space
  return DOPT_OK;
}

int dopt_phase_gather(dopt_ctx* c) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  if (c->send_fresh) return DOPT_OK;  // the last mix wrote these rows already
  int rc;
  if ((rc = rs_end(c))) return rc;
  HIPOK(launch_gather_rows(c->dtype, c->xs[c->cur], c->send_ids, c->n_send, c->ld, (int32_t)c->nchs, c->send,
                           c->stream));
  return DOPT_OK;
}

int dopt_phase_interior_count(dopt_ctx* c, int64_t* n_interior) {
  CHECK_ARG(c && n_interior, "NULL argument");
  *n_interior = c->have_topo && !c->mean_mix && c->interior ? c->n_interior : 0;
  return DOPT_OK;
}

int dopt_phase_chain(dopt_ctx* c, int mark, int* was_pending) {
  CHECK_ARG(c && was_pending, "NULL argument");
  *was_pending = c->carry_pending ? 1 : 0;
  c->carry_pending = mark != 0;
  c->carry_flags = 0;
  return DOPT_OK;
}

int dopt_phase_begin(dopt_ctx* c, int64_t batch) {
  CHECK_ARG(c, "ctx is NULL");
  c->carry_pending = false;
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  c->send_fresh = false;  // the iterates may have been set since the last mix
  int rc;
  if ((rc = rs_end(c))) return rc;
  if (c->split) {
    if ((rc = ensure_split(c))) return rc;
    if (std::min(batch, c->max_m) > kSplitMaxRows)
      return fail(DOPT_ERR_UNSUPPORTED, "column-blocked rounds hold at most %d rows per minibatch", kSplitMaxRows);
    if (batch >= c->max_m) {  // coefficients of the starting iterates
      RoundArgs p = base_args(c);
      p.x_old = c->xs[c->cur];
      HIPOK(split_dots(c, 0, p));
      HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 1, p, (int)c->n, c->stream));
    }
  }
  return DOPT_OK;
}

int dopt_phase_grad(dopt_ctx* c, int64_t batch, const int32_t* idx, double lam_grad, uint32_t metric_flags) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = check_run(c, 1, batch, idx, false))) return rc;
  const bool dev = !idx && batch < c->max_m;  // device sampler (check_run)
  if (!c->G && (rc = dalloc(&c->G, (size_t)c->n * c->ld * c->esz))) return rc;
  if (idx && (rc = upload_idx_chunk(c, idx, 0, 1, batch, true))) return rc;
  const bool cons = metric_flags & DOPT_RUN_CONSENSUS, loss = metric_flags & DOPT_RUN_OBJECTIVE;
  const bool bip = (cons || loss) && (dev ? !c->obj_sep : bip_possible(c, batch, idx));
  if ((cons || loss) && ((batch < c->max_m && !bip) || c->obj_sep))
    return fail(DOPT_ERR_UNSUPPORTED, "fused metrics need every shard row in the pass (full shards, or "
                "minibatches of shards of at most %lld rows)", (long long)kMaxBipRows);
  if (c->split) {  // the gradient is produced block by block inside the step (dopt_phase_mix)
    c->ph_batch = batch;
    c->ph_lam = lam_grad;
    c->ph_flags = metric_flags;
    c->ph_have_idx = idx != nullptr;
    if (idx) {  // this round's minibatch coefficients
      RoundArgs a = base_args(c);
      a.idx = c->idx;
      a.b = batch;
      a.b_rows = (int32_t)std::min<int64_t>(a.b_rows, batch);
      a.x_old = c->xs[c->cur];
      HIPOK(split_dots(c, 0, a));
      HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 1, a, (int)c->n, c->stream));
    }
    return DOPT_OK;
  }
  RoundArgs a = base_args(c);
  a.idx = idx ? c->idx : nullptr;
  a.b = batch;
  a.x_old = c->xs[c->cur];
  a.g_out = c->G;
  a.xbar = c->xbar[c->xb];
  a.lam = lam_grad;
  a.flags |= F_GOUT | (cons ? F_CONS : 0) | (loss ? F_LOSS : 0) | (bip || dev ? F_BIP : 0) | (dev ? F_DEVSAMPLE : 0);
  a.seed = c->sample_seed;
  a.round = c->ph_round;
  a.wid0 = c->sample_wid0;
  // interior workers: mixed and stepped here (bitwise the fused round's arithmetic; k_mix skips
  // them), when the round's step size is known (dopt_phase_set_step)
  static const bool interior_on = [] {  // DOPT_PHASE_INTERIOR=0: every worker through k_mix (A/B runs)
    const char* v = getenv("DOPT_PHASE_INTERIOR");
    return !(v && v[0] == '0');
  }();
  c->ph_interior = interior_on && c->ph_eta_set && c->have_topo && !c->mean_mix && c->n_interior > 0 && c->interior;
  c->ph_eta_set = false;
  if (c->ph_interior) {
    a.interior = c->interior;
    a.x_new = c->xs[c->cur ^ 1];
    a.eta = c->ph_eta;
  }
  if (a.flags & F_LOSS) c->loss_groups = c->slab_n[0] = c->n;  // per-worker loss slabs
  if (c->prof && (rc = prof_event(c, false))) return rc;
  HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, true, cons || loss || dev, a, (int)c->n, c->stream));
  if (c->prof && (rc = prof_event(c, true))) return rc;
  return DOPT_OK;
}

int dopt_phase_mix(dopt_ctx* c, int64_t t, double eta0) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->have_topo || !c->G) return fail(DOPT_ERR_STATE, "topology / gradient phase missing");
  RoundArgs a = base_args(c);
  a.x_old = c->xs[c->cur];
  a.x_new = c->xs[c->cur ^ 1];
  a.eta = eta0 / sqrt((double)(t + 1));  // trainer.py:138-140
  if (c->split) {  // gradient + mix + step (+ next coefficients, + metric partials) in one pass
    const bool full = !c->ph_have_idx;
    const bool cons = c->ph_flags & DOPT_RUN_CONSENSUS, loss = c->ph_flags & DOPT_RUN_OBJECTIVE;
    a.idx = full ? nullptr : c->idx;
    a.b = c->ph_batch;
    if (!full) a.b_rows = (int32_t)std::min<int64_t>(a.b_rows, c->ph_batch);
    a.lam = c->ph_lam;
    a.xbar = c->xbar[c->xb];
    a.flags |= (cons ? F_CONS : 0) | (loss ? F_LOSS : 0);
    if (a.flags & F_LOSS) c->loss_groups = c->n;  // per-worker loss slabs
    int rc;
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(split_step(c, full, cons || loss, a));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    if (full || cons || loss) {
      RoundArgs q = a;
      q.idx = nullptr;
      HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, (full ? 1 : 0) | ((cons || loss) ? 2 : 0), q, (int)c->n,
                              c->stream));
    }
    c->send_fresh = false;
  } else {
    if (c->n_send > 0) {  // refresh the send rows from the new iterates (the next round's gather)
      a.sptr = c->sptr;
      a.sslot = c->sslot;
      a.send = c->send;
    }
    if (c->ph_interior) a.interior = c->interior;  // stepped by the gradient kernel already
    a.nchunks = (int32_t)c->nchs;  // k_mix walks state chunks
    HIPOK(launch_mix(c->dtype, c->cpls, a, c->G, (int)c->n, c->stream));
    c->send_fresh = c->n_send > 0;
  }
  c->ph_interior = false;
  c->cur ^= 1;
  return DOPT_OK;
}

// ---- centralized trainer across ranks (trainer.py:41-71): per-rank gradients at the
// shared iterate, all-reduced column sums of the gradients, the step.
int dopt_phase_grad_shared(dopt_ctx* c, int64_t batch, const int32_t* idx, double lam_grad, int fuse_loss) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = check_run(c, 1, batch, idx, false))) return rc;
  if (!c->G && (rc = dalloc(&c->G, (size_t)c->n * c->ld * c->esz))) return rc;
  if (idx && (rc = upload_idx_chunk(c, idx, 0, 1, batch, true))) return rc;
  if (fuse_loss && (batch < c->max_m || c->obj_sep))
    return fail(DOPT_ERR_UNSUPPORTED, "a fused objective needs full-shard batches over the shard rows");
  RoundArgs a = base_args(c);
  a.idx = idx ? c->idx : nullptr;
  a.b = batch;
  a.w_shared = c->xg[c->gcur];
  a.g_out = c->G;
  a.lam = lam_grad;
  a.flags |= F_GOUT | F_SHARED | (fuse_loss ? (F_LOSS | F_LOSS_FROM_Z) : 0);
  if (a.flags & F_LOSS) c->loss_groups = c->n;  // per-worker loss slabs
  if (c->split) {
    if (fuse_loss) return fail(DOPT_ERR_UNSUPPORTED, "column-blocked rounds: use dopt_phase_metrics_pass_shared");
    if ((rc = ensure_split(c))) return rc;
    HIPOK(split_dots(c, 0, a));
    HIPOK(launch_split_coef(c->dtype, c->xdtype, c->problem, 1, a, (int)c->n, c->stream));
    if (c->prof && (rc = prof_event(c, false))) return rc;
    HIPOK(split_step(c, false, false, a));
    if (c->prof && (rc = prof_event(c, true))) return rc;
    return DOPT_OK;
  }
  if (c->prof && (rc = prof_event(c, false))) return rc;
  HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, true, fuse_loss != 0, a, (int)c->n, c->stream));
  if (c->prof && (rc = prof_event(c, true))) return rc;
  return DOPT_OK;
}

int dopt_phase_colsum_grad(dopt_ctx* c, double* sum_dev) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  if (!c->G) return fail(DOPT_ERR_STATE, "no gradient phase yet");
  HIPOK(launch_colsum_partial(c->dtype, c->G, c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part, nullptr,
                              c->stream));
  HIPOK(launch_colsum_final(c->dtype, c->part, c->groups, c->n, c->ld, (int32_t)c->nchs, nullptr, nullptr, 0.0, 0,
                            c->stream, sum_dev));
  return DOPT_OK;
}

int dopt_phase_central_step(dopt_ctx* c, const double* sum_dev, int64_t t, double eta0) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  HIPOK(launch_colsum_final(c->dtype, sum_dev, 1, n_div(c), c->ld, (int32_t)c->nchs, c->xg[c->gcur ^ 1],
                            c->xg[c->gcur], eta0 / sqrt((double)(t + 1)), 1, c->stream));
  c->gcur ^= 1;
  return DOPT_OK;
}

int dopt_phase_metrics_pass_shared(dopt_ctx* c) {
  CHECK_ARG(c, "ctx is NULL");
  if (c->split) {
    int rc;
    if ((rc = ensure_split(c))) return rc;
    return split_metrics(c, nullptr, c->xg[c->gcur], true, false, true);
  }
  return metrics_pass(c, nullptr, c->xg[c->gcur], true, false, true);
}

int dopt_phase_metrics_shared(dopt_ctx* c, int include_xnorm, double* out_dev) {
  CHECK_ARG(c && out_dev, "NULL argument");
  HIPOK(launch_history(c->dtype, nullptr, c->slab_loss, c->n, c->loss_groups, c->xg[c->gcur], c->ld,
                       (int32_t)c->nchs, include_xnorm != 0, out_dev, c->stream));
  return DOPT_OK;
}

int dopt_phase_colsum(dopt_ctx* c, double* sum_dev) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  int rc;
  if ((rc = rs_end(c))) return rc;
  HIPOK(launch_colsum_partial(c->dtype, c->xs[c->cur], c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part,
                              nullptr, c->stream));
  HIPOK(launch_colsum_final(c->dtype, c->part, c->groups, c->n, c->ld, (int32_t)c->nchs, nullptr, nullptr, 0.0, 0,
                            c->stream, sum_dev));
  return DOPT_OK;
}

int dopt_phase_xbar(dopt_ctx* c, const double* sum_dev) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  HIPOK(launch_colsum_final(c->dtype, sum_dev, 1, n_div(c), c->ld, (int32_t)c->nchs, c->xbar[c->xb ^ 1], nullptr,
                            0.0, 0, c->stream));
  c->xb ^= 1;
  c->S_ext = sum_dev;  // the complete-graph mix of the next round uses the global sums
  return refresh_sums_t(c);
}

int dopt_phase_fold(dopt_ctx* c, double* cons_out, double* xnorm_out, double* loss_out, int slab) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(slab == 0 || slab == 1, "slab must be 0 or 1");
  if (c->rs_live && !c->rs_sweep) {  // row-space rounds: ||xbar||^2 from the average update's block partials
    HIPOK(launch_rs_fold(rs_args(c), c->slab_cons, c->cons_n, slab ? c->slab_loss_b : c->slab_loss, c->slab_n[slab],
                         cons_out, loss_out, xnorm_out, c->stream));
    return DOPT_OK;
  }
  HIPOK(launch_fold(c->dtype, c->slab_cons, c->cons_n, slab ? c->slab_loss_b : c->slab_loss, c->slab_n[slab],
                    c->xbar[c->xb], c->ld, (int32_t)c->nchs, cons_out, loss_out, xnorm_out, c->stream));
  return DOPT_OK;
}

// ---- row-space rounds on a rank's slice (complete graph, quadratic, full shards; rowspace.hip).
// The replicated d-vectors (xbar, Z) take the all-reduced column sums, so every rank holds
// the same ones; the metric partials are this rank's workers' (folded by dopt_phase_fold).
int dopt_rs_phase_begin(dopt_ctx* c, int commit, int* ok, uint64_t* hash) {
  CHECK_ARG(c && ok && hash, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  *ok = 0;
  *hash = 0;
  if (!(rs_enabled() && c->split && c->mean_mix && c->wdiag_uniform && !c->obj_sep && c->min_m >= 1 &&
        c->max_m <= kRsMaxRows))
    return DOPT_OK;
  int rc;
  if ((rc = set_device(c))) return rc;
  if (c->rs_live) {  // (an open chain -- dopt_phase_chain -- stays open)
    if (int rc = rs_sweep_closed(c)) return rc;
    // the replicated part of the state (Z, then the float64 average), bitwise equal on every
    // rank that took the same all-reduced sums
    std::vector<double> zx(2 * (size_t)c->ld);
    HIPOK(hipMemcpyAsync(zx.data(), c->rs_Z, zx.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPOK(hipStreamSynchronize(c->stream));
    *hash = content_hash(zx.data(), zx.size() * sizeof(double));
    *ok = 1;
    return DOPT_OK;
  }
  c->carry_pending = false;
  bool equal = false, zero = false;
  if ((rc = rs_check(c, &equal, &zero, hash))) return rc;
  if (!equal) return DOPT_OK;
  *ok = 1;
  if (!commit) return DOPT_OK;
  return rs_begin(c, false) == RS_FALLBACK ? fail(DOPT_ERR_STATE, "row-space begin: iterates changed") : DOPT_OK;
}

int dopt_rs_phase_round(dopt_ctx* c, int64_t t, double eta0, double lam_grad, uint32_t metric_flags,
                        double* sum_dev) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  if (!c->rs_live) return fail(DOPT_ERR_STATE, "dopt_rs_phase_begin first");
  if (int rc = rs_sweep_closed(c)) return rc;
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  RsArgs a = rs_args(c);
  rs_round_args(c, a, t, eta0, lam_grad);
  a.xbar = c->xbar[c->xb];
  const bool met = (metric_flags & (DOPT_RUN_OBJECTIVE | DOPT_RUN_CONSENSUS)) != 0;
  a.slab_cons = (metric_flags & DOPT_RUN_CONSENSUS) ? c->slab_cons : nullptr;
  a.slab_loss = (metric_flags & DOPT_RUN_OBJECTIVE) ? c->slab_loss : nullptr;
  int rc;
  if (c->prof && (rc = prof_event(c, false))) return rc;
  HIPOK(launch_rs_pass(dt, rs_xdt(c), true, a, c->stream));
  if (c->prof && (rc = prof_event(c, true))) return rc;
  HIPOK(launch_rs_rows(dt, a, (int)c->n, 2 | (met ? 1 : 0), c->stream));
  HIPOK(launch_rs_csum(a, sum_dev, c->stream));
  c->cons_n = c->n;
  c->slab_n[0] = c->n;
  c->rs_xs_valid = false;
  return DOPT_OK;
}

int dopt_rs_phase_pass(dopt_ctx* c, int32_t chunk, int32_t n_chunks, double* sum_dev, int64_t* col_range) {
  CHECK_ARG(c && sum_dev && col_range, "NULL argument");
  if (!c->rs_live) return fail(DOPT_ERR_STATE, "dopt_rs_phase_begin first");
  CHECK_ARG(n_chunks >= 1 && chunk >= 0 && chunk < n_chunks, "chunk %d of %d", chunk, n_chunks);
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  RsArgs a = rs_args(c);
  a.xbar = c->xbar[c->rs_sweep ? c->xb ^ 1 : c->xb];  // (an open chunked update: its chunks come first)
  const int nb = std::min<int>(n_chunks, a.nblk);  // more chunks than blocks: the extra ones are empty
  const int b0 = chunk < nb ? (int)((int64_t)a.nblk * chunk / nb) : a.nblk;
  const int b1 = chunk < nb ? (int)((int64_t)a.nblk * (chunk + 1) / nb) : a.nblk;
  rs_block_cols(a, rs_xdt(c), b0, b1, &col_range[0], &col_range[1]);
  int rc;
  if (c->prof && chunk == 0 && (rc = prof_event(c, false))) return rc;  // one bracket around the whole pass
  if (b1 > b0) {
    a.blk0 = b0;
    HIPOK(launch_rs_pass(dt, rs_xdt(c), true, a, c->stream, b1 - b0));
    HIPOK(launch_rs_csum(a, sum_dev, c->stream, col_range[0], col_range[1]));
  }
  if (c->prof && chunk == n_chunks - 1 && (rc = prof_event(c, true))) return rc;
  c->rs_xs_valid = false;
  return DOPT_OK;
}

int dopt_rs_phase_rows(dopt_ctx* c, int64_t t, double eta0, double lam_grad, uint32_t metric_flags) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->rs_live) return fail(DOPT_ERR_STATE, "dopt_rs_phase_begin first");
  if (int rc = rs_sweep_closed(c)) return rc;
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  RsArgs a = rs_args(c);
  rs_round_args(c, a, t, eta0, lam_grad);
  const bool met = (metric_flags & (DOPT_RUN_OBJECTIVE | DOPT_RUN_CONSENSUS)) != 0;
  a.slab_cons = (metric_flags & DOPT_RUN_CONSENSUS) ? c->slab_cons : nullptr;
  a.slab_loss = (metric_flags & DOPT_RUN_OBJECTIVE) ? c->slab_loss : nullptr;
  HIPOK(launch_rs_rows(dt, a, (int)c->n, 2 | (met ? 1 : 0), c->stream));
  c->cons_n = c->n;
  c->slab_n[0] = c->n;
  return DOPT_OK;
}

int dopt_rs_phase_cols(dopt_ctx* c, int64_t t, double eta0, double lam_grad, const double* sum_dev) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  if (!c->rs_live) return fail(DOPT_ERR_STATE, "dopt_rs_phase_begin first");
  if (int rc = rs_sweep_closed(c)) return rc;
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  RsArgs a = rs_args(c);
  rs_round_args(c, a, t, eta0, lam_grad);
  a.csum = sum_dev;
  a.xbar_out = c->xbar[c->xb ^ 1];
  HIPOK(launch_rs_cols(dt, a, c->stream));
  c->xb ^= 1;
  return DOPT_OK;
}

// The same update for columns [c0, c1) only (a chunk of dopt_rs_phase_pass), so that the next
// round's pass over that chunk can start while the sums of later chunks are still being reduced;
// the chunks of one update in any order, the last one with last = 1.
int dopt_rs_phase_cols_range(dopt_ctx* c, int64_t t, double eta0, double lam_grad, const double* sum_dev,
                             int64_t c0, int64_t c1, int32_t last) {
  CHECK_ARG(c && sum_dev, "NULL argument");
  if (!c->rs_live) return fail(DOPT_ERR_STATE, "dopt_rs_phase_begin first");
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  RsArgs a = rs_args(c);
  CHECK_ARG(c0 >= 0 && c0 <= c1 && c1 <= a.ld &&
                (c0 == c1 || (c0 % kRsColsBlock == 0 && (c1 == a.ld || c1 % kRsColsBlock == 0))),
            "column range [%lld, %lld) of %lld: a dopt_rs_phase_pass chunk", (long long)c0, (long long)c1,
            (long long)a.ld);
  rs_round_args(c, a, t, eta0, lam_grad);
  a.csum = sum_dev;
  a.xbar_out = c->xbar[c->xb ^ 1];
  if (c1 > c0) HIPOK(launch_rs_cols(dt, a, c->stream, c0, c1));
  c->rs_sweep = last == 0;
  if (last) c->xb ^= 1;
  return DOPT_OK;
}

int dopt_rs_phase_metrics(dopt_ctx* c, uint32_t metric_flags) {
  CHECK_ARG(c, "ctx is NULL");
  if (!c->rs_live) return fail(DOPT_ERR_STATE, "dopt_rs_phase_begin first");
  if (int rc = rs_sweep_closed(c)) return rc;
  const int dt = c->dtype == DOPT_F32 ? 0 : 1;
  RsArgs a = rs_args(c);
  a.xbar = c->xbar[c->xb];
  a.slab_cons = (metric_flags & DOPT_RUN_CONSENSUS) ? c->slab_cons : nullptr;
  a.slab_loss = (metric_flags & DOPT_RUN_OBJECTIVE) ? c->slab_loss : nullptr;
  HIPOK(launch_rs_pass(dt, rs_xdt(c), false, a, c->stream));
  HIPOK(launch_rs_rows(dt, a, (int)c->n, 1, c->stream));
  c->cons_n = c->n;
  c->slab_n[0] = c->n;
  return DOPT_OK;
}

int dopt_phase_metrics_pass(dopt_ctx* c, uint32_t flags) {
  CHECK_ARG(c, "ctx is NULL");
  if (c->split) {
    int rc;
    if ((rc = ensure_split(c))) return rc;
    return split_metrics(c, c->xs[c->cur], c->xbar[c->xb], false, flags & DOPT_RUN_CONSENSUS,
                         flags & DOPT_RUN_OBJECTIVE);
  }
  return metrics_pass(c, c->xs[c->cur], c->xbar[c->xb], false, flags & DOPT_RUN_CONSENSUS,
                      flags & DOPT_RUN_OBJECTIVE);
}

int dopt_phase_metrics(dopt_ctx* c, uint32_t flags, int include_xnorm, double* out_dev) {
  CHECK_ARG(c && out_dev, "NULL argument");
  const bool cons = flags & DOPT_RUN_CONSENSUS, loss = flags & DOPT_RUN_OBJECTIVE;
  HIPOK(launch_history(c->dtype, cons ? c->slab_cons : nullptr, loss ? c->slab_loss : nullptr, c->n,
                       c->loss_groups, c->xbar[c->xb], c->ld, (int32_t)c->nchs, loss && include_xnorm, out_dev,
                       c->stream));
  return DOPT_OK;
}

// ---- the lagged schedule with the column sums in the exchange (round 4; distributed.py _run_lagged).
// Round g of a chain: dopt_lagged_grad (gradient pass of x_g; interior workers stepped; loss of
// every row at xbar_{g-1}) beside the exchange of x_g's send rows AND every rank's column sums of
// x_g, then dopt_lagged_mix (k_mixcs: xbar_g from the rank-ordered sums, consensus of x_g, x_{g+1}
// of the other workers and their send rows, the column sums of x_{g+1} into the send buffer, and
// the fold of history[g-2]; k_mixcs_final totals the column sums).  Three launches and one
// collective per round.
int dopt_lagged_exchange_layout(dopt_ctx* c, int32_t world, int32_t rank, const int64_t* sum_send_row,
                                const int64_t* sum_recv_row) {
  CHECK_ARG(c && sum_send_row && sum_recv_row, "NULL argument");
  CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "bad world / rank");
  CHECK_ARG(world <= 1024, "at most 1024 ranks");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  const int64_t rows = (int64_t)(c->esz == 4 ? 2 : 1);  // rows of T holding ld doubles
  for (int32_t p = 0; p < world; ++p) {
    if (p == rank && sum_send_row[p] < 0) {  // (a self block -- both rows >= 0 -- is checked below)
      CHECK_ARG(sum_recv_row[p] < 0, "rank %d: sum rows to itself received but not sent", rank);
      continue;
    }
    CHECK_ARG(sum_send_row[p] >= 0 && sum_recv_row[p] >= 0, "peer %d: sum rows missing", p);
    CHECK_ARG(sum_send_row[p] + rows <= std::max<int64_t>(c->n_send, 0) && sum_recv_row[p] + rows <= c->n_halo,
              "peer %d: sum rows past the send (%lld) / halo (%lld) buffers (dopt_set_halo first)", p,
              (long long)c->n_send, (long long)c->n_halo);
  }
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = dalloc_t(&c->lg_sum_in, (size_t)world * sizeof(int64_t)))) return rc;
  if ((rc = dalloc_t(&c->lg_sum_out, (size_t)world * sizeof(int64_t)))) return rc;
  HIPOK(hipMemcpy(c->lg_sum_in, sum_recv_row, (size_t)world * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(c->lg_sum_out, sum_send_row, (size_t)world * sizeof(int64_t), hipMemcpyHostToDevice));
  c->lg_in_h.assign(sum_recv_row, sum_recv_row + world);
  c->lg_out_h.assign(sum_send_row, sum_send_row + world);
  c->lg_world = world;
  c->lg_rank = rank;
  c->lg_self = sum_send_row[rank] >= 0;  // this rank's sums go through the exchange to itself too
  return DOPT_OK;
}

namespace {
int lagged_ready(dopt_ctx* c) {
  if (c->split || c->mean_mix || !c->have_topo)
    return fail(DOPT_ERR_UNSUPPORTED, "lagged rounds: row-resident contexts with CSR mixing only");
  if (c->lg_world > 1 && (int64_t)c->lg_in_h.size() != c->lg_world)
    return fail(DOPT_ERR_STATE, "lagged rounds: dopt_lagged_exchange_layout first");
  if (!c->lg_sum_in) {  // world 1 without a layout call: one rank, no peer rows
    const int64_t self = -1;
    int rc;
    if ((rc = dalloc_t(&c->lg_sum_in, sizeof(int64_t)))) return rc;
    if ((rc = dalloc_t(&c->lg_sum_out, sizeof(int64_t)))) return rc;
    HIPOK(hipMemcpy(c->lg_sum_in, &self, sizeof(int64_t), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(c->lg_sum_out, &self, sizeof(int64_t), hipMemcpyHostToDevice));
  }
  if (c->lg_alloc_n == c->n && c->lg_alloc_ld == c->ld) return DOPT_OK;
  mixcs_shape(c->dtype, c->n, (int32_t)c->nchs, &c->lg_ncb, &c->lg_r, &c->lg_ng);
  int rc;
  for (int k = 0; k < 2; ++k) {
    if ((rc = dalloc_t(&c->lg_own[k], (size_t)c->ld * sizeof(double)))) return rc;
    HIPOK(hipMemsetAsync(c->lg_own[k], 0, (size_t)c->ld * sizeof(double), c->stream));
    if ((rc = dalloc_t(&c->lg_cons[k], (size_t)std::max<int64_t>(1, c->lg_ncb * c->n) * sizeof(double)))) return rc;
  }
  if ((rc = dalloc_t(&c->lg_part, (size_t)c->lg_ng * c->ld * sizeof(double)))) return rc;
  c->lg_alloc_n = c->n;
  c->lg_alloc_ld = c->ld;
  return DOPT_OK;
}

// The lagged tail's loss pass: loss of every local objective row at the current average -> slab B,
// and with two_points also at the previous average -> slab A (one pass over the rows).
int lagged_loss_pass(dopt_ctx* c, int two_points) {
  if (!c->have_data) return fail(DOPT_ERR_STATE, "no shards loaded");
  if (c->split) return fail(DOPT_ERR_UNSUPPORTED, "lagged metrics: row-resident contexts only");
  RoundArgs a = base_args(c);
  a.X = c->obj_sep ? c->Xo : c->X;
  a.y = c->obj_sep ? c->yo : c->y;
  a.off = c->obj_sep ? c->choff_o : c->choff;
  a.defer_rows = (int32_t)kLossChunk;  // 64-row chunks
  const int64_t nc = c->obj_sep ? c->n_chunks_o : c->n_chunks;
  a.w_shared = c->xbar[c->xb];  // current average: z -> slab B
  if (two_points) {
    a.xbar = c->xbar[c->xb ^ 1];  // previous average: u -> slab A
    a.slab_loss = c->slab_loss;
    a.slab_loss2 = c->slab_loss_b;
    a.flags |= F_LOSS | F_SHARED | F_LOSS2;
    c->slab_n[0] = nc;
  } else {
    a.slab_loss = c->slab_loss_b;
    a.flags |= F_LOSS | F_SHARED | F_LOSS_FROM_Z;
  }
  c->slab_n[1] = nc;
  HIPOK(launch_round(c->dtype, c->xdtype, c->problem, c->cpl, false, true, a, (int)nc, c->stream));
  return DOPT_OK;
}

// How the lagged schedule's two streams hand off (round 5, profiles/r5_sync_ab.txt): an event recorded on
// the engine stream after k_mixcs, waited for on the side stream, and an event behind the exchange on the
// side stream that the next mix waits for -- the fastest of the forms measured (stream memory operations,
// ~5 us each as small kernels on this ROCm, made the 512-worker round ~6 % slower).
// The engine stream waits for the exchange issued on the side stream.
int lagged_xwait(dopt_ctx* c) {
  if (!c->lg_xwait) return DOPT_OK;
  HIPOK(hipStreamWaitEvent(c->stream, c->lg_xev, 0));
  c->lg_xwait = false;
  return DOPT_OK;
}

McsArgs lagged_args(dopt_ctx* c, const double* own_in, double* own_out, double* cons_part) {
  McsArgs m;
  memset(&m, 0, sizeof(m));
  m.part = c->lg_part;
  m.ng = c->lg_ng;
  m.ncb = c->lg_ncb;
  m.r = c->lg_r;
  m.world = c->lg_world;
  m.rank = c->lg_rank;
  m.own_in = own_in;
  m.own_out = own_out;
  m.sum_in = c->lg_sum_in;
  m.sum_out = c->lg_sum_out;
  m.cons_part = cons_part;
  m.n_div = (double)n_div(c);
  for (int p = 0; p < kMcsKargRanks; ++p) {  // the first ranks' rows by value (no dependent load in the kernel)
    m.kin[p] = p < (int)c->lg_in_h.size() ? (int32_t)c->lg_in_h[p] : -1;
    m.kout[p] = p < (int)c->lg_out_h.size() ? (int32_t)c->lg_out_h[p] : -1;
  }
  return m;
}
}  // namespace

int dopt_lagged_begin(dopt_ctx* c, int64_t batch) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = dopt_phase_begin(c, batch))) return rc;
  if ((rc = lagged_ready(c))) return rc;
  // the pull transport: the slot of the next record (records are numbered across chains, so a peer's
  // counter never names an older chain's round)
  if (c->ipc) c->send = c->ipc_send + (c->ipc_rec & 1) * c->ipc_slot;
  if ((rc = dopt_phase_gather(c))) return rc;  // send rows of x_0 (later rounds: k_mixcs writes them)
  // this rank's column sums of x_0 -> lg_own[0] and the send buffer's sum rows
  HIPOK(launch_colsum_partial(c->dtype, c->xs[c->cur], c->n, c->ld, (int32_t)c->nchs, kRowsPerGroup, c->part, nullptr,
                              c->stream));
  HIPOK(launch_colsum_final(c->dtype, c->part, c->groups, c->n, c->ld, (int32_t)c->nchs, nullptr, nullptr, 0.0, 0,
                            c->stream, c->lg_own[0]));
  const McsArgs m = lagged_args(c, c->lg_own[0], nullptr, nullptr);
  if (c->lg_world > 1 || c->lg_self) HIPOK(launch_xbar_ranks(c->dtype, m, c->halo, c->ld, (int32_t)c->nchs, nullptr, c->send, c->stream));
  if (c->lg_side) {  // the first exchange, issued on the side stream, follows the send rows written here
    HIPOK(hipEventRecord(c->lg_side_ev, c->stream));
    HIPOK(hipStreamWaitEvent(c->lg_side, c->lg_side_ev, 0));
  }
  c->lg = 0;
  c->lg_xwait = false;
  return ipc_publish(c);
}

namespace {
// An exchange was just enqueued on the side stream: the next mix / tail waits for it.
int lagged_mark_exchange(dopt_ctx* c) {
  // an event of the context's own (no timing, created once) behind the exchange on the side stream
  if (!c->lg_xev) HIPOK(hipEventCreateWithFlags(&c->lg_xev, kOrderEventFlags));
  HIPOK(hipEventRecord(c->lg_xev, c->lg_side));
  c->lg_xwait = true;
  return DOPT_OK;
}
}  // namespace

// ---- the pull transport (DOPT_TRANSPORT=ipc; round 6).  RCCL's kernel beside the gradient kernel slows it
// by 4-16 % on the rank proxies while a plain copy kernel there costs ~1 % (profiles/r6_xcopy_ab.txt), so
// this transport moves the rows with a copy kernel of the engine's own:
//  * every rank writes the send rows and sums of its record r (r = 1, 2, ...: the chains' begins and mixes,
//    numbered across chains and identical on every rank) into slot (r - 1) % 2 of its own allocation (exported
//    once through an IPC handle), records an interprocess event on the stream that wrote them, and publishes
//    "r events recorded" in host shared memory (ipc_publish);
//  * an exchange for record r waits on the host until every peer has published r (so that the stream wait below
//    refers to that record, not an older one), makes the exchange stream wait for the peers' events, and pulls
//    every block with one k_pull launch from the peers' slot (r - 1) % 2 into this rank's halo (ipc_pull).
// No slot is overwritten while a peer may still read it, by the schedule itself: a rank writes slot (r - 1) % 2
// again for record r + 2, in a mix that waited for its own pulls of record r + 1, which waited for every
// peer's event r + 1 -- recorded after that peer's mix that followed its pulls of record r.  The host wait is
// bounded (timeout_s, the job's collective bound).
namespace {
int ipc_publish(dopt_ctx* c) {
  if (!c->ipc) return DOPT_OK;
  HIPOK(hipEventRecord(c->ipc_ev, c->lg_side ? c->lg_side : c->stream));
  c->ipc_rec += 1;
  __atomic_store_n(c->ipc_cnt + c->lg_rank, c->ipc_rec, __ATOMIC_RELEASE);
  return DOPT_OK;
}

int ipc_pull(dopt_ctx* c) {
  const int64_t need = c->ipc_rec;  // this round's data: every peer's event number `need`
  const auto t0 = std::chrono::steady_clock::now();
  for (int32_t p : c->ipc_peers) {
    int spins = 0;
    while (__atomic_load_n(c->ipc_cnt + p, __ATOMIC_ACQUIRE) < need) {
      if (++spins > 256) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (c->ipc_timeout > 0 && el > c->ipc_timeout)
          return fail(DOPT_ERR_COMM, "rank %d: peer %d published %lld of %lld rounds in %.0f s (a peer stopped?)",
                      c->lg_rank, p, (long long)__atomic_load_n(c->ipc_cnt + p, __ATOMIC_ACQUIRE), (long long)need,
                      c->ipc_timeout);
        std::this_thread::sleep_for(std::chrono::microseconds(spins > 4096 ? 200 : 2));
      }
    }
  }
  hipStream_t xs = c->lg_side ? c->lg_side : c->stream;
  for (hipEvent_t e : c->ipc_pev) HIPOK(hipStreamWaitEvent(xs, e, 0));
  HIPOK(launch_pull(c->ipc_pa, (int)((need - 1) & 1), xs));
  return DOPT_OK;
}
}  // namespace

int dopt_lagged_exchange_issued(dopt_ctx* c, int* ordered) {
  CHECK_ARG(c && ordered, "NULL argument");
  *ordered = 0;
  if (!c->lg_side) return DOPT_OK;  // no side stream: the caller orders the engine stream
  int rc;
  if ((rc = lagged_mark_exchange(c))) return rc;
  *ordered = 1;
  return DOPT_OK;
}

int dopt_lagged_transport(dopt_ctx* c, dopt_comm* comm, const int64_t* send_rows, const int64_t* recv_rows) {
  CHECK_ARG(c, "ctx is NULL");
  c->xp = nullptr;
  c->xp_ops.clear();
  if (!comm) {  // detach either transport
    ipc_close(c);
    return DOPT_OK;
  }
  CHECK_ARG(send_rows && recv_rows, "NULL argument");
  CHECK_ARG(comm_device(comm) == c->device, "communicator on device %d, context on device %d", comm_device(comm),
            c->device);
  const int32_t world = comm_world(comm), rank = comm_rank(comm);
  CHECK_ARG(c->lg_world == world && c->lg_rank == rank,
            "communicator of rank %d of %d, exchange layout of rank %d of %d (dopt_lagged_exchange_layout first)",
            rank, world, c->lg_rank, c->lg_world);
  const int64_t row = c->ld * (int64_t)c->esz;
  int64_t so = 0, ro = 0;
  std::vector<XpOp> ops;
  for (int32_t p = 0; p < world; ++p) {
    CHECK_ARG(send_rows[p] >= 0 && recv_rows[p] >= 0, "peer %d: negative block size", p);
    if (send_rows[p] > 0) ops.push_back(XpOp{so * row, send_rows[p] * row, p, 0});
    if (recv_rows[p] > 0) ops.push_back(XpOp{ro * row, recv_rows[p] * row, p, 1});
    so += send_rows[p];
    ro += recv_rows[p];
  }
  CHECK_ARG(so <= std::max<int64_t>(c->n_send, 0) && ro <= c->n_halo,
            "blocks of %lld send / %lld halo rows past the buffers (%lld / %lld; dopt_set_halo first)", (long long)so,
            (long long)ro, (long long)c->n_send, (long long)c->n_halo);
  CHECK_ARG((so == 0 || c->send) && (ro == 0 || c->halo), "send / halo buffer missing");
  c->xp = comm;
  c->xp_ops = std::move(ops);
  ipc_close(c);
  return DOPT_OK;
}

int dopt_lagged_ipc_export(dopt_ctx* c, uint8_t* mem_handle, uint8_t* event_handle, int64_t* slot_bytes) {
  CHECK_ARG(c && mem_handle && event_handle && slot_bytes, "NULL argument");
  if (!c->have_data) return fail(DOPT_ERR_STATE, "load the shards first");
  int rc;
  if ((rc = set_device(c))) return rc;
  ipc_close(c);
  const int64_t row = c->ld * (int64_t)c->esz;
  const int64_t slot = (std::max<int64_t>(1, c->n_send) * row + 255) / 256 * 256;
  if (c->ipc_send) {
    HIPOK(hipDeviceSynchronize());  // (a previous chain's pulls by peers finished with their runner)
    HIPOK(hipFree(c->ipc_send));
    c->ipc_send = nullptr;
  }
  // uncached: the mix kernels' writes of the send rows go through to memory, where a peer's pull (on another
  // GPU: over xGMI) reads them after the interprocess event, with no dirty line left in this GPU's L2
  HIPOK(hipExtMallocWithFlags((void**)&c->ipc_send, (size_t)(2 * slot), hipDeviceMallocUncached));
  HIPOK(hipMemset(c->ipc_send, 0, (size_t)(2 * slot)));
  if (!c->ipc_ev) HIPOK(hipEventCreateWithFlags(&c->ipc_ev, hipEventInterprocess | hipEventDisableTiming));
  HIPOK(hipIpcGetMemHandle((hipIpcMemHandle_t*)mem_handle, c->ipc_send));
  HIPOK(hipIpcGetEventHandle((hipIpcEventHandle_t*)event_handle, c->ipc_ev));
  c->ipc_slot = slot;
  *slot_bytes = slot;
  return DOPT_OK;
}

int dopt_lagged_ipc_import(dopt_ctx* c, int32_t world, int32_t rank, const uint8_t* mem_handles,
                           const uint8_t* event_handles, const int64_t* slot_bytes, const int64_t* src_off,
                           const int64_t* recv_rows, int64_t* counters, double timeout_s) {
  CHECK_ARG(c && mem_handles && event_handles && slot_bytes && src_off && recv_rows && counters, "NULL argument");
  CHECK_ARG(c->ipc_send, "dopt_lagged_ipc_export first");
  CHECK_ARG(c->lg_world == world && c->lg_rank == rank,
            "pull transport of rank %d of %d, exchange layout of rank %d of %d (dopt_lagged_exchange_layout first)",
            rank, world, c->lg_rank, c->lg_world);
  CHECK_ARG(timeout_s >= 0, "timeout_s must be >= 0 (0: unbounded)");
  int rc;
  if ((rc = set_device(c))) return rc;
  ipc_close(c);
  c->xp = nullptr;
  c->xp_ops.clear();
  const int64_t row = c->ld * (int64_t)c->esz;
  CHECK_ARG(row % 16 == 0, "rows of %lld bytes: the pull copies 16-byte chunks", (long long)row);
  std::vector<const void*> src;
  std::vector<int64_t> off, n16;
  int64_t ro = 0, max16 = 0;
  for (int32_t p = 0; p < world; ++p) {
    CHECK_ARG(recv_rows[p] >= 0 && src_off[p] >= 0 && src_off[p] % 16 == 0, "peer %d: bad block", p);
    if (recv_rows[p] == 0) continue;
    const int64_t bytes = recv_rows[p] * row;
    CHECK_ARG(src_off[p] + bytes <= slot_bytes[p], "peer %d: block past its send slot (%lld + %lld > %lld bytes)", p,
              (long long)src_off[p], (long long)bytes, (long long)slot_bytes[p]);
    const char* base = c->ipc_send;
    if (p != rank) {
      void* q = nullptr;
      hipError_t e = hipIpcOpenMemHandle(&q, *(const hipIpcMemHandle_t*)(mem_handles + (size_t)p * DOPT_IPC_HANDLE_BYTES),
                                         hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess) {
        ipc_close(c);
        return fail(DOPT_ERR_HIP, "rank %d: hipIpcOpenMemHandle of peer %d: %s", rank, p, hipGetErrorString(e));
      }
      c->ipc_open.push_back(q);
      hipEvent_t ev = nullptr;
      e = hipIpcOpenEventHandle(&ev, *(const hipIpcEventHandle_t*)(event_handles + (size_t)p * DOPT_IPC_HANDLE_BYTES));
      if (e != hipSuccess) {
        ipc_close(c);
        return fail(DOPT_ERR_HIP, "rank %d: hipIpcOpenEventHandle of peer %d: %s", rank, p, hipGetErrorString(e));
      }
      c->ipc_pev.push_back(ev);
      c->ipc_peers.push_back(p);
      base = (const char*)q;
    }
    src.push_back(base + src_off[p]);
    src.push_back(base + slot_bytes[p] + src_off[p]);
    off.push_back(ro * row);
    n16.push_back(bytes / 16);
    max16 = std::max(max16, bytes / 16);
    ro += recv_rows[p];
  }
  if (ro > c->n_halo) {
    ipc_close(c);
    return fail(DOPT_ERR_INVALID, "%lld halo rows pulled, the halo holds %lld (dopt_set_halo first)", (long long)ro,
                (long long)c->n_halo);
  }
  const int nb = (int)off.size();
  if (nb > 65535) {
    ipc_close(c);
    return fail(DOPT_ERR_INVALID, "%d peer blocks: at most 65535", nb);
  }
  if ((rc = dalloc_t(&c->ipc_src_d, std::max<size_t>(1, src.size()) * sizeof(void*))) ||
      (rc = dalloc_t(&c->ipc_off_d, std::max<size_t>(1, off.size()) * sizeof(int64_t))) ||
      (rc = dalloc_t(&c->ipc_n16_d, std::max<size_t>(1, n16.size()) * sizeof(int64_t)))) {
    ipc_close(c);
    return rc;
  }
  if (nb > 0) {
    HIPOK(hipMemcpy(c->ipc_src_d, src.data(), src.size() * sizeof(void*), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(c->ipc_off_d, off.data(), off.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(c->ipc_n16_d, n16.data(), n16.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  c->ipc_pa.src = (const void* const*)c->ipc_src_d;
  c->ipc_pa.dst = (char*)c->halo;
  c->ipc_pa.dst_off = c->ipc_off_d;
  c->ipc_pa.n16 = c->ipc_n16_d;
  c->ipc_pa.nb = nb;
  c->ipc_pa.max16 = max16;
  c->ipc_cnt = counters;
  c->ipc_rec = 0;
  c->ipc_timeout = timeout_s;
  c->ipc = true;
  c->send = c->ipc_send;
  return DOPT_OK;
}

int dopt_lagged_ipc_check(dopt_ctx* c, int32_t step) {
  CHECK_ARG(c, "ctx is NULL");
  CHECK_ARG(step == 0 || step == 1, "step 0 (publish) or 1 (pull)");
  if (!c->ipc) return fail(DOPT_ERR_STATE, "no pull transport (dopt_lagged_ipc_import first)");
  int rc;
  if ((rc = set_device(c))) return rc;
  if ((rc = step == 0 ? ipc_publish(c) : ipc_pull(c))) return rc;
  HIPOK(hipStreamSynchronize(c->lg_side ? c->lg_side : c->stream));
  return DOPT_OK;
}

int dopt_lagged_exchange(dopt_ctx* c) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if (c->ipc) {
    if ((rc = ipc_pull(c))) return rc;
    return c->lg_side ? lagged_mark_exchange(c) : DOPT_OK;
  }
  if (!c->xp) return fail(DOPT_ERR_STATE, "no transport (dopt_lagged_transport first)");
  {
    if ((rc = comm_exchange(c->xp, c->xp_ops.data(), c->xp_ops.size(), c->send, c->halo,
                            c->lg_side ? c->lg_side : c->stream)))
      return rc;
  }
  if (!c->lg_side) return DOPT_OK;  // (one stream: ordered by the stream itself)
  rc = lagged_mark_exchange(c);
  return rc;
}

int dopt_lagged_side_stream(dopt_ctx* c, void* stream) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = set_device(c))) return rc;
  if (stream && !c->lg_side_ev)
    HIPOK(hipEventCreateWithFlags(&c->lg_side_ev, kOrderEventFlags));
  c->lg_side = (hipStream_t)stream;
  c->lg_xwait = false;
  return DOPT_OK;
}

int dopt_lagged_grad(dopt_ctx* c, int64_t t, double eta0, int64_t batch, const int32_t* idx, double lam_grad,
                     uint32_t metric_flags) {
  int rc;
  if ((rc = dopt_phase_set_step(c, t, eta0))) return rc;
  return dopt_phase_grad(c, batch, idx, lam_grad, metric_flags);
}

int dopt_lagged_mix(dopt_ctx* c, int64_t t, double eta0, int consensus, double* cons_out, double* xnorm_out,
                    double* loss_out) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = lagged_ready(c))) return rc;
  if (!c->G) return fail(DOPT_ERR_STATE, "gradient phase missing");
  if (c->ipc) c->send = c->ipc_send + (c->ipc_rec & 1) * c->ipc_slot;  // x_{g+1}'s rows and sums: the next record
  RoundArgs a = base_args(c);
  a.x_old = c->xs[c->cur];
  a.x_new = c->xs[c->cur ^ 1];
  a.eta = eta0 / sqrt((double)(t + 1));  // trainer.py:138-140
  a.sptr = c->n_send > 0 ? c->sptr : nullptr;
  a.sslot = c->n_send > 0 ? c->sslot : nullptr;
  a.send = c->send;
  a.xbar_out = c->xbar[c->xb ^ 1];
  if (c->ph_interior) a.interior = c->interior;  // stepped by the gradient kernel already
  c->ph_interior = false;
  a.nchunks = (int32_t)c->nchs;  // k_mixcs walks state chunks
  const int par = (int)(c->lg & 1);
  const McsArgs m = lagged_args(c, c->lg_own[par], c->lg_own[par ^ 1], consensus ? c->lg_cons[par] : nullptr);
  // history[g-2]: the consensus partials of x_{g-1} (the previous mix), the losses at xbar_{g-1} (this
  // round's gradient pass), ||xbar_{g-1}||^2
  const bool any = cons_out || xnorm_out || loss_out;
  FoldArgs f;
  memset(&f, 0, sizeof(f));
  f.sc = c->lg_cons[par ^ 1];
  f.nc = (int64_t)c->lg_ncb * c->n;
  f.sl = c->slab_loss;
  f.nl = c->slab_n[0];
  f.xbar = c->xbar[c->xb];
  f.out_c = cons_out;
  f.out_l = loss_out;
  f.out_q = xnorm_out;
  {
    if ((rc = lagged_xwait(c))) return rc;
  }
  HIPOK(launch_mixcs(c->dtype, a, c->G, (int)c->n, m, any ? &f : nullptr, c->stream, c->lg_side, c->lg_side_ev));
  c->xb ^= 1;
  c->cur ^= 1;
  c->lg += 1;
  c->S_ext = nullptr;
  c->send_fresh = c->n_send > 0;
  return ipc_publish(c);
}

int dopt_lagged_tail(dopt_ctx* c, int consensus, int objective, double* cons1, double* xnorm1, double* loss1,
                     double* cons2, double* xnorm2, double* loss2) {
  CHECK_ARG(c, "ctx is NULL");
  int rc;
  if ((rc = lagged_ready(c))) return rc;
  if ((rc = lagged_xwait(c))) return rc;
  const int par = (int)(c->lg & 1);
  // xbar_G from every rank's sums of x_G (the exchange that preceded this call)
  const McsArgs m = lagged_args(c, c->lg_own[par], nullptr, nullptr);
  HIPOK(launch_xbar_ranks(c->dtype, m, c->halo, c->ld, (int32_t)c->nchs, c->xbar[c->xb ^ 1], nullptr, c->stream));
  c->xb ^= 1;
  if (consensus) {
    HIPOK(launch_cons(c->dtype, c->xs[c->cur], c->xbar[c->xb], c->n, c->ld, (int32_t)c->nchs, c->slab_cons,
                      c->stream));
    c->cons_n = (c->n + 63) / 64;
  }
  const bool two = c->lg >= 2;
  if (objective && (rc = lagged_loss_pass(c, two ? 1 : 0))) return rc;
  // history[G-1]: consensus of x_G, loss at xbar_G (slab B), ||xbar_G||^2
  HIPOK(launch_fold(c->dtype, consensus ? c->slab_cons : nullptr, c->cons_n, objective ? c->slab_loss_b : nullptr,
                    c->slab_n[1], c->xbar[c->xb], c->ld, (int32_t)c->nchs, cons1, loss1, xnorm1, c->stream));
  // history[G-2]: consensus partials of x_{G-1} (the last mix), loss at xbar_{G-1} (slab A), ||xbar_{G-1}||^2
  if (two && (cons2 || xnorm2 || loss2))
    HIPOK(launch_fold(c->dtype, c->lg_cons[par ^ 1], (int64_t)c->lg_ncb * c->n, objective ? c->slab_loss : nullptr,
                      c->slab_n[0], c->xbar[c->xb ^ 1], c->ld, (int32_t)c->nchs, cons2, loss2, xnorm2, c->stream));
  return DOPT_OK;
}

int dopt_sync(dopt_ctx* c) {
  CHECK_ARG(c, "ctx is NULL");
  HIPOK(hipStreamSynchronize(c->stream));
  return DOPT_OK;
}

int dopt_finalize_metrics(int problem, int64_t T, const double* raw, int64_t n_workers, int64_t m_obj,
                          double lam_obj, double f_opt, double* obj_out, double* cons_out) {
  CHECK_ARG(raw && T >= 0 && n_workers >= 1 && m_obj >= 0, "bad arguments");
  finalize_metrics(raw, T, problem, n_workers, m_obj, lam_obj, f_opt, obj_out, cons_out);
  return DOPT_OK;
}

}  // extern "C"
