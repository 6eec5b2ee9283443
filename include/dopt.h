/*
 * dopt.h -- C ABI of libdopt.so, the MI355X (gfx950) engine for the
 * decentralized-SGD round of scavenx/distributed-optimization.
 *
 * The reference is pure Python/numpy and has no FFI of its own; this ABI is
 * what its Python call sites bind to (over ctypes).  Each
 * entry point names the reference code it replaces (file:line in the reference).
 *
 * Conventions
 *   - Every call returns int: DOPT_OK (0) or a negative DOPT_ERR_* code;
 *     dopt_last_error() then returns a message (thread-local, valid until the
 *     next failing call on that thread).
 *   - Host pointers are borrowed for the duration of the call and copied in/out.
 *     All device memory is owned by the context and freed by dopt_destroy().
 *   - One host thread per context; calls are synchronous at return.
 *   - Load the HIP runtime your process already uses first (import torch
 *     before loading libdopt.so when torch is in the process).
 *   - Shards are stored back to back: worker i owns rows
 *     [shard_offsets[i], shard_offsets[i+1]) of X (row-major, n_rows x d) and y.
 *   - Model state is N x d row-major float64 at the boundary; the engine keeps
 *     it on the device in the context's compute dtype.
 */
#ifndef DOPT_H_
#define DOPT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.
 *   1  round 1: contexts, shards, topology / mean mixing, D-SGD and centralized runs, single
 *      evaluations, the legacy-MT19937 sampler, the multi-GPU phase calls.
 *   2  round 2-3 additions: dopt_set_data_dtype / dopt_get_data_dtype (float32 rows under float64
 *      arithmetic), dopt_run_dsgd_pipelined, dopt_zero_models, dopt_set_sampler (device
 *      minibatches), dopt_eval_full, dopt_phase_chain / _colsum_fold / _mix_lagged / _cons /
 *      _fold / _loss_pass (lagged multi-GPU schedule), the dopt_rs_phase_* row-space calls; and
 *      one signature change: dopt_rs_phase_begin reports a 64-bit content hash (was a double
 *      checksum).
 *   3  round 4: the lagged multi-GPU schedule with the column sums in the halo exchange
 *      (dopt_lagged_exchange_layout / _begin / _grad / _mix / _tail) replaces dopt_phase_colsum_fold,
 *      dopt_phase_mix_lagged, dopt_phase_cons and dopt_phase_loss_pass; dopt_set_halo takes send_ids
 *      of -1 (rows that carry no worker); the multi-GPU runner internals form the header's last
 *      section.
 *   4  round 4: dopt_lagged_side_stream (k_mixcs_final and the exchange on a second stream).
 *   5  round 5: dopt_host_digest (threaded content digest of host arrays, the drop-in trainers'
 *      engine cache key), dopt_phase_interior_count; dopt_lagged_exchange_layout accepts a self
 *      block (a rank's own column sums routed through the exchange).
 *   6  round 5: dopt_rs_phase_cols_range (the complete graph's average update per column chunk, so
 *      the next round's pass over a chunk starts while later chunks' sums are still being reduced).
 *   7  round 5: the engine-driven RCCL transport (dopt_comm_*, dopt_lagged_transport,
 *      dopt_lagged_exchange): the lagged schedule's exchange as RCCL sends / receives issued by the
 *      engine on its side stream, without the process group's per-call cost.
 *   8  round 6: dopt_comm_create takes timeout_s -- the communicator is created non-blocking and its
 *      setup, a peer's first connection and its destroy are each bounded by that time.
 *   9  round 6: the pull transport (dopt_lagged_ipc_export / _import): the lagged exchange as a copy
 *      kernel of the engine's reading the peers' send slots through IPC handles, no RCCL kernel. */
#define DOPT_ABI_VERSION 9

typedef struct dopt_ctx dopt_ctx;
typedef struct dopt_comm dopt_comm; /* an RCCL communicator the engine drives itself (ABI 7) */

/* status codes */
#define DOPT_OK 0
#define DOPT_ERR_INVALID (-1)     /* bad argument (maps to ValueError on the Python side) */
#define DOPT_ERR_HIP (-2)         /* HIP runtime failure */
#define DOPT_ERR_STATE (-3)       /* call out of order (no data / topology loaded) */
#define DOPT_ERR_UNSUPPORTED (-4) /* shape outside what this build handles (NotImplementedError) */
#define DOPT_ERR_COMM (-5)        /* RCCL failure */
#define DOPT_ERR_NOMEM (-6)       /* host memory exhausted */
#define DOPT_ERR_RUNTIME (-7)     /* other host failure (e.g. a helper thread that cannot start) */

/* problems: obj_problems.py:3-20 (logistic), obj_problems.py:39-53 (quadratic) */
#define DOPT_LOGISTIC 0
#define DOPT_QUADRATIC 1

/* compute dtypes (the reference computes in float64) */
#define DOPT_F32 0
#define DOPT_F64 1

/* run flags */
#define DOPT_RUN_OBJECTIVE 1u /* record history['objective'] (trainer.py:188-191: X_full given) */
#define DOPT_RUN_CONSENSUS 2u /* record history['consensus_error'] (trainer.py:182-186) */

int dopt_abi_version(void);
const char *dopt_last_error(void);
/* Instance name (rocprofv3's spelling) of the last gradient-round kernel launched in this
 * process -- the fused round kernel or the column-blocked step -- or "" (reports only). */
const char *dopt_last_round_kernel(void);

/* ------------------------------------------------------------------ host only
 * Legacy-MT19937 minibatch sampler: bit-exact with np.random.choice(m, b,
 * replace=False) == RandomState.permutation(m)[:b] as called by
 * Worker.get_mini_batch (worker.py:15-28, the draw at worker.py:27).
 * key/pos are numpy's legacy state (np.random.get_state()[1], [2]) and are
 * advanced in place.  m == 0 draws nothing (worker.py:17-18).
 */
int dopt_mt_choice(uint32_t key[624], int32_t *pos, int64_t m, int64_t b, int64_t *out);

/* T rounds x N workers of Worker.get_mini_batch draws in worker order, as the
 * trainer loops draw them (trainer.py:47-50, trainer.py:166).  out is
 * [T][N][b] int32 local row ids; entries past min(b, m_i) are set to -1. */
int dopt_mt_choice_rounds(uint32_t key[624], int32_t *pos, int64_t T, int64_t n_workers,
                          const int64_t *shard_rows, int64_t b, int32_t *out);

/* The same stream advance without the indices: what T rounds x N workers of
 * Worker.get_mini_batch consume when every draw's result is discarded (full-shard
 * batches: each np.random.choice is a whole permutation of m_i whatever b is,
 * worker.py:27).  Replaces the draws of trainer.py:166 when local_batch_size >= m. */
int dopt_mt_advance_rounds(uint32_t key[624], int32_t *pos, int64_t T, int64_t n_workers,
                           const int64_t *shard_rows);

/* Content digest (128 bits) of n_arrays host buffers -- ptrs[k] / bytes[k], in order -- hashed in
 * 4 MiB chunks on `threads` threads (<= 0: min(16, this process's CPUs / LOCAL_WORLD_SIZE)).  The
 * drop-in trainers key their resident engine on it (trainer._fingerprint: the Worker.X_local /
 * y_local arrays of worker.py:7-8, compared by content on every run). */
int dopt_host_digest(int32_t n_arrays, const void *const *ptrs, const int64_t *bytes, int32_t threads,
                     uint64_t out[2]);

/* ------------------------------------------------------------------ device */
int dopt_device_count(int *count);

/* Replaces the state the reference keeps in Python objects (Worker.x,
 * Trainer.W ...): one context per GPU. */
int dopt_create(int device, int dtype, dopt_ctx **out);
int dopt_destroy(dopt_ctx *ctx);

/* Storage type of the shard rows (Worker.X_local / y_local, worker.py:7-8) on the device.
 * Default: the compute dtype.  With compute dtype DOPT_F64, DOPT_F32 stores the rows as
 * float32 while the iterates, every product, sum and transcendental stay float64
 * (trainer.py:161-193 evaluated as the reference evaluates it): rows are widened exactly
 * to float64 as they are loaded, so on data that is exactly float32-representable the
 * round is the reference's float64 round at half the HBM bytes per row.  Other values
 * are rounded to float32 on upload (the drop-in trainers only choose DOPT_F32 storage
 * when that rounding is the identity).  Every path reads such rows: the fused round kernel,
 * the column-blocked kernels and the row-space rounds (rows beyond 2048 elements).
 * Call before loading / generating the shards; it drops the loaded data. */
int dopt_set_data_dtype(dopt_ctx *ctx, int data_dtype);
int dopt_get_data_dtype(dopt_ctx *ctx, int *data_dtype);

/* Load the worker shards (utils.py:38-43 layout, Worker.X_local / y_local,
 * worker.py:7-10).  X is n_rows x d float64 (src_f32 = 0) or float32
 * (src_f32 = 1), host memory.  problem: DOPT_LOGISTIC / DOPT_QUADRATIC. */
int dopt_load_shards(dopt_ctx *ctx, int problem, int64_t n_workers, int64_t d,
                     const int64_t *shard_offsets, const void *X, const void *y, int src_f32);

/* Synthetic shards generated on the device (BASELINE.json config C3 shape):
 * X ~ N(0,1) with a ones bias column (utils.py:28), y from a planted w* --
 * logistic: sign(X w*) with a fraction `flip` of labels flipped; quadratic:
 * X w* + noise * N(0,1).  Every worker gets `rows_per_worker` rows.  Values are a
 * function of the GLOBAL row id, so a rank generating workers
 * [first_worker, first_worker + n_workers) gets exactly those rows of the
 * single-GPU data set. */
int dopt_generate_shards(dopt_ctx *ctx, int problem, int64_t n_workers, int64_t d,
                         int64_t rows_per_worker, uint64_t seed, double flip, double noise,
                         int64_t first_worker);

/* Objective dataset when it is NOT the union of the shards (the X_full /
 * y_full arguments of Trainer.run, trainer.py:154,188-189).  Without this
 * call the objective is taken over the shard rows. */
int dopt_load_objective_data(dopt_ctx *ctx, int64_t n_rows, const void *X,
                             const void *y, int src_f32);

/* Drop the separate objective dataset: the objective is again taken over the
 * shard rows (X_full == the union of the shards, the Simulator case). */
int dopt_clear_objective_data(dopt_ctx *ctx);

/* Copy worker i's shard back to the host in float64 (n_rows = shard size,
 * X_out[n_rows x d], y_out[n_rows]); used by parity checks at full size. */
int dopt_get_shard(dopt_ctx *ctx, int64_t worker, double *X_out, double *y_out);

/* Mixing matrix in CSR, diagonal included, float64 weights as the reference
 * computes them (trainer.py:91-136, Metropolis-Hastings).  row_ptr[N+1],
 * col[nnz] ascending per row, w[nnz]. */
int dopt_set_topology(dopt_ctx *ctx, int64_t n_workers, const int64_t *row_ptr,
                      const int32_t *col, const double *w);

/* Complete graph (topology 'fully_connected', trainer.py:109-110) without the N^2
 * CSR: every off-diagonal weight equals w_off (MH: 1/N), so
 * sum_j W_ij x_j = w_off * (S - x_i) + W_ii x_i with S the column sums of the
 * iterates -- one all-reduce instead of N neighbour rows.  w_diag[N] = W_ii. */
int dopt_set_mixing_mean(dopt_ctx *ctx, int64_t n_workers, double w_off, const double *w_diag);

/* Worker iterates (Worker.x, worker.py:13; trainer.py:162-163, :178-179). */
int dopt_set_models(dopt_ctx *ctx, const double *x);
int dopt_get_models(dopt_ctx *ctx, double *x);
/* Every iterate = 0 (Worker.x, worker.py:13), enqueued on the context's stream (no host copy). */
int dopt_zero_models(dopt_ctx *ctx);
/* The shared iterate of the centralized trainer (trainer.py:11). */
int dopt_set_global(dopt_ctx *ctx, const double *x);
int dopt_get_global(dopt_ctx *ctx, double *x);

/* Minibatch sampling for dopt_run_dsgd calls with idx == NULL and batch < shard size.
 * DOPT_SAMPLE_HOST (default): such calls are rejected -- parity mode draws the reference's
 * legacy MT19937 stream on the host (dopt_mt_choice_rounds) and passes idx.
 * DOPT_SAMPLE_DEVICE: the throughput mode of SURVEY section 7 (not the reference's
 * stream): worker i's minibatch in round t is a uniform subset of its shard drawn on the
 * device by Floyd's algorithm from Philox4x32-10(key = seed, counter = (k / 4, first_worker
 * + i, t)), inside the pass over all shard rows (shards of at most DOPT_MAX_BIP_ROWS rows;
 * D-SGD rounds; the phase API takes t from dopt_phase_set_round). */
#define DOPT_SAMPLE_HOST 0
#define DOPT_SAMPLE_DEVICE 1
int dopt_set_sampler(dopt_ctx *ctx, int mode, uint64_t seed, int64_t first_worker);

/* T rounds of DecentralizedTrainer.run (trainer.py:161-193), rounds t0..t0+T-1:
 *   g_i = grad f_i(x_i; minibatch)   (worker.py:30-44, obj_problems.py)
 *   x_i <- sum_j W_ij x_j - eta0/sqrt(t+1) * g_i   (trainer.py:173-175)
 *   history[t] = (objective(xbar) - f_opt, mean_i ||x_i - xbar||^2)
 * idx: [T][N][batch] local row ids from dopt_mt_choice_rounds, or NULL when
 * every worker uses its full shard (batch >= every shard size).
 * lam_grad: l2_regularization_lambda (logistic) / strong_convexity_mu
 * (quadratic) (worker.py:36-42); lam_obj: l2_regularization_lambda for both
 * (trainer.py:151-152, :189).  obj_out/cons_out/time_out: [T] or NULL. */
int dopt_run_dsgd(dopt_ctx *ctx, int64_t t0, int64_t T, double eta0, int64_t batch,
                  const int32_t *idx, double lam_grad, double lam_obj, double f_opt,
                  uint32_t flags, double *obj_out, double *cons_out, double *time_out);

/* dopt_run_dsgd with the metrics PIPELINED across calls (steady-state throughput runs;
 * bench.py): with full-shard (or in-pass minibatch) rounds the metrics of round t ride
 * round t+1's pass over the shards, and the metrics of a call's last iterate -- the only
 * ones that would need a pass of their own -- are owed to the next pipelined call on this
 * context, whose first pass computes them (entry 0 of its output).  So every pass is a
 * fused round and each round's metrics are still computed exactly once.  *n_out = the
 * entries written: T - 1 (nothing owed before) or T (owed metrics taken in); T = 0 with
 * metrics owed computes them alone (1 entry).  Any other run, dopt_set_models or new data
 * drops an owed entry; the column-blocked path runs as dopt_run_dsgd.  obj_out / cons_out:
 * [T + 1] or NULL; time_out: [T] (the end of each of this call's rounds) or NULL. */
int dopt_run_dsgd_pipelined(dopt_ctx *ctx, int64_t t0, int64_t T, double eta0, int64_t batch,
                            const int32_t *idx, double lam_grad, double lam_obj, double f_opt,
                            uint32_t flags, double *obj_out, double *cons_out, double *time_out,
                            int64_t *n_out);

/* T rounds of CentralizedTrainer.run (trainer.py:41-71): every worker's
 * gradient at the shared iterate, their mean, one step; objective at the
 * shared iterate.  Same argument meaning as dopt_run_dsgd. */
int dopt_run_centralized(dopt_ctx *ctx, int64_t t0, int64_t T, double eta0,
                         int64_t batch, const int32_t *idx, double lam_grad, double lam_obj,
                         double f_opt, uint32_t flags, double *obj_out, double *time_out);

/* Single evaluations on the device in float64 (the obj_problems.py API):
 * stochastic gradient over b rows (obj_problems.py:13-20 / :46-53) and the
 * objective over n rows (obj_problems.py:3-11 / :39-44). */
int dopt_eval_gradient(dopt_ctx *ctx, int problem, int64_t b, int64_t d,
                       const double *w, const double *X, const double *y, double reg,
                       double *g_out);
int dopt_eval_objective(dopt_ctx *ctx, int problem, int64_t n, int64_t d,
                        const double *w, const double *X, const double *y, double reg,
                        double *out);

int dopt_sync(dopt_ctx *ctx);
/* Host: raw[T x 3] (summed over ranks) -> history values, the exact formula
 * the single-GPU path applies. */
int dopt_finalize_metrics(int problem, int64_t T, const double *raw, int64_t n_workers,
                          int64_t m_obj, double lam_obj, double f_opt, double *obj_out,
                          double *cons_out);

/* Full-data objective and gradient at w over every loaded row (or the separate
 * objective dataset): f = mean loss + reg/2 ||w||^2 (obj_problems.py:3-11 /
 * :39-44), g = mean_k c_k x_k + reg w (the full-gradient shape of
 * obj_problems.py:22-36 / :55-69).  One pass over the data; the building block
 * of the device f(x*) solver (solver.py) that replaces sklearn's saga at sizes
 * sklearn cannot handle (simulator.py:32-69).  g_out may be NULL (objective only);
 * column-blocked contexts (rows beyond the row-resident kernel) evaluate the objective only,
 * with the direct kernels' dots pass (g_out must be NULL there). */
int dopt_eval_full(dopt_ctx *ctx, const double *w, double reg, double *f_out, double *g_out);

/* Device time of the dominant kernel (the fused round kernel) since the last call:
 * sampled launches and their summed milliseconds, measured with HIP events on the
 * engine's stream.  Used by bench.py for the roofline figure.
 * dopt_set_profiling: 0 = off; k >= 1 = bracket every k-th launch with an event pair
 * (a pair costs ~30 us of round time on MI355X, so bench.py samples). */
int dopt_kernel_stats(dopt_ctx *ctx, int64_t *launches, double *total_ms);
int dopt_set_profiling(dopt_ctx *ctx, int enable);

/* ------------------------------------------------------------------ multi-GPU runner internals
 * Not a user API: the calls distributed.py (DistributedDSGD / DistributedCentralized) makes to drive
 * one rank's context through the round phases.  A user runs several GPUs through the drop-in
 * trainers under torchrun and never calls these.
 * One process per GPU, each context holding a contiguous slice of the workers.
 * The round of trainer.py:161-193 is split into enqueue-only phases on the
 * context's stream, so the caller can interleave the collectives
 * (torch.distributed over RCCL, or gloo in tests) between them:
 *   gather -> [halo send/recv of x_t rows] || grad(x_t) -> metrics(prev)
 *          -> mix -> colsum -> [all-reduce of d doubles] -> xbar
 * Device pointers (halo, send, sum, out) are caller-owned device memory. */

/* Launch on `stream` (a hipStream_t, e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream. */
int dopt_set_stream(dopt_ctx *ctx, void *stream);
/* Row stride (elements) and element size of the device rows (halo / send buffers). */
int dopt_get_layout(dopt_ctx *ctx, int64_t *ld, int64_t *elem_bytes);
/* Global worker and row counts: divisors of xbar (trainer.py:182), the
 * consensus mean (:185) and the objective mean (obj_problems.py:6/:42). */
int dopt_set_partition(dopt_ctx *ctx, int64_t n_global, int64_t rows_global);
/* Halo plan: CSR columns >= n_local address halo rows [n_halo x ld]; rows
 * send_ids[n_send] (local ids) are gathered into send [n_send x ld].  Call
 * before dopt_set_topology (the local CSR indexes local + halo rows). */
int dopt_set_halo(dopt_ctx *ctx, int64_t n_halo, void *halo_dev, int64_t n_send, void *send_dev,
                  const int32_t *send_ids);
/* Pipelined multi-GPU runs (distributed.py DistributedDSGD.run_pipelined): *was_pending =
 * whether the previous pipelined phase run on this context left its lagged schedule open
 * (nothing else -- dopt_set_models, new data, any other run, dopt_phase_begin -- has
 * touched the context since); then the mark is set (mark = 1: this run leaves it open) or
 * cleared. */
int dopt_phase_chain(dopt_ctx *ctx, int mark, int *was_pending);
/* Workers of this rank's slice that dopt_phase_grad / dopt_lagged_grad mix and step itself (no halo
 * column in their CSR row, no peer reading their row), as set by dopt_set_topology after
 * dopt_set_halo; 0 without a halo plan or with column-sum mixing. */
int dopt_phase_interior_count(dopt_ctx *ctx, int64_t *n_interior);
/* Start of a run of phases: column-blocked contexts (large d) compute the
 * coefficients of the starting iterates here (full-shard batches). */
int dopt_phase_begin(dopt_ctx *ctx, int64_t batch);
/* Round index t (trainer.py:138) of the next dopt_phase_grad: the counter of the device
 * sampler (dopt_set_sampler), so every rank draws worker i's minibatch of round t alike. */
int dopt_phase_set_round(dopt_ctx *ctx, int64_t t);
/* dopt_phase_set_round plus the round's step size eta0 / sqrt(t + 1) (trainer.py:138-140): the
 * next dopt_phase_grad then also mixes and steps the workers whose CSR row needs no halo row and
 * who send no row (rank slices), and the next mix skips them -- the same arithmetic as the fused
 * round, one pass less over their iterates (round 3; ABI version 2 addition). */
int dopt_phase_set_step(dopt_ctx *ctx, int64_t t, double eta0);
/* Rows send_ids of the current iterates -> send.  A no-op when the last dopt_phase_mix
 * already wrote them (the mix kernel refreshes the send rows as it writes the iterates). */
int dopt_phase_gather(dopt_ctx *ctx);
/* Gradients of every local worker at its current iterate (worker.py:30-44);
 * metric_flags (DOPT_RUN_*) also accumulate the current iterate's metric
 * partials at the current xbar from the same pass over every shard row (full-shard
 * batches, or minibatches when every shard has at most DOPT_MAX_BIP_ROWS rows: the
 * minibatch rows then feed the gradient inside that pass). */
#define DOPT_MAX_BIP_ROWS 65536
int dopt_phase_grad(dopt_ctx *ctx, int64_t batch, const int32_t *idx, double lam_grad,
                    uint32_t metric_flags);
/* x_{t+1} = W [x_t | halo] - eta0/sqrt(t+1) g  (trainer.py:173-175), and the send rows
 * of x_{t+1}.  Column-blocked contexts compute the gradient here, block by block, in the
 * same pass (and leave the send rows to dopt_phase_gather). */
int dopt_phase_mix(dopt_ctx *ctx, int64_t t, double eta0);
/* Local column sums of the current iterates -> sum_dev[ld] (float64). */
int dopt_phase_colsum(dopt_ctx *ctx, double *sum_dev);
/* xbar = sum_dev / n_global. */
int dopt_phase_xbar(dopt_ctx *ctx, const double *sum_dev);
/* Metrics-only pass over the local shard rows at the current xbar. */
int dopt_phase_metrics_pass(dopt_ctx *ctx, uint32_t flags);
/* Raw sums -> out_dev[3] = (sum of consensus partials, sum of loss terms,
 * ||xbar||^2 if include_xnorm else 0). */
int dopt_phase_metrics(dopt_ctx *ctx, uint32_t flags, int include_xnorm, double *out_dev);
/* dopt_phase_fold: *cons_out = the sum of the consensus slab, *xnorm_out = ||xbar||^2, *loss_out =
 *   sum of loss slab `slab` (slab 0: the last pass with DOPT_RUN_OBJECTIVE; slab 1: unused outside
 *   the lagged tail); NULL outputs are skipped (the row-space rounds' history rows). */
int dopt_phase_fold(dopt_ctx *ctx, double *cons_out, double *xnorm_out, double *loss_out, int slab);
/* Row-space rounds on a rank's slice (complete graph with one W_ii, quadratic, full shards of
 * 1..64 rows) -- replace the serial phase order of DistributedDSGD for that case
 * (trainer.py:161-193 with the mix of trainer.py:173 through the all-reduced column sums):
 * dopt_rs_phase_begin: *ok = 1 when this rank's iterates are all equal (or the row-space state
 *   is live already), *hash = a 64-bit content hash of that common iterate's bytes (of the
 *   replicated Z and average when the state is live; the caller compares it across ranks);
 *   commit = 1 also enters row-space mode (Gram matrices, Z = xbar = the iterate).
 * dopt_rs_phase_round: round t's pass at the current average: the next row state, the metric
 *   partials of the current iterates (metric_flags, folded by dopt_phase_fold slab 0) and this
 *   rank's column sums into sum_dev[ld] (to be all-reduced).
 * dopt_rs_phase_cols: the average / Z update of round t from the all-reduced sums.
 * dopt_rs_phase_metrics: the metric partials of the current iterates (a dots pass).
 * dopt_get_models forms the iterates; dopt_phase_begin, dopt_phase_colsum / _fold / _gather,
 * dopt_set_models, dopt_set_mixing_mean and dopt_set_topology leave row-space mode. */
int dopt_rs_phase_begin(dopt_ctx *ctx, int commit, int *ok, uint64_t *hash);
int dopt_rs_phase_round(dopt_ctx *ctx, int64_t t, double eta0, double lam_grad, uint32_t metric_flags,
                        double *sum_dev);
int dopt_rs_phase_cols(dopt_ctx *ctx, int64_t t, double eta0, double lam_grad, const double *sum_dev);
/* The same round with the pass split into column chunks, so the caller can all-reduce chunk k's
 * sums while chunk k + 1 streams (distributed.py, the complete-graph average across ranks):
 * dopt_rs_phase_pass: the pass over column chunk `chunk` of `n_chunks` (contiguous column
 *   blocks) at the current average; this rank's column sums of those columns -> sum_dev[c0:c1),
 *   col_range[2] = {c0, c1} (empty when there are more chunks than column blocks).
 * dopt_rs_phase_rows: after every chunk's pass, round t's next row state and (metric_flags) the
 *   metric partials of the current iterates; then dopt_rs_phase_cols with the reduced sums. */
int dopt_rs_phase_pass(dopt_ctx *ctx, int32_t chunk, int32_t n_chunks, double *sum_dev, int64_t *col_range);
int dopt_rs_phase_rows(dopt_ctx *ctx, int64_t t, double eta0, double lam_grad, uint32_t metric_flags);
/* dopt_rs_phase_cols_range: dopt_rs_phase_cols for the columns [c0, c1) of one dopt_rs_phase_pass chunk
 *   (sum_dev[c0:c1) reduced), so round t + 1's pass over that chunk may run before the later chunks'
 *   sums arrive: until the call with last = 1 the update is open, dopt_rs_phase_pass reads the updated
 *   chunks' new average, and every other dopt_rs_phase_* call (and leaving row-space mode) fails with
 *   DOPT_ERR_STATE.  Each chunk once per round, in any order; the round's metrics (dopt_rs_phase_rows)
 *   after the last. */
int dopt_rs_phase_cols_range(dopt_ctx *ctx, int64_t t, double eta0, double lam_grad, const double *sum_dev,
                             int64_t c0, int64_t c1, int32_t last);
int dopt_rs_phase_metrics(dopt_ctx *ctx, uint32_t metric_flags);
/* The lagged schedule (round 4, ABI version 3; distributed.py DistributedDSGD._run_lagged): one
 * collective per round -- the halo rows of x_g AND every rank's column sums of x_g in one exchange
 * (an all-to-all-v: the send / halo buffers hold, per peer in rank order, that peer's rows then
 * 8 ld bytes of float64 sums) -- and three launches per round (gradient, k_mixcs, k_mixcs_final):
 *   exchange(x_g rows + sums) ----------------------------------------------.
 *   dopt_lagged_grad: gradient pass of x_g (+ loss of every row at xbar_{g-1}) +--> dopt_lagged_mix
 * dopt_lagged_exchange_layout: the send-buffer row where the sums for peer p go and the halo-buffer
 *   row where peer p's sums arrive, p = 0 .. world-1 (-1 for p == rank, or -- a self block, the
 *   one-GPU rehearsal of the RCCL path at world 1 -- rows for the rank's own sums, which the mix then
 *   reads back from the halo buffer); after dopt_set_halo, whose send_ids are -1 on those rows.
 * dopt_lagged_begin: dopt_phase_begin + the send rows and this rank's column sums of x_0.
 * dopt_lagged_grad: dopt_phase_set_step + dopt_phase_grad (replaces the worker loop of
 *   trainer.py:164-170; interior workers mixed and stepped too).
 * dopt_lagged_mix: xbar_g = (sum over ranks p in rank order of p's column sums of x_g) / n_global
 *   (trainer.py:182), the consensus partials of x_g (trainer.py:183-186, with consensus), x_{g+1} =
 *   W [x_g | halo] - eta g (trainer.py:173-175) and its send rows, this rank's column sums of
 *   x_{g+1} into the send buffer's sum rows, and into the non-NULL outputs the history row g-2
 *   (consensus partials of x_{g-1}, the losses of the preceding dopt_lagged_grad, ||xbar_{g-1}||^2).
 * dopt_lagged_tail: after one more exchange: xbar_G, and the history rows G-1 (cons1 / xnorm1 /
 *   loss1) and G-2 (cons2 / xnorm2 / loss2) of a chain of G rounds.
 * dopt_lagged_side_stream: a second stream (NULL: none) for the column-sum totals of each mix
 *   (k_mixcs_final, after an event wait on the engine stream) and for the caller's exchange, so the
 *   next gradient kernel does not wait for them; dopt_lagged_begin makes it wait for x_0's send rows.
 *   The caller issues the exchange on it and makes the engine stream wait for the exchange (RCCL:
 *   work.wait() on the engine stream; host transports: a stream wait on the side stream). */
int dopt_lagged_exchange_layout(dopt_ctx *ctx, int32_t world, int32_t rank, const int64_t *sum_send_row,
                                const int64_t *sum_recv_row);
int dopt_lagged_begin(dopt_ctx *ctx, int64_t batch);
int dopt_lagged_grad(dopt_ctx *ctx, int64_t t, double eta0, int64_t batch, const int32_t *idx, double lam_grad,
                     uint32_t metric_flags);
int dopt_lagged_mix(dopt_ctx *ctx, int64_t t, double eta0, int consensus, double *cons_out, double *xnorm_out,
                    double *loss_out);
int dopt_lagged_tail(dopt_ctx *ctx, int consensus, int objective, double *cons1, double *xnorm1, double *loss1,
                     double *cons2, double *xnorm2, double *loss2);
int dopt_lagged_side_stream(dopt_ctx *ctx, void *stream);
/* Right after the caller has enqueued a round's exchange ON the side stream (a transport of its own that
 * runs on the stream it is issued on, or a host transport's halo copy): the context records an event
 * behind it on the side stream and the next dopt_lagged_mix / _tail makes the engine stream wait for it --
 * *ordered = 1, the caller does not order the engine stream itself.  *ordered = 0 without a side stream
 * (the caller orders it). */
int dopt_lagged_exchange_issued(dopt_ctx *ctx, int *ordered);
/* Engine-driven RCCL transport (ABI 7; csrc/transport.cpp).  It replaces, for the lagged schedule's
 * per-round exchange, the caller's process-group all-to-all-v (torch.distributed all_to_all_single in
 * distributed.py HaloExchange: ~22 us of host time per call, 36-40 us with its wait, against 4.5-6 us for
 * RCCL's own group of sends and receives -- profiles/r5_rccl_probe.txt).
 * dopt_comm_unique_id: rank 0's RCCL unique id (DOPT_COMM_ID_BYTES bytes), which the caller hands to every
 *   rank (the job's existing process group broadcasts it).
 * dopt_comm_create: RCCL communicator of rank `rank` of `world` on `device`; collective -- every rank
 *   calls it with the same id.  Created non-blocking (ncclCommInitRankConfig, blocking = 0) and waited
 *   for at most timeout_s seconds (0: unbounded): a rank that never joins ends the others' call with
 *   DOPT_ERR_COMM, the half-built communicator aborted, instead of a hang.  The same bound applies to an
 *   exchange's first connection to a peer and to dopt_comm_destroy's finalize.
 *   dopt_comm_destroy (abort = 1: without waiting for pending work, after a peer failed);
 *   dopt_comm_check: DOPT_ERR_COMM if RCCL reported an asynchronous error.
 * dopt_comm_library: the path of the RCCL library in use (the process's copy when one is loaded).
 * dopt_lagged_transport: route the context's exchange through comm (NULL: detach, the pull transport's
 *   too): per peer p in rank
 *   order, send_rows[p] rows of the send buffer go to p and recv_rows[p] rows of the halo buffer come
 *   from p (the blocks of the all-to-all-v layout; the rank's own block at world 1 with a self block);
 *   after dopt_set_halo and dopt_lagged_exchange_layout, whose rank and world must match comm's.
 * dopt_lagged_exchange: the round's exchange as one RCCL group on the side stream (the engine stream
 *   without one), ordered before the next dopt_lagged_mix / _tail as dopt_lagged_exchange_issued orders
 *   the caller's; where the caller would have issued its all-to-all.
 * A context keeps the communicator it was given: destroy a communicator only after the contexts using it
 * are closed or detached (dopt_lagged_transport(ctx, NULL, ...)) and their streams are idle. */
#define DOPT_COMM_ID_BYTES 128
int dopt_comm_unique_id(uint8_t *id_out, int64_t n);
int dopt_comm_create(dopt_comm **out, int32_t world, int32_t rank, int32_t device, const uint8_t *id, int64_t n,
                     double timeout_s);
int dopt_comm_check(dopt_comm *comm);
int dopt_comm_destroy(dopt_comm *comm, int32_t abort);
const char *dopt_comm_library(void);
int dopt_lagged_transport(dopt_ctx *ctx, dopt_comm *comm, const int64_t *send_rows, const int64_t *recv_rows);
int dopt_lagged_exchange(dopt_ctx *ctx);
/* Pull transport (ABI 9): the same exchange without RCCL, for ranks of one node.  Replaces, like
 * dopt_lagged_transport, the neighbour reads of the reference's mix (trainer.py:173) across ranks.
 * dopt_lagged_ipc_export: after dopt_set_halo -- the context keeps its send rows in two slots (round
 *   parity) of an allocation of its own instead of the caller's send buffer; returns that allocation's IPC
 *   handle, an interprocess event's handle (DOPT_IPC_HANDLE_BYTES each) and the bytes of one slot.
 * dopt_lagged_ipc_import: after every rank exported and dopt_lagged_exchange_layout: per rank p (rank order,
 *   world entries of each array), p's two handles and slot bytes, the byte offset in p's slot of the block
 *   p sends to this rank and recv_rows[p] rows that block holds (this rank's own entry: its self block,
 *   if any).  counters: world int64 in host memory shared by the ranks (zeroed), where each rank publishes
 *   how many rounds of send rows it has recorded; a rank waits at most timeout_s (0: unbounded) for a peer's
 *   round before DOPT_ERR_COMM.  Detaches an RCCL transport; dopt_lagged_transport or dopt_set_halo
 *   detaches this one.  dopt_lagged_exchange then pulls every block with one copy kernel on the side stream
 *   (the engine stream without one), ordered before the next dopt_lagged_mix / _tail.
 * dopt_lagged_ipc_check: the transport tried once before any round, in two collective steps with the
 *   caller's agreement between them -- step 0 publishes a record (the slots' current content), step 1 pulls
 *   every peer's; each waits for its stream.  A failure in either (an IPC event the runtime cannot wait on,
 *   a peer's memory it cannot read) lets every rank choose another transport before the first round. */
#define DOPT_IPC_HANDLE_BYTES 64
int dopt_lagged_ipc_export(dopt_ctx *ctx, uint8_t *mem_handle, uint8_t *event_handle, int64_t *slot_bytes);
int dopt_lagged_ipc_import(dopt_ctx *ctx, int32_t world, int32_t rank, const uint8_t *mem_handles,
                           const uint8_t *event_handles, const int64_t *slot_bytes, const int64_t *src_off,
                           const int64_t *recv_rows, int64_t *counters, double timeout_s);
int dopt_lagged_ipc_check(dopt_ctx *ctx, int32_t step);
/* Centralized trainer across ranks (trainer.py:41-71): gradients of the local
 * workers at the shared iterate (fuse_loss: the objective partial of the shared
 * iterate over the same rows, full shards only), local column sums of the
 * gradients, then x <- x - eta0/sqrt(t+1) * sum_dev / n_global once the sums
 * are all-reduced. */
int dopt_phase_grad_shared(dopt_ctx *ctx, int64_t batch, const int32_t *idx, double lam_grad,
                           int fuse_loss);
int dopt_phase_colsum_grad(dopt_ctx *ctx, double *sum_dev);
int dopt_phase_central_step(dopt_ctx *ctx, const double *sum_dev, int64_t t, double eta0);
/* Objective partial at the shared iterate over the local rows, and its raw sums
 * out_dev[3] = (0, sum of loss terms, ||x||^2 if include_xnorm). */
int dopt_phase_metrics_pass_shared(dopt_ctx *ctx);
int dopt_phase_metrics_shared(dopt_ctx *ctx, int include_xnorm, double *out_dev);
#ifdef __cplusplus
}
#endif

#endif /* DOPT_H_ */
