"""Trainers (drop-in for trainer.py): the round loop runs on the GPU.

CentralizedTrainer   trainer.py:7-74     parameter-server mini-batch SGD
DecentralizedTrainer trainer.py:76-197   D-SGD with Metropolis-Hastings mixing

Same constructor signatures, attributes (workers, W, adj, degrees, topology,
history, total_floats_transmitted, x_global), prints, errors and return values
as the reference.  What changes is underneath `run`: instead of a Python loop
over workers per round, the shards live in HBM and every round is one fused
HIP launch (gradient + mix + step, with the metrics of the previous round folded
into the same pass over the data), driven through libdopt.so.

Config keys beyond the reference's (all optional):
  dtype      'float64' (default, trajectory parity) or 'float32' (throughput)
  device     GPU ordinal (default: $LOCAL_RANK or $DOPT_DEVICE or 0)
  sampling   'legacy' (default): minibatch indices are the exact numpy legacy
             RNG stream (np.random.choice per worker per round, worker.py:27);
             'full': with full-shard batches skip the RNG entirely;
             'device': D-SGD minibatches drawn on the GPU (Philox + Floyd, seed
             'sampling_seed', default 0) inside the pass over every shard row -- the
             throughput mode, NOT the reference's stream (numpy's RNG is not advanced)
  regular_degree / topology_seed   for topology='random_regular'
  spectral_gap   force / skip the spectral-gap print (default: N <= 4096)
  mean_mixing_min  complete graphs of at least this many workers mix through the
                 column sums (default 128)
  distributed    False disables the multi-process mode below

Multi-process mode: when torch.distributed is initialised with more than one rank
(e.g. `python -m torch.distributed.run --nproc-per-node 8 main.py`), every rank
keeps all Worker objects (same data, same RNG stream) but loads only its
contiguous slice of workers onto its own GPU; the rounds run through
distributed.DistributedDSGD / DistributedCentralized (halo send/recv and
all-reduces over RCCL) and every rank ends with the same history and iterates.
"""
import os
import time
from contextlib import closing

import numpy as np

import _dopt
import topology as _topology
from obj_problems import logistic_objective, quadratic_objective

DENSE_LIMIT = 4096          # dense adj / W attributes up to this many workers
MEAN_MIX_MIN = 128          # complete graphs from this size mix through the column sums
ROW_RESIDENT_MAX = 2048     # longer float64 rows take the column-blocked rounds (complete graphs: the
                            # row-space rounds, DESIGN.md 6c, which mix through the column sums)
IDX_CHUNK_ELEMS = 1 << 24   # host index buffer per device call (64 MiB of int32)
IDX_CHUNK_ROUNDS = 512      # rounds per device call when indices are drawn (the next chunk's draw
                            # runs on a host thread while the device runs this one)
IDX_CHUNK_DRAWS = 1 << 24   # pipelined D-SGD: draws per chunk (~25 ms of host stream at 1.4 ns; C3: 8 rounds)


# ---------------------------------------------------------------------------- shared helpers
def _dist_info(config):
    """(rank, world, backend) when running under an initialised multi-rank torch.distributed."""
    if not config.get("distributed", True):
        return None
    try:
        import torch.distributed as dist
    except Exception:
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size(), dist.get_backend()
    return None


def _say(msg, config):
    info = _dist_info(config)
    if info is None or info[0] == 0:
        print(msg)


def _warn_nonfinite(history, config):
    """Failure detection: the reference only skips non-finite values
    when plotting (simulator.py:181-183); here a diverged run also says so once."""
    for key in ("objective", "consensus_error"):
        v = np.asarray(history.get(key, []), dtype=np.float64)
        if v.size and not np.all(np.isfinite(v)):
            first = int(np.argmin(np.isfinite(v)))
            _say(f"Warning: non-finite {key} from round {first} on (diverged? lower learning_rate_eta0)", config)


def _device(config):
    """The GPU of this process: config 'device', else DOPT_DEVICE (an explicit override, e.g. every rank
    of a gloo rehearsal on one GPU), else the launcher's LOCAL_RANK, else 0."""
    return int(config.get("device", os.environ.get("DOPT_DEVICE", os.environ.get("LOCAL_RANK", 0))))


def _pack(workers, n_features, f32=False):
    """Shards back to back (utils.py:38-43 order) + row offsets.  f32: pack as float32 (the
    engine stores float32 rows: exact values, or a float32 engine) -- half the host bytes."""
    rows = np.array([w.X_local.shape[0] for w in workers], dtype=np.int64)
    off = np.zeros(len(workers) + 1, dtype=np.int64)
    np.cumsum(rows, out=off[1:])
    dt = np.float32 if f32 else np.float64
    if off[-1] > 0:
        X = np.concatenate([np.asarray(w.X_local, dtype=dt).reshape(-1, n_features) for w in workers])
        y = np.concatenate([np.asarray(w.y_local, dtype=dt).reshape(-1) for w in workers])
    else:
        X, y = np.zeros((0, n_features), dtype=dt), np.zeros(0, dtype=dt)
    return X, y, off


def _all_f32(workers):
    return all(np.asarray(w.X_local).dtype == np.float32 and np.asarray(w.y_local).dtype == np.float32
               for w in workers)


def _full_digest(arrays, algo="xxh3"):
    """Content hash of arrays (dtype, shape and bytes): xxh3_128 (~7 GB/s) or blake2b."""
    if algo == "xxh3":
        import xxhash

        h = xxhash.xxh3_128()
    else:
        import hashlib

        h = hashlib.blake2b(digest_size=16)
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(repr((a.dtype.str, a.shape)).encode())
        if a.size:
            h.update(memoryview(a.reshape(-1).view(np.uint8)))
    return h.hexdigest()


def _hash_algo():
    try:
        import xxhash  # noqa: F401

        return "xxh3"
    except ImportError:  # pragma: no cover - xxhash ships in this image
        return "blake2b"


_FP_CACHE = {}            # identity of a list of arrays -> (sampled digest, full digest): opt-in only
_FP_FULL_BELOW = 64 << 20  # with the sampled key, arrays totalling fewer bytes are still hashed in full
_FP_SAMPLES = 64          # 256-byte pieces per array in the sampled digest


def _sampled_digest(arrays):
    """A digest of 64 evenly spaced 256-byte pieces (and the last bytes) of every array."""
    import hashlib

    h = hashlib.blake2b(digest_size=16)
    for a in arrays:
        h.update(repr((a.dtype.str, a.shape)).encode())
        if not a.size:
            continue
        b = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        n = b.shape[0]
        if n <= _FP_SAMPLES * 256:
            h.update(memoryview(b))
            continue
        starts = np.linspace(0, n - 256, _FP_SAMPLES).astype(np.int64)
        h.update(b[(starts[:, None] + np.arange(256)).reshape(-1)].tobytes())
    return h.hexdigest()


def _content_digest(arrays):
    """Every byte of the arrays (dtype and shape too), hashed natively on several threads
    (dopt_host_digest: C3's 8.6 GB of host shards without one Python thread's ~6 GB/s limit)."""
    import hashlib

    meta = hashlib.blake2b(repr([(a.dtype.str, a.shape) for a in arrays]).encode(), digest_size=8).hexdigest()
    return meta + _dopt.host_digest(arrays)


def _fingerprint(arrays, sampled=False):
    """Content key of arrays, for the engine cache (it compares data by content, not by id(): ids of
    freed arrays are reused by CPython, and shards edited in place keep their ids, trainer.py's
    reference semantics being that every run uses the arrays as they are now).  By default every
    byte is hashed on every call.  sampled=True (trainer config content_key='sampled', an opt-in):
    data of 64 MiB or more is hashed in full the first time a list of arrays is seen, and later calls
    with the same arrays (object ids, buffer addresses, shapes, dtypes, strides) re-hash only 64
    pieces of each array, reusing the full digest while those are unchanged -- an in-place edit
    that touches none of the sampled bytes is then NOT seen (call trainer.forget_data() after one)."""
    arrays = [np.asarray(a) for a in arrays]
    if not sampled or sum(a.nbytes for a in arrays) < _FP_FULL_BELOW:
        return _content_digest(arrays)
    ident = tuple((id(a), a.__array_interface__["data"][0], a.shape, a.dtype.str, a.strides) for a in arrays)
    samp = _sampled_digest(arrays)
    hit = _FP_CACHE.get(ident)
    if hit is not None and hit[0] == samp:
        return hit[1]
    full = _content_digest(arrays)
    if len(_FP_CACHE) >= 16:
        _FP_CACHE.pop(next(iter(_FP_CACHE)))
    _FP_CACHE[ident] = (samp, full)
    return full


def _sampled_key(config):
    """Trainer config content_key: 'full' (default, every byte hashed per run) or 'sampled'."""
    v = (config or {}).get("content_key", "full")
    if v not in ("full", "sampled"):
        raise ValueError(f"content_key must be 'full' or 'sampled', not {v!r}")
    return v == "sampled"


def forget_data():
    """Drop the cached content digests of the opt-in sampled key (after editing large shard arrays
    in place)."""
    _FP_CACHE.clear()


def _f32_exact(arrays):
    """True when every value is exactly representable in float32 (so float32 storage under
    float64 arithmetic changes nothing; dopt_set_data_dtype)."""
    for a in arrays:
        if a is None:
            continue
        a = np.asarray(a)
        if a.dtype == np.float32:
            continue
        a = np.asarray(a, dtype=np.float64)
        if a.size and not np.array_equal(a.astype(np.float32).astype(np.float64), a):
            return False
    return True


def _data_dtype(config, d, arrays):
    """Shard storage: config 'data_dtype' = 'auto' (default: float32 when dtype is float64 and
    every value -- shards and a separate X_full -- is exactly float32; the arithmetic stays
    float64, on every path: fused, column-blocked and row-space rounds), 'float32' or 'float64'."""
    dtype = config.get("dtype", "float64")
    want = config.get("data_dtype", "auto")
    if _dopt.DTYPES[dtype] == _dopt.F32:
        return dtype
    if want == "auto":
        return "float32" if d > 0 and _f32_exact(arrays) else "float64"
    return want


def _same_rows(A, ya, B, yb):
    """True when (A, ya) and (B, yb) hold the same multiset of (row, label) pairs."""
    A, B = np.asarray(A), np.asarray(B)
    if A.dtype != B.dtype or A.dtype.kind != "f":
        A = np.asarray(A, dtype=np.float64)
        B = np.asarray(B, dtype=np.float64)
    ya = np.asarray(ya, dtype=np.float64).reshape(-1)
    yb = np.asarray(yb, dtype=np.float64).reshape(-1)
    if A.shape != B.shape or ya.shape[0] != A.shape[0] or yb.shape[0] != B.shape[0]:
        return False
    if np.array_equal(A, B) and np.array_equal(ya, yb):
        return True
    v = np.random.default_rng(12345).standard_normal(A.shape[1] + 1)
    ha = A @ v[:-1] + ya * v[-1]
    hb = B @ v[:-1] + yb * v[-1]
    oa, ob = np.argsort(ha, kind="stable"), np.argsort(hb, kind="stable")
    return bool(np.array_equal(A[oa], B[ob]) and np.array_equal(ya[oa], yb[ob]))


_ENGINES = {}
_WARNED_CENTRAL_DEVICE = False


def _engine(workers, n_features, config, lo=0, hi=None, X_full=None, y_full=None):
    """One resident engine per (device, dtype), holding one data set: reused by the four
    trainers Simulator.run_all builds over the same worker data.  [lo, hi) is the slice of
    workers this process holds (multi-process mode).  Reuse is decided by CONTENT (a hash
    of every byte of the slice's shards), so freed-and-reallocated or edited-in-place arrays reload
    (with the opt-in content_key='sampled': edits the sample sees)."""
    hi = len(workers) if hi is None else hi
    arrays = [a for w in workers[lo:hi] for a in (w.X_local, w.y_local)]
    dev, dtype = _device(config), config.get("dtype", "float64")
    xdt = _data_dtype(config, n_features, arrays + [X_full, y_full])
    key = (config["problem_type"], xdt, lo, hi, _fingerprint(arrays, _sampled_key(config)))
    eng = _ENGINES.get((dev, dtype))
    if eng is None or eng.data_key != key:
        if eng is not None:
            _ENGINES.pop((dev, dtype)).close()  # free the previous data set's HBM
        eng = _dopt.Engine(dev, dtype, data_dtype=xdt)
        X, y, off = _pack(workers[lo:hi], n_features, f32=eng.data_dtype == _dopt.F32)
        eng.load_shards(config["problem_type"], X, y, off)
        eng.obj_key = None
        eng.data_key = key
        _ENGINES[(dev, dtype)] = eng
    device_sampling = config.get("sampling", "legacy") == "device"
    eng.set_sampler("device" if device_sampling else "host", seed=int(config.get("sampling_seed", 0)), first_worker=lo)
    return eng


def _dist_objective(eng, workers, n_features, X_full, y_full, rank, world, sampled=False):
    """Objective rows for a rank: its own shards when X_full is their union, else its
    array_split slice of X_full.  Returns (want_obj, rows_global, separate)."""
    if X_full is None or y_full is None:
        eng.clear_objective_data()
        eng.obj_key = None
        return False, 1, False
    X, y, _ = _pack(workers, n_features, f32=_all_f32(workers))
    if _same_rows(X_full, y_full, X, y):
        eng.clear_objective_data()
        eng.obj_key = None
        return True, X.shape[0], False
    Xf = np.asarray(X_full, dtype=np.float64).reshape(-1, n_features)
    yf = np.asarray(y_full, dtype=np.float64).reshape(-1)
    parts = np.array_split(np.arange(Xf.shape[0]), world)[rank]
    eng.load_objective_data(Xf[parts], yf[parts])
    eng.obj_key = ("dist", _fingerprint([X_full, y_full], sampled))
    return True, Xf.shape[0], True


def _set_objective_data(eng, workers, n_features, X_full, y_full, sampled=False):
    """trainer.py:188: the objective is recorded only when X_full and y_full are given.
    When they hold exactly the shard rows (the Simulator case) the objective is fused
    into the round's pass over the shards; otherwise X_full is uploaded separately."""
    if X_full is None or y_full is None:
        if eng.obj_key is not None:
            eng.clear_objective_data()
            eng.obj_key = None
        return False
    key = _fingerprint([X_full, y_full], sampled)  # by content: ids are reused once arrays are freed
    if eng.obj_key != key:
        X, y, _ = _pack(workers, n_features, f32=_all_f32(workers))
        if _same_rows(X_full, y_full, X, y):
            eng.clear_objective_data()
        else:
            eng.load_objective_data(np.asarray(X_full).reshape(-1, n_features), y_full)
        eng.obj_key = key
    return True


def _grad_reg(cfg, n_iterations, workers):
    """Gradient regulariser (worker.py:36-42): lambda for logistic, mu for quadratic.  The
    reference's Worker.compute_gradient reads BOTH keys on every call, so a run that takes
    any gradient raises KeyError when either is missing, whatever the problem."""
    if int(n_iterations) > 0 and len(workers) > 0:
        lam, mu = cfg["l2_regularization_lambda"], cfg["strong_convexity_mu"]
    else:
        lam, mu = cfg.get("l2_regularization_lambda", 0.0), cfg.get("strong_convexity_mu", 0.0)
    return lam if cfg["problem_type"] == "logistic" else mu


def _batch_size(workers):
    bs = {int(w.batch_size) for w in workers}
    if len(bs) > 1:
        raise NotImplementedError("workers with different batch sizes")
    return bs.pop() if bs else 0


def _index_chunks(workers, T, config, t_begin=0, max_chunk=0, overlap=False):
    """Yield (t_start, n_rounds, b, idx or None, rng_state): minibatch indices drawn on the
    host in trainer order (trainer.py:47-50 / :166), `None` when every batch is the full
    shard; rng_state = numpy's legacy state right after this chunk's draws (what a
    checkpoint taken after the chunk records).  Rounds t_begin .. T-1; chunks of at most
    max_chunk rounds (0: no limit) starting at multiples of it.  The legacy MT19937 stream
    is sequential, so the draw runs one chunk AHEAD on a host thread (the C sampler
    releases the GIL) while the device runs the current chunk.  overlap: chunks of about
    IDX_CHUNK_DRAWS stream words, so the device starts after a short first draw and the
    draw of chunk k+1 overlaps the device run of chunk k even in short runs (callers whose
    chunk calls carry no extra metrics pass: pipelined D-SGD runs)."""
    b = _batch_size(workers)
    rows = np.array([w.n_local_samples for w in workers], dtype=np.int64)
    full = b >= (rows.max() if len(rows) else 0)
    mode = config.get("sampling", "legacy")
    skip_rng = (full and mode == "full") or mode == "device"  # device: the GPU draws the minibatches

    def bounds(ch):  # chunks of <= ch rounds that never cross a multiple of max_chunk
        t = t_begin
        while t < T:
            n = min(ch, T - t)
            if max_chunk > 0:
                n = min(n, max_chunk - t % max_chunk)
            yield t, n
            t += n

    if skip_rng:
        for t, n in bounds(max(1, T)):
            yield t, n, b, None, np.random.get_state()
        return
    # Full shards: the indices are discarded but the stream must still advance (every
    # choice() is a whole permutation of m_i, whatever b is): advance it without making them.
    b_draw = 1 if full else b
    ch = max(1, min(IDX_CHUNK_ROUNDS, IDX_CHUNK_ELEMS // max(1, len(workers) * max(b_draw, 1))))
    if overlap:  # every choice() draws a whole permutation: about m_i - 1 words per worker
        per_round = max(1, int(np.sum(np.maximum(rows - 1, 0))))
        ch = max(1, min(ch, IDX_CHUNK_DRAWS // per_round))

    def draws():
        for t, n in bounds(ch):
            if full:  # the stream advance alone (dopt_mt_advance_rounds): no indices are made
                _dopt.mt_advance_rounds(n, rows)
                yield t, n, b, None, np.random.get_state()
            else:
                idx = _dopt.mt_choice_rounds(n, rows, b_draw)  # advances np.random exactly like the reference
                yield t, n, b, idx, np.random.get_state()

    yield from _one_ahead(draws())


class _Checkpoint:
    """Checkpoint / resume (the reference keeps its state in memory only):
    config 'checkpoint_path' + 'checkpoint_every' (rounds; 0 = at the end of run only) save,
    after every such round, the iterates (N x d, or the global model), the round count t,
    the history so far, floats transmitted and numpy's legacy RNG state as of the last
    consumed draw; config 'resume_from' restarts run(n_iterations) at round t of that file.
    A resumed run continues bit for bit: the iterates, the learning-rate schedule
    (eta0 / sqrt(t+1), trainer.py:138-140) and the minibatch stream pick up where they were.
    The file is an .npz (no pickles) written to a temporary name and renamed."""

    def __init__(self, cfg, kind, trainer, rank=0):
        self.path = cfg.get("checkpoint_path")
        self.every = int(cfg.get("checkpoint_every", 0) or 0)
        self.resume = cfg.get("resume_from")
        self.kind, self.tr, self.rank = kind, trainer, rank
        self.meta = {"kind": kind, "n_workers": trainer.n_workers, "n_features": trainer.n_features,
                     "problem_type": cfg["problem_type"], "topology": getattr(trainer, "topology", "")}
        if self.path or self.resume:
            # everything else a resumed run must share with the saved one to continue bit for bit:
            # the step size (trainer.py:138-140), the minibatch size, the arithmetic, both regulariser
            # keys (worker.py:36-37) and the shard contents
            ws = trainer.workers
            self.meta.update(
                learning_rate_eta0=float(cfg.get("learning_rate_eta0", 0.0)),
                local_batch_size=int(_batch_size(ws)), dtype=str(cfg.get("dtype", "float64")),
                l2_regularization_lambda=float(cfg.get("l2_regularization_lambda", 0.0)),
                strong_convexity_mu=float(cfg.get("strong_convexity_mu", 0.0)),
                # one fixed hash (blake2b, named in the file), so a checkpoint resumes in an environment
                # with or without xxhash
                data_hash="blake2b",
                data=_full_digest([a for w in ws for a in (w.X_local, w.y_local)], "blake2b"))

    @staticmethod
    def _meta_value(v):
        k = v.dtype.kind
        return str(v) if k == "U" else float(v) if k == "f" else int(v)

    def max_chunk(self):
        return self.every if self.path and self.every > 0 else 0

    def due(self, t_done, T):
        return bool(self.path) and ((self.every > 0 and t_done % self.every == 0) or t_done == T)

    def load(self, T):
        """(t, state array, time offset) from 'resume_from', history / floats / RNG restored,
        or (0, None, 0.0) without one."""
        if not self.resume:
            return 0, None, 0.0
        with np.load(self.resume, allow_pickle=False) as z:
            missing = [k for k in self.meta if k not in z.files]
            if missing:
                raise ValueError(f"checkpoint {self.resume} lacks {missing}: written by another version")
            got = {k: self._meta_value(z[k]) for k in self.meta}
            if "data" in self.meta and got.get("data") != self.meta["data"]:
                raise ValueError(f"checkpoint {self.resume} was written for other shard data "
                                 f"({got.get('data_hash')} digest {got.get('data')} vs {self.meta['data']})")
            if got != self.meta:
                diff = {k: (got[k], self.meta[k]) for k in self.meta if got[k] != self.meta[k]}
                raise ValueError(f"checkpoint {self.resume} does not match this trainer (saved, this run): {diff}")
            t = int(z["t"])
            if t > T:
                raise ValueError(f"checkpoint {self.resume} is at round {t} > n_iterations = {T}")
            for key in self.tr.history:
                self.tr.history[key] = list(z[f"history_{key}"])
            self.tr.total_floats_transmitted = int(z["floats"])
            np.random.set_state(("MT19937", z["rng_key"], int(z["rng_pos"]), int(z["rng_has_gauss"]),
                                 float(z["rng_gauss"])))
            state = np.array(z["state"])
            offset = float(self.tr.history["time"][-1]) if self.tr.history["time"] else 0.0
        return t, state, offset

    def save(self, t, state, rng_state):
        if self.rank != 0:
            return
        arrays = {k: np.array(v) for k, v in self.meta.items()}
        arrays.update({f"history_{k}": np.asarray(v, dtype=np.float64) for k, v in self.tr.history.items()})
        arrays.update(t=np.int64(t), state=np.asarray(state, dtype=np.float64),
                      floats=np.int64(self.tr.total_floats_transmitted),
                      rng_key=np.asarray(rng_state[1], dtype=np.uint32), rng_pos=np.int64(rng_state[2]),
                      rng_has_gauss=np.int64(rng_state[3]), rng_gauss=np.float64(rng_state[4]))
        tmp = self.path + ".tmp.npz"
        np.savez(tmp, **arrays)
        os.replace(tmp, self.path)


def _one_ahead(gen):
    """Items of `gen`, each produced on a worker thread while the caller consumes the
    previous one.  Exactly the items of gen are produced (no draw past the end).

    The draws advance numpy's global legacy stream.  If the consumer stops early (the
    device run of a chunk raised, or the loop was left), the chunk drawn ahead was never
    used: numpy's state goes back to where the last CONSUMED chunk left it, so a later
    trainer in the process continues the reference's stream (trainer.py:166, worker.py:27)."""
    from concurrent.futures import ThreadPoolExecutor

    done = object()
    with ThreadPoolExecutor(max_workers=1) as ex:
        fut = ex.submit(next, gen, done)
        finished = False
        try:
            while True:
                item = fut.result()
                if item is done:
                    finished = True
                    return
                consumed = np.random.get_state()  # the stream after the chunk handed out now
                fut = ex.submit(next, gen, done)
                yield item
        finally:
            if not finished:
                try:
                    fut.result()  # let the in-flight draw finish, then undo it
                except Exception:
                    pass
                if "consumed" in locals():
                    np.random.set_state(consumed)


# ---------------------------------------------------------------------------- centralized
class CentralizedTrainer:
    def __init__(self, workers, n_features, config):
        self.workers = workers
        self.n_workers = len(workers)
        self.x_global = np.zeros(n_features)
        self.config = config
        self.history = {"objective": [], "time": []}
        self.n_features = n_features
        self.total_floats_transmitted = 0

    def _get_learning_rate(self, t):
        return self.config["learning_rate_eta0"] / np.sqrt(t + 1)

    def _get_objective_func(self):
        problem_type = self.config["problem_type"]
        if problem_type == "logistic":
            return logistic_objective
        elif problem_type == "quadratic":
            return quadratic_objective
        raise ValueError(f"Unknown problem type: {problem_type}")

    def _get_regularization_param(self):
        return self.config["l2_regularization_lambda"]

    def run(self, n_iterations, X_full=None, y_full=None, f_opt=0.0):
        print("\n--- Running Centralized Synchronous mini-batch SGD ---")
        start_time = time.time()
        self._get_objective_func()
        reg_param = self._get_regularization_param()
        self.total_floats_transmitted = 0
        cfg = self.config
        if cfg.get("sampling", "legacy") == "device":
            # the device sampler draws inside the D-SGD row pass only; the centralized trainer
            # (which Simulator.run_all runs first) takes the reference's legacy stream instead
            global _WARNED_CENTRAL_DEVICE
            if not _WARNED_CENTRAL_DEVICE:
                _say("Note: sampling='device' applies to D-SGD; the centralized trainer draws its "
                     "minibatches from numpy's legacy stream (sampling='legacy')", cfg)
                _WARNED_CENTRAL_DEVICE = True
            cfg = dict(cfg, sampling="legacy")
        lam_grad = _grad_reg(cfg, n_iterations, self.workers)
        info = _dist_info(cfg)
        if info is not None:
            return self._run_distributed(info, int(n_iterations), X_full, y_full, f_opt, lam_grad, reg_param,
                                         start_time, cfg)
        eng = _engine(self.workers, self.n_features, cfg, X_full=X_full, y_full=y_full)
        want_obj = _set_objective_data(eng, self.workers, self.n_features, X_full, y_full, _sampled_key(cfg))
        T = int(n_iterations)
        ck = _Checkpoint(cfg, "centralized", self)
        t_begin, state, t_off = ck.load(T)
        if state is not None:
            self.x_global = state
        eng.set_global(self.x_global)
        with closing(_index_chunks(self.workers, T, cfg, t_begin, ck.max_chunk())) as chunks:
            for t0, n, b, idx, rng in chunks:
                t_host = time.time() - start_time + t_off
                obj, tim = eng.run_centralized(n, cfg["learning_rate_eta0"], b, lam_grad, reg_param, f_opt, idx=idx,
                                               t0=t0, objective=want_obj)
                if want_obj:
                    self.history["objective"].extend(list(obj))
                self.history["time"].extend((tim + t_host).tolist())
                # trainer.py:50,60-61: N*d up + N*d down per round (Python ints)
                self.total_floats_transmitted += n * (self.n_workers * self.n_features * 2)
                if ck.due(t0 + n, T):
                    ck.save(t0 + n, eng.get_global(), rng)
        self.x_global = eng.get_global()
        _warn_nonfinite(self.history, self.config)
        print(f"C-SGD training finished. Time: {time.time() - start_time:.2f}sseconds")
        return self.history, self.x_global

    def _run_distributed(self, info, T, X_full, y_full, f_opt, lam_grad, reg_param, start_time, cfg):
        import distributed

        rank, world, _ = info
        bounds = distributed.partition_bounds(self.n_workers, world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        eng = _engine(self.workers, self.n_features, cfg, lo, hi, X_full=X_full, y_full=y_full)
        want_obj, rows_global, sep = _dist_objective(eng, self.workers, self.n_features, X_full, y_full, rank, world,
                                                    _sampled_key(cfg))
        plan = distributed.HaloPlan(rank, world, bounds, lo, hi, np.zeros(0, np.int64), np.zeros(world + 1, np.int64),
                                    np.zeros(0, np.int32), np.zeros(world + 1, np.int64), None, None, None)
        runner = distributed.DistributedCentralized(eng, plan, self.n_workers, rows_global, device=_device(cfg),
                                                    obj_sep=sep)
        ck = _Checkpoint(cfg, "centralized", self, rank)
        t_begin, state, t_off = ck.load(T)
        if state is not None:
            self.x_global = state
        eng.set_global(self.x_global)
        with closing(_index_chunks(self.workers, T, cfg, t_begin, ck.max_chunk())) as chunks:
            for t0, n, b, idx, rng in chunks:
                t_host = time.time() - start_time + t_off
                obj = runner.run(n, cfg["learning_rate_eta0"], b, lam_grad, reg_param, f_opt, t0=t0, objective=want_obj,
                                 idx=None if idx is None else idx[:, lo:hi])
                if want_obj:
                    self.history["objective"].extend(list(obj))
                self.history["time"].extend(list(np.linspace(t_host, time.time() - start_time + t_off, n + 1)[1:]))
                self.total_floats_transmitted += n * (self.n_workers * self.n_features * 2)
                if ck.due(t0 + n, T):
                    ck.save(t0 + n, eng.get_global(), rng)  # every rank holds the same global model
        self.x_global = eng.get_global()
        _warn_nonfinite(self.history, self.config)
        _say(f"C-SGD training finished. Time: {time.time() - start_time:.2f}sseconds", cfg)
        return self.history, self.x_global


# ---------------------------------------------------------------------------- decentralized
class DecentralizedTrainer:
    def __init__(self, workers, topology, n_features, config):
        self.workers = workers
        self.n_workers = len(workers)
        self.topology = topology
        self.n_features = n_features
        self.config = config
        self.adj = None
        self.degrees = None
        self.W = self._create_mixing_matrix()
        print(f"\n--- Running Decentralized SGD ({self.topology} - {self.config['problem_type']}) ---")
        self.history = {"objective": [], "consensus_error": [], "time": []}
        self.total_floats_transmitted = 0

    def _create_mixing_matrix(self):
        """Metropolis-Hastings mixing matrix (trainer.py:91-136), built sparse."""
        topo = _topology.build(self.topology, self.n_workers, self.config)
        self._topo = topo
        self.degrees = topo.degrees
        dense = self.n_workers <= DENSE_LIMIT
        self.adj = topo.dense_adjacency() if dense else None
        W = topo.dense_W() if dense else topo.sparse_W()
        if self.n_workers > 0:
            topo.check()
            if self.n_workers > 1 and self.config.get("spectral_gap", dense):
                print(f"Mixing Matrix Spectral gap (1 - rho): {topo.spectral_gap():.4f} for topology: {self.topology}")
        return W

    def _get_learning_rate(self, t):
        return self.config["learning_rate_eta0"] / np.sqrt(t + 1)

    def _get_objective_func(self):
        problem_type = self.config["problem_type"]
        if problem_type == "logistic":
            return logistic_objective
        elif problem_type == "quadratic":
            return quadratic_objective
        raise NotImplementedError(f"Wrong {problem_type}")

    def _get_regularization_param(self):
        return self.config["l2_regularization_lambda"]

    def run(self, n_iterations, X_full=None, y_full=None, f_opt=0.0):
        start_time = time.time()
        self._get_objective_func()
        reg_param = self._get_regularization_param()
        self.total_floats_transmitted = 0
        cfg = self.config
        lam_grad = _grad_reg(cfg, n_iterations, self.workers)
        info = _dist_info(cfg)
        if info is not None:
            return self._run_distributed(info, int(n_iterations), X_full, y_full, f_opt, lam_grad, reg_param,
                                         start_time)
        eng = _engine(self.workers, self.n_features, cfg, X_full=X_full, y_full=y_full)
        want_obj = _set_objective_data(eng, self.workers, self.n_features, X_full, y_full, _sampled_key(cfg))
        t = self._topo
        uni = t.uniform_offdiag() if self._mean_mixing() else None
        if uni is not None:  # complete graph: w_off (S - x_i) + W_ii x_i, no N^2 neighbour reads
            eng.set_mixing_mean(*uni)
        else:
            eng.set_topology(t.row_ptr, t.col, t.w)
        T = int(n_iterations)
        ck = _Checkpoint(cfg, "decentralized", self)
        t_begin, state, t_off = ck.load(T)
        eng.set_models(state if state is not None else np.stack([np.asarray(w.x, dtype=np.float64)
                                                                 for w in self.workers]))
        iteration_transmission = np.sum(self.degrees) * self.n_features  # trainer.py:169
        eta0 = cfg["learning_rate_eta0"]
        loop_start = time.perf_counter()
        # chunks run as one pipelined chain (dopt_run_dsgd_pipelined: each chunk's last metrics ride
        # the next chunk's first pass), closed where the history must be complete: at a
        # checkpoint and at the end -- the same values as one run_dsgd over all the rounds
        with closing(_index_chunks(self.workers, T, cfg, t_begin, ck.max_chunk(), overlap=True)) as chunks:
            for t0, n, b, idx, rng in chunks:
                t_host = time.time() - start_time + t_off
                obj, cons, tim = eng.run_dsgd_pipelined(n, eta0, b, lam_grad, reg_param, f_opt, idx=idx, t0=t0,
                                                        objective=want_obj, consensus=True, want_time=True)
                end = t0 + n == T or ck.due(t0 + n, T)
                if end:  # the owed metrics of the last iterate
                    o2, c2 = eng.run_dsgd_pipelined(0, eta0, b, lam_grad, reg_param, f_opt, objective=want_obj,
                                                    consensus=True)
                    cons = np.concatenate([cons, c2])
                    obj = np.concatenate([obj, o2]) if want_obj else obj
                self.history["consensus_error"].extend(list(cons))
                if want_obj:
                    self.history["objective"].extend(list(obj))
                self.history["time"].extend((tim + t_host).tolist())
                for _ in range(n):
                    self.total_floats_transmitted += iteration_transmission
                if ck.due(t0 + n, T):
                    ck.save(t0 + n, eng.get_models(), rng)
        # wall time of the round loop alone (the draws, the device rounds, the history), without
        # the per-run data checks before it; bench.py's drop-in leg reads it
        self.loop_seconds = time.perf_counter() - loop_start
        models = eng.get_models()
        for i, worker in enumerate(self.workers):  # trainer.py:178-179: row views
            worker.x = models[i, :]
        _warn_nonfinite(self.history, self.config)
        print(f"Decentralized ({self.topology}) training finished. Time: {time.time() - start_time:.2f}s")
        final_avg_model = np.mean([worker.x for worker in self.workers], axis=0)
        return self.history, final_avg_model

    def _mean_mixing(self):
        """Complete graphs mix through the column sums from MEAN_MIX_MIN workers on, and at any
        size when the rows are longer than the row-resident kernel holds."""
        return (self.n_workers >= self.config.get("mean_mixing_min", MEAN_MIX_MIN) or
                self.n_features > ROW_RESIDENT_MAX)

    def _run_distributed(self, info, T, X_full, y_full, f_opt, lam_grad, reg_param, start_time):
        import distributed

        rank, world, _ = info
        cfg = self.config
        t = self._topo
        uni = t.uniform_offdiag() if self._mean_mixing() else None
        plan = distributed.build_plan(t, world, rank)
        eng = _engine(self.workers, self.n_features, cfg, plan.lo, plan.hi, X_full=X_full, y_full=y_full)
        want_obj, rows_global, sep = _dist_objective(eng, self.workers, self.n_features, X_full, y_full, rank, world,
                                                    _sampled_key(cfg))
        ck = _Checkpoint(cfg, "decentralized", self, rank)
        t_begin, state, t_off = ck.load(T)
        x0 = state if state is not None else np.stack([np.asarray(w.x, dtype=np.float64) for w in self.workers])
        eng.set_models(np.ascontiguousarray(x0[plan.lo:plan.hi]))
        runner = distributed.DistributedDSGD(eng, plan, self.n_workers, rows_global, device=_device(cfg),
                                             mean=None if uni is None else (uni[0], uni[1][plan.lo:plan.hi]),
                                             obj_sep=sep)
        iteration_transmission = np.sum(self.degrees) * self.n_features  # trainer.py:169
        with closing(_index_chunks(self.workers, T, cfg, t_begin, ck.max_chunk())) as chunks:
            for t0, n, b, idx, rng in chunks:
                t_host = time.time() - start_time + t_off
                obj, cons = runner.run(n, cfg["learning_rate_eta0"], b, lam_grad, reg_param, f_opt, t0=t0,
                                       objective=want_obj, consensus=True,
                                       idx=None if idx is None else idx[:, plan.lo:plan.hi])
                self.history["consensus_error"].extend(list(cons))
                if want_obj:
                    self.history["objective"].extend(list(obj))
                self.history["time"].extend(list(np.linspace(t_host, time.time() - start_time + t_off, n + 1)[1:]))
                for _ in range(n):
                    self.total_floats_transmitted += iteration_transmission
                if ck.due(t0 + n, T):
                    ck.save(t0 + n, runner.gather_models(), rng)  # collective: every rank gathers, rank 0 writes
        models = runner.gather_models()
        for i, worker in enumerate(self.workers):
            worker.x = models[i, :]
        _warn_nonfinite(self.history, self.config)
        _say(f"Decentralized ({self.topology}) training finished. Time: {time.time() - start_time:.2f}s", cfg)
        final_avg_model = np.mean([worker.x for worker in self.workers], axis=0)
        return self.history, final_avg_model
