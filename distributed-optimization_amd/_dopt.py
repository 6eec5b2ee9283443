"""ctypes binding of libdopt.so (the C ABI in include/dopt.h).

This is the only place the Python host code touches the engine.  There is no
CPU fallback: if libdopt.so is missing or no GPU is visible, device calls raise.

Error mapping (so the drop-in modules raise what the reference raises):
  DOPT_ERR_INVALID      -> ValueError
  DOPT_ERR_UNSUPPORTED  -> NotImplementedError
  anything else         -> RuntimeError
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DOPT_LIB", os.path.join(_HERE, "libdopt.so"))

OK, ERR_INVALID, ERR_HIP, ERR_STATE, ERR_UNSUPPORTED, ERR_COMM, ERR_NOMEM, ERR_RUNTIME = 0, -1, -2, -3, -4, -5, -6, -7
LOGISTIC, QUADRATIC = 0, 1
F32, F64 = 0, 1
RUN_OBJECTIVE, RUN_CONSENSUS = 1, 2
SAMPLE_HOST, SAMPLE_DEVICE = 0, 1
MAX_BIP_ROWS = 65536  # dopt.h DOPT_MAX_BIP_ROWS: minibatch gradient inside the metrics pass
PROBLEMS = {"logistic": LOGISTIC, "quadratic": QUADRATIC}
DTYPES = {"float32": F32, "fp32": F32, "f32": F32, np.float32: F32,
          "float64": F64, "fp64": F64, "f64": F64, np.float64: F64}

_lib = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_D = ctypes.c_double

_SIGS = {
    "dopt_abi_version": ([], ctypes.c_int),
    "dopt_last_error": ([], ctypes.c_char_p),
    "dopt_mt_choice": ([_P, _P, _I64, _I64, _P], ctypes.c_int),
    "dopt_mt_choice_rounds": ([_P, _P, _I64, _I64, _P, _I64, _P], ctypes.c_int),
    "dopt_mt_advance_rounds": ([_P, _P, _I64, _I64, _P], ctypes.c_int),
    "dopt_last_round_kernel": ([], ctypes.c_char_p),
    "dopt_device_count": ([_P], ctypes.c_int),
    "dopt_create": ([ctypes.c_int, ctypes.c_int, _P], ctypes.c_int),
    "dopt_destroy": ([_P], ctypes.c_int),
    "dopt_set_data_dtype": ([_P, ctypes.c_int], ctypes.c_int),
    "dopt_get_data_dtype": ([_P, _P], ctypes.c_int),
    "dopt_load_shards": ([_P, ctypes.c_int, _I64, _I64, _P, _P, _P, ctypes.c_int], ctypes.c_int),
    "dopt_generate_shards": ([_P, ctypes.c_int, _I64, _I64, _I64, ctypes.c_uint64, _D, _D, _I64], ctypes.c_int),
    "dopt_load_objective_data": ([_P, _I64, _P, _P, ctypes.c_int], ctypes.c_int),
    "dopt_clear_objective_data": ([_P], ctypes.c_int),
    "dopt_get_shard": ([_P, _I64, _P, _P], ctypes.c_int),
    "dopt_set_topology": ([_P, _I64, _P, _P, _P], ctypes.c_int),
    "dopt_set_mixing_mean": ([_P, _I64, _D, _P], ctypes.c_int),
    "dopt_set_models": ([_P, _P], ctypes.c_int),
    "dopt_get_models": ([_P, _P], ctypes.c_int),
    "dopt_set_global": ([_P, _P], ctypes.c_int),
    "dopt_get_global": ([_P, _P], ctypes.c_int),
    "dopt_run_dsgd": ([_P, _I64, _I64, _D, _I64, _P, _D, _D, _D, ctypes.c_uint32, _P, _P, _P], ctypes.c_int),
    "dopt_run_dsgd_pipelined": ([_P, _I64, _I64, _D, _I64, _P, _D, _D, _D, ctypes.c_uint32, _P, _P, _P, _P],
                                ctypes.c_int),
    "dopt_run_centralized": ([_P, _I64, _I64, _D, _I64, _P, _D, _D, _D, ctypes.c_uint32, _P, _P], ctypes.c_int),
    "dopt_eval_gradient": ([_P, ctypes.c_int, _I64, _I64, _P, _P, _P, _D, _P], ctypes.c_int),
    "dopt_eval_objective": ([_P, ctypes.c_int, _I64, _I64, _P, _P, _P, _D, _P], ctypes.c_int),
    "dopt_set_stream": ([_P, _P], ctypes.c_int),
    "dopt_get_layout": ([_P, _P, _P], ctypes.c_int),
    "dopt_set_partition": ([_P, _I64, _I64], ctypes.c_int),
    "dopt_set_halo": ([_P, _I64, _P, _I64, _P, _P], ctypes.c_int),
    "dopt_phase_begin": ([_P, _I64], ctypes.c_int),
    "dopt_phase_chain": ([_P, ctypes.c_int, _P], ctypes.c_int),
    "dopt_phase_gather": ([_P], ctypes.c_int),
    "dopt_phase_grad_shared": ([_P, _I64, _P, _D, ctypes.c_int], ctypes.c_int),
    "dopt_phase_colsum_grad": ([_P, _P], ctypes.c_int),
    "dopt_phase_central_step": ([_P, _P, _I64, _D], ctypes.c_int),
    "dopt_phase_metrics_pass_shared": ([_P], ctypes.c_int),
    "dopt_phase_metrics_shared": ([_P, ctypes.c_int, _P], ctypes.c_int),
    "dopt_phase_grad": ([_P, _I64, _P, _D, ctypes.c_uint32], ctypes.c_int),
    "dopt_phase_mix": ([_P, _I64, _D], ctypes.c_int),
    "dopt_phase_colsum": ([_P, _P], ctypes.c_int),
    "dopt_phase_xbar": ([_P, _P], ctypes.c_int),
    "dopt_phase_metrics_pass": ([_P, ctypes.c_uint32], ctypes.c_int),
    "dopt_phase_metrics": ([_P, ctypes.c_uint32, ctypes.c_int, _P], ctypes.c_int),
    "dopt_phase_fold": ([_P, _P, _P, _P, ctypes.c_int], ctypes.c_int),
    "dopt_lagged_exchange_layout": ([_P, _I32, _I32, _P, _P], ctypes.c_int),
    "dopt_lagged_begin": ([_P, _I64], ctypes.c_int),
    "dopt_lagged_grad": ([_P, _I64, _D, _I64, _P, _D, ctypes.c_uint32], ctypes.c_int),
    "dopt_lagged_mix": ([_P, _I64, _D, ctypes.c_int, _P, _P, _P], ctypes.c_int),
    "dopt_lagged_tail": ([_P, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "dopt_lagged_side_stream": ([_P, _P], ctypes.c_int),
    "dopt_lagged_exchange_issued": ([_P, _P], ctypes.c_int),
    "dopt_rs_phase_begin": ([_P, ctypes.c_int, _P, _P], ctypes.c_int),
    "dopt_rs_phase_round": ([_P, _I64, _D, _D, ctypes.c_uint32, _P], ctypes.c_int),
    "dopt_rs_phase_cols": ([_P, _I64, _D, _D, _P], ctypes.c_int),
    "dopt_rs_phase_metrics": ([_P, ctypes.c_uint32], ctypes.c_int),
    "dopt_rs_phase_pass": ([_P, ctypes.c_int32, ctypes.c_int32, _P, _P], ctypes.c_int),
    "dopt_rs_phase_cols_range": ([_P, _I64, _D, _D, _P, _I64, _I64, ctypes.c_int32], ctypes.c_int),
    "dopt_rs_phase_rows": ([_P, _I64, _D, _D, ctypes.c_uint32], ctypes.c_int),
    "dopt_zero_models": ([_P], ctypes.c_int),
    "dopt_sync": ([_P], ctypes.c_int),
    "dopt_finalize_metrics": ([ctypes.c_int, _I64, _P, _I64, _I64, _D, _D, _P, _P], ctypes.c_int),
    "dopt_eval_full": ([_P, _P, _D, _P, _P], ctypes.c_int),
    "dopt_kernel_stats": ([_P, _P, _P], ctypes.c_int),
    "dopt_set_profiling": ([_P, ctypes.c_int], ctypes.c_int),
    "dopt_set_sampler": ([_P, ctypes.c_int, ctypes.c_uint64, _I64], ctypes.c_int),
    "dopt_phase_set_round": ([_P, _I64], ctypes.c_int),
    "dopt_phase_set_step": ([_P, _I64, ctypes.c_double], ctypes.c_int),
    "dopt_phase_interior_count": ([_P, _P], ctypes.c_int),
    "dopt_host_digest": ([_I32, _P, _P, _I32, _P], ctypes.c_int),
    "dopt_comm_unique_id": ([_P, _I64], ctypes.c_int),
    "dopt_comm_create": ([_P, _I32, _I32, _I32, _P, _I64, ctypes.c_double], ctypes.c_int),
    "dopt_comm_check": ([_P], ctypes.c_int),
    "dopt_comm_destroy": ([_P, _I32], ctypes.c_int),
    "dopt_comm_library": ([], ctypes.c_char_p),
    "dopt_lagged_transport": ([_P, _P, _P, _P], ctypes.c_int),
    "dopt_lagged_exchange": ([_P], ctypes.c_int),
    "dopt_lagged_ipc_export": ([_P, _P, _P, _P], ctypes.c_int),
    "dopt_lagged_ipc_import": ([_P, _I32, _I32, _P, _P, _P, _P, _P, _P, ctypes.c_double], ctypes.c_int),
    "dopt_lagged_ipc_check": ([_P, _I32], ctypes.c_int),
}
EXPORTED = tuple(_SIGS)
ABI_VERSION = 9  # DOPT_ABI_VERSION of include/dopt.h


def lib():
    """Load libdopt.so once.  torch (when installed) is imported first so the
    process has ONE HIP runtime: libdopt.so binds to torch's libamdhip64."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if os.environ.get("DOPT_NO_TORCH", "0") != "1":
            try:
                import torch  # noqa: F401
            except Exception:  # pragma: no cover - torch is optional plumbing
                pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libdopt.so not built at {LIB_PATH}: run `make -C "
                               f"distributed-optimization_amd/csrc` or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.dopt_abi_version() != ABI_VERSION:
            raise RuntimeError(f"libdopt.so ABI {L.dopt_abi_version()} != {ABI_VERSION} (include/dopt.h): rebuild it")
        _lib = L
    return _lib


def check(rc):
    if rc == OK:
        return
    msg = (lib().dopt_last_error() or b"").decode(errors="replace")
    if rc == ERR_INVALID:
        raise ValueError(msg)
    if rc == ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == ERR_NOMEM:
        raise MemoryError("libdopt: host memory exhausted")
    if rc == ERR_RUNTIME:
        raise RuntimeError("libdopt: host failure (a helper thread could not start)")
    raise RuntimeError(f"libdopt error {rc}: {msg}")


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def host_digest(buffers, threads=0):
    """128-bit content digest (32 hex digits) of C-contiguous host arrays, in order, hashed in 4 MiB
    chunks on several threads (dopt_host_digest; host code, no GPU needed)."""
    bufs = [np.ascontiguousarray(b) for b in buffers]
    n = len(bufs)
    ptrs = (ctypes.c_void_p * max(1, n))(*[b.ctypes.data if b.nbytes else None for b in bufs])
    sizes = np.array([b.nbytes for b in bufs] or [0], dtype=np.int64)
    out = np.zeros(2, dtype=np.uint64)
    check(lib().dopt_host_digest(n, ptrs, _ptr(sizes), int(threads), _ptr(out)))
    return f"{int(out[0]):016x}{int(out[1]):016x}"


COMM_ID_BYTES = 128  # DOPT_COMM_ID_BYTES


def comm_unique_id():
    """dopt_comm_unique_id: rank 0's RCCL unique id (bytes) for Comm()."""
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    check(lib().dopt_comm_unique_id(buf, COMM_ID_BYTES))
    return bytes(buf)


def comm_library():
    """dopt_comm_library: path of the RCCL library the transport uses ('' before the first use / none)."""
    return (lib().dopt_comm_library() or b"").decode()


class Comm:
    """An RCCL communicator the engine drives itself (dopt_comm_create; csrc/transport.cpp): rank `rank` of
    `world` on `device`, from rank 0's comm_unique_id() -- every rank constructs it with the same id.  Its
    setup waits at most `timeout_s` seconds for the other ranks (0: unbounded), then raises RuntimeError."""

    def __init__(self, world, rank, device, uid, timeout_s=0.0):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"RCCL unique id of {COMM_ID_BYTES} bytes expected, got {len(uid)}")
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        check(lib().dopt_comm_create(ctypes.byref(h), int(world), int(rank), int(device), buf, COMM_ID_BYTES,
                                     float(timeout_s)))
        self._h = h
        self.world, self.rank, self.device = int(world), int(rank), int(device)
        self.users = weakref.WeakSet()  # engines whose exchange runs through it (Engine.lagged_transport)

    @property
    def closed(self):
        return not getattr(self, "_h", None)

    def check(self):
        """Raise if RCCL reported an asynchronous error on this communicator."""
        if self.closed:
            raise RuntimeError("the RCCL communicator is closed")
        check(lib().dopt_comm_check(self._h))

    def close(self, abort=False):
        """Detach every engine still routed through it (so none can reach the freed communicator: its next
        dopt_lagged_exchange fails with 'no transport'), then destroy it (abort: without waiting for
        pending work, after a peer failed).  The caller drains the engines' streams first unless aborting."""
        h = getattr(self, "_h", None)
        if not h:
            return
        for eng in list(self.users):
            eng.lagged_transport(None)
        self._h = None
        check(lib().dopt_comm_destroy(h, 1 if abort else 0))


def device_count():
    n = ctypes.c_int(0)
    check(lib().dopt_device_count(ctypes.byref(n)))
    return n.value


# ---------------------------------------------------------------------------- sampler
def _get_np_state():
    st = np.random.get_state()
    if st[0] != "MT19937":
        raise RuntimeError("numpy global RNG is not the legacy MT19937")
    return st, np.array(st[1], dtype=np.uint32, copy=True), ctypes.c_int32(int(st[2]))


def _set_np_state(st, key, pos):
    np.random.set_state((st[0], key, int(pos.value), st[3], st[4]))


def mt_choice(m, b):
    """np.random.choice(m, min(b, m), replace=False) on numpy's global state (worker.py:27)."""
    st, key, pos = _get_np_state()
    eb = 0 if m == 0 else min(b, m)
    out = np.empty(max(eb, 0), dtype=np.int64)
    check(lib().dopt_mt_choice(_ptr(key), ctypes.byref(pos), int(m), int(b), _ptr(out)))
    _set_np_state(st, key, pos)
    return out


def mt_choice_rounds(T, shard_rows, b):
    """[T, N, b] int32 index draws of T rounds x N workers, advancing numpy's global state."""
    st, key, pos = _get_np_state()
    rows = np.ascontiguousarray(shard_rows, dtype=np.int64)
    out = np.empty((int(T), len(rows), int(b)), dtype=np.int32)
    check(lib().dopt_mt_choice_rounds(_ptr(key), ctypes.byref(pos), int(T), len(rows), _ptr(rows),
                                      int(b), _ptr(out)))
    _set_np_state(st, key, pos)
    return out


def last_round_kernel():
    """Instance name of the last gradient-round kernel launched in this process ('' before any)."""
    return lib().dopt_last_round_kernel().decode()


def mt_advance_rounds(T, shard_rows):
    """Advance numpy's global legacy state as T rounds x N workers of choice() draws would
    (full-shard batches: the indices are discarded, worker.py:27)."""
    st, key, pos = _get_np_state()
    rows = np.ascontiguousarray(shard_rows, dtype=np.int64)
    check(lib().dopt_mt_advance_rounds(_ptr(key), ctypes.byref(pos), int(T), len(rows), _ptr(rows)))
    _set_np_state(st, key, pos)


# ---------------------------------------------------------------------------- device engine
class Engine:
    """One dopt context (one GPU): shards, topology and iterates resident in HBM.

    dtype: iterates and arithmetic.  data_dtype: storage of the shard rows (default: dtype);
    'float32' under dtype 'float64' keeps every operation in float64 and reads the rows as
    float32 (exact for float32-representable data: half the HBM bytes per round)."""

    def __init__(self, device=0, dtype="float64", data_dtype=None):
        self.dtype = DTYPES[dtype] if not isinstance(dtype, int) else dtype
        self.np_dtype = np.float32 if self.dtype == F32 else np.float64
        self.device = int(device)
        h = ctypes.c_void_p()
        check(lib().dopt_create(self.device, self.dtype, ctypes.byref(h)))
        self._h = h
        self.data_dtype = self.dtype
        if data_dtype is not None:
            xd = DTYPES[data_dtype] if not isinstance(data_dtype, int) else data_dtype
            check(lib().dopt_set_data_dtype(self._h, xd))
            self.data_dtype = xd
        self.n = 0
        self.d = 0
        self.problem = None
        self.shard_rows = None
        self.tag = None  # identity of the loaded data, for caching in the trainers

    def close(self):
        if getattr(self, "_h", None):
            lib().dopt_destroy(self._h)
            self._h = None
        comm = getattr(self, "_comm", None)
        if comm is not None:
            comm.users.discard(self)
            self._comm = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order varies
        try:
            self.close()
        except Exception:
            pass

    # -- data
    def load_shards(self, problem, X, y, shard_offsets):
        X = np.ascontiguousarray(X)
        src_f32 = 1 if X.dtype == np.float32 else 0
        X = np.ascontiguousarray(X, dtype=np.float32 if src_f32 else np.float64)
        y = np.ascontiguousarray(y, dtype=X.dtype)
        off = np.ascontiguousarray(shard_offsets, dtype=np.int64)
        n = len(off) - 1
        d = X.shape[1]
        check(lib().dopt_load_shards(self._h, PROBLEMS[problem], n, d, _ptr(off), _ptr(X), _ptr(y), src_f32))
        self.n, self.d, self.problem = n, d, problem
        self.shard_rows = np.diff(off)

    def generate_shards(self, problem, n_workers, d, rows_per_worker, seed=0, flip=0.05, noise=10.0,
                        first_worker=0):
        check(lib().dopt_generate_shards(self._h, PROBLEMS[problem], int(n_workers), int(d),
                                         int(rows_per_worker), int(seed) & (2 ** 64 - 1), float(flip),
                                         float(noise), int(first_worker)))
        self.n, self.d, self.problem = int(n_workers), int(d), problem
        self.shard_rows = np.full(int(n_workers), int(rows_per_worker), dtype=np.int64)

    def load_objective_data(self, X, y):
        X = np.ascontiguousarray(X, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.float64)
        check(lib().dopt_load_objective_data(self._h, X.shape[0], _ptr(X), _ptr(y), 0))

    def clear_objective_data(self):
        check(lib().dopt_clear_objective_data(self._h))

    def get_shard(self, i):
        m = int(self.shard_rows[i])
        X = np.empty((m, self.d), dtype=np.float64)
        y = np.empty(m, dtype=np.float64)
        check(lib().dopt_get_shard(self._h, int(i), _ptr(X), _ptr(y)))
        return X, y

    def set_topology(self, row_ptr, col, w):
        rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
        ci = np.ascontiguousarray(col, dtype=np.int32)
        cw = np.ascontiguousarray(w, dtype=np.float64)
        check(lib().dopt_set_topology(self._h, len(rp) - 1, _ptr(rp), _ptr(ci), _ptr(cw)))

    def set_mixing_mean(self, w_off, w_diag):
        wd = np.ascontiguousarray(w_diag, dtype=np.float64)
        check(lib().dopt_set_mixing_mean(self._h, len(wd), float(w_off), _ptr(wd)))

    def set_models(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64).reshape(self.n, self.d)
        check(lib().dopt_set_models(self._h, _ptr(x)))

    def zero_models(self):
        """Every iterate = 0 on the device (no host copy)."""
        check(lib().dopt_zero_models(self._h))

    def get_models(self):
        x = np.empty((self.n, self.d), dtype=np.float64)
        check(lib().dopt_get_models(self._h, _ptr(x)))
        return x

    def set_global(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64).reshape(self.d)
        check(lib().dopt_set_global(self._h, _ptr(x)))

    def get_global(self):
        x = np.empty(self.d, dtype=np.float64)
        check(lib().dopt_get_global(self._h, _ptr(x)))
        return x

    # -- rounds
    def run_dsgd(self, T, eta0, batch, lam_grad, lam_obj, f_opt=0.0, idx=None, t0=0,
                 objective=True, consensus=True, want_time=True):
        T = int(T)
        obj = np.zeros(T) if objective else None
        cons = np.zeros(T) if consensus else None
        tim = np.zeros(T) if want_time else None
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int32)
        flags = (RUN_OBJECTIVE if objective else 0) | (RUN_CONSENSUS if consensus else 0)
        check(lib().dopt_run_dsgd(self._h, int(t0), T, float(eta0), int(batch), _ptr(idx), float(lam_grad),
                                  float(lam_obj), float(f_opt), flags, _ptr(obj), _ptr(cons), _ptr(tim)))
        return obj, cons, tim

    def run_dsgd_pipelined(self, T, eta0, batch, lam_grad, lam_obj, f_opt=0.0, idx=None, t0=0,
                           objective=True, consensus=True, want_time=False):
        """dopt_run_dsgd_pipelined: the metrics of the last iterate are owed to the next such
        call (entry 0 of its output); returns (objective, consensus) of the entries written,
        and with want_time also the end-of-round times of this call's T rounds."""
        T = int(T)
        obj = np.zeros(T + 1) if objective else None
        cons = np.zeros(T + 1) if consensus else None
        tim = np.zeros(T) if want_time else None
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int32)
        flags = (RUN_OBJECTIVE if objective else 0) | (RUN_CONSENSUS if consensus else 0)
        n = ctypes.c_int64(0)
        check(lib().dopt_run_dsgd_pipelined(self._h, int(t0), T, float(eta0), int(batch), _ptr(idx),
                                            float(lam_grad), float(lam_obj), float(f_opt), flags, _ptr(obj),
                                            _ptr(cons), _ptr(tim), ctypes.byref(n)))
        k = n.value
        res = (None if obj is None else obj[:k]), (None if cons is None else cons[:k])
        return res + (tim,) if want_time else res

    def run_centralized(self, T, eta0, batch, lam_grad, lam_obj, f_opt=0.0, idx=None, t0=0,
                        objective=True, want_time=True):
        T = int(T)
        obj = np.zeros(T) if objective else None
        tim = np.zeros(T) if want_time else None
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int32)
        flags = RUN_OBJECTIVE if objective else 0
        check(lib().dopt_run_centralized(self._h, int(t0), T, float(eta0), int(batch), _ptr(idx),
                                         float(lam_grad), float(lam_obj), float(f_opt), flags, _ptr(obj),
                                         _ptr(tim)))
        return obj, tim

    # -- single evaluations (float64)
    def eval_gradient(self, problem, w, X, y, reg):
        w = np.ascontiguousarray(w, dtype=np.float64)
        X = np.ascontiguousarray(X, dtype=np.float64).reshape(-1, w.shape[0])
        y = np.ascontiguousarray(y, dtype=np.float64)
        g = np.empty(w.shape[0], dtype=np.float64)
        check(lib().dopt_eval_gradient(self._h, PROBLEMS[problem], X.shape[0], w.shape[0], _ptr(w), _ptr(X),
                                       _ptr(y), float(reg), _ptr(g)))
        return g

    def eval_objective(self, problem, w, X, y, reg):
        w = np.ascontiguousarray(w, dtype=np.float64)
        X = np.ascontiguousarray(X, dtype=np.float64).reshape(-1, w.shape[0])
        y = np.ascontiguousarray(y, dtype=np.float64)
        out = np.zeros(1, dtype=np.float64)
        check(lib().dopt_eval_objective(self._h, PROBLEMS[problem], X.shape[0], w.shape[0], _ptr(w), _ptr(X),
                                        _ptr(y), float(reg), _ptr(out)))
        return np.float64(out[0])

    # -- multi-GPU phases (enqueue only; pointers are device addresses)
    def set_stream(self, stream_handle):
        check(lib().dopt_set_stream(self._h, ctypes.c_void_p(stream_handle) if stream_handle else None))

    def layout(self):
        ld, esz = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().dopt_get_layout(self._h, ctypes.byref(ld), ctypes.byref(esz)))
        return ld.value, esz.value

    def set_partition(self, n_global, rows_global):
        check(lib().dopt_set_partition(self._h, int(n_global), int(rows_global)))

    def set_halo(self, n_halo, halo_ptr, send_ids, send_ptr):
        ids = np.ascontiguousarray(send_ids, dtype=np.int32)
        check(lib().dopt_set_halo(self._h, int(n_halo), ctypes.c_void_p(halo_ptr) if halo_ptr else None, len(ids),
                                  ctypes.c_void_p(send_ptr) if send_ptr else None, _ptr(ids)))

    def phase_interior_count(self):
        """Workers this rank's gradient kernel mixes and steps itself (dopt_phase_interior_count)."""
        n = ctypes.c_int64(0)
        check(lib().dopt_phase_interior_count(self._h, ctypes.byref(n)))
        return n.value

    def phase_chain(self, mark):
        """dopt_phase_chain: whether the last pipelined phase run left its schedule open (and
        nothing has touched the context since); then set (mark) or clear the mark."""
        was = ctypes.c_int(0)
        check(lib().dopt_phase_chain(self._h, 1 if mark else 0, ctypes.byref(was)))
        return bool(was.value)

    def phase_begin(self, batch):
        check(lib().dopt_phase_begin(self._h, int(batch)))

    def phase_grad_shared(self, batch, lam_grad, fuse_loss=False, idx=None):
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int32)
        check(lib().dopt_phase_grad_shared(self._h, int(batch), _ptr(idx), float(lam_grad), 1 if fuse_loss else 0))

    def phase_colsum_grad(self, sum_ptr):
        check(lib().dopt_phase_colsum_grad(self._h, ctypes.c_void_p(sum_ptr)))

    def phase_central_step(self, sum_ptr, t, eta0):
        check(lib().dopt_phase_central_step(self._h, ctypes.c_void_p(sum_ptr), int(t), float(eta0)))

    def phase_metrics_pass_shared(self):
        check(lib().dopt_phase_metrics_pass_shared(self._h))

    def phase_metrics_shared(self, include_xnorm, out_ptr):
        check(lib().dopt_phase_metrics_shared(self._h, 1 if include_xnorm else 0, ctypes.c_void_p(out_ptr)))

    def phase_set_round(self, t):
        check(lib().dopt_phase_set_round(self._h, int(t)))

    def phase_set_step(self, t, eta0):
        check(lib().dopt_phase_set_step(self._h, int(t), float(eta0)))

    def phase_gather(self):
        check(lib().dopt_phase_gather(self._h))

    def phase_grad(self, batch, lam_grad, metric_flags=0, idx=None):
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int32)
        check(lib().dopt_phase_grad(self._h, int(batch), _ptr(idx), float(lam_grad), int(metric_flags)))

    def phase_mix(self, t, eta0):
        check(lib().dopt_phase_mix(self._h, int(t), float(eta0)))

    def phase_colsum(self, sum_ptr):
        check(lib().dopt_phase_colsum(self._h, ctypes.c_void_p(sum_ptr)))

    def phase_xbar(self, sum_ptr):
        check(lib().dopt_phase_xbar(self._h, ctypes.c_void_p(sum_ptr)))

    def phase_metrics_pass(self, flags):
        check(lib().dopt_phase_metrics_pass(self._h, int(flags)))

    def phase_metrics(self, flags, include_xnorm, out_ptr):
        check(lib().dopt_phase_metrics(self._h, int(flags), 1 if include_xnorm else 0, ctypes.c_void_p(out_ptr)))

    def phase_fold(self, cons_ptr=None, xnorm_ptr=None, loss_ptr=None, slab=0):
        """Device-side sums into the given device addresses (None: skip that output)."""
        vp = lambda p: ctypes.c_void_p(p) if p else None  # noqa: E731
        check(lib().dopt_phase_fold(self._h, vp(cons_ptr), vp(xnorm_ptr), vp(loss_ptr), int(slab)))

    # -- the lagged schedule (dopt_lagged_*; distributed.py _run_lagged): two calls per round
    def lagged_exchange_layout(self, world, rank, sum_send_row, sum_recv_row):
        so = np.ascontiguousarray(sum_send_row, dtype=np.int64)
        ri = np.ascontiguousarray(sum_recv_row, dtype=np.int64)
        check(lib().dopt_lagged_exchange_layout(self._h, int(world), int(rank), _ptr(so), _ptr(ri)))

    def lagged_begin(self, batch):
        check(lib().dopt_lagged_begin(self._h, int(batch)))

    def lagged_grad(self, t, eta0, batch, lam_grad, metric_flags=0, idx=None):
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.int32)
        rc = lib().dopt_lagged_grad(self._h, t, eta0, batch, _ptr(idx), lam_grad, metric_flags)
        if rc:
            check(rc)

    def lagged_mix(self, t, eta0, consensus, cons_ptr=None, xnorm_ptr=None, loss_ptr=None):
        """Per round; device addresses of the history row g-2 (None: not folded)."""
        rc = lib().dopt_lagged_mix(self._h, t, eta0, 1 if consensus else 0, cons_ptr, xnorm_ptr, loss_ptr)
        if rc:
            check(rc)

    def lagged_side_stream(self, stream_ptr):
        """dopt_lagged_side_stream: the stream (a hipStream_t as int, or None) that takes each mix's
        column-sum totals and that the caller issues the exchange on."""
        check(lib().dopt_lagged_side_stream(self._h, ctypes.c_void_p(stream_ptr or None)))

    def lagged_exchange_issued(self):
        """dopt_lagged_exchange_issued: after the caller issued an exchange on the side stream, True when the
        engine stream will wait for it (an event the context records there), False without a side stream
        (the caller orders the engine stream)."""
        o = ctypes.c_int(0)
        check(lib().dopt_lagged_exchange_issued(self._h, ctypes.byref(o)))
        return bool(o.value)

    def lagged_transport(self, comm, send_rows=None, recv_rows=None):
        """dopt_lagged_transport: route the exchange through `comm` (a Comm; None: detach), blocks of
        send_rows[p] / recv_rows[p] rows per peer p in rank order."""
        old = getattr(self, "_comm", None)
        self._ipc_owner = None  # (a pull transport set up later marks itself again: distributed.IpcTransport)
        if comm is None:
            if self._h:  # (a closed context holds no transport)
                check(lib().dopt_lagged_transport(self._h, None, None, None))
            if old is not None:
                old.users.discard(self)
            self._comm = None
            return
        if comm.closed:
            raise ValueError("the RCCL communicator is closed")
        s = np.ascontiguousarray(send_rows, dtype=np.int64)
        r = np.ascontiguousarray(recv_rows, dtype=np.int64)
        if s.shape != (comm.world,) or r.shape != (comm.world,):
            raise ValueError(f"{comm.world} block sizes per direction expected")
        check(lib().dopt_lagged_transport(self._h, comm._h, _ptr(s), _ptr(r)))
        if old is not None and old is not comm:
            old.users.discard(self)
        comm.users.add(self)
        self._comm = comm

    IPC_HANDLE_BYTES = 64  # DOPT_IPC_HANDLE_BYTES

    def lagged_ipc_export(self):
        """dopt_lagged_ipc_export: (memory handle bytes, event handle bytes, slot bytes) of this context's
        send slots for the pull transport."""
        mh = (ctypes.c_uint8 * self.IPC_HANDLE_BYTES)()
        eh = (ctypes.c_uint8 * self.IPC_HANDLE_BYTES)()
        slot = ctypes.c_int64(0)
        self.lagged_transport(None)  # (detaches any RCCL transport: the engine's exchange is this one's next)
        check(lib().dopt_lagged_ipc_export(self._h, mh, eh, ctypes.byref(slot)))
        return bytes(mh), bytes(eh), int(slot.value)

    def lagged_ipc_import(self, world, rank, mem_handles, event_handles, slot_bytes, src_off, recv_rows,
                          counters_addr, timeout_s):
        """dopt_lagged_ipc_import: the peers' exported handles (bytes each, rank order), their slot bytes, the
        byte offset of this rank's block in each peer's slot, recv_rows per peer, the address of `world`
        shared int64 counters (kept alive by the caller while the context uses them) and the host wait bound."""
        n = self.IPC_HANDLE_BYTES
        if len(mem_handles) != world or len(event_handles) != world or any(
                len(h) != n for h in list(mem_handles) + list(event_handles)):
            raise ValueError(f"{world} handles of {n} bytes per kind expected")
        mh = (ctypes.c_uint8 * (n * world)).from_buffer_copy(b"".join(mem_handles))
        eh = (ctypes.c_uint8 * (n * world)).from_buffer_copy(b"".join(event_handles))
        arrs = [np.ascontiguousarray(a, dtype=np.int64) for a in (slot_bytes, src_off, recv_rows)]
        if any(a.shape != (world,) for a in arrs):
            raise ValueError(f"{world} entries per array expected")
        check(lib().dopt_lagged_ipc_import(self._h, int(world), int(rank), mh, eh, *[_ptr(a) for a in arrs],
                                           ctypes.c_void_p(int(counters_addr)), float(timeout_s)))

    def lagged_ipc_check(self, step):
        """dopt_lagged_ipc_check: step 0 publishes a record, step 1 pulls every peer's (each synchronous)."""
        check(lib().dopt_lagged_ipc_check(self._h, int(step)))

    def lagged_exchange(self):
        """dopt_lagged_exchange: the round's exchange through the attached communicator."""
        rc = lib().dopt_lagged_exchange(self._h)
        if rc:
            check(rc)

    def lagged_tail(self, consensus, objective, row1, row2):
        """row1 / row2: (cons, xnorm, loss) device addresses of the history rows G-1 / G-2 (None: skip)."""
        check(lib().dopt_lagged_tail(self._h, 1 if consensus else 0, 1 if objective else 0, *row1, *row2))

    def rs_phase_begin(self, commit):
        """(ok, hash): this rank's iterates all equal (row-space rounds possible) and the 64-bit
        content hash of that common iterate (of the replicated state when already live, as a
        signed int64); commit=True also enters row-space mode."""
        ok = ctypes.c_int(0)
        h = ctypes.c_uint64(0)
        check(lib().dopt_rs_phase_begin(self._h, 1 if commit else 0, ctypes.byref(ok), ctypes.byref(h)))
        v = int(h.value)
        return bool(ok.value), v - (1 << 64) if v >= (1 << 63) else v

    def rs_phase_round(self, t, eta0, lam_grad, metric_flags, sum_ptr):
        check(lib().dopt_rs_phase_round(self._h, int(t), float(eta0), float(lam_grad), int(metric_flags),
                                        ctypes.c_void_p(sum_ptr)))

    def rs_phase_cols(self, t, eta0, lam_grad, sum_ptr):
        check(lib().dopt_rs_phase_cols(self._h, int(t), float(eta0), float(lam_grad), ctypes.c_void_p(sum_ptr)))

    def rs_phase_cols_range(self, t, eta0, lam_grad, sum_ptr, c0, c1, last):
        """The average / Z update of round t for the columns [c0, c1) of one pass chunk (last=True on
        the round's last chunk: the update is complete)."""
        check(lib().dopt_rs_phase_cols_range(self._h, int(t), float(eta0), float(lam_grad), ctypes.c_void_p(sum_ptr),
                                             int(c0), int(c1), 1 if last else 0))

    def rs_phase_pass(self, chunk, n_chunks, sum_ptr):
        """The row-space pass over column chunk `chunk` of `n_chunks`; returns the column range
        (c0, c1) whose local sums it wrote to sum_ptr[c0:c1)."""
        rng = np.zeros(2, dtype=np.int64)
        check(lib().dopt_rs_phase_pass(self._h, int(chunk), int(n_chunks), ctypes.c_void_p(sum_ptr), _ptr(rng)))
        return int(rng[0]), int(rng[1])

    def rs_phase_rows(self, t, eta0, lam_grad, metric_flags):
        check(lib().dopt_rs_phase_rows(self._h, int(t), float(eta0), float(lam_grad), int(metric_flags)))

    def rs_phase_metrics(self, metric_flags):
        check(lib().dopt_rs_phase_metrics(self._h, int(metric_flags)))

    def sync(self):
        check(lib().dopt_sync(self._h))

    def eval_full(self, w, reg, gradient=True):
        """(objective, gradient) over all loaded rows at w, one device pass; gradient=False:
        (objective, None) -- the only form for column-blocked (large d) contexts."""
        w = np.ascontiguousarray(w, dtype=np.float64)
        g = np.empty(self.d, dtype=np.float64) if gradient else None
        f = np.zeros(1)
        check(lib().dopt_eval_full(self._h, _ptr(w), float(reg), _ptr(f), _ptr(g)))
        return float(f[0]), g

    def set_sampler(self, mode, seed=0, first_worker=0):
        """'host' (default: minibatch rounds need idx) or 'device' (Philox + Floyd draws on
        the GPU inside the pass over all rows; not the reference's RNG stream)."""
        m = {"host": SAMPLE_HOST, "device": SAMPLE_DEVICE}[mode] if isinstance(mode, str) else int(mode)
        check(lib().dopt_set_sampler(self._h, m, int(seed) & (2 ** 64 - 1), int(first_worker)))

    # -- profiling
    def set_profiling(self, on, every=1):
        """HIP-event timing of the round kernel: every `every`-th launch (0 / False: off)."""
        check(lib().dopt_set_profiling(self._h, int(every) if on else 0))

    def kernel_stats(self):
        n = ctypes.c_int64(0)
        ms = ctypes.c_double(0.0)
        check(lib().dopt_kernel_stats(self._h, ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value


def finalize_metrics(problem, raw, n_workers, m_obj, lam_obj, f_opt):
    """raw [T, 3] metric sums -> (objective, consensus) with the engine's own formula."""
    raw = np.ascontiguousarray(raw, dtype=np.float64).reshape(-1, 3)
    T = raw.shape[0]
    obj, cons = np.zeros(T), np.zeros(T)
    check(lib().dopt_finalize_metrics(PROBLEMS[problem], T, _ptr(raw), int(n_workers), int(m_obj),
                                      float(lam_obj), float(f_opt), _ptr(obj), _ptr(cons)))
    return obj, cons


_default = {}


def default_engine(device=None):
    """Float64 engine used by the obj_problems / Worker single-call API."""
    dev = int(os.environ.get("DOPT_DEVICE", "0")) if device is None else int(device)
    eng = _default.get(dev)
    if eng is None:
        eng = Engine(dev, "float64")
        _default[dev] = eng
    return eng
