"""CPU oracle for the D-SGD round -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the HIP engine.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only
as the checker (or the timed CPU baseline), never as part of the product path.

It is a from-scratch numpy restatement of the reference's hot path
(scavenx/distributed-optimization @ /root/reference), written in the plainest
per-worker form so it reads against the reference line by line:

  objectives / gradients ........ obj_problems.py:3-20 (logistic), :39-53 (quadratic),
                                  :22-36 / :55-69 (full-data gradients, dead code upstream)
  minibatch sampling ............ worker.py:15-28 (np.random.choice == legacy
                                  MT19937 permutation(m)[:b]; numpy itself is the
                                  reference's RNG, so it is used here as is)
  gradient dispatch ............. worker.py:30-44 (lambda for logistic, mu for quadratic)
  MH mixing matrix .............. trainer.py:91-136
  learning rate ................. trainer.py:138-140  eta0 / sqrt(t+1)
  D-SGD round + metrics ......... trainer.py:154-197
  centralized round ............. trainer.py:33-74

Pinning: every function here is checked against the golden fixtures in
tests/golden/ that tests/golden/make_golden.py produced by importing and running
the reference itself (test_oracle_golden.py).  The fixtures reproduce the
report's Table II exactly (5425 / 7214 / 5666 / 5549 iterations).

dtype=np.float32 runs the same algorithm in fp32 numpy (the fp32 CPU
restatement used to bound the fp32 GPU path); dtype=np.float64 is the parity mode.
The partitioned variant (`run_decentralized(..., partitions=P)`) splits workers
into P contiguous ranges, copies every remote neighbour row into a halo buffer
explicitly, mixes from local+halo only, and must equal the unpartitioned round
bit for bit (last paragraph).
"""
from __future__ import annotations

import numpy as np
from scipy.special import expit

# --------------------------------------------------------------------------- objectives


def logistic_objective(w, X, y, lam):
    """obj_problems.py:3-11 (np.log(1 + ...), not log1p; regulariser includes the bias)."""
    if X.shape[0] == 0:
        return 0.0
    z = X @ w
    yz = y * z
    t = np.maximum(0, -yz) + np.log(1 + np.exp(-np.abs(yz)))
    return np.mean(t) + (lam / 2.0) * np.dot(w, w)


def logistic_gradient(w, Xb, yb, lam):
    """obj_problems.py:13-20."""
    if Xb.shape[0] == 0:
        return np.zeros_like(w)
    z = Xb @ w
    p = expit(-yb * z)
    return np.mean(-yb[:, None] * Xb * p[:, None], axis=0) + lam * w


def quadratic_objective(w, X, y, mu):
    """obj_problems.py:39-44."""
    if X.shape[0] == 0:
        return 0.0
    e = X @ w - y
    return 0.5 * np.mean(e ** 2) + (mu / 2.0) * np.dot(w, w)


def quadratic_gradient(w, Xb, yb, mu):
    """obj_problems.py:46-53."""
    if Xb.shape[0] == 0:
        return np.zeros_like(w)
    e = Xb @ w - yb
    return np.mean(Xb * e[:, None], axis=0) + mu * w


def full_gradient(problem, w, shards, reg):
    """obj_problems.py:22-36 / :55-69: sum over every shard, divided by the row count."""
    acc = np.zeros_like(w)
    n = 0
    for X, y in shards:
        if X.shape[0] == 0:
            continue
        z = X @ w
        if problem == "logistic":
            acc = acc + np.sum(-y[:, None] * X * expit(-y * z)[:, None], axis=0)
        else:
            acc = acc + np.sum(X * (z - y)[:, None], axis=0)
        n += X.shape[0]
    if n == 0:
        return np.zeros_like(w)
    return acc / n + reg * w


def objective(problem, w, X, y, reg):
    if problem == "logistic":
        return logistic_objective(w, X, y, reg)
    if problem == "quadratic":
        return quadratic_objective(w, X, y, reg)
    raise NotImplementedError(f"Wrong {problem}")


def gradient(problem, w, Xb, yb, config):
    """worker.py:36-44: logistic uses l2_regularization_lambda, quadratic strong_convexity_mu."""
    if problem == "logistic":
        return logistic_gradient(w, Xb, yb, config["l2_regularization_lambda"])
    if problem == "quadratic":
        return quadratic_gradient(w, Xb, yb, config["strong_convexity_mu"])
    raise NotImplementedError(f"Wrong {problem}")


# --------------------------------------------------------------------------- sampling


def minibatch_indices(rs, m, b):
    """worker.py:15-28 on RandomState `rs`: empty shard -> no draw; else choice(m, min(b,m))."""
    if m == 0:
        return np.zeros(0, dtype=np.int64)
    eb = min(b, m)
    if eb <= 0:
        return np.zeros(0, dtype=np.int64)
    return rs.choice(m, eb, replace=eb > m)


# --------------------------------------------------------------------------- topology


def adjacency(topology, n):
    """trainer.py:93-112, dense (small N only).  Torus ids are row-major (r, c)."""
    adj = np.zeros((n, n))
    if topology == "ring":
        for i in range(n):
            adj[i, (i + 1) % n] = 1
            adj[i, (i - 1 + n) % n] = 1
    elif topology == "grid":
        side = int(np.sqrt(n))
        if side * side != n:
            raise ValueError(f"Warning: N_WORKERS ({n}) is not a perfect square.")
        # nx.grid_2d_graph(side, side, periodic=True): simple graph, no self loops
        for r in range(side):
            for c in range(side):
                u = r * side + c
                for rr, cc in (((r + 1) % side, c), (r, (c + 1) % side)):
                    v = rr * side + cc
                    if u != v:
                        adj[u, v] = 1
                        adj[v, u] = 1
    elif topology == "fully_connected":
        adj = np.ones((n, n)) - np.eye(n)
    else:
        raise ValueError(f"Wrong topology: {topology}")
    return adj


def mh_matrix(adj):
    """trainer.py:114-126: W_ij = 1/(1+max(d_i,d_j)), W_ii = 1 - sum(W[i, neighbours])."""
    n = adj.shape[0]
    deg = np.sum(adj, axis=1)
    W = np.zeros((n, n))
    for i in range(n):
        nb = np.where(adj[i, :] > 0)[0]
        for j in nb:
            if i != j:
                W[i, j] = 1.0 / (1.0 + max(deg[i], deg[j]))
        W[i, i] = 1.0 - np.sum(W[i, nb])
    return W, deg


def spectral_gap(W):
    """trainer.py:133-135."""
    ev = np.linalg.eigvalsh(W)
    return 1.0 - np.sort(np.abs(ev))[-2]


# --------------------------------------------------------------------------- rounds


def _lr(eta0, t):
    return eta0 / np.sqrt(t + 1)  # trainer.py:138-140


def _mix(W, X, partitions):
    """Dense W @ X, or the partitioned form with explicit halo copies."""
    if partitions is None or partitions <= 1:
        return W @ X
    n = W.shape[0]
    bounds = np.linspace(0, n, partitions + 1).astype(np.int64)
    out = np.empty_like(X)
    for p in range(partitions):
        lo, hi = bounds[p], bounds[p + 1]
        rows = W[lo:hi]
        cols = np.where(np.any(rows != 0, axis=0))[0]
        halo = cols[(cols < lo) | (cols >= hi)]
        halo_buf = X[halo].copy()  # the "received" boundary iterates
        for i in range(lo, hi):
            acc = np.zeros(X.shape[1], dtype=X.dtype)
            nz = np.where(W[i] != 0)[0]
            for j in nz:  # ascending column order, same as the unpartitioned sparse sum
                src = X[j] if lo <= j < hi else halo_buf[np.searchsorted(halo, j)]
                acc = acc + W[i, j].astype(X.dtype) * src
            out[i] = acc
    return out


def _mix_sparse(W, X):
    out = np.empty_like(X)
    for i in range(W.shape[0]):
        acc = np.zeros(X.shape[1], dtype=X.dtype)
        for j in np.where(W[i] != 0)[0]:
            acc = acc + W[i, j].astype(X.dtype) * X[j]
        out[i] = acc
    return out


def run_decentralized(shards, W, T, config, X_full=None, y_full=None, f_opt=0.0,
                      rng_state=None, dtype=np.float64, mixing="dense", partitions=None,
                      x0=None, indices=None):
    """trainer.py:154-197 for the worker shards [(X_i, y_i)].

    Returns (history, final_avg_model, final_models, rng_state_after).
    `indices[t][i]` overrides sampling (same index vectors the RNG would draw).
    """
    problem = config["problem_type"]
    b = config["local_batch_size"]
    reg_obj = config["l2_regularization_lambda"]  # trainer.py:151-152,189 (both problems)
    n = len(shards)
    d = shards[0][0].shape[1]
    rs = np.random.RandomState()
    if rng_state is not None:
        rs.set_state(rng_state)
    Xs = [(np.asarray(X, dtype=dtype), np.asarray(y, dtype=dtype)) for X, y in shards]
    Wd = W.astype(dtype)
    models = np.zeros((n, d), dtype=dtype) if x0 is None else np.array(x0, dtype=dtype)
    if X_full is not None:
        Xf, yf = np.asarray(X_full, dtype=dtype), np.asarray(y_full, dtype=dtype)
    hist = {"objective": [], "consensus_error": [], "time": []}
    for t in range(T):
        grads = np.zeros_like(models)
        for i, (X, y) in enumerate(Xs):
            idx = indices[t][i] if indices is not None else minibatch_indices(rs, X.shape[0], b)
            grads[i] = gradient(problem, models[i], X[idx], y[idx], config)
        if mixing == "dense" and not partitions:
            mixed = Wd @ models
        elif partitions:
            mixed = _mix(Wd, models, partitions)
        else:
            mixed = _mix_sparse(Wd, models)
        eta = _lr(config["learning_rate_eta0"], t)
        models = mixed - np.asarray(eta, dtype=dtype) * grads
        avg = np.mean(models, axis=0)
        hist["consensus_error"].append(float(np.mean([np.linalg.norm(models[i] - avg) ** 2 for i in range(n)])))
        if X_full is not None:
            hist["objective"].append(float(objective(problem, avg, Xf, yf, reg_obj) - f_opt))
        hist["time"].append(0.0)
    return hist, np.mean(models, axis=0), models, rs.get_state()


def run_centralized(shards, T, config, X_full=None, y_full=None, f_opt=0.0,
                    rng_state=None, dtype=np.float64, indices=None):
    """trainer.py:33-74."""
    problem = config["problem_type"]
    b = config["local_batch_size"]
    reg_obj = config["l2_regularization_lambda"]
    d = shards[0][0].shape[1]
    rs = np.random.RandomState()
    if rng_state is not None:
        rs.set_state(rng_state)
    Xs = [(np.asarray(X, dtype=dtype), np.asarray(y, dtype=dtype)) for X, y in shards]
    x = np.zeros(d, dtype=dtype)
    if X_full is not None:
        Xf, yf = np.asarray(X_full, dtype=dtype), np.asarray(y_full, dtype=dtype)
    hist = {"objective": [], "time": []}
    for t in range(T):
        cur = x.copy()
        gs = []
        for i, (X, y) in enumerate(Xs):
            idx = indices[t][i] if indices is not None else minibatch_indices(rs, X.shape[0], b)
            gs.append(gradient(problem, cur, X[idx], y[idx], config))
        g = np.mean(gs, axis=0)
        x = x - np.asarray(_lr(config["learning_rate_eta0"], t), dtype=dtype) * g
        if X_full is not None:
            hist["objective"].append(float(objective(problem, x, Xf, yf, reg_obj) - f_opt))
        hist["time"].append(0.0)
    return hist, x, rs.get_state()


def iterations_to_threshold(objective_history, threshold):
    """simulator.py:71-79."""
    h = np.asarray(objective_history)
    if len(h) == 0:
        return -1
    hit = np.where(h <= threshold)[0]
    return int(hit[0] + 1) if len(hit) else -1
