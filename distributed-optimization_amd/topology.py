"""Topologies and Metropolis-Hastings mixing weights in CSR form.

Replaces the dense construction of DecentralizedTrainer._create_mixing_matrix
(trainer.py:91-136), which needs two N x N float64 matrices (64 GiB at
N = 65536).  Here a topology is a list of sorted neighbour ids per worker and
W is built directly in CSR with the diagonal included.

Bit-exactness with the reference: W_ij = 1 / (1 + max(d_i, d_j)) is one IEEE
division, and W_ii = 1 - np.sum(W[i, neighbours]) is evaluated with the same
numpy call on the same float64 vector the reference sums (neighbour weights in
ascending column order, 0.0 in the slot of a self loop), so every entry equals
the reference's W to the bit (tests/test_topology.py checks the fixtures).

Topologies:
  ring              trainer.py:95-98 (N = 1 gives a self loop, N = 2 degree 1)
  grid              trainer.py:99-108, nx.grid_2d_graph(side, side, periodic=True)
                    with row-major ids over sorted (r, c) nodes; side 2 has degree 2
  fully_connected   trainer.py:109-110
  random_regular    not in the reference: the random k-regular graph of
                    BASELINE.json config C3 (pairing model, fixed seed)
"""
from __future__ import annotations

import numpy as np


class Topology:
    """Neighbour lists + MH weights.  `row_ptr`, `col`, `w` include the diagonal."""

    def __init__(self, name, neighbours):
        self.name = name
        self.n = len(neighbours)
        self.neighbours = neighbours
        # reference degrees = row sums of the 0/1 adjacency (float64), self loop included
        self.degrees = np.array([float(len(nb)) for nb in neighbours], dtype=np.float64)
        self.row_ptr, self.col, self.w = _mh_csr(neighbours, self.degrees)

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def dense_adjacency(self):
        adj = np.zeros((self.n, self.n))
        for i, nb in enumerate(self.neighbours):
            adj[i, nb] = 1.0
        return adj

    def dense_W(self):
        W = np.zeros((self.n, self.n))
        for i in range(self.n):
            s, e = self.row_ptr[i], self.row_ptr[i + 1]
            W[i, self.col[s:e]] = self.w[s:e]
        return W

    def sparse_W(self):
        from scipy.sparse import csr_matrix

        return csr_matrix((self.w, self.col, self.row_ptr), shape=(self.n, self.n))

    def uniform_offdiag(self):
        """(w_off, diag) when every off-diagonal weight is present and equal (the
        complete graph), else None: then sum_j W_ij x_j = w_off (S - x_i) + W_ii x_i."""
        n = self.n
        if n < 2 or self.nnz != n * n:
            return None
        diag_mask = self.col == np.repeat(np.arange(n), n)
        off = self.w[~diag_mask]
        if not np.all(off == off[0]):
            return None
        return float(off[0]), self.w[diag_mask].copy()

    def check(self):
        """trainer.py:129-131 on the CSR form: rows sum to 1 and W is symmetric."""
        if self.n == 0:
            return
        rs = np.add.reduceat(self.w, self.row_ptr[:-1]) if self.nnz else np.zeros(self.n)
        assert np.allclose(rs, 1.0), f"Rows of W do not sum to 1 (Topology: {self.name})"
        S = self.sparse_W()
        assert abs(S - S.T).max() <= 1e-8 + 1e-5 * abs(S).max(), f"W is not symmetric (Topology: {self.name})"

    def spectral_gap(self, dense_limit=4096):
        """trainer.py:133-135: 1 - (second largest |eigenvalue|).  Dense eigvalsh up to
        `dense_limit` workers, Lanczos (scipy eigsh) on the CSR matrix above it."""
        if self.n <= 1:
            return None
        if self.n <= dense_limit:
            ev = np.linalg.eigvalsh(self.dense_W())
            return 1.0 - np.sort(np.abs(ev))[-2]
        from scipy.sparse.linalg import eigsh

        ev = eigsh(self.sparse_W(), k=2, which="LM", return_eigenvectors=False, tol=1e-10)
        return 1.0 - np.sort(np.abs(ev))[0]


def _mh_csr(neighbours, degrees):
    n = len(neighbours)
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    cols, vals = [], []
    for i, nb in enumerate(neighbours):
        nb = np.asarray(nb, dtype=np.int64)
        # off-diagonal weights, one IEEE division each (trainer.py:125)
        wn = 1.0 / (1.0 + np.maximum(degrees[i], degrees[nb]))
        wn[nb == i] = 0.0  # W[i, i] is still 0 when the reference sums the row
        wii = 1.0 - np.sum(wn)  # trainer.py:126, same numpy reduction on the same vector
        if np.any(nb == i):
            row_c, row_w = nb, wn.copy()
            row_w[nb == i] = wii
        else:
            pos = int(np.searchsorted(nb, i))
            row_c = np.concatenate([nb[:pos], [i], nb[pos:]])
            row_w = np.concatenate([wn[:pos], [wii], wn[pos:]])
        cols.append(row_c)
        vals.append(row_w)
        row_ptr[i + 1] = row_ptr[i] + len(row_c)
    col = np.concatenate(cols).astype(np.int32) if cols else np.zeros(0, np.int32)
    w = np.concatenate(vals).astype(np.float64) if vals else np.zeros(0)
    return row_ptr, col, w


def ring(n):
    nbrs = []
    for i in range(n):
        nbrs.append(sorted({(i + 1) % n, (i - 1 + n) % n}))
    return Topology("ring", nbrs)


def grid(n):
    side = int(np.sqrt(n))
    if side * side != n:
        raise ValueError(f"Warning: N_WORKERS ({n}) is not a perfect square.")
    nbrs = [set() for _ in range(n)]
    for r in range(side):
        for c in range(side):
            u = r * side + c
            for v in (((r + 1) % side) * side + c, r * side + (c + 1) % side):
                if u != v:  # nx.grid_2d_graph has no self loops
                    nbrs[u].add(v)
                    nbrs[v].add(u)
    return Topology("grid", [sorted(s) for s in nbrs])


def fully_connected(n):
    allv = np.arange(n)
    return Topology("fully_connected", [np.delete(allv, i) for i in range(n)])


def random_regular(n, k, seed=0, max_tries=10000):
    """Uniform-ish random simple k-regular graph by the pairing model with restarts."""
    if (n * k) % 2 or k >= n:
        raise ValueError(f"no simple {k}-regular graph on {n} vertices")
    rng = np.random.default_rng(seed)
    stubs = np.repeat(np.arange(n), k)
    for _ in range(max_tries):
        p = rng.permutation(stubs).reshape(-1, 2)
        a, b = p[:, 0], p[:, 1]
        if np.any(a == b):
            continue
        lo, hi = np.minimum(a, b), np.maximum(a, b)
        key = lo.astype(np.int64) * n + hi
        if len(np.unique(key)) != len(key):
            continue
        nbrs = [[] for _ in range(n)]
        for u, v in zip(lo.tolist(), hi.tolist()):
            nbrs[u].append(v)
            nbrs[v].append(u)
        return Topology("random_regular", [sorted(x) for x in nbrs])
    raise RuntimeError("random_regular: no simple graph found")


def relabel(topo, order):
    """The same graph with new vertex ids: new id k is old vertex order[k] (a permutation).
    MH weights are recomputed on the new ids (per edge the same value; W_ii can differ in
    the last bit, as it sums the row in the new column order)."""
    order = np.asarray(order, dtype=np.int64)
    inv = np.empty_like(order)
    inv[order] = np.arange(len(order))
    nbrs = [np.sort(inv[np.asarray(topo.neighbours[o], dtype=np.int64)]) for o in order]
    return Topology(topo.name, nbrs)


def build(name, n, config=None):
    """trainer.py:95-112 dispatch; unknown names raise the reference's ValueError."""
    config = config or {}
    if name == "ring":
        return ring(n)
    if name == "grid":
        return grid(n)
    if name == "fully_connected":
        return fully_connected(n)
    if name == "random_regular":
        return random_regular(n, int(config.get("regular_degree", 4)), int(config.get("topology_seed", 0)))
    raise ValueError(f"Wrong topology: {name}")
