"""Multi-GPU D-SGD: one process per GPU, contiguous worker slices, halo exchange.

The reference simulates every worker in one process (trainer.py:161-193).  Here
rank r of a torch.distributed job (backend "nccl" = RCCL over xGMI on MI355X;
"gloo" in tests) owns workers [lo_r, hi_r) -- their shards, iterates and rows of
W -- on its own GPU.  Per round:

  gather x_t rows the peers need --> all-to-all of the halo rows ---.
  gradient of every local worker at x_t (+ metrics of x_t) ---------+--> mix + step
  local column sums --> all_reduce(d doubles) --> xbar_{t+1}

The mix uses the same CSR entry order as the single-GPU kernel, so the iterates
are bitwise the single-GPU iterates; only the metric sums are reduced in a
different order (per rank, then across ranks).  Metric partial sums stay on the
device per round and are all-reduced once per run.

With CSR mixing and metrics that ride the gradient pass the rounds run LAGGED
(`_run_lagged`): the column sums of x_t are all-reduced while the gradient kernel of
round t runs, and that kernel's fused objective pass is taken at xbar_{t-1}
(history[t-2]) instead of xbar_t; the mix kernel forms xbar_t from the reduced sums
and the consensus of x_t from the rows it reads anyway.  So no collective sits
between two rounds' kernels; the halo exchange of x_t overlaps the same gradient
kernel, and the mix kernel writes the next round's send rows (no gather kernel).

Plan construction (`build_plan`) is pure host logic over the global CSR, so it
is tested on CPU with gloo against the oracle (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

import _dopt


DEFAULT_TIMEOUT_S = 300.0
# Column chunks of the complete graph's row-space pass across ranks, pipelined across rounds:
# chunk k's sums are all-reduced while the later chunks stream, and round h's average update of chunk k runs
# just before round h + 1's pass over chunk k, so only what the next round's earlier chunks cannot cover of
# the last chunk's all-reduce stays exposed; every extra chunk costs a launch boundary and a hand-off.
# The model that picks the chunk count per world size ("Column chunks across ranks"): exposed
# time (K - 1) * boundary + max(0, allreduce(S / K, N) - (K - 1) / K * pass(N)), where the ring all-reduce of
# S bytes over N ranks on xGMI costs ALPHA + 2 (N - 1) / N * S / BUSBW (assumed: no multi-GPU run here to
# measure them on) and the pass of one rank reads 68.7 GB / N at 6.5 TB/s.
AR_ALPHA_S = 30e-6       # per all-reduce latency (8 ranks, ring steps, launch): assumed
AR_BUSBW = 100e9         # RCCL bus bandwidth for MB-sized messages over xGMI, bytes/s: assumed
RS_BOUNDARY_S = 15e-6    # one extra chunk (boundary + hand-off), measured at one rank's shape of 8 (128 workers,
                         # RCCL world 1 forced, K = 2 / 4 vs 1: 0-12 / 13 us per chunk; profiles/r5_rs_chunks.txt)
RS_PASS_BYTES = 68.72e9  # C5's row bytes per round (all ranks)
RS_PASS_BW = 6.5e12


def rs_chunks_for(world, sum_bytes=8 << 20, max_chunks=8, pass_bytes=RS_PASS_BYTES):
    """Chunk count K (a power of two: chunks of equal column blocks -- 3 chunks of C5's 2048 blocks cost
    0.4 ms at world 1) minimising the modelled exposed time; 1 at world 1 (nothing to overlap).  With
    the constants above it is 2 for 2-8 ranks: the half all-reduce of the last chunk hides behind the
    next round's first chunk, for one ~15 us boundary."""
    if world <= 1:
        return 1
    pass_s = pass_bytes / world / RS_PASS_BW

    def exposed(k):
        ar = AR_ALPHA_S + 2.0 * (world - 1) / world * (sum_bytes / k) / AR_BUSBW
        return (k - 1) * RS_BOUNDARY_S + max(0.0, ar - (k - 1) / k * pass_s)

    ks = [k for k in (1, 2, 4, 8, 16) if k <= max_chunks]
    return min(ks, key=exposed)


class CollectiveError(RuntimeError):
    """A collective or halo transfer of the round failed or timed out on this rank (peer and
    operation named), instead of a hang until the driver's limit."""


def timeout_seconds():
    """Bound on every collective of a job (DOPT_PG_TIMEOUT seconds, default 300): a peer that
    never joins a send/recv or all-reduce ends the job with an error within this time."""
    return float(os.environ.get("DOPT_PG_TIMEOUT", DEFAULT_TIMEOUT_S))


def init_process_group(backend, timeout=None, **kw):
    """torch.distributed.init_process_group with a bounded collective timeout (`timeout`
    seconds, default timeout_seconds()); for "nccl" (RCCL) with high-priority internal
    streams, so the halo send/recv and the all-reduce of a round get CU slots ahead of the
    4096-workgroup gradient kernel they overlap.
    With RCCL the watchdog aborts a rank whose collective exceeds the timeout (the work, its
    sequence number and op type in the message) and the launcher ends the other ranks; with
    gloo the waiting call raises, which the transport below turns into CollectiveError."""
    import datetime

    import torch.distributed as dist

    kw.setdefault("timeout", datetime.timedelta(seconds=timeout if timeout is not None else timeout_seconds()))
    if backend == "nccl":
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        opts._timeout = kw["timeout"]  # the options carry the job's bound too (no override warning)
        kw["pg_options"] = opts
    dist.init_process_group(backend, **kw)


def _wait(work, what, rank, timeout_s=None):
    """work.wait(), with a failure or timeout re-raised as CollectiveError naming the rank and
    the operation (`what`: op and peer).  For RCCL works the wait only orders the current
    stream after the transfer (no host block); the process group's watchdog bounds them."""
    import datetime

    try:
        if timeout_s is None:
            work.wait()
        else:
            work.wait(datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # gloo: timeout / peer gone; RCCL: aborted communicator
        raise CollectiveError(f"rank {rank}: {what} failed: {e}") from e


def partition_bounds(n, world):
    """Contiguous slices, np.array_split sizes (the first n % world ranks get one more)."""
    sizes = [n // world + (1 if r < n % world else 0) for r in range(world)]
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)


def _adjacency(topo):
    from scipy.sparse import csr_matrix

    rows = np.repeat(np.arange(topo.n), np.diff(topo.row_ptr))
    cols = topo.col.astype(np.int64)
    off = rows != cols
    return csr_matrix((np.ones(int(off.sum())), (rows[off], cols[off])), shape=(topo.n, topo.n))


def _fiedler(A, seed):
    """Second-smallest Laplacian eigenvector (Lanczos on c I - L, a fixed start vector)."""
    from scipy.sparse import diags
    from scipy.sparse.linalg import eigsh

    deg = np.asarray(A.sum(axis=1)).ravel()
    M = diags(2.0 * deg.max() + 1.0 - deg) + A
    v0 = np.random.default_rng(seed).standard_normal(A.shape[0])
    w, V = eigsh(M, k=2, which="LA", v0=v0, tol=1e-6, maxiter=20000)
    return V[:, np.argsort(w)[0]]


def _refine(A, right, passes=20):
    """Balanced greedy refinement of a bisection: swap the best-gain vertices of the two
    sides pairwise while a pair's gain exceeds what their mutual edge could cost."""
    deg = np.asarray(A.sum(axis=1)).ravel()
    for _ in range(passes):
        on_right = A @ right.astype(np.float64)
        ext = np.where(right, deg - on_right, on_right)
        gain = 2.0 * ext - deg  # cut edges removed by moving the vertex alone
        lv, rv = np.where(~right)[0], np.where(right)[0]
        lv = lv[np.argsort(-gain[lv], kind="stable")]
        rv = rv[np.argsort(-gain[rv], kind="stable")]
        k = min(len(lv), len(rv))
        good = int(np.sum(gain[lv[:k]] + gain[rv[:k]] > 2.0))
        if good == 0:
            break
        take = max(1, good // 2)  # half the candidates per pass: their gains interact
        right[lv[:take]] = True
        right[rv[:take]] = False
    return right


def graph_partition(topo, parts, seed=0):
    """Worker -> rank for `parts` ranks by recursive spectral bisection (Fiedler vector of
    the graph Laplacian) with balanced greedy refinement; part r gets exactly the
    partition_bounds(n, parts) size of slice r.  On a random 4-regular graph it cuts
    2.5x (8 parts) to 3x (2 parts) fewer edges than contiguous id ranges, i.e. that many
    fewer halo rows per round.  Deterministic for a given seed (run it on one rank and
    broadcast the result: eigensolvers are not bitwise reproducible across libraries)."""
    n = topo.n
    sizes = np.diff(partition_bounds(n, parts))
    part = np.zeros(n, dtype=np.int32)
    A = _adjacency(topo)

    def split(ids, p0, p1):
        if p1 - p0 == 1:
            part[ids] = p0
            return
        mid = (p0 + p1) // 2
        n_left = int(sizes[p0:mid].sum())
        sub = A[ids][:, ids]
        right = np.ones(len(ids), dtype=bool)
        if n_left > 0 and len(ids) > 2 and sub.nnz:
            right[np.argsort(_fiedler(sub, seed), kind="stable")[:n_left]] = False
            right = _refine(sub, right)
        else:
            right[:n_left] = False
        split(ids[~right], p0, mid)
        split(ids[right], mid, p1)

    split(np.arange(n), 0, parts)
    return part


def partition_order(part):
    """Relabelling that makes every part a contiguous id range (topology.relabel order)."""
    return np.argsort(part, kind="stable")


def cut_edges(topo, part):
    A = _adjacency(topo).tocoo()
    return int(np.sum(part[A.row] != part[A.col]) // 2)


@dataclass
class HaloPlan:
    rank: int
    world: int
    bounds: np.ndarray      # [world+1] global worker ranges
    lo: int
    hi: int
    halo_ids: np.ndarray    # [n_halo] global ids of the remote rows this rank reads, ascending
    recv_off: np.ndarray    # [world+1] halo rows coming from each peer (contiguous blocks)
    send_ids: np.ndarray    # [n_send] LOCAL ids of rows peers need, grouped by peer, ascending
    send_off: np.ndarray    # [world+1]
    row_ptr: np.ndarray     # local CSR, columns in local (< n_local) + halo (>= n_local) space
    col: np.ndarray
    w: np.ndarray

    @property
    def n_local(self):
        return self.hi - self.lo

    @property
    def n_halo(self):
        return len(self.halo_ids)

    def peers(self):
        return [p for p in range(self.world) if p != self.rank and
                (self.send_off[p + 1] > self.send_off[p] or self.recv_off[p + 1] > self.recv_off[p])]


def build_plan(topo, world, rank):
    """Halo plan of `rank` for a topology.Topology (global CSR incl. diagonal)."""
    bounds = partition_bounds(topo.n, world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    e0, e1 = topo.row_ptr[lo], topo.row_ptr[hi]
    cols = topo.col[e0:e1].astype(np.int64)
    remote = np.unique(cols[(cols < lo) | (cols >= hi)])
    n_local = hi - lo
    local_col = np.where((cols >= lo) & (cols < hi), cols - lo, n_local + np.searchsorted(remote, cols))
    recv_off = np.searchsorted(remote, bounds).astype(np.int64)
    send, send_off = [], [0]
    for p in range(world):
        if p != rank:
            pc = topo.col[topo.row_ptr[bounds[p]]:topo.row_ptr[bounds[p + 1]]].astype(np.int64)
            need = np.unique(pc[(pc >= lo) & (pc < hi)])
            send.append(need - lo)
        else:
            send.append(np.zeros(0, np.int64))
        send_off.append(send_off[-1] + len(send[-1]))
    return HaloPlan(rank=rank, world=world, bounds=bounds, lo=lo, hi=hi, halo_ids=remote, recv_off=recv_off,
                    send_ids=np.concatenate(send).astype(np.int32), send_off=np.array(send_off, np.int64),
                    row_ptr=(topo.row_ptr[lo:hi + 1] - e0).astype(np.int64), col=local_col.astype(np.int32),
                    w=topo.w[e0:e1].copy())


@dataclass
class ExchangeLayout:
    """Send / halo buffer rows of the lagged schedule's exchange (round 4): per peer p in rank order
    (p != rank), p's plan rows, then `ks` rows holding this rank's (send) or p's (halo) float64 column
    sums of the current iterates (ks = 8 / element bytes: one row of float64, two of float32).  One
    all-to-all-v per round then moves the halo rows and the sums every rank needs for xbar; every
    peer gets a block (the sums), so every pair of ranks exchanges each round."""
    ks: int
    send_sizes: list        # [world] rows per peer block of the send buffer
    recv_sizes: list        # [world] rows per peer block of the halo buffer
    send_rows: np.ndarray   # [n_send] buffer row of plan send slot k
    halo_rows: np.ndarray   # [n_halo] buffer row of plan halo row j
    sum_send_row: np.ndarray  # [world] send-buffer row of the sums for peer p (-1: self)
    sum_recv_row: np.ndarray  # [world] halo-buffer row of peer p's sums (-1: self)

    @property
    def n_send_rows(self):
        return int(sum(self.send_sizes))

    @property
    def n_recv_rows(self):
        return int(sum(self.recv_sizes))

    def send_ids(self, plan):
        """Local worker of every send-buffer row, -1 on the sum rows (dopt_set_halo)."""
        ids = np.full(self.n_send_rows, -1, dtype=np.int32)
        ids[self.send_rows] = plan.send_ids
        return ids

    def local_col(self, plan):
        """The plan's local CSR columns with halo columns moved to their buffer rows."""
        col = plan.col.astype(np.int64).copy()
        h = col >= plan.n_local
        col[h] = plan.n_local + self.halo_rows[col[h] - plan.n_local]
        return col.astype(np.int32)


def exchange_layout(plan, ks, self_block=False):
    """ExchangeLayout of a HaloPlan with ks sum rows per peer (ks = 0: the plan's rows only).
    self_block: this rank gets a block too -- its own plan rows (if any) and sum rows, sent to itself
    -- so the one-GPU rehearsal of the RCCL path (world 1, collectives forced) moves real rows
    through the all-to-all and the mix reads them back from the halo buffer."""
    W, r = plan.world, plan.rank

    def shift(p):  # sum rows of the blocks before rank p's rows
        p = np.asarray(p)
        return ks * (p if self_block else p - (p > r))

    def block(off, p):
        return int(off[p + 1] - off[p]) + ks if (p != r or self_block) else 0

    send_sizes = [block(plan.send_off, p) for p in range(W)]
    recv_sizes = [block(plan.recv_off, p) for p in range(W)]
    k = np.arange(len(plan.send_ids))
    send_rows = k + shift(np.searchsorted(plan.send_off, k, side="right") - 1)
    j = np.arange(plan.n_halo)
    halo_rows = j + shift(np.searchsorted(plan.recv_off, j, side="right") - 1)
    ps = np.arange(W)
    mine = (ps == r) & (not self_block)
    sum_send = np.where(mine, -1, plan.send_off[1:] + shift(ps)).astype(np.int64)
    sum_recv = np.where(mine, -1, plan.recv_off[1:] + shift(ps)).astype(np.int64)
    if ks == 0:
        sum_send[:] = -1
        sum_recv[:] = -1
    return ExchangeLayout(ks, send_sizes, recv_sizes, send_rows.astype(np.int64), halo_rows.astype(np.int64),
                          sum_send, sum_recv)


class _StreamOrdered:
    """The 'work' of a collective that ProcessGroupNCCL enqueued on the caller's stream (asyncOp=False):
    wait() makes the current stream wait for that stream's work so far (the host does not block)."""

    def __init__(self, stream):
        self.stream = stream

    def wait(self, timeout=None):
        import torch

        torch.cuda.current_stream().wait_stream(self.stream)


class HaloExchange:
    """The per-round halo transfer of a HaloPlan: rows send[send_off[p]:send_off[p+1]] go to
    peer p, rows halo[recv_off[p]:recv_off[p+1]] come from peer p.

    RCCL (device_comm): the whole exchange is ONE all_to_all_single over the device buffers --
    the send rows are grouped by peer and the halo rows come in per-peer blocks, exactly the
    split layout of an all-to-all-v -- enqueued behind the current stream's work; finish() makes
    the current stream wait for it (the host does not block; the process group's watchdog
    bounds it).  One collective call per round instead of an isend and an irecv per peer (14
    P2P ops per rank at 8 ranks on the spectral partition of C3's graph), so the host's issue
    cost per round stays far below a round kernel even at the strong leg's 512 workers per rank
    (~0.19 ms per round).  Every rank of the group joins it each round, with or without rows
    to move (zero split sizes).  gloo: per-peer isend / irecv through host memory, and finish()
    waits on the host with the job's timeout, so a peer that never sends ends this rank with a
    CollectiveError naming it."""

    def __init__(self, plan, send, halo, group=None, device_comm=False, layout=None):
        """layout: an ExchangeLayout (the blocks carry column-sum rows too), or None: the plan's rows."""
        import torch.distributed as dist

        self.dist, self.plan, self.group, self.device_comm = dist, plan, group, device_comm
        self.send, self.halo = send, halo
        self.rank = plan.rank
        # the RCCL all-to-all: at world > 1, or at world 1 with the collectives forced (the one-GPU
        # box runs the call then, with zero rows or rows to itself)
        self.collective = device_comm and (plan.world > 1 or os.environ.get("DOPT_FORCE_COLLECTIVES") == "1")
        if layout is None:
            self.send_sizes = [int(plan.send_off[p + 1] - plan.send_off[p]) for p in range(plan.world)]
            self.recv_sizes = [int(plan.recv_off[p + 1] - plan.recv_off[p]) for p in range(plan.world)]
        else:
            self.send_sizes, self.recv_sizes = list(layout.send_sizes), list(layout.recv_sizes)
        self.send_off = np.concatenate([[0], np.cumsum(self.send_sizes)]).astype(np.int64)
        self.recv_off = np.concatenate([[0], np.cumsum(self.recv_sizes)]).astype(np.int64)
        self.peers = [p for p in range(plan.world) if p != self.rank and (self.send_sizes[p] or self.recv_sizes[p])]
        self.ns, self.nr = int(self.send_off[-1]), int(self.recv_off[-1])
        self.what = f"all_to_all_single of {self.ns} rows out / {self.nr} halo rows in (peers {self.peers})"
        self._direct = None
        if self.collective:  # the process group's all-to-all-v, called as dist.all_to_all_single calls it,
            try:             # minus its per-call argument checks (host cost per round: VERDICT r3 item 3)
                opts = dist.AllToAllOptions()
                # on the process group's stream, behind the current stream's work (the round-5 A/B against
                # asyncOp=False on the current stream: the engine then waited ~24 us longer per round)
                pg = group if group is not None else dist.distributed_c10d._get_default_group()
                self._direct = (pg.alltoall_base, self.halo[:self.nr], self.send[:self.ns], opts)
            except (AttributeError, RuntimeError):
                self._direct = None

    def disable(self):
        """No exchange at all (complete-graph mixing on every rank: no rows move)."""
        self.peers = []
        self.collective = False

    def peers_or_collective(self):
        """True when start() moves anything (a collective, or host transfers with peers)."""
        return bool(self.collective or self.peers)

    def _ops(self, send, halo):
        """(kind, peer, buffer, rows) for every transfer, sends first per peer, peers ascending."""
        for p in self.peers:
            s0, s1 = self.send_off[p], self.send_off[p + 1]
            r0, r1 = self.recv_off[p], self.recv_off[p + 1]
            if s1 > s0:
                yield "isend", p, send[s0:s1], int(s1 - s0)
            if r1 > r0:
                yield "irecv", p, halo[r0:r1], int(r1 - r0)

    def start(self):
        dist = self.dist
        if self.collective:
            if self._direct is not None:
                fn, out, inp, opts = self._direct
                w = fn(out, inp, self.recv_sizes, self.send_sizes, opts)
                if w is None:  # asyncOp=False: enqueued on the current stream; finish() orders after it
                    import torch

                    w = _StreamOrdered(torch.cuda.current_stream())
                return [(w, self.what)]
            w = dist.all_to_all_single(self.halo[:self.nr], self.send[:self.ns], output_split_sizes=self.recv_sizes,
                                       input_split_sizes=self.send_sizes, group=self.group, async_op=True)
            return [(w, self.what)]
        if not self.peers or self.device_comm:
            return None
        send = self.send.cpu()
        halo = self.halo.cpu()
        works = []
        for k, p, buf, rows in self._ops(send, halo):
            fn = dist.isend if k == "isend" else dist.irecv
            what = f"{k} of {rows} halo rows {'to' if k == 'isend' else 'from'} rank {p}"
            works.append((fn(buf, p, group=self.group), what))
        for w, what in works:
            _wait(w, what, self.rank, timeout_seconds())
        if halo.data_ptr() != self.halo.data_ptr():
            self.halo.copy_(halo)
        return None

    def finish(self, works):
        for w, what in works or ():
            _wait(w, what, self.rank)


_STREAMS = {}
_COMMS = {}


def transport_kind():
    """The lagged schedule's exchange: "ipc" -- the engine's pull transport (ABI 9, ranks of one node: a copy
    kernel reads the peers' send slots through IPC handles, no RCCL kernel beside the gradient kernel;
    IpcTransport), "rccl" -- the engine's own communicator, RCCL sends and receives issued by
    dopt_lagged_exchange on the side stream (ABI 7, csrc/transport.cpp: 4.5-6 us of host time per round against
    22 us for the process group's alltoall_base, profiles/r5_rccl_probe.txt) --, or "pg": torch's process group
    all-to-all-v (rounds 3-4).  "auto" (the default): the pull transport over RCCL jobs whose ranks share one
    node, RCCL otherwise and whenever the pull transport cannot be set up (every rank falls back together);
    DOPT_TRANSPORT overrides."""
    v = os.environ.get("DOPT_TRANSPORT", "auto").strip().lower()
    if v not in ("auto", "rccl", "pg", "ipc"):
        raise ValueError(f"DOPT_TRANSPORT={v!r}: 'auto', 'ipc', 'rccl' or 'pg'")
    return v


def _one_node(group):
    """Whether every rank of `group` runs on this host (hostnames all-gathered once per call)."""
    import socket

    import torch.distributed as dist

    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


class IpcTransport:
    """The pull transport's setup for one runner (dopt_lagged_ipc_*; DESIGN.md section 6, "A transport
    without RCCL's kernel").  Every rank exports its context's send slots and event, the handles and each
    rank's send-block offsets travel over the job's process group (any backend: gloo in the one-GPU
    multi-process tests), rank 0 creates the shared counters (POSIX shared memory, one int64 per rank) the
    others attach to, and every rank opens its peers' handles.  The ranks must share one node."""

    def __init__(self, engine, plan, layout, group, row_bytes, timeout_s):
        import torch.distributed as dist
        from multiprocessing import resource_tracker, shared_memory

        import weakref

        world, rank = plan.world, plan.rank
        self._shm = self._cnt = None
        self._creator = rank == 0
        self._eng = weakref.ref(engine)

        def agree(err):  # every rank learns every rank's failure: all raise together, none waits for a peer
            errs = [None] * world
            dist.all_gather_object(errs, err, group=group)
            bad = [e for e in errs if e]
            if bad:
                engine.lagged_transport(None)  # (no context keeps the counters about to be unmapped)
                self.close()
                raise CollectiveError("pull transport setup failed: " + "; ".join(bad))

        err, mh, eh, slot = None, b"", b"", 0
        try:
            mh, eh, slot = engine.lagged_ipc_export()
        except Exception as e:  # noqa: BLE001  (reported to every rank below)
            err = f"rank {rank}: {e}"
        send_off = np.concatenate([[0], np.cumsum(layout.send_sizes)]).astype(np.int64) * int(row_bytes)
        mine = (err, mh, eh, slot, [int(v) for v in send_off[:-1]])
        name = None
        infos = [None] * world  # (world 1 too: the same object collectives as a job's, over its backend)
        dist.all_gather_object(infos, mine, group=group)
        bad = [i[0] for i in infos if i[0]]
        if bad:
            raise CollectiveError("pull transport setup failed: " + "; ".join(bad))
        if self._creator:
            try:
                shm = shared_memory.SharedMemory(create=True, size=max(4096, 8 * world))
                shm.buf[:8 * world] = bytes(8 * world)
                name = shm.name
            except Exception as e:  # noqa: BLE001  (sent to every rank instead of the segment's name)
                name = "ERR:" + repr(e)[:200]
        box = [name]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        name = box[0]
        if name.startswith("ERR:"):
            raise CollectiveError(f"pull transport setup failed: rank 0's shared counters: {name[4:]}")
        err = None
        try:
            if not self._creator:
                shm = shared_memory.SharedMemory(name=name)
                resource_tracker.unregister(shm._name, "shared_memory")  # rank 0 owns the segment
            self._shm = shm
            self._cnt = np.ndarray((world,), dtype=np.int64, buffer=shm.buf)
            engine.lagged_ipc_import(world, rank, [i[1] for i in infos], [i[2] for i in infos],
                                     [i[3] for i in infos], [infos[p][4][rank] for p in range(world)],
                                     list(layout.recv_sizes), self._cnt.ctypes.data, timeout_s)
        except Exception as e:  # noqa: BLE001
            err = f"rank {rank}: {e}"
        # (also the barrier: every rank has opened its peers' handles before any rank's first round publishes)
        agree(err)
        # one trial exchange before any round, every step agreed: a runtime that cannot wait on a peer's
        # interprocess event or read its memory fails here, on every rank, instead of in a round
        for step in (0, 1):
            err = None
            try:
                engine.lagged_ipc_check(step)
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank}: trial {'publish' if step == 0 else 'pull'}: {e}"
            agree(err)
        engine._ipc_owner = self  # (Engine.lagged_transport clears it: another transport took over)

    def close(self):
        """Detach the context if this transport is still its exchange, then unmap the counters (rank 0
        removes the segment).  A new runner exports and imports again."""
        eng = self._eng() if getattr(self, "_eng", None) is not None else None
        if eng is not None and getattr(eng, "_ipc_owner", None) is self:
            eng.lagged_transport(None)  # (no context keeps the counters about to be unmapped)
        self._cnt = None
        if self._shm is not None:
            self._shm.close()
            if self._creator:
                self._shm.unlink()
            self._shm = None


def _comm(group, dev):
    """The process's engine-driven RCCL communicator over `group` on device `dev` (created once, collectively:
    rank 0's unique id is broadcast over the group's process group; every runner of the process shares it)."""
    import torch
    import torch.distributed as dist

    # keyed by the group's member ranks (a group object that is gone cannot alias a new one's id)
    key = (None if group is None else tuple(dist.get_process_group_ranks(group)), int(dev.index))
    c = _COMMS.get(key)
    if c is not None:
        return c
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    # one byte of status ahead of the id: rank 0's failure reaches every rank instead of leaving them in the
    # broadcast until the timeout
    buf = torch.zeros(1 + _dopt.COMM_ID_BYTES, dtype=torch.uint8, device=dev)
    err = None
    if rank == 0:
        try:
            buf[1:].copy_(torch.frombuffer(bytearray(_dopt.comm_unique_id()), dtype=torch.uint8))
        except RuntimeError as e:
            err = e
            buf[0] = 1
    src = 0 if group is None else dist.get_global_rank(group, 0)
    dist.broadcast(buf, src=src, group=group)
    if err is not None:
        raise err
    if int(buf[0].item()) != 0:
        raise RuntimeError("rank 0 could not create the engine's RCCL communicator id (DOPT_TRANSPORT=pg avoids it)")
    buf = buf[1:]
    if not _COMMS:
        import atexit

        atexit.register(close_comms)
    try:  # non-blocking setup, bounded like the process group's collectives (csrc/transport.cpp)
        c = _dopt.Comm(world, rank, int(dev.index), bytes(buf.cpu().numpy().tobytes()), timeout_s=timeout_seconds())
    except RuntimeError as e:
        raise CollectiveError(f"rank {rank}: the engine's RCCL communicator over {world} ranks could not be set up: "
                              f"{e}") from e
    _COMMS[key] = c
    return c


def close_comms(abort=False):
    """Destroy the engine-driven communicators, before the process group (bench.py and main.py call it; an
    atexit hook too).  Every engine still routed through one is detached first (Comm.close), so none can reach
    a freed communicator; without `abort` the devices are drained first, so no exchange is in flight."""
    if not _COMMS:
        return
    if not abort:
        import torch

        for dev in {c.device for c in _COMMS.values()}:
            torch.cuda.synchronize(dev)
    while _COMMS:
        _, c = _COMMS.popitem()
        c.close(abort)


def _stream(dev, role):
    """The process's stream `role` (0: the engine's rounds, 1: the lagged schedule's side stream) on device
    `dev`, created once and shared by every runner of the process (bench.py's strong leg builds a second
    DistributedDSGD after the weak leg's; a fresh pair of pool streams for it measured slower on the box,
    tools/rank_proxy.py --reps 2).  Runners of one process are used one at a time; if two were used at
    once, sharing a stream would order their work, not corrupt it."""
    import torch

    key = (int(dev.index if dev.index is not None else torch.cuda.current_device()), role)
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(dev)
    return st


class DistributedDSGD:
    """Drives one rank's engine through the round phases with torch.distributed."""

    def __init__(self, engine, plan, n_global, rows_global, device=0, group=None, mean=None, obj_sep=False,
                 rs_chunks=None):
        """`mean` = (w_off, W_ii of the local workers) for the complete graph: the mix then
        uses the all-reduced column sums and no halo rows move at all.  `rows_global` is
        the row count of the objective data (all shards, or the X_full slices loaded with
        Engine.load_objective_data when obj_sep).  `rs_chunks`: column chunks of the row-space
        pass (complete graph), each chunk's sums all-reduced while the next one streams
        (default: 1 at world size 1, else rs_chunks_for at this context's sums and row bytes)."""
        self.obj_sep = obj_sep
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.eng, self.plan, self.group = engine, plan, group
        self.n_global, self.rows_global = int(n_global), int(rows_global)
        self.dev = torch.device("cuda", device)
        self.device_comm = dist.get_backend(group) == "nccl"
        self.stream = _stream(self.dev, 0)
        ld, esz = engine.layout()
        self.ld = ld
        tdt = torch.float32 if esz == 4 else torch.float64
        # the lagged schedule: CSR mixing on row-resident contexts (DOPT_LAGGED=0: the serial one)
        nch = (ld * esz) // 16
        self._lagged_ok = (mean is None and nch <= 16 * 64 and
                           os.environ.get("DOPT_LAGGED", "1") != "0")
        # RCCL at world 1 with the collectives forced (the one-GPU rehearsal): this rank's own sums go
        # through the all-to-all to itself (a self block), so the side-stream chain carries real data
        forced = plan.world == 1 and self.device_comm and os.environ.get("DOPT_FORCE_COLLECTIVES") == "1"
        # the lagged schedule's exchange also carries every rank's column sums (its xbar, no all-reduce
        # per round); ks rows of T per block hold ld float64 sums.  Other schedules: the plan's rows only
        ks = (8 // esz) if (self._lagged_ok and (plan.world > 1 or forced)) else 0
        self.layout = exchange_layout(plan, ks, self_block=forced and ks > 0)
        lay = self.layout
        self.halo = torch.zeros((max(1, lay.n_recv_rows), ld), dtype=tdt, device=self.dev)
        self.send = torch.zeros((max(1, lay.n_send_rows), ld), dtype=tdt, device=self.dev)
        self.sum = torch.zeros(ld, dtype=torch.float64, device=self.dev)
        self.exchange = HaloExchange(plan, self.send, self.halo, group, self.device_comm, layout=lay)
        if rs_chunks:
            self.rs_chunks = int(rs_chunks)
        elif self._solo() or mean is None:
            self.rs_chunks = 1
        else:  # the model at this context's real sizes: ld float64 sums, this rank's rows times the ranks
            rows = engine.shard_rows
            xesz = 4 if engine.data_dtype == _dopt.F32 else 8
            nrows = int(np.sum(rows)) if rows is not None and len(rows) else 0
            self.rs_chunks = rs_chunks_for(plan.world, sum_bytes=ld * 8, pass_bytes=nrows * ld * xesz * plan.world)
        engine.set_partition(self.n_global, self.rows_global)
        if mean is None:
            engine.set_halo(lay.n_recv_rows, self.halo.data_ptr(), lay.send_ids(plan), self.send.data_ptr())
            engine.set_topology(plan.row_ptr, lay.local_col(plan), plan.w)
            if lay.ks > 0:
                engine.lagged_exchange_layout(plan.world, plan.rank, lay.sum_send_row, lay.sum_recv_row)
            self._peers = self.exchange.peers
        else:
            engine.set_halo(0, None, np.zeros(0, np.int32), None)
            engine.set_mixing_mean(mean[0], mean[1])
            self._peers = []
            self.exchange.disable()
        self.mean = mean
        engine.set_stream(self.stream.cuda_stream)
        # a second stream for each mix's column-sum totals (k_mixcs_final) and the exchange, so the
        # next gradient kernel does not wait for them -- whenever there is an exchange to order it
        # (DOPT_LAGGED_SIDE=0: one stream, the exchange serialised between the mix and the next gradient
        # kernel; DESIGN.md section 6, "Which form of the exchange")
        self.side = None
        self._stream_switch = None
        if (self._lagged_ok and not self._solo() and self.exchange.peers_or_collective()
                and os.environ.get("DOPT_LAGGED_SIDE", "1") != "0"):
            self.side = _stream(self.dev, 1)
        engine.lagged_side_stream(self.side.cuda_stream if self.side is not None else None)
        # the lagged exchange's transport (transport_kind): the engine's pull transport (ranks of one node) or
        # its own RCCL communicator (dopt_lagged_exchange); otherwise the process group / host transfers
        self.comm = None
        self.ipc = None
        kind = transport_kind()
        lagged_x = self._lagged_ok and mean is None and (plan.world > 1 or forced) and lay.ks > 0
        if kind == "auto":  # (every rank computes the same answer: the inputs are the job's, the test collective)
            kind = "ipc" if (lagged_x and self.device_comm and plan.world > 1 and _one_node(group)) else "rccl"
            if kind == "ipc":
                try:
                    engine.lagged_transport(None)
                    self.ipc = IpcTransport(engine, plan, lay, group, ld * esz, timeout_seconds())
                except CollectiveError as e:  # raised on every rank together: all fall back to RCCL
                    import sys

                    print(f"[distributed] rank {plan.rank}: {e}; the exchange goes over RCCL", file=sys.stderr)
                    self.ipc = None
                    kind = "rccl"
        elif kind == "ipc" and lagged_x:
            engine.lagged_transport(None)
            self.ipc = IpcTransport(engine, plan, lay, group, ld * esz, timeout_seconds())
        if self.ipc is not None:  # the shared counters go with the runner (rank 0 removes the segment)
            import weakref

            weakref.finalize(self, self.ipc.close)
        if self.ipc is None:
            if (self.device_comm and self._lagged_ok and mean is None and self.exchange.collective
                    and kind == "rccl"):
                self.comm = _comm(group, self.dev)
                engine.lagged_transport(self.comm, lay.send_sizes, lay.recv_sizes)
            else:
                engine.lagged_transport(None)
        # the communicator is created by one small collective here, not inside the first round
        # (the halo all-to-all and the all-reduces of the rounds then find it ready)
        if self.device_comm and dist.get_world_size(group) > 1:
            dist.all_reduce(torch.zeros(1, device=self.dev), group=group)

    # -- transport
    def _start_exchange(self):
        return self.exchange.start()

    def _start_exchange_lagged(self):
        """The lagged schedule's exchange: on the side stream when there is one (queued behind
        k_mixcs_final), with the engine stream current again afterwards.  The current stream is switched
        through torch._C._cuda_setStream with the two streams' cached ids (what torch.cuda.stream's
        context manager does, without its per-call Python: VERDICT r4 item 4, host cost per round)."""
        if self.comm is not None or self.ipc is not None:  # the engine issues it on the side stream and orders
            if self.comm is not None and self.comm.closed:  # the engine stream after it
                raise CollectiveError(f"rank {self.plan.rank}: the engine's RCCL communicator was aborted")
            if self.ipc is None:
                self.eng.lagged_exchange()
                return None
            try:  # (a peer that stopped publishing its rounds: the engine's bounded host wait)
                self.eng.lagged_exchange()
            except RuntimeError as e:
                raise CollectiveError(f"rank {self.plan.rank}: {e}") from e
            return None
        side = self.side
        if side is None:
            return self.exchange.start()
        sw = self._stream_switch
        if sw is None:
            set_id = getattr(self.torch._C, "_cuda_setStream", None)
            if set_id is not None:
                ids = [dict(stream_id=st.stream_id, device_index=st.device_index, device_type=st.device_type)
                       for st in (side, self.stream)]
            else:  # (a torch without the private setter: the public one, same effect)
                set_id = lambda stream: self.torch.cuda.set_stream(stream)  # noqa: E731
                ids = [dict(stream=side), dict(stream=self.stream)]
            sw = self._stream_switch = (set_id, ids[0], ids[1])
        set_id, to_side, to_eng = sw
        set_id(**to_side)
        try:
            w = self.exchange.start()
        finally:
            set_id(**to_eng)
        # the process group's all-to-all runs on its internal stream: finish() waits on its work; the host
        # transport wrote the halo rows on the side stream, which the engine stream then waits for
        if w is None:
            self.stream.wait_stream(side)
        return w

    def _finish_exchange(self, works):
        self.exchange.finish(works)

    def _sync(self, stream):
        """stream.synchronize(), bounded like the process group's collectives when the engine's own
        communicator has exchanges in it: a peer that never joins ends this rank with CollectiveError
        (the communicator aborted) within timeout_seconds() instead of a hang."""
        if self.comm is None:
            stream.synchronize()
            return
        import time

        t0 = time.monotonic()
        last = t0
        nap = 20e-6  # backs off to 1 ms: the host does not hold a core while the GPU works
        while not stream.query():
            now = time.monotonic()
            if now - last > 1.0:
                last = now
                try:
                    self.comm.check()
                except RuntimeError as e:
                    raise CollectiveError(f"rank {self.plan.rank}: the engine's RCCL exchange failed: {e}") from e
                if now - t0 > timeout_seconds():
                    # every communicator of the process aborted, every engine routed through one detached
                    # first (Comm.close), so no context keeps a freed communicator
                    comm, self.comm = self.comm, None
                    comm.close(abort=True)
                    close_comms(abort=True)
                    raise CollectiveError(f"rank {self.plan.rank}: the engine's RCCL exchange "
                                          f"({self.exchange.what}) did not finish in {timeout_seconds():.0f} s")
            time.sleep(nap)
            nap = min(2 * nap, 1e-3)

    def _solo(self):
        """One rank: the reductions are identities and are skipped, unless
        DOPT_FORCE_COLLECTIVES=1 (exercises the RCCL calls on a one-GPU box)."""
        return self.dist.get_world_size(self.group) == 1 and os.environ.get("DOPT_FORCE_COLLECTIVES") != "1"

    def _all_reduce(self, t):
        w = self._all_reduce_start(t)
        if w is not None:
            _wait(w, f"all_reduce of {t.numel()} float64", self.plan.rank)

    def _all_reduce_start(self, t):
        """Enqueue an all-reduce of t behind the current stream's work; returns the work to
        wait on (RCCL: the current stream waits at .wait(), the host does not), or None
        when the reduction is already complete (world 1, gloo: done here on the host, bounded
        by the job's timeout)."""
        if self._solo():
            return None
        what = f"all_reduce of {t.numel()} float64"
        if self.device_comm:
            return self.dist.all_reduce(t, group=self.group, async_op=True)
        c = t.cpu()
        _wait(self.dist.all_reduce(c, group=self.group, async_op=True), what, self.plan.rank, timeout_seconds())
        if c.data_ptr() != t.data_ptr():
            t.copy_(c)
        return None

    # -- rounds
    def run(self, T, eta0, batch, lam_grad, lam_obj, f_opt=0.0, t0=0, objective=True, consensus=True, idx=None):
        """T rounds; returns the GLOBAL (objective, consensus) history on every rank.

        idx: [T, n_local, batch] minibatch row ids of this rank's workers (the slice of
        the global draw), or None for full-shard batches.  With full shards the metrics
        of round t ride on round t+1's pass over the rows; otherwise a metrics pass
        over all local rows follows every round."""
        torch = self.torch
        eng = self.eng
        flags = (_dopt.RUN_OBJECTIVE if objective else 0) | (_dopt.RUN_CONSENSUS if consensus else 0)
        fused = idx is None and not self.obj_sep
        rows = self.eng.shard_rows
        bip = (idx is not None and not self.obj_sep and rows is not None and len(rows) > 0 and
               batch < int(rows.max()) <= _dopt.MAX_BIP_ROWS and os.environ.get("DOPT_BIP", "1") != "0")
        if (fused or bip) and flags and self._lagged_ok:
            return self._run_lagged(T, eta0, batch, lam_grad, lam_obj, f_opt, t0, objective, consensus, idx)
        if self.mean is not None and fused and T > 0 and self._full_batch(batch) and self._rowspace_ready():
            return self._run_rowspace(T, eta0, lam_grad, lam_obj, f_opt, t0, objective, consensus)
        xnorm = self.plan.rank == 0  # ||xbar||^2 is global already: count it once
        with torch.cuda.stream(self.stream):
            partials = torch.zeros((max(1, T), 3), dtype=torch.float64, device=self.dev)
            # prologue: global column sums / xbar of the starting iterates (complete-graph mix, metrics)
            eng.phase_colsum(self.sum.data_ptr())
            self._all_reduce(self.sum)
            eng.phase_xbar(self.sum.data_ptr())
            eng.phase_begin(batch)
            for h in range(T):
                met = fused and h > 0 and flags
                if self._peers:
                    eng.phase_gather()
                pending = self._start_exchange()
                eng.phase_set_step(t0 + h, eta0)  # (the gradient kernel steps the interior workers)
                eng.phase_grad(batch, lam_grad, flags if met else 0, idx=None if idx is None else idx[h])
                self._finish_exchange(pending)
                eng.phase_mix(t0 + h, eta0)
                if met:  # metric partials of x_t at xbar_t (slabs from this round's pass)
                    eng.phase_metrics(flags, xnorm, partials[h - 1].data_ptr())
                eng.phase_colsum(self.sum.data_ptr())
                self._all_reduce(self.sum)
                eng.phase_xbar(self.sum.data_ptr())
                if flags and not fused:
                    eng.phase_metrics_pass(flags)
                    eng.phase_metrics(flags, xnorm, partials[h].data_ptr())
            if flags and fused and T > 0:
                eng.phase_metrics_pass(flags)
                eng.phase_metrics(flags, xnorm, partials[T - 1].data_ptr())
            self._all_reduce(partials)
            raw = partials[:T].cpu().numpy()
        self.stream.synchronize()
        obj, cons = _dopt.finalize_metrics(self.eng.problem, raw, self.n_global, self.rows_global, lam_obj, f_opt)
        return (obj if objective else None), (cons if consensus else None)

    def _full_batch(self, batch):
        """Every local worker's minibatch is its whole shard (the row-space rounds take full-shard
        gradients only; a smaller batch goes to the phase path, which draws it or refuses)."""
        rows = self.eng.shard_rows
        return rows is None or len(rows) == 0 or int(batch) >= int(np.max(rows))

    def _rowspace_ready(self):
        """Complete graph + quadratic + full shards of <= 64 rows and iterates that are equal on
        every rank (checked here: the 64-bit content hash of each rank's common iterate -- of the
        replicated state once live -- must be the same on all ranks): the row-space rounds."""
        torch = self.torch
        ok, h = self.eng.rs_phase_begin(False)
        hi, lo = (h >> 32), (h & 0xFFFFFFFF)  # 32-bit halves: their negations fit an int64
        v = torch.tensor([1 if ok else 0, hi, -hi, lo, -lo], dtype=torch.int64,
                         device=self.dev if self.device_comm else "cpu")
        if not self._solo():
            self._all_reduce_op(v, self.dist.ReduceOp.MIN)
        v = [int(a) for a in v.cpu()]
        return v[0] == 1 and v[1] == -v[2] and v[3] == -v[4]

    def _all_reduce_op(self, t, op):
        what = f"all_reduce ({op}) of {t.numel()} values"
        if self.device_comm:
            _wait(self.dist.all_reduce(t, op=op, group=self.group, async_op=True), what, self.plan.rank)
        else:
            _wait(self.dist.all_reduce(t, op=op, group=self.group, async_op=True), what, self.plan.rank,
                  timeout_seconds())

    def _run_rowspace(self, T, eta0, lam_grad, lam_obj, f_opt, t0, objective, consensus, pipelined=False):
        """Complete graph: the iterates stay Z + X_i^T beta_i.  Per round one
        read-only pass over this rank's rows (row state, metric partials of the current iterates,
        local column sums), the all-reduce of the d column sums, the replicated average / Z
        update; history[h] = metrics of x_{h+1} from the next pass (the last from a dots pass).
        pipelined: the last metrics stay owed and the next pipelined call's first pass takes
        them (T = 0: a dots pass for them), as Engine.run_dsgd_pipelined on one context.  The
        iterates are formed when asked for (gather_models)."""
        torch, eng = self.torch, self.eng
        xnorm = self.plan.rank == 0
        mf = (_dopt.RUN_OBJECTIVE if objective else 0) | (_dopt.RUN_CONSENSUS if consensus else 0)
        was_open = eng.phase_chain(False)  # any call ends an open chain; a pipelined one continues it
        if pipelined and was_open and getattr(self, "_rs_flags", None) != mf:
            # the open chain owes an entry with the other flags: refuse (as dopt_run_dsgd_pipelined
            # does on one context) rather than drop it; the chain stays open
            eng.phase_chain(True)
            raise ValueError("pipelined run: the open chain owes the metrics of its last iterate with other "
                             "objective / consensus flags; continue or close it (T = 0) with the same flags")
        owed = pipelined and was_open
        leave = pipelined and T > 0 and mf != 0
        n_out = (T + (1 if owed else 0) - (1 if leave else 0)) if mf else 0
        if not owed:
            if T == 0:
                return (np.zeros(0) if objective else None), (np.zeros(0) if consensus else None)
            eng.rs_phase_begin(True)
        with torch.cuda.stream(self.stream):
            partials = torch.zeros((max(1, n_out), 3), dtype=torch.float64, device=self.dev)
            e = 0

            def fold(k):
                base = partials.data_ptr() + 3 * k * 8
                eng.phase_fold(base if consensus else None, base + 16 if objective and xnorm else None,
                               base + 8 if objective else None, 0)

            # K column chunks, pipelined across rounds: chunk k's sums are all-reduced while the later chunks
            # stream, and round h's average update of chunk k (which needs those sums) runs just before
            # round h + 1's pass over chunk k -- so the all-reduce of the last chunk is hidden behind the
            # next round's first chunks instead of sitting between two passes (K = 1: the serial order
            # pass, rows, all-reduce, cols).  Every column's arithmetic is the same in either order.
            K = self.rs_chunks
            sp = self.sum.data_ptr()
            pend = None  # (round, [(c0, c1, work)] per chunk) whose average update is still to run
            for h in range(T):
                met = mf and (h > 0 or owed)
                cur = []
                for k in range(K):
                    if pend is not None:
                        self._rs_cols_chunk(pend, k, eta0, lam_grad, sp)
                    c0, c1 = eng.rs_phase_pass(k, K, sp)
                    cur.append((c0, c1, self._all_reduce_start(self.sum[c0:c1]) if c1 > c0 else None))
                pend = (t0 + h, cur)
                eng.rs_phase_rows(t0 + h, eta0, lam_grad, mf if met else 0)
                if met:
                    fold(e)
                    e += 1
            if pend is not None:
                for k in range(K):
                    self._rs_cols_chunk(pend, k, eta0, lam_grad, sp)
            if mf and not leave:
                eng.rs_phase_metrics(mf)
                fold(e)
                e += 1
            assert e == n_out
            self._all_reduce(partials[:n_out])
            raw = partials[:n_out].cpu().numpy()
        self.stream.synchronize()
        if leave:
            eng.phase_chain(True)
            self._rs_flags = mf
        obj, cons = _dopt.finalize_metrics(self.eng.problem, raw, self.n_global, self.rows_global, lam_obj, f_opt)
        return (obj if objective else None), (cons if consensus else None)

    def _rs_cols_chunk(self, pend, k, eta0, lam_grad, sum_ptr):
        """Round pend[0]'s average / Z update of pass chunk k, once that chunk's all-reduce is done."""
        t, chunks = pend
        c0, c1, w = chunks[k]
        if w is not None:
            _wait(w, f"all_reduce of column chunk [{c0}, {c1}) of the {self.ld} column sums", self.plan.rank)
        self.eng.rs_phase_cols_range(t, eta0, lam_grad, sum_ptr, c0, c1, k == len(chunks) - 1)

    def run_pipelined(self, T, eta0, batch, lam_grad, lam_obj, f_opt=0.0, t0=0, objective=True, consensus=True,
                      idx=None):
        """The lagged schedule continued across calls (steady-state timing, bench.py; the
        multi-GPU counterpart of Engine.run_dsgd_pipelined).  A chain of such calls is one
        long lagged run: no call ends with the tail of _run_lagged (xbar_T, the consensus of
        x_T and a pass for the last losses); T = 0 runs that tail and closes the chain.  Each
        call returns the GLOBAL (objective, consensus) entries that became complete during it
        -- T of them in the steady state (history[t] is complete once the loss at xbar_t has
        been folded, two rounds later: round t + 2's mix).  Rounds use learning-rate index t0 + h per call.
        Any other run or dopt_set_models ends a chain (dopt_phase_chain)."""
        rows = self.eng.shard_rows
        bip = (idx is not None and not self.obj_sep and rows is not None and len(rows) > 0 and
               batch < int(rows.max()) <= _dopt.MAX_BIP_ROWS and os.environ.get("DOPT_BIP", "1") != "0")
        if (self.mean is not None and idx is None and not self.obj_sep and (objective or consensus) and
                self._full_batch(batch) and self._rowspace_ready()):  # complete graph: row-space rounds continued across calls
            return self._run_rowspace(T, eta0, lam_grad, lam_obj, f_opt, t0, objective, consensus, pipelined=True)
        if not ((idx is None and not self.obj_sep) or bip) or not (objective or consensus) or not self._lagged_ok:
            raise NotImplementedError("pipelined runs: the lagged schedule (CSR mixing, fused metrics) or the "
                                      "row-space rounds (complete graph, equal iterates)")
        return self._run_lagged(T, eta0, batch, lam_grad, lam_obj, f_opt, t0, objective, consensus, idx,
                                pipelined=True)

    def _run_lagged(self, T, eta0, batch, lam_grad, lam_obj, f_opt, t0, objective, consensus, idx=None,
                    pipelined=False):
        """Rounds with CSR mixing whose metrics ride the gradient pass (full shards, or
        minibatches taken inside a pass over every row); history[t] = metrics of x_{t+1}.
        Round g (counted from the start of the chain; one call = one chain unless pipelined):

          exchange: halo rows of x_g + every rank's column sums of x_g (ONE all-to-all-v) ---.
          lagged_grad: gradient pass of x_g + loss of every row at xbar_{g-1} -------------+--> lagged_mix
          lagged_mix: xbar_g (rank-ordered sums), consensus of x_g, x_{g+1} and its send rows,
                      the column sums of x_{g+1} into the send buffer, fold of history[g-2]

        Three launches, two engine calls and one collective per round (round 4; round 3 had four
        kernels, two collectives and five engine calls); history row t is complete once round t + 2's
        mix has folded it.  After the last round of a chain (the tail): one more exchange for the
        sums of x_T, then xbar_T, the consensus of x_T and one pass for the losses at xbar_{T-1} and
        xbar_T (dopt_lagged_tail)."""
        torch, eng = self.torch, self.eng
        xnorm = self.plan.rank == 0  # ||xbar||^2 is global already: count it once
        obj_f = _dopt.RUN_OBJECTIVE if objective else 0
        flags = (objective, consensus)
        # every rank makes the same calls, so all see the same chain state
        was_open = pipelined and eng.phase_chain(False) and getattr(self, "_chain", None) is not None
        if was_open and self._chain["flags"] != flags:
            # the open chain owes history rows with the other flags: refuse, as the row-space rounds and
            # dopt_run_dsgd_pipelined on one context do; the chain stays open
            eng.phase_chain(True)
            raise ValueError("pipelined run: the open chain owes the metrics of its last iterates with other "
                             "objective / consensus flags; continue or close it (T = 0) with the same flags")
        cont = was_open
        if not cont:
            if not pipelined and T == 0:
                return (np.zeros(0) if objective else None), (np.zeros(0) if consensus else None)
            self._chain = {"g": 0, "done": 0, "flags": flags, "hist": None}
        ch = self._chain
        G0, G1 = ch["g"], ch["g"] + T
        tail = not pipelined or T == 0
        exchange = self.exchange
        with torch.cuda.stream(self.stream):
            cap = max(1, G1)
            if ch["hist"] is None or ch["hist"].shape[0] < cap:  # history rows by global entry, grown by doubling
                new = torch.zeros((max(cap, 2 * (0 if ch["hist"] is None else ch["hist"].shape[0])), 3),
                                  dtype=torch.float64, device=self.dev)
                if ch["hist"] is not None:
                    new[:ch["hist"].shape[0]].copy_(ch["hist"])
                ch["hist"] = new
            partials = ch["hist"]
            base = partials.data_ptr()

            def at(e, k, want=True):  # device address of history row e, column k, or None
                return base + (3 * e + k) * 8 if want and 0 <= e < G1 else None

            if not cont:
                eng.lagged_begin(batch)  # send rows and column sums of x_0
            lagged_grad, lagged_mix = eng.lagged_grad, eng.lagged_mix
            side = self.side

            start = self._start_exchange_lagged
            for g in range(G0, G1):
                h = g - G0
                pending = start()
                # loss at xbar_{g-1} (history[g-2]); at g = 1 it is the loss of x_0, which no history row
                # holds -- taken anyway so round 1's gradient dots reduce in the same (paired) butterfly
                # as the fused single-context round 1, whose pass carries the metrics of x_1
                lagged_grad(t0 + h, eta0, batch, lam_grad, obj_f if g >= 1 else 0, None if idx is None else idx[h])
                if pending is not None:
                    exchange.finish(pending)
                e = g - 2
                lagged_mix(t0 + h, eta0, consensus, at(e, 0, consensus), at(e, 2, objective and xnorm),
                           at(e, 1, objective))
            if tail and G1 > 0:
                exchange.finish(start())  # every rank's column sums of x_T
                eng.lagged_tail(consensus, objective,
                                (at(G1 - 1, 0, consensus), at(G1 - 1, 2, objective and xnorm), at(G1 - 1, 1, objective)),
                                (at(G1 - 2, 0, consensus), at(G1 - 2, 2, objective and xnorm), at(G1 - 2, 1, objective)))
            upto = G1 if tail else max(ch["done"], G1 - 2)  # history rows complete on every rank
            done = ch["done"]
            if upto > done:
                self._all_reduce(partials[done:upto])
        # the streams drained first (bounded: _sync), then the history rows copied out
        self._sync(self.stream)
        if self.side is not None:
            self._sync(self.side)  # no side-stream work outlives the call
        raw = partials[done:upto].cpu().numpy()
        ch["g"], ch["done"] = G1, upto
        if tail:
            self._chain = None
        else:
            eng.phase_chain(True)
        obj, cons = _dopt.finalize_metrics(self.eng.problem, raw, self.n_global, self.rows_global, lam_obj, f_opt)
        return (obj if objective else None), (cons if consensus else None)

    def gather_models(self):
        """All ranks' iterates, concatenated in global worker order (on every rank)."""
        torch = self.torch
        sizes = np.diff(self.plan.bounds)
        top = int(sizes.max())
        x = torch.zeros((top, self.eng.d), dtype=torch.float64)
        x[:self.plan.n_local] = torch.from_numpy(self.eng.get_models())
        if self.device_comm:
            x = x.to(self.dev)
        buf = [torch.zeros_like(x) for _ in sizes]
        self.dist.all_gather(buf, x, group=self.group)
        return torch.cat([b[:int(s)] for b, s in zip(buf, sizes)]).cpu().numpy()


class DistributedCentralized:
    """CentralizedTrainer rounds across ranks (trainer.py:41-71): each rank's workers take
    their gradients at the shared iterate, the column sums of the gradients are
    all-reduced (d doubles), and every rank applies the same step."""

    def __init__(self, engine, plan, n_global, rows_global, device=0, group=None, obj_sep=False):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.eng, self.plan, self.group = engine, plan, group
        self.n_global, self.rows_global, self.obj_sep = int(n_global), int(rows_global), obj_sep
        self.dev = torch.device("cuda", device)
        self.device_comm = dist.get_backend(group) == "nccl"
        self.stream = _stream(self.dev, 0)
        ld, _ = engine.layout()
        self.sum = torch.zeros(ld, dtype=torch.float64, device=self.dev)
        engine.set_partition(self.n_global, self.rows_global)
        engine.set_stream(self.stream.cuda_stream)

    _solo = DistributedDSGD._solo
    _all_reduce = DistributedDSGD._all_reduce
    _all_reduce_start = DistributedDSGD._all_reduce_start

    def run(self, T, eta0, batch, lam_grad, lam_obj, f_opt=0.0, t0=0, objective=True, idx=None):
        torch = self.torch
        eng = self.eng
        split = ((eng.d + 16 // eng.layout()[1] - 1) // (16 // eng.layout()[1])) > 16 * 64
        fused = idx is None and not self.obj_sep and not split
        xnorm = self.plan.rank == 0
        with torch.cuda.stream(self.stream):
            partials = torch.zeros((max(1, T), 3), dtype=torch.float64, device=self.dev)
            for h in range(T):
                met = fused and h > 0 and objective
                eng.phase_grad_shared(batch, lam_grad, fuse_loss=met, idx=None if idx is None else idx[h])
                if met:  # objective of the iterate the gradients were taken at
                    eng.phase_metrics_shared(xnorm, partials[h - 1].data_ptr())
                eng.phase_colsum_grad(self.sum.data_ptr())
                self._all_reduce(self.sum)
                eng.phase_central_step(self.sum.data_ptr(), t0 + h, eta0)
                if objective and not fused:
                    eng.phase_metrics_pass_shared()
                    eng.phase_metrics_shared(xnorm, partials[h].data_ptr())
            if objective and fused and T > 0:
                eng.phase_metrics_pass_shared()
                eng.phase_metrics_shared(xnorm, partials[T - 1].data_ptr())
            self._all_reduce(partials)
            raw = partials[:T].cpu().numpy()
        self.stream.synchronize()
        obj, _ = _dopt.finalize_metrics(eng.problem, raw, self.n_global, self.rows_global, lam_obj, f_opt)
        return obj if objective else None
