"""libdopt.so's legacy-MT19937 sampler (host code, no GPU) vs numpy and the fixtures."""
import os

import numpy as np
import pytest

import _dopt

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_choice_matches_fixture_stream():
    z = np.load(os.path.join(G, "rng.npz"))
    np.random.seed(203)
    for k, (m, b) in enumerate(z["specs"]):
        np.testing.assert_array_equal(_dopt.mt_choice(int(m), int(b)), z[f"call{k}_idx"])
        assert np.random.get_state()[2] == z[f"call{k}_pos"]
    np.testing.assert_array_equal(np.random.get_state()[1], z["final_key"])


def test_rounds_match_fixture():
    z = np.load(os.path.join(G, "rng.npz"))
    np.random.seed(203)
    np.testing.assert_array_equal(_dopt.mt_choice_rounds(3, [500] * 10, 16), z["rounds_c2"])


@pytest.mark.parametrize("seed", [0, 1, 203, 2 ** 31 - 1])
def test_choice_matches_numpy_random_shapes(seed):
    rng = np.random.default_rng(seed)
    np.random.seed(seed)
    calls = [(int(rng.integers(0, 3000)), int(rng.integers(0, 700))) for _ in range(200)]
    ours = [_dopt.mt_choice(m, b) for m, b in calls]
    st_ours = np.random.get_state()
    np.random.seed(seed)
    for (m, b), got in zip(calls, ours):
        eb = 0 if m == 0 else min(b, m)
        want = np.random.choice(m, eb, replace=False) if eb > 0 else np.zeros(0, dtype=np.int64)
        np.testing.assert_array_equal(got, want)
    st = np.random.get_state()
    assert st[2] == st_ours[2]
    np.testing.assert_array_equal(st[1], st_ours[1])


def test_rounds_padding_and_ragged():
    np.random.seed(5)
    rows = [0, 1, 3, 7, 600]
    out = _dopt.mt_choice_rounds(4, rows, 5)
    np.random.seed(5)
    for t in range(4):
        for i, m in enumerate(rows):
            eb = 0 if m == 0 else min(5, m)
            want = np.random.choice(m, eb, replace=False) if eb else np.zeros(0, dtype=np.int64)
            np.testing.assert_array_equal(out[t, i, :eb], want)
            assert np.all(out[t, i, eb:] == -1)


def test_large_interval_uses_numpy_semantics():
    np.random.seed(77)
    got = _dopt.mt_choice(100003, 3)
    np.random.seed(77)
    np.testing.assert_array_equal(got, np.random.choice(100003, 3, replace=False))


def test_bad_state_rejected():
    key = np.zeros(624, dtype=np.uint32)
    import ctypes

    pos = ctypes.c_int32(1000)
    out = np.zeros(4, dtype=np.int64)
    rc = _dopt.lib().dopt_mt_choice(key.ctypes.data_as(ctypes.c_void_p), ctypes.byref(pos), 10, 4,
                                    out.ctypes.data_as(ctypes.c_void_p))
    assert rc == _dopt.ERR_INVALID


@pytest.mark.parametrize("rows,b", [([500] * 10, 16), ([1, 2, 3, 700, 0, 64, 65], 9), ([4096] * 3, 4096)])
def test_rounds_leave_numpy_state_where_numpy_does(rows, b):
    """After T rounds the generator state (key words and position) is exactly where the
    reference's T x N np.random.choice calls leave it, so later draws continue the stream."""
    np.random.seed(11)
    _dopt.mt_choice_rounds(3, rows, b)
    ours = np.random.get_state()
    np.random.seed(11)
    for _ in range(3):
        for m in rows:
            if m > 0 and min(b, m) > 0:
                np.random.choice(m, min(b, m), replace=False)
    ref = np.random.get_state()
    assert ours[2] == ref[2]
    np.testing.assert_array_equal(ours[1], ref[1])


@pytest.mark.parametrize("b", [10 ** 6, 501, 16, 0])
def test_trainer_index_chunks_advance_stream_like_choice(b):
    """Trainer draws (full shards use b = 1 internally) leave numpy's global state exactly
    where the reference's per-worker np.random.choice(m, min(b, m)) calls leave it
    (worker.py:17-27), including empty shards and b far above m."""
    from trainer import _index_chunks

    class W:
        def __init__(self, m):
            self.n_local_samples, self.batch_size = m, b

    rows = [500, 499, 0, 501]
    np.random.seed(5)
    chunks = list(_index_chunks([W(m) for m in rows], 37, {}))
    key, pos = np.random.get_state()[1].copy(), np.random.get_state()[2]
    np.random.seed(5)
    for _ in range(37):
        for m in rows:
            if m > 0 and b > 0:
                np.random.choice(m, min(b, m), replace=False)
    np.testing.assert_array_equal(key, np.random.get_state()[1])
    assert pos == np.random.get_state()[2]
    assert sum(c[1] for c in chunks) == 37
    assert (chunks[0][3] is None) == (b >= max(rows))


def test_prefetched_draw_is_undone_when_the_run_stops_early():
    """trainer._one_ahead draws the next chunk of legacy-MT19937 indices on a helper thread.
    When the consumer stops after the first chunk (e.g. the device run raised), numpy's
    global stream must be where the CONSUMED chunk left it, not one chunk further."""
    from contextlib import closing

    import trainer

    class W:
        def __init__(self, m):
            self.n_local_samples, self.batch_size = m, 4

    ws = [W(30), W(17), W(30)]
    rows = [30, 17, 30]
    np.random.seed(11)
    expect_first = _dopt.mt_choice_rounds(trainer.IDX_CHUNK_ROUNDS, rows, 4)
    expect_state = np.random.get_state()
    np.random.seed(11)
    with closing(trainer._index_chunks(ws, 3 * trainer.IDX_CHUNK_ROUNDS, {})) as chunks:
        t0, n, b, idx, _ = next(chunks)
    assert (t0, n, b) == (0, trainer.IDX_CHUNK_ROUNDS, 4)
    np.testing.assert_array_equal(idx, expect_first)
    st = np.random.get_state()
    assert st[2] == expect_state[2]
    np.testing.assert_array_equal(st[1], expect_state[1])


@pytest.mark.parametrize("start_draws", [0, 1, 313])
def test_rounds_long_stream_through_the_block_ring(start_draws):
    """Many more MT19937 blocks than the generator thread's ring holds (BlockRing::kSlots = 64),
    starting mid-block: indices and the state left behind equal numpy's, call by call."""
    rows, T, b = [300, 0, 1, 257, 300, 31], 40, 7
    np.random.seed(19)
    np.random.randint(0, 2 ** 16, size=start_draws)  # leaves pos mid-block
    st0 = np.random.get_state()
    out = _dopt.mt_choice_rounds(T, rows, b)
    st_ours = np.random.get_state()
    np.random.set_state(st0)
    for t in range(T):
        for i, m in enumerate(rows):
            eb = 0 if m == 0 else min(b, m)
            if eb:
                np.testing.assert_array_equal(out[t, i, :eb], np.random.choice(m, eb, replace=False))
    st = np.random.get_state()
    assert st[2] == st_ours[2]
    np.testing.assert_array_equal(st[1], st_ours[1])


@pytest.mark.parametrize("rows", [[512] * 64, [0, 1, 2, 999, 5000]])
def test_advance_rounds_leaves_numpy_state_where_numpy_does(rows):
    """dopt_mt_advance_rounds (full-shard batches: indices discarded) consumes exactly what
    T x N np.random.choice calls consume (trainer.py:166, worker.py:27)."""
    T = 12
    np.random.seed(23)
    np.random.randint(0, 10, size=5)
    st0 = np.random.get_state()
    _dopt.mt_advance_rounds(T, rows)
    st_ours = np.random.get_state()
    np.random.set_state(st0)
    for _ in range(T):
        for m in rows:
            if m:
                np.random.choice(m, m, replace=False)
    st = np.random.get_state()
    assert st[2] == st_ours[2]
    np.testing.assert_array_equal(st[1], st_ours[1])


@pytest.mark.parametrize("batch,max_chunk,t_begin", [(4, 7, 0), (4, 7, 10), (10 ** 6, 5, 3), (4, 0, 0)])
def test_index_chunks_boundaries_and_rng_states(batch, max_chunk, t_begin):
    """trainer._index_chunks (host side of checkpoint / resume): chunks cover rounds
    t_begin .. T-1 in order, never cross a multiple of max_chunk, and each carries numpy's
    state right after its own draws (the state a checkpoint after that chunk records)."""
    from contextlib import closing

    from trainer import _index_chunks

    class W:
        def __init__(self, m):
            self.n_local_samples, self.batch_size = m, batch

    ws = [W(m) for m in (30, 30, 17)]
    T = 23
    np.random.seed(4)
    st0 = np.random.get_state()
    with closing(_index_chunks(ws, T, {"sampling": "legacy"}, t_begin, max_chunk)) as chunks:
        got = [(t0, n, idx, st) for t0, n, _, idx, st in chunks]
    assert [g[0] for g in got] == list(np.cumsum([t_begin] + [g[1] for g in got[:-1]]))
    assert got[-1][0] + got[-1][1] == T
    if max_chunk:
        assert all((t0 % max_chunk) + n <= max_chunk for t0, n, _, _ in got)
    np.random.set_state(st0)
    for t0, n, idx, st in got:
        for t in range(n):
            for i, w in enumerate(ws):
                eb = min(batch, w.n_local_samples)
                want = np.random.choice(w.n_local_samples, eb, replace=False)
                if idx is not None:
                    np.testing.assert_array_equal(idx[t, i, :eb], want)
        now = np.random.get_state()
        assert now[2] == st[2] and np.array_equal(now[1], st[1])


@pytest.mark.parametrize("seg,win,start_draws", [("64", "8", 0), ("64", "64", 101), ("48", "20", 7), (None, None, 3)])
def test_parallel_advance_matches_numpy(monkeypatch, seg, win, start_draws):
    """The speculative parallel stream advance (uniform shards: segments filtered from a guessed
    state on their own threads, stitched where each meets the true run) leaves numpy's state
    exactly where T x N np.random.choice calls do.  Small segments / windows force many stitches
    and windows without a meeting point (the stitch then runs the segment itself); the last
    case runs the default shape.  Workers with 0 / 1 rows draw nothing and keep the shards
    uniform."""
    monkeypatch.setenv("DOPT_MT_THREADS", "3")
    if seg:
        monkeypatch.setenv("DOPT_MT_SEG_BLOCKS", seg)
        monkeypatch.setenv("DOPT_MT_WIN_BLOCKS", win)
    rows = [512, 0, 512, 1] * 16 if seg else [512] * 64
    T = 12 if seg else 200  # the default shape needs >= 3 segments of 4096 blocks
    np.random.seed(29)
    np.random.randint(0, 10, size=start_draws)
    st0 = np.random.get_state()
    _dopt.mt_advance_rounds(T, rows)
    st_ours = np.random.get_state()
    np.random.set_state(st0)
    for _ in range(T):
        for m in rows:
            if m:
                np.random.choice(m, m, replace=False)
    st = np.random.get_state()
    assert st[2] == st_ours[2]
    np.testing.assert_array_equal(st[1], st_ours[1])


@pytest.mark.parametrize("seg,win,rows,T,b", [("64", "8", [512, 0, 512, 1] * 16, 12, 16),
                                              ("40", "40", [300] * 64, 10, 300),
                                              ("40", "12", [3, 1, 3] * 50, 1500, 2),
                                              (None, None, [512] * 64, 200, 16)])
def test_parallel_minibatch_draws_match_numpy(monkeypatch, seg, win, rows, T, b):
    """Minibatch draws (b < m) over uniform shards through the speculative parallel filter: the
    kept words of every segment after its meeting point, spliced after the stitch's own, give
    every worker's np.random.choice(m, b, replace=False) bit for bit, and numpy's state after the
    call is numpy's.  m = 3 is the smallest shard the kept-word splice handles (every kept word
    changes k); tiny segments / windows force windows without a meeting point."""
    monkeypatch.setenv("DOPT_MT_THREADS", "4")
    if seg:
        monkeypatch.setenv("DOPT_MT_SEG_BLOCKS", seg)
        monkeypatch.setenv("DOPT_MT_WIN_BLOCKS", win)
    np.random.seed(31)
    np.random.randint(0, 10, size=3)
    st0 = np.random.get_state()
    out = _dopt.mt_choice_rounds(T, rows, b)
    st_ours = np.random.get_state()
    np.random.set_state(st0)
    for t in range(T):
        for i, m in enumerate(rows):
            eb = 0 if m == 0 else min(b, m)
            if eb:
                np.testing.assert_array_equal(out[t, i, :eb], np.random.choice(m, eb, replace=False))
            assert np.all(out[t, i, eb:] == -1)
    st = np.random.get_state()
    assert st[2] == st_ours[2]
    np.testing.assert_array_equal(st[1], st_ours[1])


_RSS_PROBE = r"""
import resource, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import _dopt
_dopt.lib()
np.random.seed(7)
base = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
t0 = time.time()
mode = sys.argv[2]
if mode == "choice":  # C3 minibatch draws, 256 rounds in one call (the trainer's non-overlapped chunk)
    _dopt.mt_choice_rounds(256, [512] * 4096, 16)
else:  # C3 full-shard stream advance, 512 rounds in one call
    _dopt.mt_advance_rounds(512, [512] * 4096)
peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
print((peak - base) / 1024.0, time.time() - t0)
"""


@pytest.mark.parametrize("mode,cap_mb", [("choice", 900), ("advance", 300)])
def test_parallel_draw_memory_is_bounded(mode, cap_mb):
    """the parallel filter keeps at most a bounded number of segments' buffers
    (run-ahead bound, stitched segments released) and minibatch draws go in parts of at most
    32 segments of kept values -- a C3-sized call no longer holds ~3 GB.  Run in a fresh process
    so the peak resident set is this call's (4 filter threads)."""
    import subprocess
    import sys

    env = dict(os.environ, DOPT_MT_THREADS="4", DOPT_NO_TORCH="1")
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-optimization_amd")
    r = subprocess.run([sys.executable, "-c", _RSS_PROBE, pkg, mode], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr
    grew_mb, secs = (float(v) for v in r.stdout.split())
    assert grew_mb < cap_mb, (grew_mb, secs)
