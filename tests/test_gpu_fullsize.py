"""Configs C3, C4 and C5 at full size on ONE MI355X (288 GB of HBM holds any of them).

C3: the headline benchmark's exact instance (bench.py): 4096 workers, d = 1024, m = b = 512, random
    4-regular graph, float64 over float32-stored rows, pipelined as the bench times it; every round
    and the objective over all 2M rows recomputed on the host.
C4: logistic, N = 65536 workers on the 256 x 256 torus, d = 1024, m = b = 512 -- the
    configuration the reference cannot run (trainer.py:93,118 build dense N x N matrices:
    64 GiB at this N).  Float64 arithmetic over float32-stored exact rows (137 GB of shards).
C5: quadratic, N = 1024 workers, d = 2^20, m = b = 16, complete graph mixed through the
    column sums (trainer.py:109-110, 173), float32 (64 GiB of shards): the column-blocked
    round kernels.

Both run T = 3 rounds in one call and are checked against host recomputation in float64 of
the reference's round (trainer.py:161-193) from the downloaded shards: the updates of
workers on the torus wrap-around rows / columns and random ones, every worker's consensus,
and (C5) every round, re-run round by round from the same start.  C4's float64 checks are
rtol 1e-10 (summation order only); C5's float32 ones 2e-4 (the float32 engine vs the
float64 host recomputation of one round).
"""
import numpy as np
import pytest

import _dopt
import dsgd_oracle as O
import topology as TP

pytestmark = pytest.mark.gpu


def _free_gb():
    import torch

    free, _ = torch.cuda.mem_get_info(0)
    return free / 1e9


def _mix_row(top, x, i):
    s, e = top.row_ptr[i], top.row_ptr[i + 1]
    acc = np.zeros(x.shape[1])
    for k in range(s, e):  # CSR order, as the kernel sums
        acc = acc + top.w[k] * x[top.col[k]]
    return acc


def test_c3_headline_instance_full_size():
    """C3 exactly as bench.py times it (4096 workers, d = 1024, m = b = 512, the random 4-regular
    graph of seed 0, the same device-generated shards, float64 arithmetic over float32-stored rows,
    a pipelined chain from the reference's zero start, worker.py:13): the chain runs the headline
    kernel instance, and its history equals three one-round calls, each checked on the host --
    sampled workers' updates (trainer.py:166-175), the consensus over all 4096 iterates
    (trainer.py:182-186), and the objective at xbar over all 2M rows (trainer.py:188-191) by the
    oracle's numpy formula, shard by shard."""
    n, d, m, T, eta0, lam = 4096, 1024, 512, 3, 0.05, 1e-4
    if _free_gb() < 20:
        pytest.skip("needs ~15 GB of free HBM")
    top = TP.random_regular(n, 4, seed=0)
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    try:
        eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
        eng.set_topology(top.row_ptr, top.col, top.w)
        # the bench's form: pipelined calls (the last iterate's metrics owed to the next call)
        eng.zero_models()
        o0, c0 = eng.run_dsgd_pipelined(1, eta0, m, lam, lam, 0.0, t0=0)
        o1, c1 = eng.run_dsgd_pipelined(2, eta0, m, lam, lam, 0.0, t0=1)
        assert _dopt.last_round_kernel().startswith("void dopt::k_round<double, float, 4, 0, true, true,")
        o2, c2 = eng.run_dsgd_pipelined(0, eta0, m, lam, lam, 0.0, t0=3)
        obj_p, cons_p = np.concatenate([o0, o1, o2]), np.concatenate([c0, c1, c2])
        assert len(obj_p) == T and len(cons_p) == T
        x_p = eng.get_models()

        eng.zero_models()
        x = np.zeros((n, d))
        rng = np.random.default_rng(5)
        picks = [0, 1, n - 1] + [int(i) for i in rng.choice(n, 9, replace=False)]
        shards = {i: eng.get_shard(i) for i in picks}
        xbars = []
        for t in range(T):  # one round per call: every round's updates and metrics pinned on the host
            obj, cons, _ = eng.run_dsgd(1, eta0, m, lam, lam, 0.0, t0=t)
            xn = eng.get_models()
            eta = eta0 / np.sqrt(t + 1)  # trainer.py:138-140
            for i in picks:
                X, y = shards[i]
                ref = _mix_row(top, x, i) - eta * O.logistic_gradient(x[i], X, y, lam)
                np.testing.assert_allclose(xn[i], ref, rtol=1e-10, atol=1e-13)
            xbar = xn.mean(axis=0)
            np.testing.assert_allclose(cons[0], np.mean(np.sum((xn - xbar) ** 2, axis=1)), rtol=1e-10)
            np.testing.assert_allclose(cons_p[t], cons[0], rtol=1e-11)
            np.testing.assert_allclose(obj_p[t], obj[0], rtol=1e-12)
            xbars.append((xbar, obj[0]))
            x = xn
        np.testing.assert_allclose(x_p, x, rtol=1e-11, atol=1e-14)
        # the objective at every round's xbar over all 4096 x 512 rows: the oracle's formula
        # (obj_problems.py:3-11) per shard, summed over shards
        W = np.stack([xb for xb, _ in xbars], axis=1)
        loss = np.zeros(T)
        for i in range(n):
            X, y = eng.get_shard(i)
            yz = y[:, None] * (X @ W)
            loss += np.sum(np.maximum(0, -yz) + np.log(1 + np.exp(-np.abs(yz))), axis=0)
        for t, (xb, f) in enumerate(xbars):
            np.testing.assert_allclose(f, loss[t] / (n * m) + lam / 2.0 * np.dot(xb, xb), rtol=1e-10)
    finally:
        eng.close()


def test_c4_torus_65536_workers_full_size():
    n, d, m, T, eta0, lam = 65536, 1024, 512, 3, 0.05, 1e-4
    if _free_gb() < 150:
        pytest.skip("needs ~140 GB of free HBM")
    top = TP.grid(n)
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    try:
        eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
        eng.set_topology(top.row_ptr, top.col, top.w)
        rng = np.random.default_rng(2)
        x0 = rng.standard_normal((n, d)) * 1e-2
        # torus corners / wrap-around rows and columns (neighbours ids i +- 1 mod 256, i +- 256 mod 65536)
        picks = [0, 255, 256, 511, 65280, 65535, 32767, 32768] + [int(i) for i in rng.choice(n, 8, replace=False)]
        shards = {i: eng.get_shard(i) for i in picks}
        eng.set_models(x0)
        x, per_obj, per_cons = x0, [], []
        for t in range(T):  # one round per call: every round's updates, consensus and objective pinned
            obj, cons, _ = eng.run_dsgd(1, eta0, m, lam, lam, 0.0, t0=t)
            xn = eng.get_models()
            eta = eta0 / np.sqrt(t + 1)  # trainer.py:138-140
            for i in picks:
                X, y = shards[i]
                g = O.logistic_gradient(x[i], X, y, lam)
                np.testing.assert_allclose(xn[i], _mix_row(top, x, i) - eta * g, rtol=1e-10, atol=1e-13)
            xbar = xn.mean(axis=0)
            np.testing.assert_allclose(cons[0], np.mean(np.sum((xn - xbar) ** 2, axis=1)), rtol=1e-10)
            # the objective at xbar over all 33.5M rows (trainer.py:188-191): an independent device
            # evaluation (dopt_eval_full, pinned to the oracle in test_full_evaluation_and_device_optimum)
            f_ref, _ = eng.eval_full(xbar, lam)
            np.testing.assert_allclose(obj[0], f_ref, rtol=1e-10)
            per_obj.append(obj[0])
            per_cons.append(cons[0])
            x = xn
        # the same T rounds in one call (the fused path: the metrics of round t in round t+1's pass)
        eng.set_models(x0)
        obj_all, cons_all, _ = eng.run_dsgd(T, eta0, m, lam, lam, 0.0)
        np.testing.assert_allclose(obj_all, per_obj, rtol=1e-12)
        np.testing.assert_allclose(cons_all, per_cons, rtol=1e-12)
        np.testing.assert_allclose(eng.get_models(), x, rtol=1e-13, atol=1e-16)
    finally:
        eng.close()


def test_c5_d2pow20_1024_workers_full_size():
    n, d, m, T, eta0, lam = 1024, 1 << 20, 16, 3, 1e-5, 1e-4
    if _free_gb() < 75:
        pytest.skip("needs ~70 GB of free HBM")
    top = TP.fully_connected(n)
    w_off, diag = top.uniform_offdiag()
    eng = _dopt.Engine(0, "float32")
    try:
        eng.generate_shards("quadratic", n, d, m, seed=3, noise=10.0)
        eng.set_mixing_mean(w_off, diag)
        rng = np.random.default_rng(1)
        x0 = (rng.standard_normal((n, d)) * 1e-3).astype(np.float32).astype(np.float64)
        eng.set_models(x0)
        obj_all, cons_all, _ = eng.run_dsgd(T, eta0, m, lam, lam, 0.0)  # T rounds, one call
        x_all = eng.get_models()
        eng.set_models(x0)
        x = x0
        picks = [0, 1, 511, 1023] + list(rng.choice(n, 4, replace=False))
        shards = {int(i): eng.get_shard(int(i)) for i in picks}
        for t in range(T):  # the same rounds one call each: every round checked on the host
            obj, cons, _ = eng.run_dsgd(1, eta0, m, lam, lam, 0.0, t0=t)
            xn = eng.get_models()
            S = x.sum(axis=0)
            eta = eta0 / np.sqrt(t + 1)
            for i in picks:
                X, y = shards[int(i)]
                g = O.quadratic_gradient(x[i], X, y, lam)
                ref = w_off * (S - x[i]) + diag[i] * x[i] - eta * g
                np.testing.assert_allclose(xn[i], ref, rtol=2e-4, atol=2e-6 * np.abs(ref).max())
            xb = xn.mean(axis=0)
            np.testing.assert_allclose(cons[0], np.mean(np.sum((xn - xb) ** 2, axis=1)), rtol=1e-3)
            np.testing.assert_allclose(cons[0], cons_all[t], rtol=1e-5)
            np.testing.assert_allclose(obj[0], obj_all[t], rtol=1e-5)
            # the objective at xbar over all 16384 rows (trainer.py:188-191) by an independent pass
            # (dopt_eval_full: the dots-only kernel at the shared point), float32 engine
            np.testing.assert_allclose(obj[0], eng.eval_full(xb, lam, gradient=False)[0], rtol=1e-5)
            x = xn
        # one call (next round's coefficients fused into the step) or T calls (a dots pass per call):
        # the same rounds up to the row-dot summation tree
        np.testing.assert_allclose(x, x_all, rtol=1e-5, atol=1e-7 * np.abs(x_all).max())
    finally:
        eng.close()


def test_c5_rowspace_full_size_vs_direct(monkeypatch):
    """C5 from the reference's start (Worker.x = zeros, worker.py:13) through the row-space rounds
    (rowspace.hip, the bench's C5 path): round 1 recomputed on the host for several workers,
    then rounds 2-3 continued from the live row-space state, against the direct column-blocked
    rounds (DOPT_ROWSPACE=0) on the same 64 GiB of float32 shards."""
    n, d, m, T, eta0, lam = 1024, 1 << 20, 16, 3, 1e-5, 1e-4
    if _free_gb() < 80:
        pytest.skip("needs ~75 GB of free HBM")
    top = TP.fully_connected(n)
    w_off, diag = top.uniform_offdiag()
    eng = _dopt.Engine(0, "float32")
    try:
        eng.generate_shards("quadratic", n, d, m, seed=3, noise=10.0)
        eng.set_mixing_mean(w_off, diag)
        monkeypatch.setenv("DOPT_ROWSPACE", "1")
        o1, c1, _ = eng.run_dsgd(1, eta0, m, lam, lam, 0.0)
        assert "k_rs_pass<float, true," in _dopt.last_round_kernel()
        x1 = eng.get_models()
        for i in (0, 1, 700, 1023):  # x_1 = mix(0) - eta (X^T (0 - y) / m + lam 0)
            X, y = eng.get_shard(i)
            ref = -eta0 * O.quadratic_gradient(np.zeros(d), X, y, lam)
            np.testing.assert_allclose(x1[i], ref, rtol=2e-5, atol=1e-7 * np.abs(ref).max())
        xb = x1.mean(axis=0)
        np.testing.assert_allclose(c1[0], np.mean(np.sum((x1 - xb) ** 2, axis=1)), rtol=1e-4)
        np.testing.assert_allclose(o1[0], eng.eval_full(xb, lam, gradient=False)[0], rtol=1e-5)
        del x1
        o23, c23, _ = eng.run_dsgd(T - 1, eta0, m, lam, lam, 0.0, t0=1)
        x_rs = eng.get_models()
        monkeypatch.setenv("DOPT_ROWSPACE", "0")
        eng.set_models(np.zeros((n, d), dtype=np.float32))
        od, cd, _ = eng.run_dsgd(T, eta0, m, lam, lam, 0.0)
        assert "k_split_step" in _dopt.last_round_kernel()
        np.testing.assert_allclose(np.concatenate([o1, o23]), od, rtol=1e-4)
        np.testing.assert_allclose(np.concatenate([c1, c23]), cd, rtol=1e-4)
        x_d = eng.get_models()
        np.testing.assert_allclose(x_rs, x_d, rtol=1e-4, atol=1e-5 * np.abs(x_d).max())
    finally:
        eng.close()


def test_c5_x32_full_size_host_rounds(monkeypatch):
    """C5 at the reference's float64 arithmetic over float32-stored rows (k_rs_pass_x32, the bench's
    C5 default) from Worker.x = zeros: every round recomputed on the host for several workers
    (mixing sum over all iterates, float64 gradient; trainer.py:173-175) at rtol 1e-8, consensus
    over all iterates, and the per-round calls equal to one 3-round call."""
    n, d, m, T, eta0, lam = 1024, 1 << 20, 16, 3, 1e-5, 1e-4
    if _free_gb() < 90:
        pytest.skip("needs ~85 GB of free HBM")
    top = TP.fully_connected(n)
    w_off, diag = top.uniform_offdiag()
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    try:
        eng.generate_shards("quadratic", n, d, m, seed=3, noise=10.0)
        eng.set_mixing_mean(w_off, diag)
        o_all, c_all, _ = eng.run_dsgd(T, eta0, m, lam, lam, 0.0)
        assert _dopt.last_round_kernel().startswith("void dopt::k_rs_pass_x32<true,")
        x_all = eng.get_models()
        eng.set_models(np.zeros((n, d)))
        picks = [0, 1, 511, 1023, 77, 640]
        shards = {i: eng.get_shard(i) for i in picks}
        x = None
        for t in range(T):
            o, c, _ = eng.run_dsgd(1, eta0, m, lam, lam, 0.0, t0=t)
            xn = eng.get_models()
            eta = eta0 / np.sqrt(t + 1)
            S = x.sum(axis=0) if x is not None else None
            for i in picks:
                X, y = shards[i]
                xi = x[i] if x is not None else np.zeros(d)
                mix = w_off * (S - xi) + diag[i] * xi if x is not None else np.zeros(d)
                ref = mix - eta * O.quadratic_gradient(xi, X, y, lam)
                np.testing.assert_allclose(xn[i], ref, rtol=1e-8, atol=1e-10 * np.abs(ref).max())
            xb = xn.mean(axis=0)
            np.testing.assert_allclose(c[0], np.mean(np.sum((xn - xb) ** 2, axis=1)), rtol=1e-8)
            np.testing.assert_allclose(c[0], c_all[t], rtol=1e-12)
            np.testing.assert_allclose(o[0], o_all[t], rtol=1e-12)
            # the objective at xbar over all 16384 rows (trainer.py:188-191) by an independent pass:
            # dopt_eval_full's dots-only kernel over the float32 rows, float64 arithmetic
            np.testing.assert_allclose(o[0], eng.eval_full(xb, lam, gradient=False)[0], rtol=1e-10)
            x = xn
        np.testing.assert_allclose(x, x_all, rtol=1e-12, atol=1e-14 * np.abs(x_all).max())
        # the same 3 rounds by the DIRECT column-blocked kernels over the float32 rows (k_split_step
        # <double, float, ...>: the row-space rounds off), from the same zero start
        monkeypatch.setenv("DOPT_ROWSPACE", "0")
        eng.set_models(np.zeros((n, d)))
        od, cd, _ = eng.run_dsgd(T, eta0, m, lam, lam, 0.0)
        assert _dopt.last_round_kernel().startswith("void dopt::k_split_step<double, float,")
        np.testing.assert_allclose(od, o_all, rtol=1e-10)
        np.testing.assert_allclose(cd, c_all, rtol=1e-9)
        np.testing.assert_allclose(eng.get_models(), x_all, rtol=1e-10, atol=1e-12 * np.abs(x_all).max())
    finally:
        eng.close()
