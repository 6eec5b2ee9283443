"""Column-blocked rounds (d beyond the row-resident kernel: config C5, d = 2^20) and
complete-graph mean mixing, against the oracle (float64, rtol 1e-9) and against
host recomputation at full C5 row length."""

import numpy as np
import pytest

import _dopt
import dsgd_oracle as O
import topology as TP

pytestmark = pytest.mark.gpu


def _data(n, d, m, seed, problem):
    rng = np.random.default_rng(seed)
    shards = []
    for _ in range(n):
        X = np.hstack([rng.standard_normal((m, d - 1)), np.ones((m, 1))])
        y = rng.choice([-1.0, 1.0], m) if problem == "logistic" else rng.standard_normal(m) * 3
        shards.append((X, y))
    return shards


def _engine(shards, problem, dtype="float64"):
    """dtype 'float64/x32': float64 arithmetic over float32-stored rows."""
    if dtype == "float64/x32":
        eng = _dopt.Engine(0, "float64", data_dtype="float32")
    else:
        eng = _dopt.Engine(0, dtype)
    off = np.concatenate([[0], np.cumsum([len(s[1]) for s in shards])])
    eng.load_shards(problem, np.vstack([s[0] for s in shards]), np.concatenate([s[1] for s in shards]), off)
    return eng


def _f32_exact(shards):
    return [(X.astype(np.float32).astype(np.float64), y.astype(np.float32).astype(np.float64)) for X, y in shards]


@pytest.mark.parametrize("dtype", ["float64", "float64/x32"])
@pytest.mark.parametrize("problem,topo,batch,mean,m,rowspace", [
    ("logistic", "ring", 12, False, 12, "1"),        # full shard: next-round dots fused into the step
    ("logistic", "ring", 5, False, 12, "1"),         # minibatches: separate dots pass per round
    ("quadratic", "fully_connected", 12, True, 12, "0"),  # complete graph through column sums
    ("quadratic", "fully_connected", 12, True, 12, "1"),  # ... in row space (rowspace.hip)
    ("quadratic", "fully_connected", 5, True, 12, "1"),   # minibatches: direct rounds
    ("logistic", "fully_connected", 12, True, 12, "1"),   # logistic in row space
    ("quadratic", "grid", 4, False, 12, "1"),
    ("logistic", "ring", 24, False, 24, "1"),        # > 16 rows per worker: the row-split step kernel
])
def test_split_rounds_vs_oracle(problem, topo, batch, mean, m, rowspace, dtype, monkeypatch):
    """float64/x32: the same rounds over float32-stored rows under float64 arithmetic (data exactly
    float32; k_split_* / k_rs_pass_x32 <double, float>), against the same float64 oracle."""
    monkeypatch.setenv("DOPT_ROWSPACE", rowspace)
    n, d, T = 9, 2100, 6  # d = 2100 fp64 -> 1050 chunks > 1024: column-blocked path
    shards = _data(n, d, m, 1, problem)
    if dtype == "float64/x32":
        shards = _f32_exact(shards)
    cfg = {"problem_type": problem, "local_batch_size": batch, "learning_rate_eta0": 0.05,
           "l2_regularization_lambda": 1e-3, "strong_convexity_mu": 2e-3}
    top = TP.build(topo, n)
    eng = _engine(shards, problem, dtype)
    if mean:
        eng.set_mixing_mean(*top.uniform_offdiag())
    else:
        eng.set_topology(top.row_ptr, top.col, top.w)
    np.random.seed(4)
    st = np.random.get_state()
    idx = None if batch >= m else _dopt.mt_choice_rounds(T, [m] * n, batch)
    lam_g = cfg["l2_regularization_lambda"] if problem == "logistic" else cfg["strong_convexity_mu"]
    Xf = np.vstack([s[0] for s in shards])
    yf = np.concatenate([s[1] for s in shards])
    obj, cons, _ = eng.run_dsgd(T, 0.05, batch, lam_g, 1e-3, 0.1, idx=idx)
    x = eng.get_models()
    h, _, xr, _ = O.run_decentralized(shards, top.dense_W(), T, dict(cfg, l2_regularization_lambda=1e-3), Xf, yf,
                                      0.1, rng_state=st)
    np.testing.assert_allclose(x, xr, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(obj, h["objective"], rtol=1e-9)
    np.testing.assert_allclose(cons, h["consensus_error"], rtol=1e-9)
    eng.close()


def test_split_centralized_vs_oracle():
    n, d, m, T, b = 5, 2100, 10, 4, 3
    shards = _data(n, d, m, 2, "logistic")
    cfg = {"problem_type": "logistic", "local_batch_size": b, "learning_rate_eta0": 0.05,
           "l2_regularization_lambda": 1e-3, "strong_convexity_mu": 1e-3}
    eng = _engine(shards, "logistic")
    np.random.seed(8)
    st = np.random.get_state()
    idx = _dopt.mt_choice_rounds(T, [m] * n, b)
    Xf = np.vstack([s[0] for s in shards])
    yf = np.concatenate([s[1] for s in shards])
    obj, _ = eng.run_centralized(T, 0.05, b, 1e-3, 1e-3, 0.0, idx=idx)
    h, xg, _ = O.run_centralized(shards, T, cfg, Xf, yf, 0.0, rng_state=st)
    np.testing.assert_allclose(obj, h["objective"], rtol=1e-9)
    np.testing.assert_allclose(eng.get_global(), xg, rtol=1e-9, atol=1e-13)
    eng.close()


def test_c5_shape_round_spot_check():
    """C5 row length: quadratic, d = 2^20, m = b = 16, complete graph via column sums,
    fp32; 128 workers (8 GiB) on one GPU.  Two workers recomputed on the host."""
    n, d, m = 128, 1 << 20, 16
    eng = _dopt.Engine(0, "float32")
    eng.generate_shards("quadratic", n, d, m, seed=3, noise=10.0)
    top = TP.fully_connected(n)
    eng.set_mixing_mean(*top.uniform_offdiag())
    rng = np.random.default_rng(1)
    x0 = (rng.standard_normal((n, d)) * 1e-3).astype(np.float32).astype(np.float64)
    eng.set_models(x0)
    obj, cons, _ = eng.run_dsgd(1, 0.05, m, 1e-4, 1e-4, 0.0)
    x1 = eng.get_models()
    S = x0.sum(axis=0)
    w_off, diag = top.uniform_offdiag()
    for i in (0, 77):
        X, y = eng.get_shard(i)
        g = O.quadratic_gradient(x0[i], X, y, 1e-4)
        mix = w_off * (S - x0[i]) + diag[i] * x0[i]
        np.testing.assert_allclose(x1[i], mix - 0.05 * g, rtol=1e-3, atol=1e-5)
    xbar = x1.mean(axis=0)
    np.testing.assert_allclose(cons[0], np.mean(np.sum((x1 - xbar) ** 2, axis=1)), rtol=1e-3)
    assert np.isfinite(obj[0])
    eng.close()


@pytest.mark.parametrize("d", [2100, 5000])
def test_single_evaluations_wide_rows_vs_oracle(d):
    """The obj_problems.py API for rows beyond the row-resident kernel (d > 2048 in float64):
    k_wide_* kernels, rtol 1e-12 against the oracle -- the Simulator's f(x*) evaluation
    (simulator.py:32-69 calls the objectives) must work at any n_features."""
    import obj_problems as P

    rng = np.random.default_rng(d)
    w = rng.standard_normal(d) * 0.05
    for rows in (1, 13, 700):
        X = np.hstack([rng.standard_normal((rows, d - 1)), np.ones((rows, 1))])
        yl = rng.choice([-1.0, 1.0], rows)
        yq = rng.standard_normal(rows) * 3
        gl, gq = O.logistic_gradient(w, X, yl, 1e-3), O.quadratic_gradient(w, X, yq, 2e-3)
        # atol: entries that cancel to ~0 carry the rounding of the others (summation order only)
        np.testing.assert_allclose(P.logistic_stochastic_gradient(w, X, yl, 1e-3), gl, rtol=1e-12,
                                   atol=1e-13 * np.abs(gl).max())
        np.testing.assert_allclose(P.quadratic_stochastic_gradient(w, X, yq, 2e-3), gq, rtol=1e-12,
                                   atol=1e-13 * np.abs(gq).max())
        np.testing.assert_allclose(P.logistic_objective(w, X, yl, 1e-3), O.logistic_objective(w, X, yl, 1e-3),
                                   rtol=1e-12)
        np.testing.assert_allclose(P.quadratic_objective(w, X, yq, 2e-3), O.quadratic_objective(w, X, yq, 2e-3),
                                   rtol=1e-12)


@pytest.mark.parametrize("mean,rowspace", [(True, "0"), (True, "1"), (False, "1")])
def test_split_pipelined_runs_equal_one_run(mean, rowspace, monkeypatch):
    """Column-blocked rounds pipelined across calls (bench.py's C5 timing): the last step's
    next-round coefficients, S and xbar carry over, the owed metrics ride the next call's
    first step -- concatenated, exactly one run's history and iterates."""
    monkeypatch.setenv("DOPT_ROWSPACE", rowspace)
    n, d, m = 9, 2100, 12
    shards = _data(n, d, m, 7, "quadratic")
    eng = _engine(shards, "quadratic")
    top = TP.build("fully_connected" if mean else "ring", n)
    if mean:
        eng.set_mixing_mean(*top.uniform_offdiag())
    else:
        eng.set_topology(top.row_ptr, top.col, top.w)
    eng.set_models(np.zeros((n, d)))
    obj_ref, cons_ref, _ = eng.run_dsgd(9, 0.05, m, 2e-3, 2e-3, 0.1)
    x_ref = eng.get_models()
    eng.set_models(np.zeros((n, d)))
    objs, conss, t0 = [], [], 0
    for k in (3, 1, 5, 0):
        o, c = eng.run_dsgd_pipelined(k, 0.05, m, 2e-3, 2e-3, 0.1, t0=t0)
        objs.append(o)
        conss.append(c)
        t0 += k
    assert np.array_equal(np.concatenate(objs), obj_ref)
    assert np.array_equal(np.concatenate(conss), cons_ref)
    assert np.array_equal(eng.get_models(), x_ref)
    eng.close()


@pytest.mark.parametrize("dtype", ["float64", "float64/x32", "float32"])
def test_tiled_rows_round_trip(dtype):
    """Column-blocked contexts store the shards column-block tiled (kcommon.h XAddr): uploads
    (ragged shards, a partial last tile) come back unchanged through dopt_get_shard, and generated
    shards hold exactly the values of the same rows generated into a row-major (row-resident)
    float32 context -- the generator is a function of (global row, column) only."""
    rng = np.random.default_rng(11)
    d = 2100 if dtype != "float32" else 5000
    sizes = [3, 1, 7, 0, 5]
    shards = [(rng.standard_normal((m, d)), rng.standard_normal(m)) for m in sizes]
    if dtype == "float64/x32":
        shards = _f32_exact(shards)
    eng = _engine(shards, "quadratic", dtype)
    for (X, y), i in zip(shards, range(len(sizes))):
        Xg, yg = eng.get_shard(i)
        np.testing.assert_array_equal(Xg, X.astype(np.float32) if dtype == "float32" else X)
        np.testing.assert_array_equal(yg, y.astype(np.float32) if dtype == "float32" else y)
    eng.close()
    # generated: the x32 context (tiled, d = 2100 past the mixed row-resident kernel) vs the float32
    # engine (row-resident at d = 2100, row-major): the same float32 values
    if dtype == "float64/x32":
        a = _dopt.Engine(0, "float64", data_dtype="float32")
        b = _dopt.Engine(0, "float32")
        for e in (a, b):
            e.generate_shards("logistic", 6, 2100, 5, seed=17, flip=0.1, first_worker=3)
        for i in range(6):
            for u, v in zip(a.get_shard(i), b.get_shard(i)):
                np.testing.assert_array_equal(u, v)
        a.close()
        b.close()


@pytest.mark.parametrize("dtype", ["float64", "float64/x32"])
def test_split_rounds_separate_objective_data_vs_oracle(dtype, monkeypatch):
    """A separate X_full (trainer.py:154, 188-189) on a column-blocked context: the objective rows
    are uploaded tiled too (their own tile stride) and read by the dots-only pass; every round's
    objective and consensus vs the oracle (rtol 1e-9)."""
    monkeypatch.setenv("DOPT_ROWSPACE", "1")
    n, d, m, T = 7, 2100, 6, 5
    shards = _data(n, d, m, 21, "logistic")
    rng = np.random.default_rng(22)
    Xo = np.hstack([rng.standard_normal((37, d - 1)), np.ones((37, 1))])
    yo = rng.choice([-1.0, 1.0], 37)
    if dtype == "float64/x32":
        shards = _f32_exact(shards)
        Xo, yo = _f32_exact([(Xo, yo)])[0]
    cfg = {"problem_type": "logistic", "local_batch_size": m, "learning_rate_eta0": 0.05,
           "l2_regularization_lambda": 1e-3, "strong_convexity_mu": 1e-3}
    top = TP.build("ring", n)
    eng = _engine(shards, "logistic", dtype)
    eng.set_topology(top.row_ptr, top.col, top.w)
    eng.load_objective_data(Xo, yo)
    obj, cons, _ = eng.run_dsgd(T, 0.05, m, 1e-3, 1e-3, 0.05)
    x = eng.get_models()
    h, _, xr, _ = O.run_decentralized(shards, top.dense_W(), T, cfg, Xo, yo, 0.05,
                                      indices=[[np.arange(m)] * n] * T)
    np.testing.assert_allclose(obj, h["objective"], rtol=1e-9)
    np.testing.assert_allclose(cons, h["consensus_error"], rtol=1e-9)
    np.testing.assert_allclose(x, xr, rtol=1e-9, atol=1e-13)
    eng.close()
