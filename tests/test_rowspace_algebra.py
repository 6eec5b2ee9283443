"""CPU check of the row-space algebra the C5 kernels implement (csrc/rowspace.hip): the
recurrences for xbar, Z, z, v, beta and the consensus expansion, restated in numpy exactly as
k_rs_pass / k_rs_rows / k_rs_cols order them, reproduce the oracle's D-SGD trajectory
(trainer.py:161-193, complete graph, quadratic and logistic objectives) and iterates to float64 rounding."""
import numpy as np
import pytest

import dsgd_oracle as O
import topology as TP


def rowspace_run(shards, W_off, W_ii, T, eta0, mu, lam_obj, x0, problem="quadratic"):
    """Row-space D-SGD from equal starting iterates x0 (one vector); returns (obj, cons, models).
    The gradient's row weights: z - y (quadratic) or -y expit(-y z) (logistic), over m_i."""
    n = len(shards)
    d = x0.shape[0]
    m = [len(s[1]) for s in shards]
    gram = [X @ X.T for X, _ in shards]
    Z = x0.copy()
    xbar = x0.copy()
    z = [X @ x0 for X, _ in shards]
    v = [zi.copy() for zi in z]
    beta = [np.zeros(mi) for mi in m]

    def weight(zi, yi, mi):
        return ((zi - yi) if problem == "quadratic" else -yi / (1.0 + np.exp(yi * zi))) / mi

    def loss(ui, yi):
        if problem == "quadratic":
            return 0.5 * np.sum((ui - yi) ** 2)
        t = yi * ui
        return np.sum(np.maximum(0.0, -t) + np.log(1.0 + np.exp(-np.abs(t))))

    coef = [weight(z[i], shards[i][1], m[i]) for i in range(n)]
    a1 = W_off * n
    rows = sum(m)
    obj, cons = [], []

    def metrics(u):
        ls = sum(loss(u[i], shards[i][1]) for i in range(n))
        dn = np.sum((Z - xbar) ** 2)
        cs = sum(dn + np.sum(beta[i] * (2.0 * (v[i] - u[i]) + gram[i] @ beta[i])) for i in range(n))
        return ls / rows + lam_obj / 2 * np.dot(xbar, xbar), cs / n

    for t in range(T + 1):
        u = [X @ xbar for X, _ in shards]  # the pass's dots at xbar_t
        if t > 0:
            o, c = metrics(u)  # metrics of x_t (history[t-1])
            obj.append(o)
            cons.append(c)
        if t == T:
            break
        eta = eta0 / np.sqrt(t + 1)
        q = W_ii - W_off - eta * mu
        C = sum(shards[i][0].T @ coef[i] for i in range(n))  # the pass's column sums
        for i in range(n):
            zn = a1 * u[i] + q * z[i] - eta * (gram[i] @ coef[i])
            v[i] = a1 * u[i] + q * v[i]
            beta[i] = q * beta[i] - eta * coef[i]
            z[i] = zn
            coef[i] = weight(zn, shards[i][1], m[i])
        Z, xbar = a1 * xbar + q * Z, (a1 + q) * xbar - (eta / n) * C
    models = np.stack([Z + shards[i][0].T @ beta[i] for i in range(n)])
    return np.array(obj), np.array(cons), models


@pytest.mark.parametrize("problem", ["quadratic", "logistic"])
@pytest.mark.parametrize("sizes,d,start", [([6] * 7, 40, "zero"), ([5, 1, 8, 3, 8, 2], 30, "common"),
                                           ([4] * 9, 10, "common")])  # d < N m: rows span R^d
def test_rowspace_recurrences_match_oracle(sizes, d, start, problem):
    rng = np.random.default_rng(len(sizes) * d)
    shards = [(np.hstack([rng.standard_normal((mi, d - 1)), np.ones((mi, 1))]),
               rng.standard_normal(mi) * 3 if problem == "quadratic" else rng.choice([-1.0, 1.0], mi))
              for mi in sizes]
    n, T, eta0, mu, lam = len(sizes), 25, 0.05, 2e-3, 1e-3
    top = TP.fully_connected(n)
    w_off, diag = top.uniform_offdiag()
    x0 = np.zeros(d) if start == "zero" else rng.standard_normal(d) * 0.1
    reg = mu if problem == "quadratic" else lam  # worker.py:36-42
    obj, cons, models = rowspace_run(shards, w_off, diag[0], T, eta0, reg, lam, x0, problem)
    cfg = {"problem_type": problem, "local_batch_size": max(sizes), "learning_rate_eta0": eta0,
           "l2_regularization_lambda": lam, "strong_convexity_mu": mu}
    Xf = np.vstack([s[0] for s in shards])
    yf = np.concatenate([s[1] for s in shards])
    h, _, xr, _ = O.run_decentralized(shards, top.dense_W(), T, cfg, Xf, yf, 0.0, x0=np.tile(x0, (n, 1)))
    np.testing.assert_allclose(obj, h["objective"], rtol=1e-11)
    np.testing.assert_allclose(cons, h["consensus_error"], rtol=1e-8)
    np.testing.assert_allclose(models, xr, rtol=1e-10, atol=1e-12)
