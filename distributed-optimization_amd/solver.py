"""Device f(x*) solver.

The reference gets the optimum from sklearn's saga solver on the host
(simulator.py:32-69: LogisticRegression / Ridge with alpha = lambda * n_samples and a
fitted intercept, evaluated afterwards with obj_problems.py:3-11 / :39-44).  At the
BASELINE sizes
(2M-33M rows x 1024, or 16k rows x 2^20) that is out of reach, so this module
minimises the SAME objective the trainers report -- f(w) = mean loss + lam/2 ||w||^2,
bias included in the regulariser as obj_problems.py does -- with L-BFGS on the
host driving one fused device pass per evaluation (Engine.eval_full).

Note: sklearn does not regularise its intercept, so its w* is not the minimiser
of f; the Simulator keeps sklearn for parity with the reference's f_opt.
"""
import numpy as np


def reference_optimum(engine, lam, w0=None, max_iter=1000, gtol=1e-10):
    """Minimise the engine's full-data objective; returns (f_opt, w_opt, info)."""
    from scipy.optimize import minimize

    w0 = np.zeros(engine.d) if w0 is None else np.asarray(w0, dtype=np.float64)
    calls = [0]

    def fg(w):
        calls[0] += 1
        return engine.eval_full(w, lam)

    res = minimize(fg, w0, jac=True, method="L-BFGS-B",
                   options={"maxiter": max_iter, "gtol": gtol, "ftol": 1e-15, "maxcor": 20})
    return float(res.fun), res.x, {"evaluations": calls[0], "iterations": int(res.nit),
                                   "grad_norm": float(np.linalg.norm(res.jac)), "message": str(res.message)}
