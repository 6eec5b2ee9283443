"""Objectives and gradients (drop-in for obj_problems.py), evaluated on the GPU.

Same names, signatures, return types and edge cases as the reference:
  logistic_objective(w, X, y, lambda_reg)            obj_problems.py:3-11
  logistic_stochastic_gradient(w, Xb, yb, lambda_reg) obj_problems.py:13-20
  logistic_full_gradient(w, workers, lambda_reg)     obj_problems.py:22-36
  quadratic_objective(w, X, y, mu_reg)               obj_problems.py:39-44
  quadratic_stochastic_gradient(w, Xb, yb, mu_reg)   obj_problems.py:46-53
  quadratic_full_gradient(w, workers, mu_reg)        obj_problems.py:55-69
Empty inputs return 0.0 / zeros_like(w) on the host exactly as upstream; every
other call runs the float64 HIP kernels through libdopt.so (no CPU fallback).
The trainers do NOT call these per worker: their rounds run batched on the
device (trainer.py in this package).
"""
import numpy as np

import _dopt


def _eng():
    return _dopt.default_engine()


def logistic_objective(w, X, y, lambda_reg):
    if X.shape[0] == 0:
        return 0.0
    return _eng().eval_objective("logistic", w, X, y, lambda_reg)


def logistic_stochastic_gradient(w, X_batch, y_batch, lambda_reg):
    if X_batch.shape[0] == 0:
        return np.zeros_like(w)
    return _eng().eval_gradient("logistic", w, X_batch, y_batch, lambda_reg)


def _full(problem, w, workers, reg):
    Xs = [wk.X_local for wk in workers if wk.X_local.shape[0] > 0]
    if not Xs:
        return np.zeros_like(w)
    ys = [wk.y_local for wk in workers if wk.X_local.shape[0] > 0]
    # sum over every shard / total rows + reg * w == the gradient over the union
    return _eng().eval_gradient(problem, w, np.vstack(Xs), np.concatenate(ys), reg)


def logistic_full_gradient(w, workers, lambda_reg):
    """full gradient for across all workers' data."""
    return _full("logistic", w, workers, lambda_reg)


def quadratic_objective(w, X, y, mu_reg):
    if X.shape[0] == 0:
        return 0.0
    return _eng().eval_objective("quadratic", w, X, y, mu_reg)


def quadratic_stochastic_gradient(w, X_batch, y_batch, mu_reg):
    if X_batch.shape[0] == 0:
        return np.zeros_like(w)
    return _eng().eval_gradient("quadratic", w, X_batch, y_batch, mu_reg)


def quadratic_full_gradient(w, workers, mu_reg):
    """full gradient across all workers' data"""
    return _full("quadratic", w, workers, mu_reg)
