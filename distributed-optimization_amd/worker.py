"""Worker (drop-in for worker.py:4-44).

Holds one shard and the local iterate.  Minibatch indices come from the native
legacy-MT19937 sampler in libdopt.so operating on numpy's global RandomState, so
the index stream is bit-identical to np.random.choice(m, b, replace=False)
(worker.py:27); the gradient runs on the GPU (obj_problems.py in this package).
Inside DecentralizedTrainer / CentralizedTrainer.run the per-worker calls are
replaced by one batched device launch per round; these methods keep the
single-worker API.
"""
import numpy as np

import _dopt
from obj_problems import logistic_stochastic_gradient, quadratic_stochastic_gradient


class Worker:
    def __init__(self, worker_id, local_data, batch_size, n_features, config):
        self.worker_id = worker_id
        self.X_local = local_data["X"]
        self.y_local = local_data["y"]
        self.batch_size = batch_size
        self.n_local_samples = self.X_local.shape[0]
        self.config = config
        self.n_features = n_features
        self.x = np.zeros(n_features)

    def get_mini_batch(self):
        if self.n_local_samples == 0:  # worker.py:17-18
            return np.array([]).reshape(0, self.n_features), np.array([])
        eb = min(self.batch_size, self.n_local_samples)
        if eb <= 0:  # worker.py:21-23
            return np.array([]).reshape(0, self.n_features), np.array([])
        idxs = _dopt.mt_choice(self.n_local_samples, eb)
        return self.X_local[idxs], self.y_local[idxs]

    def compute_gradient(self, model_params=None):
        params = model_params if model_params is not None else self.x
        X_batch, y_batch = self.get_mini_batch()
        problem = self.config["problem_type"]
        # worker.py:36-37 reads BOTH keys before dispatching: a config without either raises
        # KeyError whatever the problem (after the draw, as in the reference)
        lambda_reg = self.config["l2_regularization_lambda"]
        mu_reg = self.config["strong_convexity_mu"]
        if problem == "logistic":
            return logistic_stochastic_gradient(params, X_batch, y_batch, lambda_reg)
        elif problem == "quadratic":
            return quadratic_stochastic_gradient(params, X_batch, y_batch, mu_reg)
        raise NotImplementedError(f"Wrong {problem}")
