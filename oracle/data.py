"""Shard generation for the oracle -- TEST INFRASTRUCTURE ONLY.

Restates utils.generate_and_preprocess_data (utils.py:5-50): sklearn
make_classification / make_regression with random_state=203, StandardScaler,
a ones bias column (utils.py:28), non-IID split by argsort(y) + array_split
(utils.py:34-43).  `order` overrides the argsort result so a fixture's recorded
shard order is used verbatim (the unstable argsort over +-1 ties is
platform-dependent).
"""
import hashlib

import numpy as np
from sklearn.datasets import make_classification, make_regression
from sklearn.preprocessing import StandardScaler


def generate(config, order=None):
    problem = config["problem_type"]
    n, nf = config["n_samples"], config["n_features"]
    ni = config["n_informative_features"]
    if problem == "logistic":
        X, y = make_classification(n_samples=n, n_features=nf, n_informative=ni,
                                   n_redundant=nf - ni, n_clusters_per_class=1, flip_y=0.05,
                                   class_sep=config.get("classification_sep", 0.8),
                                   random_state=203)
        y = 2 * y - 1
    elif problem == "quadratic":
        X, y, _ = make_regression(n_samples=n, n_features=nf, n_informative=ni,
                                  noise=10.0, coef=True, random_state=203)
    else:
        raise NotImplementedError(f"Wrong {problem}")
    Xb = np.hstack([StandardScaler().fit_transform(X), np.ones((X.shape[0], 1))])
    if order is None:
        order = np.argsort(y)
    shards = [(Xb[idx, :], y[idx]) for idx in np.array_split(order, config["n_workers"])]
    return shards, Xb, y


def digest(shards):
    h = hashlib.sha256()
    for X, y in shards:
        h.update(np.ascontiguousarray(X, dtype=np.float64).tobytes())
        h.update(np.ascontiguousarray(y).astype(np.float64).tobytes())
    return h.hexdigest()
