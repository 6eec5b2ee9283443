"""Synthetic non-IID shards (drop-in for utils.py:5-50).

Same sklearn generators, seeds, scaling, bias column and argsort/array_split
sharding as the reference; setup-time host code, not on the hot path.  For the
large BASELINE configs the shards are generated on the device instead
(_dopt.Engine.generate_shards).
"""
import numpy as np
from sklearn.datasets import make_classification, make_regression
from sklearn.preprocessing import StandardScaler


def _make(config):
    kind = config["problem_type"]
    n, nf, ni = config["n_samples"], config["n_features"], config["n_informative_features"]
    if kind == "logistic":
        X, y = make_classification(n_samples=n, n_features=nf, n_informative=ni, n_redundant=nf - ni,
                                   n_clusters_per_class=1, flip_y=0.05,
                                   class_sep=config.get("classification_sep", 0.8), random_state=203)
        return X, 2 * y - 1  # labels in {-1, +1}
    if kind == "quadratic":
        X, y, _ = make_regression(n_samples=n, n_features=nf, n_informative=ni, noise=10.0, coef=True,
                                  random_state=203)
        return X, y
    raise NotImplementedError(f"Wrong {kind}")


def generate_and_preprocess_data(n_workers, config):
    print("Generating Non-IID data")
    X, y = _make(config)
    Xs = StandardScaler().fit_transform(X)
    X_bias = np.concatenate([Xs, np.ones((Xs.shape[0], 1))], axis=1)
    shards = []
    for i, idx in enumerate(np.array_split(np.argsort(y), n_workers)):  # non-IID: sorted labels
        Xi, yi = X_bias[idx, :], y[idx]
        shards.append({"X": Xi, "y": yi})
        print(f"Worker {i}: {len(idx)} samples, Target y range: [{np.min(yi):.2f}, {np.max(yi):.2f}], "
              f"Mean y: {np.mean(yi):.2f}")
    print(f"Generated {X.shape[0]} samples, {X_bias.shape[1]} features")
    return shards, X_bias.shape[1], X_bias, y
