"""The oracle (oracle/dsgd_oracle.py) pinned against the reference's own outputs.

Every fixture here was produced by importing and running the reference
(tests/golden/make_golden.py).  float64 oracle vs float64 reference: the oracle
uses the same numpy calls, so most trajectories agree to the bit; the bound
used is rtol 1e-12.
"""
import json
import os

import numpy as np
import pytest

import data as odata
import dsgd_oracle as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(tag):
    return json.load(open(os.path.join(G, f"traj_{tag}.json"))), np.load(os.path.join(G, f"traj_{tag}.npz"))


def test_gradients_and_objectives():
    z = np.load(os.path.join(G, "grads.npz"))
    for k, (prob, d, b, scale) in enumerate(z["cases"]):
        w, X, y = z[f"c{k}_w"], z[f"c{k}_X"], z[f"c{k}_y"]
        name = "logistic" if prob == 0 else "quadratic"
        cfg = {"l2_regularization_lambda": 1e-4, "strong_convexity_mu": 1e-4}
        np.testing.assert_array_equal(O.gradient(name, w, X, y, cfg), z[f"c{k}_g"])
        assert O.objective(name, w, X, y, 1e-4) == z[f"c{k}_f"]
    for prob in ("logistic", "quadratic"):
        sh = [(z[f"full_{prob}_X{j}"], z[f"full_{prob}_y{j}"]) for j in range(3)]
        np.testing.assert_allclose(O.full_gradient(prob, z[f"full_{prob}_w"], sh, 1e-4), z[f"full_{prob}_g"],
                                   rtol=1e-14)
        np.testing.assert_array_equal(O.full_gradient(prob, z[f"full_{prob}_w"], [sh[1]], 1e-4),
                                      z[f"full_{prob}_gempty"])


def test_mixing_matrices_and_gaps():
    z = np.load(os.path.join(G, "mixing.npz"))
    gaps = json.load(open(os.path.join(G, "mixing_gaps.json")))
    for topo in ("ring", "grid", "fully_connected"):
        for n in (1, 2, 3, 4, 5, 9, 10, 16, 25, 36):
            key = f"{topo}_{n}"
            if key + "_error" in z:
                with pytest.raises(ValueError, match="not a perfect square"):
                    O.adjacency(topo, n)
                continue
            adj = O.adjacency(topo, n)
            np.testing.assert_array_equal(adj, z[key + "_adj"])
            W, deg = O.mh_matrix(adj)
            np.testing.assert_array_equal(W, z[key + "_W"])
            np.testing.assert_array_equal(deg, z[key + "_deg"])
            if n > 1:
                assert round(O.spectral_gap(W), 4) == gaps[key]
    # the report's values (PDF p.8), N = 25
    assert (gaps["ring_25"], gaps["grid_25"], gaps["fully_connected_25"]) == (0.0209, 0.2764, 1.0)


def test_rng_stream():
    z = np.load(os.path.join(G, "rng.npz"))
    rs = np.random.RandomState(203)
    for k, (m, b) in enumerate(z["specs"]):
        np.testing.assert_array_equal(O.minibatch_indices(rs, int(m), int(b)), z[f"call{k}_idx"])
        assert rs.get_state()[2] == z[f"call{k}_pos"]


@pytest.mark.parametrize("tag,rounds", [("c2", 400), ("c1", 400), ("n1", 200), ("n2", 300), ("n4", 300),
                                        ("ragged", 300), ("fullbatch", 60)])
def test_trajectories(tag, rounds):
    meta, z = _load(tag)
    cfg = meta["config"]
    shards, Xf, yf = odata.generate(cfg, order=z["order"])
    assert odata.digest(shards) == meta["data_sha256"]
    T = min(rounds, cfg["n_iterations"])
    for j, label in enumerate(meta["labels"]):
        st = ("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0)
        if label == "Centralized":
            h, _, _ = O.run_centralized(shards, T, cfg, Xf, yf, meta["f_opt"], rng_state=st)
        else:
            topo = {"D-SGD (Ring)": "ring", "D-SGD (Grid)": "grid", "D-SGD (Fully Connected)": "fully_connected"}[label]
            W, _ = O.mh_matrix(O.adjacency(topo, cfg["n_workers"]))
            h, _, _, _ = O.run_decentralized(shards, W, T, cfg, Xf, yf, meta["f_opt"], rng_state=st)
            np.testing.assert_allclose(h["consensus_error"], z[f"L{j}_consensus"][:T], rtol=1e-12)
        np.testing.assert_allclose(h["objective"], z[f"L{j}_objective"][:T], rtol=1e-12)


def test_table2_numbers_in_fixture():
    meta, z = _load("table2")
    its = [meta["numerical_results"][k]["iterations_to_threshold"] for k in meta["labels"]]
    assert its == [5425, 7214, 5666, 5549]  # PDF p.9, Table II
    tx = [meta["numerical_results"][k]["total_transmission_floats"] for k in meta["labels"]]
    assert tx == [4.05e7, 4.05e7, 8.10e7, 4.86e8]
    for j, k in enumerate(meta["labels"]):
        assert O.iterations_to_threshold(z[f"L{j}_objective"], 0.08) == its[j]


def test_direct_fixtures():
    z = np.load(os.path.join(G, "direct.npz"))
    for prob in ("logistic", "quadratic"):
        shards = [(z[f"{prob}_X{j}"], z[f"{prob}_y{j}"]) for j in range(6)]
        Xf = np.vstack([s[0] for s in shards])
        yf = np.concatenate([s[1] for s in shards])
        cfg = {"local_batch_size": 2, "learning_rate_eta0": 0.05, "l2_regularization_lambda": 1e-4,
               "strong_convexity_mu": 1e-4, "problem_type": prob}
        st = np.random.RandomState(203).get_state()
        h, x, _ = O.run_centralized(shards, 40, cfg, Xf, yf, 0.125, rng_state=st)
        np.testing.assert_allclose(h["objective"], z[f"{prob}_central_objective"], rtol=1e-12)
        for name, topo in (("ring", "ring"), ("fc", "fully_connected")):
            W, _ = O.mh_matrix(O.adjacency(topo, 6))
            h, xf, _, _ = O.run_decentralized(shards, W, 40, cfg, Xf, yf, 0.125, rng_state=st)
            np.testing.assert_allclose(h["objective"], z[f"{prob}_{name}_objective"], rtol=1e-12)
            np.testing.assert_allclose(h["consensus_error"], z[f"{prob}_{name}_consensus"], rtol=1e-12)
            np.testing.assert_allclose(xf, z[f"{prob}_{name}_final"], rtol=1e-12, atol=1e-15)


def test_partitioned_round_is_bit_exact():
    """P contiguous partitions with explicit halo copies == the unpartitioned sparse mix."""
    meta, z = _load("c2")
    cfg = meta["config"]
    shards, Xf, yf = odata.generate(cfg, order=z["order"])
    W, _ = O.mh_matrix(O.adjacency("ring", 10))
    st = ("MT19937", z["state1_key"], int(z["state1_pos"]), 0, 0.0)
    ref, _, xr, _ = O.run_decentralized(shards, W, 30, cfg, Xf, yf, meta["f_opt"], rng_state=st, mixing="sparse")
    for P in (2, 3, 4):
        h, _, xp, _ = O.run_decentralized(shards, W, 30, cfg, Xf, yf, meta["f_opt"], rng_state=st, partitions=P)
        np.testing.assert_array_equal(xp, xr)
        assert h["objective"] == ref["objective"]


def test_device_sampler_restatement_uniform_subsets():
    """oracle/device_sampler.py (the GPU's Philox + Floyd minibatch, restated): exactly
    min(b, m) distinct rows in [0, m), deterministic in (seed, round, worker), and uniform:
    over 4000 draws of 5 of 20 rows each row's count stays within 5 sigma of 1000."""
    import device_sampler as DS

    for m, b in ((20, 5), (7, 7), (5, 9), (1, 1), (300, 16)):
        s = DS.minibatch(3, 11, 2, m, b)
        assert len(s) == min(b, m) and len(np.unique(s)) == len(s) and s.min() >= 0 and s.max() < m
        np.testing.assert_array_equal(s, DS.minibatch(3, 11, 2, m, b))
    assert not np.array_equal(DS.minibatch(3, 11, 2, 300, 16), DS.minibatch(3, 12, 2, 300, 16))
    counts = np.zeros(20)
    for t in range(4000):
        counts[DS.minibatch(7, t, 0, 20, 5)] += 1
    p = 5 / 20
    assert np.all(np.abs(counts - 4000 * p) < 5 * np.sqrt(4000 * p * (1 - p)))
    idx = DS.rounds(1, 4, 2, [3, 10, 0], 4, first_worker=5)
    assert idx.shape == (2, 3, 4)
    np.testing.assert_array_equal(idx[1, 1], DS.minibatch(1, 5, 6, 10, 4))
    assert np.all(idx[:, 0, 3] == -1) and np.all(idx[:, 2] == -1)


def test_float32_rounded_reference_data_tracks_the_fixtures():
    """The north star's fp32 tolerance, checked on the restatement: the reference's own C2 data
    (StandardScaler float64 output, not float32-representable) rounded to float32 -- what the engine's
    float32 storage of such data computes on -- gives the reference's D-SGD / centralized trajectories
    within 1e-9 relative (objective) and 1e-7 (consensus) over 400 rounds."""
    meta, z = _load("c2")
    cfg = meta["config"]
    shards, Xf, yf = odata.generate(cfg, order=z["order"])
    r = [(X.astype(np.float32).astype(np.float64), y) for X, y in shards]
    Xr = Xf.astype(np.float32).astype(np.float64)
    assert not np.array_equal(Xr, Xf)
    T = 400
    for j, label in enumerate(meta["labels"]):
        st = ("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0)
        if label == "Centralized":
            h, _, _ = O.run_centralized(r, T, cfg, Xr, yf, meta["f_opt"], rng_state=st)
        else:
            topo = {"D-SGD (Ring)": "ring", "D-SGD (Grid)": "grid", "D-SGD (Fully Connected)": "fully_connected"}[label]
            W, _ = O.mh_matrix(O.adjacency(topo, cfg["n_workers"]))
            h, _, _, _ = O.run_decentralized(r, W, T, cfg, Xr, yf, meta["f_opt"], rng_state=st)
            np.testing.assert_allclose(h["consensus_error"], z[f"L{j}_consensus"][:T], rtol=1e-7)
        np.testing.assert_allclose(h["objective"], z[f"L{j}_objective"][:T], rtol=1e-9)
