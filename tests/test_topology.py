"""Product topology builder (CSR MH weights) vs the reference's dense matrices, bit for bit."""
import json
import os

import numpy as np
import pytest

import topology as T

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_against_reference_fixtures():
    z = np.load(os.path.join(G, "mixing.npz"))
    gaps = json.load(open(os.path.join(G, "mixing_gaps.json")))
    for topo in ("ring", "grid", "fully_connected"):
        for n in (1, 2, 3, 4, 5, 9, 10, 16, 25, 36):
            key = f"{topo}_{n}"
            if key + "_error" in z:
                with pytest.raises(ValueError) as e:
                    T.build(topo, n)
                assert str(e.value) == str(z[key + "_error"])
                continue
            t = T.build(topo, n)
            np.testing.assert_array_equal(t.dense_W(), z[key + "_W"])
            np.testing.assert_array_equal(t.dense_adjacency(), z[key + "_adj"])
            np.testing.assert_array_equal(t.degrees, z[key + "_deg"])
            t.check()
            if n > 1:
                assert round(t.spectral_gap(), 4) == gaps[key]
    with pytest.raises(ValueError) as e:
        T.build("star", 4)
    assert str(e.value) == str(z["star_4_error"])


@pytest.mark.parametrize("n,k", [(64, 4), (4096, 4), (1000, 6), (10, 3)])
def test_random_regular(n, k):
    t = T.random_regular(n, k, seed=1)
    assert np.all(t.degrees == k)
    for i, nb in enumerate(t.neighbours):
        assert len(set(nb)) == k and i not in nb
        for j in nb:
            assert i in t.neighbours[j]
    t.check()
    assert np.array_equal(T.random_regular(n, k, seed=1).col, t.col)  # deterministic


def test_csr_layout():
    t = T.grid(16)
    assert t.nnz == 16 * 5
    for i in range(16):
        cols = t.col[t.row_ptr[i]:t.row_ptr[i + 1]]
        assert list(cols) == sorted(cols) and i in cols


def test_large_torus_sparse_only():
    t = T.grid(256 * 256)  # C4 topology: never densified
    assert t.n == 65536 and t.nnz == 65536 * 5
    np.testing.assert_allclose(np.add.reduceat(t.w, t.row_ptr[:-1]), 1.0)
    diag = t.w[t.col == np.repeat(np.arange(t.n), 5)]
    assert diag.shape == (t.n,) and np.all(diag == 1.0 - np.sum(np.full(4, 0.2)))


@pytest.mark.parametrize("name,n", [("ring", 4097), ("grid", 6400), ("random_regular", 4100), ("random_regular", 4098)])
def test_lanczos_spectral_gap_matches_dense(name, n):
    """trainer.py:133-135 computes 1 - (second largest |eigenvalue|) with dense eigvalsh;
    above 4096 workers Topology.spectral_gap switches to Lanczos (scipy eigsh on the CSR
    W).  Just past the crossover, both must agree: on the ring (gap ~ 1e-6, nearly
    degenerate top eigenvalues), the 80 x 80 torus (4-fold degenerate lambda_2) and
    random 4-regular expanders."""
    t = T.build(name, n, {"regular_degree": 4, "topology_seed": 2})
    assert t.n > 4096
    dense = 1.0 - np.sort(np.abs(np.linalg.eigvalsh(t.dense_W())))[-2]
    lanczos = t.spectral_gap()
    np.testing.assert_allclose(lanczos, dense, rtol=1e-6, atol=1e-9)
    assert round(lanczos, 4) == round(dense, 4)  # the value trainer.py:135 prints
