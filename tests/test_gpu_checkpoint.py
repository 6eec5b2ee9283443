"""Checkpoint / resume of the drop-in trainers (trainer._Checkpoint).

A run interrupted at round t and resumed from its checkpoint must continue bit for bit:
the iterates, history, floats transmitted and numpy's legacy RNG stream equal those of an
uninterrupted run with the same chunk boundaries (checkpoint_every).  The resumed run is
also pinned to the reference's own trajectory (the C2 fixture, rtol 1e-9)."""
import json
import os

import numpy as np
import pytest

import data as odata
from trainer import CentralizedTrainer, DecentralizedTrainer
from worker import Worker

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture():
    meta = json.load(open(os.path.join(G, "traj_c2.json")))
    z = np.load(os.path.join(G, "traj_c2.npz"))
    shards, Xf, yf = odata.generate(meta["config"], order=z["order"])
    return meta, z, shards, Xf, yf


def _trainer(label, shards, cfg):
    d = shards[0][0].shape[1]
    ws = [Worker(i, {"X": X, "y": y}, cfg["local_batch_size"], d, cfg) for i, (X, y) in enumerate(shards)]
    if label == "Centralized":
        return CentralizedTrainer(ws, d, cfg)
    return DecentralizedTrainer(ws, {"D-SGD (Ring)": "ring", "D-SGD (Fully Connected)": "fully_connected"}[label],
                                d, cfg)


@pytest.mark.parametrize("label", ["D-SGD (Ring)", "Centralized"])
@pytest.mark.parametrize("batch", [None, 10 ** 6])  # the fixture's minibatches; full shards (stream advance)
def test_resume_continues_bit_for_bit(tmp_path, label, batch):
    meta, z, shards, Xf, yf = _fixture()
    j = meta["labels"].index(label)
    cfg = dict(meta["config"])
    if batch:
        cfg["local_batch_size"] = batch
    T, K = 60, 25  # checkpoints at rounds 25 and 50; the interrupted run stops after 25
    ck = str(tmp_path / "ck.npz")

    # uninterrupted, same chunk boundaries
    np.random.set_state(("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0))
    full = _trainer(label, shards, dict(cfg, checkpoint_path=str(tmp_path / "full.npz"), checkpoint_every=K))
    h_full, x_full = full.run(T, Xf, yf, meta["f_opt"])
    st_full = np.random.get_state()

    # interrupted after round K ...
    np.random.set_state(("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0))
    first = _trainer(label, shards, dict(cfg, checkpoint_path=ck, checkpoint_every=K))
    first.run(K, Xf, yf, meta["f_opt"])
    np.random.seed(12345)  # whatever the process did in between
    # ... and resumed by a fresh trainer
    second = _trainer(label, shards, dict(cfg, resume_from=ck, checkpoint_path=str(tmp_path / "b.npz"),
                                          checkpoint_every=K))
    h_res, x_res = second.run(T, Xf, yf, meta["f_opt"])
    st_res = np.random.get_state()

    assert np.array_equal(x_res, x_full)
    for key in ("objective", "consensus_error"):
        if key in h_full:
            assert len(h_res[key]) == T
            assert np.array_equal(np.asarray(h_res[key]), np.asarray(h_full[key])), key
    assert len(h_res["time"]) == T and np.all(np.diff(h_res["time"]) >= 0)
    assert second.total_floats_transmitted == full.total_floats_transmitted
    assert st_res[2] == st_full[2] and np.array_equal(st_res[1], st_full[1])
    if not batch:  # the reference's own trajectory (trainer.py:161-193 / :33-74)
        np.testing.assert_allclose(h_res["objective"], z[f"L{j}_objective"][:T], rtol=1e-9)
    with np.load(str(tmp_path / "b.npz"), allow_pickle=False) as f:
        assert int(f["t"]) == T  # the end of run is always checkpointed


def test_resume_rejects_a_mismatched_checkpoint(tmp_path):
    meta, z, shards, Xf, yf = _fixture()
    cfg = dict(meta["config"])
    ck = str(tmp_path / "ck.npz")
    _trainer("D-SGD (Ring)", shards, dict(cfg, checkpoint_path=ck)).run(5, Xf, yf, meta["f_opt"])
    with pytest.raises(ValueError):
        _trainer("D-SGD (Fully Connected)", shards, dict(cfg, resume_from=ck)).run(10, Xf, yf, meta["f_opt"])
    with pytest.raises(ValueError):
        _trainer("D-SGD (Ring)", shards, dict(cfg, resume_from=ck)).run(3, Xf, yf, meta["f_opt"])
    # anything else the saved trajectory depends on: step size, minibatch size, arithmetic, the
    # regulariser keys (worker.py:36-37), the shard contents
    for change in ({"learning_rate_eta0": cfg["learning_rate_eta0"] * 2}, {"dtype": "float32"},
                   {"l2_regularization_lambda": 3e-3}, {"strong_convexity_mu": 3e-3}):
        with pytest.raises(ValueError):
            _trainer("D-SGD (Ring)", shards, dict(cfg, resume_from=ck, **change)).run(10, Xf, yf, meta["f_opt"])
    edited = [(X.copy(), y.copy()) for X, y in shards]
    edited[0][0][0, 0] += 1.0
    with pytest.raises(ValueError):
        _trainer("D-SGD (Ring)", edited, dict(cfg, resume_from=ck)).run(10, Xf, yf, meta["f_opt"])
    # the unchanged configuration still resumes
    _trainer("D-SGD (Ring)", shards, dict(cfg, resume_from=ck)).run(10, Xf, yf, meta["f_opt"])
