"""Generate the golden fixtures by importing the reference simulator.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference (override with DOPT_REFERENCE).  It imports the reference's own
modules (trainer.py, worker.py, obj_problems.py, utils.py, simulator.py), calls
them, and records their OUTPUTS as small .npz / .json fixtures next to this
script.  No reference source text is copied; the GPU box never sees the
reference, only these data files.

Fixture groups:
  mixing.npz    - MH mixing matrices / degrees / spectral gaps per topology, N
                  (trainer.py:91-136), plus the ValueError cases (:101-102, :112)
  rng.npz       - np.random.choice(m, b, replace=False) index vectors drawn by
                  Worker.get_mini_batch after np.random.seed(203) (worker.py:15-28)
  grads.npz     - known answers of the four objective / gradient functions and
                  the two full-gradient functions (obj_problems.py)
  traj_<tag>.npz + traj_<tag>.json
                - per-round objective and consensus trajectories of
                  Simulator.run_all (simulator.py:94-137), the RNG state at the
                  start of every trainer, f(x*), the shard order and a data hash,
                  and numerical_results (iterations to threshold, floats sent)

Usage:  python tests/golden/make_golden.py [--only TAG ...]
"""
import argparse
import contextlib
import hashlib
import io
import json
import os
import re
import sys
import time

os.environ.setdefault("MPLBACKEND", "Agg")
REF = os.environ.get("DOPT_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

import obj_problems as r_obj  # noqa: E402
import simulator as r_sim  # noqa: E402
import trainer as r_trainer  # noqa: E402
import worker as r_worker  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def _quiet():
    return contextlib.redirect_stdout(io.StringIO())


def data_digest(worker_data):
    """sha256 over every shard's X then y bytes, in worker order."""
    h = hashlib.sha256()
    for wd in worker_data:
        h.update(np.ascontiguousarray(wd["X"], dtype=np.float64).tobytes())
        h.update(np.ascontiguousarray(wd["y"]).astype(np.float64).tobytes())
    return h.hexdigest()


# --------------------------------------------------------------------------- mixing
def gen_mixing():
    out, gaps = {}, {}
    for topo in ("ring", "grid", "fully_connected"):
        for n in (1, 2, 3, 4, 5, 9, 10, 16, 25, 36):
            buf = io.StringIO()
            try:
                with contextlib.redirect_stdout(buf):
                    tr = r_trainer.DecentralizedTrainer([None] * n, topo, 3, {"problem_type": "logistic"})
            except ValueError as e:
                out[f"{topo}_{n}_error"] = np.array(str(e))
                continue
            out[f"{topo}_{n}_W"] = tr.W
            out[f"{topo}_{n}_adj"] = tr.adj
            out[f"{topo}_{n}_deg"] = tr.degrees
            m = re.search(r"Spectral gap \(1 - rho\): ([0-9.]+)", buf.getvalue())
            if m:
                gaps[f"{topo}_{n}"] = float(m.group(1))
    try:
        with _quiet():
            r_trainer.DecentralizedTrainer([None] * 4, "star", 3, {"problem_type": "logistic"})
    except ValueError as e:
        out["star_4_error"] = np.array(str(e))
    np.savez_compressed(os.path.join(OUT, "mixing.npz"), **out)
    with open(os.path.join(OUT, "mixing_gaps.json"), "w") as f:
        json.dump(gaps, f, indent=1, sort_keys=True)


# --------------------------------------------------------------------------- rng
def gen_rng():
    """Index vectors of Worker.get_mini_batch for a sequence of (m, b) shapes."""
    np.random.seed(203)
    specs = [(500, 16), (501, 16), (1, 16), (2, 1), (0, 16), (37, 37), (37, 100),
             (1000, 1000), (70001, 5), (500, 16), (3, 2)]
    out = {"specs": np.array(specs, dtype=np.int64)}
    for k, (m, b) in enumerate(specs):
        X = np.arange(m, dtype=np.float64).reshape(m, 1)
        w = r_worker.Worker(k, {"X": X, "y": np.arange(m)}, b, 1, {})
        Xb, yb = w.get_mini_batch()
        out[f"call{k}_idx"] = Xb[:, 0].astype(np.int64)
        st = np.random.get_state()
        out[f"call{k}_pos"] = np.int64(st[2])
    st = np.random.get_state()
    out["final_key"] = np.asarray(st[1], dtype=np.uint32)
    out["final_pos"] = np.int64(st[2])
    # a D-SGD-shaped stream: 3 rounds x 10 workers x choice(500, 16)
    np.random.seed(203)
    ws = [r_worker.Worker(i, {"X": np.arange(500.0).reshape(500, 1), "y": np.arange(500)}, 16, 1, {})
          for i in range(10)]
    rounds = np.zeros((3, 10, 16), dtype=np.int64)
    for t in range(3):
        for i, w in enumerate(ws):
            rounds[t, i] = w.get_mini_batch()[0][:, 0].astype(np.int64)
    out["rounds_c2"] = rounds
    np.savez_compressed(os.path.join(OUT, "rng.npz"), **out)


# --------------------------------------------------------------------------- grads
class _FakeWorker:
    def __init__(self, X, y):
        self.X_local, self.y_local = X, y


def gen_grads():
    rng = np.random.default_rng(7)
    out, cases = {}, []
    for prob in ("logistic", "quadratic"):
        for d in (1, 5, 81):
            for b in (0, 1, 16, 37):
                for scale in (1.0, 40.0):
                    k = len(cases)
                    w = rng.standard_normal(d) * scale
                    X = rng.standard_normal((b, d))
                    if prob == "logistic":
                        y = rng.choice(np.array([-1, 1]), size=b)
                        g = r_obj.logistic_stochastic_gradient(w, X, y, 1e-4)
                        f = r_obj.logistic_objective(w, X, y, 1e-4)
                    else:
                        y = rng.standard_normal(b) * 10
                        g = r_obj.quadratic_stochastic_gradient(w, X, y, 1e-4)
                        f = r_obj.quadratic_objective(w, X, y, 1e-4)
                    out[f"c{k}_w"], out[f"c{k}_X"], out[f"c{k}_y"] = w, X, y
                    out[f"c{k}_g"], out[f"c{k}_f"] = np.asarray(g), np.float64(f)
                    cases.append((prob, d, b, scale))
    # full-gradient functions (dead code in the reference, kept for API parity)
    for prob in ("logistic", "quadratic"):
        d = 7
        w = rng.standard_normal(d)
        shards = []
        for m in (5, 0, 3):
            X = rng.standard_normal((m, d))
            y = rng.choice(np.array([-1, 1]), size=m) if prob == "logistic" else rng.standard_normal(m)
            shards.append(_FakeWorker(X, y))
        fn = r_obj.logistic_full_gradient if prob == "logistic" else r_obj.quadratic_full_gradient
        out[f"full_{prob}_w"] = w
        for j, s in enumerate(shards):
            out[f"full_{prob}_X{j}"], out[f"full_{prob}_y{j}"] = s.X_local, s.y_local
        out[f"full_{prob}_g"] = fn(w, shards, 1e-4)
        out[f"full_{prob}_gempty"] = fn(w, [shards[1]], 1e-4)
    out["cases"] = np.array([[0 if p == "logistic" else 1, d, b, s] for p, d, b, s in cases], dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "grads.npz"), **out)


# --------------------------------------------------------------------------- trajectories
def base_config(**kw):
    cfg = {
        "n_workers": 25, "local_batch_size": 16, "n_iterations": 10000,
        "learning_rate_eta0": 0.05, "l2_regularization_lambda": 1e-4,
        "strong_convexity_mu": 1e-4, "problem_type": "quadratic",
        "n_samples": 25 * 500, "n_features": 80, "n_informative_features": 50,
        "classification_sep": 0.7, "suboptimality_threshold": 0.08,
    }
    cfg.update(kw)
    return cfg


TRAJ = {
    # tag: config overrides  (n_samples defaults to n_workers * 500 like main.py:14)
    "c1": dict(n_workers=10, problem_type="quadratic", n_iterations=2000),
    "c2": dict(n_workers=10, problem_type="logistic", n_iterations=2000),
    "table2": dict(n_workers=25, problem_type="quadratic", n_iterations=10000),
    "table1": dict(n_workers=25, problem_type="logistic", n_iterations=10000),
    "fullbatch": dict(n_workers=9, problem_type="logistic", n_iterations=300, local_batch_size=600),
    "n1": dict(n_workers=1, problem_type="logistic", n_iterations=200),
    "n2": dict(n_workers=2, problem_type="logistic", n_iterations=300),
    "n4": dict(n_workers=4, problem_type="quadratic", n_iterations=300),
    "ragged": dict(n_workers=7, problem_type="quadratic", n_iterations=300, n_samples=3503),
}
# NOTE: empty shards cannot come out of the reference's data generator
# (utils.py:44 takes np.min of an empty label array and raises ValueError), so
# the empty-shard case is pinned by gen_direct() through the trainer API.


def gen_traj(tag):
    over = dict(TRAJ[tag])
    n = over["n_workers"]
    over.setdefault("n_samples", n * 500)
    cfg = base_config(**over)
    np.random.seed(203)  # main.py:24
    t0 = time.time()
    with _quiet():
        sim = r_sim.Simulator(cfg)
    states = []
    orig_reset = sim._reset_workers

    def reset_and_record():
        st = np.random.get_state()
        states.append((np.asarray(st[1], dtype=np.uint32).copy(), int(st[2])))
        orig_reset()

    sim._reset_workers = reset_and_record
    with _quiet():
        sim.run_all()
    wall = time.time() - t0

    order = np.argsort(sim.y_full)  # the same call utils.py:34 makes, same numpy
    splits = np.array_split(order, n)
    for i, idx in enumerate(splits):  # confirm the recorded order is the one used
        assert np.array_equal(sim.worker_data[i]["X"], sim.X_full[idx]), tag
    arrays = {"order": order.astype(np.int64),
              "shard_sizes": np.array([len(s) for s in splits], dtype=np.int64)}
    labels = list(sim.results.keys())
    for j, lab in enumerate(labels):
        h = sim.results[lab]
        key = f"L{j}"
        arrays[f"{key}_objective"] = np.asarray(h.get("objective", []), dtype=np.float64)
        if "consensus_error" in h:
            arrays[f"{key}_consensus"] = np.asarray(h["consensus_error"], dtype=np.float64)
    for j, (key, pos) in enumerate(states):
        arrays[f"state{j}_key"], arrays[f"state{j}_pos"] = key, np.int64(pos)
    np.savez_compressed(os.path.join(OUT, f"traj_{tag}.npz"), **arrays)

    def _py(v):
        if isinstance(v, (np.integer,)):
            return int(v)
        if isinstance(v, (np.floating,)):
            return float(v)
        return v

    meta = {
        "config": cfg,
        "labels": labels,
        "f_opt": float(sim.f_opt),
        "n_features_bias": int(sim.n_features),
        "data_sha256": data_digest(sim.worker_data),
        "numerical_results": {k: {kk: _py(vv) for kk, vv in v.items()} for k, v in sim.numerical_results.items()},
        "numerical_results_types": {k: {kk: type(vv).__name__ for kk, vv in v.items()} for k, v in sim.numerical_results.items()},
        "reference_wall_s": wall,
    }
    with open(os.path.join(OUT, f"traj_{tag}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"[golden] traj_{tag}: {labels} in {wall:.1f}s", flush=True)


def gen_direct():
    """Trainer-level fixtures with hand-built shards, incl. empty and 1-row ones.

    Drives Worker / CentralizedTrainer / DecentralizedTrainer directly
    (worker.py:15-23 empty-batch path, obj_problems.py:14-15 zero gradient).
    """
    rng = np.random.default_rng(11)
    out, meta = {}, {}
    for prob in ("logistic", "quadratic"):
        d = 6
        sizes = [3, 0, 2, 1, 0, 4]
        shards = []
        for m in sizes:
            X = np.hstack([rng.standard_normal((m, d - 1)), np.ones((m, 1))])
            y = (rng.choice(np.array([-1, 1]), size=m) if prob == "logistic"
                 else rng.standard_normal(m) * 3)
            shards.append({"X": X, "y": y})
        X_full = np.vstack([s["X"] for s in shards])
        y_full = np.concatenate([s["y"] for s in shards])
        cfg = base_config(problem_type=prob, n_workers=len(sizes), local_batch_size=2)
        for j, s in enumerate(shards):
            out[f"{prob}_X{j}"], out[f"{prob}_y{j}"] = s["X"], s["y"]
        T = 40
        runs = [("central", None), ("ring", "ring"), ("fc", "fully_connected")]
        for name, topo in runs:
            np.random.seed(203)
            ws = [r_worker.Worker(i, shards[i], 2, d, cfg) for i in range(len(sizes))]
            with _quiet():
                if topo is None:
                    tr = r_trainer.CentralizedTrainer(ws, d, cfg)
                else:
                    tr = r_trainer.DecentralizedTrainer(ws, topo, d, cfg)
                hist, xf = tr.run(T, X_full, y_full, 0.125)
            out[f"{prob}_{name}_objective"] = np.asarray(hist["objective"])
            if "consensus_error" in hist:
                out[f"{prob}_{name}_consensus"] = np.asarray(hist["consensus_error"])
            out[f"{prob}_{name}_final"] = np.asarray(xf)
            out[f"{prob}_{name}_final_pos"] = np.int64(np.random.get_state()[2])
            meta[f"{prob}_{name}_tx"] = float(tr.total_floats_transmitted)
        # X_full different from the union of the shards (first 5 rows only)
        np.random.seed(203)
        ws = [r_worker.Worker(i, shards[i], 2, d, cfg) for i in range(len(sizes))]
        with _quiet():
            tr = r_trainer.DecentralizedTrainer(ws, "ring", d, cfg)
            hist, xf = tr.run(T, X_full[:5], y_full[:5], 0.0)
        out[f"{prob}_subset_objective"] = np.asarray(hist["objective"])
        # no X_full: objective history stays empty (trainer.py:188)
        np.random.seed(203)
        ws = [r_worker.Worker(i, shards[i], 2, d, cfg) for i in range(len(sizes))]
        with _quiet():
            tr = r_trainer.DecentralizedTrainer(ws, "ring", d, cfg)
            hist, xf = tr.run(7, None, None, 0.0)
        meta[f"{prob}_noobj_lens"] = [len(hist["objective"]), len(hist["consensus_error"]), len(hist["time"])]
    np.savez_compressed(os.path.join(OUT, "direct.npz"), **out)
    with open(os.path.join(OUT, "direct.json"), "w") as f:
        json.dump(meta, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    jobs = {"mixing": gen_mixing, "rng": gen_rng, "grads": gen_grads, "direct": gen_direct}
    for tag in TRAJ:
        jobs[f"traj_{tag}"] = (lambda t=tag: gen_traj(t))
    for name, fn in jobs.items():
        if args.only and name not in args.only:
            continue
        t0 = time.time()
        fn()
        print(f"[golden] {name} done in {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
