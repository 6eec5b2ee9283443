#!/usr/bin/env python3
"""Where the drop-in trainer's C3 round goes with the exact legacy stream (host draws vs
device calls, and how much they overlap): the C3 shards as host arrays, 128 rounds of
DecentralizedTrainer.run with the stream draw and the device calls wrapped in timers."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import _dopt  # noqa: E402
from trainer import DecentralizedTrainer  # noqa: E402
from worker import Worker  # noqa: E402

n, d, m, R = 4096, 1024, 512, int(os.environ.get("PROBE_ROUNDS", "128"))
eng = _dopt.Engine(0, "float64", data_dtype="float32")
eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
X = np.empty((n * m, d), dtype=np.float32)
y = np.empty(n * m, dtype=np.float32)
for i in range(n):
    Xi, yi = eng.get_shard(i)
    X[i * m:(i + 1) * m] = Xi
    y[i * m:(i + 1) * m] = yi
eng.close()
log, lock = [], threading.Lock()


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        with lock:
            log.append((name, t0, time.perf_counter()))
        return r
    return w


_dopt.mt_advance_rounds = timed("draw", _dopt.mt_advance_rounds)
_dopt.Engine.run_dsgd_pipelined = timed("device", _dopt.Engine.run_dsgd_pipelined)
cfg = {"problem_type": "logistic", "local_batch_size": m, "learning_rate_eta0": 0.05,
       "l2_regularization_lambda": 1e-4, "strong_convexity_mu": 1e-4, "dtype": "float64", "sampling": "legacy",
       "regular_degree": 4, "topology_seed": 0, "spectral_gap": False}
ws = [Worker(i, {"X": X[i * m:(i + 1) * m], "y": y[i * m:(i + 1) * m]}, m, d, cfg) for i in range(n)]
np.random.seed(203)
DecentralizedTrainer(ws, "random_regular", d, cfg).run(2, X, y)  # loads the engine
log.clear()
tr = DecentralizedTrainer(ws, "random_regular", d, cfg)
t0 = time.perf_counter()
tr.run(R, X, y)
wall = time.perf_counter() - t0
draw = [e - s for k, s, e in log if k == "draw"]
dev = [e - s for k, s, e in log if k == "device"]
first = min(s for _, s, _ in log) - t0
print(json.dumps({"rounds": R, "wall_ms_per_round": wall / R * 1e3, "draws": len(draw),
                  "draw_ms_total": sum(draw) * 1e3, "draw_ms_per_round": sum(draw) / R * 1e3,
                  "device_calls": len(dev), "device_ms_total": sum(dev) * 1e3,
                  "setup_ms_before_first_call": first * 1e3,
                  "timeline": [(k, round((s - t0) * 1e3, 2), round((e - t0) * 1e3, 2)) for k, s, e in log[:12]]}))
