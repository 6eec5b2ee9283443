#!/usr/bin/env python3
"""Where a small-config round goes (main.py's N = 25 quadratic run, d = 81, b = 16,
T = 10^4 rounds, ring): the drop-in DecentralizedTrainer with the exact legacy sampler
(host MT19937, drawn one chunk ahead on a host thread), the same trainer with device
sampling (no host RNG), full-shard batches (no sampler at all), and the host sampler
alone for the same T x N draws.  One GPU; prints one line per leg."""
import io
import contextlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402

import _dopt  # noqa: E402
import main as M  # noqa: E402
from trainer import CentralizedTrainer, DecentralizedTrainer  # noqa: E402
from utils import generate_and_preprocess_data  # noqa: E402
from worker import Worker  # noqa: E402

T = int(os.environ.get("C2_T", "10000"))


def leg(name, cfg, shards, d, X, y, central=False):
    workers = [Worker(i, shards[i], cfg["local_batch_size"], d, cfg) for i in range(cfg["n_workers"])]
    tr = CentralizedTrainer(workers, d, cfg) if central else DecentralizedTrainer(workers, "ring", d, cfg)
    with contextlib.redirect_stdout(io.StringIO()):
        tr.run(50, X, y, 0.0)  # warm: engine, data upload, kernels
        for w in workers:
            w.x = np.zeros(d)
        if central:
            tr.x_global = np.zeros(d)
        t0 = time.perf_counter()
        tr.run(T, X, y, 0.0)
        dt = time.perf_counter() - t0
    print(f"{name:28s} {dt:7.3f} s  {dt / T * 1e6:7.2f} us/round", flush=True)


def main():
    np.random.seed(203)
    cfg = M.make_config(problem_type=os.environ.get("C2_PROBLEM", "quadratic"))
    with contextlib.redirect_stdout(io.StringIO()):
        shards, d, X, y = generate_and_preprocess_data(cfg["n_workers"], cfg)
    leg("legacy sampler (exact)", cfg, shards, d, X, y)
    leg("device sampler", dict(cfg, sampling="device"), shards, d, X, y)
    leg("full shard (b = m)", dict(cfg, local_batch_size=10 ** 6), shards, d, X, y)
    leg("centralized, legacy sampler", cfg, shards, d, X, y, central=True)
    rows = np.array([len(s["y"]) for s in shards])
    _dopt.mt_choice_rounds(1, rows, cfg["local_batch_size"])
    t0 = time.perf_counter()
    _dopt.mt_choice_rounds(T, rows, cfg["local_batch_size"])
    dt = time.perf_counter() - t0
    print(f"{'host MT19937 alone':28s} {dt:7.3f} s  {dt / T * 1e6:7.2f} us/round", flush=True)


if __name__ == "__main__":
    main()
