#!/usr/bin/env python3
"""Host legacy-stream advance (or, --batch b, minibatch draws) at the C3 chunk shape (8 rounds x 4096 workers x permutations of 512):
the sequential filter (DOPT_MT_THREADS=0) vs the speculative parallel advance, alternated, with
the resulting numpy state checked equal.  python tools/mt_advance_probe.py [--threads 0,4,8]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
os.environ.setdefault("DOPT_NO_TORCH", "1")

import numpy as np  # noqa: E402

import _dopt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="0,4,8")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--batch", type=int, default=0, help="b < 512: minibatch draws (dopt_mt_choice_rounds)")
    a = ap.parse_args()
    rows = np.full(4096, 512, np.int64)
    res = {}
    for rep in range(a.reps):
        for th in a.threads.split(","):
            os.environ["DOPT_MT_THREADS"] = th
            np.random.seed(100 + rep)
            t0 = time.perf_counter()
            if a.batch:
                _dopt.mt_choice_rounds(a.rounds, rows, a.batch)
            else:
                _dopt.mt_advance_rounds(a.rounds, rows)
            dt = time.perf_counter() - t0
            st = np.random.get_state()
            res.setdefault(th, []).append((dt, st[2], st[1][:4].tolist()))
    for th, v in res.items():
        ms = sorted(x[0] * 1e3 for x in v)
        print(f"threads {th}: median {ms[len(ms) // 2]:.1f} ms per {a.rounds} rounds "
              f"({ms[len(ms) // 2] / a.rounds:.2f} ms/round), min {ms[0]:.1f}")
    ref = res[a.threads.split(",")[0]]
    for th, v in res.items():
        assert all(x[1:] == y[1:] for x, y in zip(v, ref)), f"threads {th}: state differs"
    print("states equal across thread counts")


if __name__ == "__main__":
    main()
