"""A/B of the row-space pass shapes (DOPT_RS_CB / DOPT_RS_NBUF / DOPT_RS_WG [/ DOPT_RS_LDOT]) at C5 on one GPU:
one engine, the shape re-planned by set_mixing_mean, interleaved repetitions; prints the
round-kernel average (HIP events) and the wall time per round of a pipelined call."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402  (one HIP runtime: torch first)

import _dopt  # noqa: E402
import topology as TP  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4,2,16 4,3,16 2,3,16 2,4,16 2,6,16 1,8,16")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--data-dtype", default=None, help="float32: rows stored as float32 under float64 arithmetic")
    args = ap.parse_args()
    n, d, m = args.n, 1 << 20, 16
    eng = _dopt.Engine(0, args.dtype, data_dtype=args.data_dtype)
    xesz = 4 if (args.data_dtype or args.dtype) == "float32" else 8
    eng.generate_shards("quadratic", n, d, m, seed=3, noise=10.0)
    top = TP.fully_connected(n)
    zeros = np.zeros((n, d), dtype=np.float32)
    res = {}
    for rep in range(args.reps):
        for sh in args.shapes.replace("_", " ").split():
            parts = sh.split(",")
            cb, nb, wg = parts[:3]
            os.environ["DOPT_RS_CB"], os.environ["DOPT_RS_NBUF"] = cb, nb
            os.environ["DOPT_RS_WG"] = wg
            os.environ["DOPT_RS_LDOT"] = parts[3] if len(parts) > 3 else "1"  # row dots through LDS (2,8 only)
            eng.set_mixing_mean(*top.uniform_offdiag())  # re-plans the pass
            eng.set_models(zeros)  # the reference's start (row-space rounds need equal iterates)
            t = time.perf_counter()
            eng.run_dsgd_pipelined(3, 1e-5, m, 1e-4, 1e-4, 0.0)  # begin (check, Gram, init) + warmup
            tb = time.perf_counter() - t
            eng.kernel_stats()
            eng.set_profiling(True, every=1)
            eng.sync()
            t = time.perf_counter()
            eng.run_dsgd_pipelined(args.steps, 1e-5, m, 1e-4, 1e-4, 0.0, t0=3)
            eng.sync()
            dt = (time.perf_counter() - t) / args.steps
            k, ms = eng.kernel_stats()
            eng.set_profiling(False)
            eng.run_dsgd_pipelined(0, 1e-5, m, 1e-4, 1e-4, 0.0)
            res.setdefault(sh, []).append((ms / k, dt * 1e3))
            print(f"rep {rep} shape {sh}: kernel {ms / k:.3f} ms, round {dt * 1e3:.3f} ms "
                  f"({n * m * d * xesz / (ms / k) / 1e9:.2f} TB/s), setup {tb:.2f} s "
                  f"[{_dopt.last_round_kernel()}]", flush=True)
    for sh, v in res.items():
        print(sh, "best kernel %.3f ms, best round %.3f ms" % (min(a for a, _ in v), min(b for _, b in v)))
    eng.close()


if __name__ == "__main__":
    main()
