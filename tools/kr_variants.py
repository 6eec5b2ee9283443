#!/usr/bin/env python3
"""In-process A/B of k_round tuning variants on the C3 workload (guide rule 24:
interleaved rounds in ONE process, median and min reported).  Each variant's
histories must match variant 0 (fp32 tolerance) -- a faster wrong kernel is not a win.

  python tools/kr_variants.py [--variants 0,1,2,3,4,6,7] [--reps 5] [--rounds 10]
  python tools/kr_variants.py --mode x32 --variants -1,30755,129059   (float64 over float32 rows)

Variant -1 is the default build (env knob unset).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime)

import _dopt  # noqa: E402
import topology  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="14627,291,6435")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--workers", type=int, default=4096)
    ap.add_argument("--mode", default="f32", choices=["f32", "x32", "f64"],
                    help="f32: float32 engine (DOPT_KR_VARIANT); x32: float64 arithmetic over float32 rows "
                         "(DOPT_KRX_VARIANT); f64: float64 rows (DOPT_KRD_VARIANT)")
    args = ap.parse_args()
    n, d, m = args.workers, 1024, 512
    knob = {"f32": "DOPT_KR_VARIANT", "x32": "DOPT_KRX_VARIANT", "f64": "DOPT_KRD_VARIANT"}[args.mode]
    eng = {"f32": lambda: _dopt.Engine(0, "float32"), "x32": lambda: _dopt.Engine(0, "float64", data_dtype="float32"),
           "f64": lambda: _dopt.Engine(0, "float64")}[args.mode]()
    eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
    top = topology.random_regular(n, 4, seed=0)
    eng.set_topology(top.row_ptr, top.col, top.w)
    eng.set_profiling(True)
    variants = [int(v) for v in args.variants.split(",")]
    times = {v: [] for v in variants}
    ref = None
    xs = 8 if args.mode == "f64" else 4
    bytes_per = xs * n * (m * d + m) + (4 if args.mode == "f32" else 8) * n * 2 * d
    for rep in range(args.reps):
        for v in variants:
            if v < 0:
                os.environ.pop(knob, None)
            else:
                os.environ[knob] = str(v)
            eng.set_models(np.zeros((n, d)))
            eng.kernel_stats()
            obj, cons, _ = eng.run_dsgd(args.rounds, 0.05, m, 1e-4, 1e-4, 0.0, want_time=False)
            k, ms = eng.kernel_stats()
            times[v].append(ms / k)
            if ref is None:
                ref = (obj, cons)
            else:
                tol = (2e-5, 2e-4) if args.mode == "f32" else (1e-11, 1e-9)
                np.testing.assert_allclose(obj, ref[0], rtol=tol[0])
                np.testing.assert_allclose(cons, ref[1], rtol=tol[1])
        print(f"rep {rep}: " + " ".join(f"v{v}={times[v][-1]:.4f}ms" for v in variants), file=sys.stderr, flush=True)
    out = {}
    for v in variants:
        t = np.array(times[v])
        out[v] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                  "tbps_median": bytes_per / (np.median(t) * 1e-3) / 1e12}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
