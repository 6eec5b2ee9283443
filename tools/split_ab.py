#!/usr/bin/env python3
"""In-process A/B of two column-blocked step variants selected by an environment knob
(AB_KNOB, default DOPT_SPLIT_PREFETCH: next-block prefetch in the row-split kernel; AB_VALUES,
default "1,0", the knob values interleaved), on
the C5 shape (quadratic, d = 2^20, m = b = 16, complete graph through column sums).
Results of both variants must agree.  Measured on MI355X: prefetch 13.75 vs 13.58 ms;
a barrier-free column-streaming kernel (every wave holds all 16 rows of a block, 183
VGPRs, 2 waves/SIMD) 16.8 vs 14.1 ms -- both kept off."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import _dopt  # noqa: E402
import topology  # noqa: E402


def main():
    n, d, m = int(os.environ.get("AB_WORKERS", "1024")), 1 << 20, 16
    eng = _dopt.Engine(0, "float32")
    eng.generate_shards("quadratic", n, d, m, seed=1000)
    eng.set_mixing_mean(*topology.fully_connected(n).uniform_offdiag())
    eng.set_profiling(True)
    bytes_per = 4 * n * (m * d + m + 2 * d)
    vals = os.environ.get("AB_VALUES", "1,0").split(",")
    times, ref = {v: [] for v in vals}, None
    for rep in range(4):
        for v in vals:
            os.environ[os.environ.get("AB_KNOB", "DOPT_SPLIT_PREFETCH")] = v
            eng.set_models(np.zeros((n, d), dtype=np.float32))
            eng.kernel_stats()
            obj, cons, _ = eng.run_dsgd(4, 1e-5, m, 1e-4, 1e-4, 0.0, want_time=False)
            k, ms = eng.kernel_stats()
            times[v].append(ms / k)
            if v in os.environ.get("AB_NOCHECK", "").split(","):  # timing diagnostics: results not comparable
                pass
            elif ref is None:
                ref = (obj, cons)
            elif os.environ.get("AB_EXACT") == "1":  # variants that claim the same arithmetic
                assert np.array_equal(obj, ref[0]) and np.array_equal(cons, ref[1]), (v, obj, ref[0], cons, ref[1])
            else:
                np.testing.assert_allclose(obj, ref[0], rtol=1e-6)
                np.testing.assert_allclose(cons, ref[1], rtol=1e-5)
        print(f"rep {rep}: " + ", ".join(f"knob={v} {times[v][-1]:.3f} ms" for v in vals), file=sys.stderr, flush=True)
    print(json.dumps({v: {"median_ms": float(np.median(t)), "tbps": bytes_per / (np.median(t) * 1e-3) / 1e12}
                      for v, t in times.items()}))


if __name__ == "__main__":
    main()
