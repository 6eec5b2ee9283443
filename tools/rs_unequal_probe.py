#!/usr/bin/env python3
"""C5 (float64 arithmetic over float32 rows) row-space rounds from UNEQUAL iterates: one direct
column-blocked round from zeros (DOPT_ROWSPACE=0) leaves iterates that differ, then row-space
rounds continue from them (the start kept as a term of its own).  Reports the one-time start cost
(x(0) mean / deviations / row dots) and the per-round time beside the direct rounds' and the
zero-start row-space rounds'; histories checked against the direct rounds."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime)

import _dopt  # noqa: E402
import topology  # noqa: E402


def main():
    n, d, m, T, eta0, lam = 1024, 1 << 20, 16, 10, 1e-5, 1e-4
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    eng.generate_shards("quadratic", n, d, m, seed=3, noise=10.0)
    eng.set_mixing_mean(*topology.fully_connected(n).uniform_offdiag())

    def run(knob, first):
        os.environ["DOPT_ROWSPACE"] = knob
        eng.zero_models()
        os.environ["DOPT_ROWSPACE"] = "0"
        eng.run_dsgd(1, eta0, m, lam, lam, 0.0)  # direct round 1: unequal iterates
        os.environ["DOPT_ROWSPACE"] = knob
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o1, c1, _ = eng.run_dsgd(first, eta0, m, lam, lam, 0.0, t0=1)  # start (+ rounds)
        t1 = time.perf_counter()
        o2, c2, _ = eng.run_dsgd(T, eta0, m, lam, lam, 0.0, t0=1 + first)
        t2 = time.perf_counter()
        return t1 - t0, (t2 - t1) / T, np.concatenate([o1, o2]), np.concatenate([c1, c2]), _dopt.last_round_kernel()

    for rep in range(2):
        s_rs, r_rs, o_rs, c_rs, k_rs = run("1", 1)
        s_d, r_d, o_d, c_d, k_d = run("0", 1)
        print(f"rep {rep}: row-space from unequal iterates: first call {s_rs * 1e3:.1f} ms (start + 1 round + "
              f"metrics), {r_rs * 1e3:.2f} ms per round ({k_rs[:40]}); direct {s_d * 1e3:.1f} ms, "
              f"{r_d * 1e3:.2f} ms per round ({k_d[:40]})", flush=True)
        np.testing.assert_allclose(o_rs, o_d, rtol=1e-9)
        np.testing.assert_allclose(c_rs, c_d, rtol=1e-8)
    print("histories agree (objective rtol 1e-9, consensus 1e-8)")
    # minibatches of 4 of the 16 rows (the reference's legacy stream, host indices), from zeros
    b = 4
    np.random.seed(7)
    idx = _dopt.mt_choice_rounds(T + 2, [m] * n, b)
    for rep in range(2):
        res = {}
        for knob in ("1", "0"):
            os.environ["DOPT_ROWSPACE"] = knob
            eng.zero_models()
            eng.run_dsgd(2, eta0, b, lam, lam, 0.0, idx=idx[:2])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            o, c, _ = eng.run_dsgd(T, eta0, b, lam, lam, 0.0, idx=idx[2:], t0=2)
            res[knob] = ((time.perf_counter() - t0) / T, o, c, _dopt.last_round_kernel())
        print(f"rep {rep}: b = {b} of {m}: row-space {res['1'][0] * 1e3:.2f} ms per round ({res['1'][3][:40]}), "
              f"direct {res['0'][0] * 1e3:.2f} ms ({res['0'][3][:40]})", flush=True)
        np.testing.assert_allclose(res["1"][1], res["0"][1], rtol=1e-9)
        np.testing.assert_allclose(res["1"][2], res["0"][2], rtol=1e-8)
    print("minibatch histories agree")
    eng.close()


if __name__ == "__main__":
    main()
