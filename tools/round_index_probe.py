#!/usr/bin/env python3
"""Is the headline round kernel slower in the first rounds of a run because of the iterates (training just
started from zeros) or because of the time since the device started working?  Two chains of ROUNDS
pipelined C3 rounds, each from zero iterates, back to back on one engine (run it under
`rocprofv3 --kernel-trace`); `--analyse <run_kernel_trace.csv>` prints each chain's round-kernel durations
(first 40, and the medians of rounds 0-19 / 20-39 / the last 20).  The same pattern in both chains
points at the iterates; a first-chain-only slowdown at the device's state."""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
HEAD = "k_round<double, float, 4, 0, true, true"


def run(rounds):
    import torch  # noqa: F401

    import _dopt
    import topology

    n, d, m = 4096, 1024, 512
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
    top = topology.random_regular(n, 4, seed=0)
    eng.set_topology(top.row_ptr, top.col, top.w)
    for _ in range(2):
        eng.zero_models()
        eng.run_dsgd_pipelined(rounds, 0.05, m, 1e-4, 1e-4, 0.0)
        eng.run_dsgd_pipelined(0, 0.05, m, 1e-4, 1e-4, 0.0)  # closes the chain (a metrics-only pass)
    eng.close()


def analyse(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    chains, cur = [], []
    for s, e, name in ev:
        if HEAD in name:
            cur.append((e - s) / 1e3)
        elif "k_round" in name and cur:  # the metrics-only pass that closes a chain
            chains.append(cur)
            cur = []
    out = {}
    for k, ts in enumerate(chains):
        out[f"chain{k + 1}"] = {"rounds": len(ts), "first40_us": [round(t, 1) for t in ts[:40]],
                                "median_0_19": statistics.median(ts[:20]), "median_20_39": statistics.median(ts[20:40]),
                                "median_last20": statistics.median(ts[-20:])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run(int(os.environ.get("PROBE_ROUNDS", "120")))
