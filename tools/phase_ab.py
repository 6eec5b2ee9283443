#!/usr/bin/env python3
"""In-process A/B of the round kernel as the fused single-GPU path launches it (gradient +
mix + step) and as the multi-GPU phase path launches it (gradient only, F_GOUT), on the
same C3 data, interleaved: per-launch HIP-event times and round times of both paths.
AB_DTYPE: float32 | x32 (float64 arithmetic over float32 rows, the headline; default) |
float64.  The phase path also runs with one wave per worker in the mix (DOPT_MIX_ONEWAVE=1,
"phase1"); all use pipelined runs (bench.py's timing).  Measured (two boxes, medians of 5):
fused 1.323 / 1.322 ms per round, phase 1.304 / 1.364, phase1 1.303 / 1.371 -- the phase
path's gradient-only kernel was 5 % faster than the fused one on the first box and equal
on the second.  The fused epilogue with every neighbour load in flight at once (instead of
one CSR entry at a time) measured 1.332 vs 1.322 there: not kept."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _dopt  # noqa: E402
import distributed  # noqa: E402
import topology  # noqa: E402


def main():
    n, d, m, R = 4096, 1024, 512, int(os.environ.get("AB_ROUNDS", "20"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29577")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    top = topology.random_regular(n, 4, seed=0)
    engs = {}
    dt_ = os.environ.get("AB_DTYPE", "x32")
    for k in ("fused", "phase"):
        e = (_dopt.Engine(0, "float64", data_dtype="float32") if dt_ == "x32" else _dopt.Engine(0, dt_))
        e.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
        engs[k] = e
    engs["fused"].set_topology(top.row_ptr, top.col, top.w)
    plan = distributed.build_plan(top, 1, 0)
    runner = distributed.DistributedDSGD(engs["phase"], plan, n, n * m, device=0)
    res = {k: {"kernel_ms": [], "round_ms": []} for k in ("fused", "phase", "phase1")}
    for rep in range(int(os.environ.get("AB_REPS", "5"))):
        for k in res:
            e = engs["fused" if k.startswith("fused") else "phase"]
            os.environ["DOPT_MIX_ONEWAVE"] = "1" if k == "phase1" else "0"
            e.set_models(np.zeros((n, d)))
            if k.startswith("fused"):
                e.run_dsgd_pipelined(3, 0.05, m, 1e-4, 1e-4, 0.0)
            else:
                runner.run_pipelined(3, 0.05, m, 1e-4, 1e-4, 0.0)
            e.set_profiling(True)
            e.kernel_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if k.startswith("fused"):
                e.run_dsgd_pipelined(R, 0.05, m, 1e-4, 1e-4, 0.0)
            else:
                runner.run_pipelined(R, 0.05, m, 1e-4, 1e-4, 0.0)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            launches, ms = e.kernel_stats()
            res[k]["kernel_ms"].append(ms / launches)
            res[k]["round_ms"].append(dt / R * 1e3)
        print(f"rep {rep}: " + ", ".join(f"{k} kernel {v['kernel_ms'][-1]:.4f} round {v['round_ms'][-1]:.4f}"
                                         for k, v in res.items()), file=sys.stderr, flush=True)
    print(json.dumps({k: {q: float(np.median(v)) for q, v in r.items()} for k, r in res.items()}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
