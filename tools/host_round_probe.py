#!/usr/bin/env python3
"""Host cost per round of the multi-GPU lagged schedule (distributed.py: _run_lagged) at RCCL
world 1 with the collectives forced (DOPT_FORCE_COLLECTIVES=1), PROBE_WORKERS workers (default
512, the strong leg's share of N = 4096 at 8 ranks): the Python time spent in each call of the
round loop (the exchange's start / finish, the two engine calls), accumulated over PROBE_ROUNDS
rounds, and the whole loop's host time per round (everything but the device), against the round's
GPU time.  A loop whose host time per round exceeds the GPU's leaves the GPU waiting between
kernels."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
os.environ.setdefault("DOPT_FORCE_COLLECTIVES", "1")

import torch  # noqa: E402

import _dopt  # noqa: E402
import distributed  # noqa: E402
import topology  # noqa: E402


def main():
    n, d, m = int(os.environ.get("PROBE_WORKERS", "512")), 1024, 512
    R = int(os.environ.get("PROBE_ROUNDS", "100"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29581")
    torch.cuda.set_device(0)
    distributed.init_process_group("nccl", rank=0, world_size=1)
    top = topology.random_regular(n, 4, seed=0)
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
    plan = distributed.build_plan(top, 1, 0)
    run = distributed.DistributedDSGD(eng, plan, n, n * m, device=0)
    acc = {}

    def wrap(obj, name):
        f = getattr(obj, name)

        def g(*a, **k):
            t = time.perf_counter()
            r = f(*a, **k)
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
            return r
        setattr(obj, name, g)

    for name in ("lagged_grad", "lagged_mix"):
        wrap(eng, name)
    for name in ("start", "finish"):
        wrap(run.exchange, name)
    wrap(run, "_start_exchange_lagged")  # the exchange call with the stream switch around it
    run.run_pipelined(5, 0.05, m, 1e-4, 1e-4, 0.0)
    torch.cuda.synchronize()
    acc.clear()
    issued = []
    ar = run._all_reduce

    def mark(*a, **k):  # the first call after the round loop: every round is issued by now
        issued.append(time.perf_counter())
        return ar(*a, **k)
    run._all_reduce = mark
    t0 = time.perf_counter()
    run.run_pipelined(R, 0.05, m, 1e-4, 1e-4, 0.0)
    wall = time.perf_counter() - t0
    run._all_reduce = ar
    run.run_pipelined(0, 0.05, m, 1e-4, 1e-4, 0.0)
    out = {"workers": n, "rounds": R, "transport": "rccl (engine)" if run.comm is not None else "process group", "wall_us_per_round": wall / R * 1e6,
           "host_us_per_round": {k: v / R * 1e6 for k, v in sorted(acc.items())},
           # ("start" -- the process group's all-to-all call -- runs inside _start_exchange_lagged; with the
           # engine's own communicator that call is dopt_lagged_exchange and start / finish are not used)
           "host_us_per_round_total": sum(v for k, v in acc.items() if k != "start") / R * 1e6,
           "loop_issue_us_per_round": (issued[0] - t0) / R * 1e6 if issued else None}
    print(json.dumps(out))
    eng.close()
    distributed.close_comms()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
