#!/usr/bin/env python3
"""C5's row-space rounds at one rank's shape of an N-rank run (1024 / N workers of 16 rows, d = 2^20,
complete graph over 1024 workers) on one GPU, through DistributedDSGD at RCCL world 1 with the
collectives forced: the column-chunked, cross-round pipelined schedule (distributed.py _run_rowspace)
at K = 1, 2, 3, ... chunks, interleaved on one engine, as pipelined calls.  At world 1 the all-reduce
of the column sums is a local RCCL kernel, so what this measures is the price of chunking (launch
tails, per-chunk hand-offs); the all-reduce time it hides across ranks is not measurable on one GPU.

  python3 tools/rs_chunk_proxy.py --workers 128 --chunks 1,2,3,4 --reps 2 --steps 40 --warmup 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=128, help="this rank's workers (C5 over 8 ranks: 128)")
    ap.add_argument("--n-global", type=int, default=1024)
    ap.add_argument("--chunks", default="1,2,3,4")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    os.environ["DOPT_FORCE_COLLECTIVES"] = "1"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import torch

    import _dopt
    import bench
    import distributed as Dm
    import topology

    torch.cuda.set_device(0)
    Dm.init_process_group("nccl", store=bench._solo_store(), rank=0, world_size=1)
    n, d, m, eta0, lam = args.workers, 1 << 20, 16, 1e-5, 1e-4
    eng = _dopt.Engine(0, "float64", data_dtype="float32")
    eng.generate_shards("quadratic", n, d, m, seed=1000, flip=0.05)
    w_off, diag = topology.fully_connected(args.n_global).uniform_offdiag()
    plan = Dm.HaloPlan(0, 1, np.array([0, n]), 0, n, np.zeros(0, np.int64), np.zeros(2, np.int64),
                       np.zeros(0, np.int32), np.zeros(2, np.int64), None, None, None)
    run = Dm.DistributedDSGD(eng, plan, args.n_global, args.n_global * m, device=0, mean=(w_off, diag[:n]))
    if not run._rowspace_ready():
        raise SystemExit("the row-space rounds do not apply")
    t = 0
    res = []
    for rep in range(args.reps):
        for K in [int(k) for k in args.chunks.split(",")]:
            run.rs_chunks = K
            run.run_pipelined(args.warmup, eta0, m, lam, lam, 0.0, t0=t)
            t += args.warmup
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            obj, cons = run.run_pipelined(args.steps, eta0, m, lam, lam, 0.0, t0=t)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            t += args.steps
            res.append({"K": K, "rep": rep, "ms_per_round": dt / args.steps * 1e3,
                        "worker_iters_per_s": n * args.steps / dt, "last_objective": float(obj[-1])})
            print(json.dumps(res[-1]), file=sys.stderr, flush=True)
    run.run_pipelined(0, eta0, m, lam, lam, 0.0, t0=t)
    print(json.dumps({"workers": n, "n_global": args.n_global, "d": d, "m": m, "steps": args.steps, "legs": res,
                      "kernel": bench.kernel_name()}), flush=True)
    eng.close()
    torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
