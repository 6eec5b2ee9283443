#!/usr/bin/env python3
"""One GPU runs what rank R of an N-rank `bench.py --gpus N` run does, and times it beside the fused
one-GPU round (the N = 1 line), to predict the per-rank efficiency of the driver's scaling run.

This pool gives one GPU per call, so the N-rank path itself only runs over gloo (host-staged) or over
RCCL at world 1.  The proxy takes rank R's real halo plan of the bench's graph -- the random 4-regular
graph over 4096 x N workers (weak leg) or 4096 in all (strong leg), spectrally partitioned as
bench.py partitions it -- and turns it into a world-1 plan with the same local CSR, boundary share and
interior set: the rows any peer reads (the rank's send set, each row once) go through the RCCL
all-to-all to the rank itself, and every halo column h of the CSR reads slot h mod |send set| of that
copy (a local row stands in for the remote one: the values differ, the schedule, the kernels, their
bytes and the exchange's kernel do not).  So one GPU runs the lagged schedule exactly as rank R would:
the gradient kernel with the interior workers stepped inside it, `k_mixcs` over the real boundary
workers, `k_mixcs_final` and an all-to-all that moves |send set| rows plus the sum rows, with the
collectives forced (DOPT_FORCE_COLLECTIVES=1).  The exchange goes over the transport DOPT_TRANSPORT names:
at world 1 the default is the engine's RCCL communicator; DOPT_TRANSPORT=ipc pulls the rank's blocks from
its own send slot with k_pull (the pull transport, the default of a multi-GPU job on one node).  What it
cannot show: xGMI itself (the self copy is a local device copy), the peers' latency, and rank imbalance.

  python3 tools/rank_proxy.py --world 8 --rank 0 --scaling weak --reps 2 --steps 400 --warmup 50
  python3 tools/rank_proxy.py --world 8 --plan-only          # plan statistics only (CPU)

Prints one JSON object: per leg (fused 4096, proxy) and repetition the worker-iters/s, ms per round,
the gradient kernel's average by HIP events, and the proxy / fused ratio (the per-rank efficiency the
weak-scaling line can reach at most on that rank, before xGMI and RCCL peer latency).
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


def rank_plan(world, rank, n_global, degree=4, config="c3"):
    """Rank `rank`'s HaloPlan of the bench's graph and the partition's cut: C3 (bench.setup_leg: random_regular,
    seed 0, spectral partition, relabel) or C4 (the 256 x 256 torus in contiguous strips of torus rows)."""
    import distributed as Dm
    import topology

    if config == "c4":
        top = topology.grid(n_global)
        part = np.repeat(np.arange(world), np.diff(Dm.partition_bounds(n_global, world)))
        return Dm.build_plan(top, world, rank), Dm.cut_edges(top, part)
    top = topology.random_regular(n_global, degree, seed=0)
    part = Dm.graph_partition(top, world)
    cut = Dm.cut_edges(top, part)
    top = topology.relabel(top, Dm.partition_order(part))
    return Dm.build_plan(top, world, rank), cut


def self_plan(plan):
    """The world-1 stand-in of a rank's plan (module docstring)."""
    import distributed as Dm

    n = plan.n_local
    S = np.unique(plan.send_ids.astype(np.int64))
    ns = len(S)
    if ns == 0:
        raise SystemExit("the rank sends no rows: nothing to stand in for")
    col = plan.col.astype(np.int64).copy()
    h = col >= n
    col[h] = n + (col[h] - n) % ns
    return Dm.HaloPlan(0, 1, np.array([0, n], np.int64), 0, n, np.arange(ns, dtype=np.int64),
                       np.array([0, ns], np.int64), S.astype(np.int32), np.array([0, ns], np.int64),
                       plan.row_ptr.astype(np.int64).copy(), col.astype(np.int32), plan.w.copy())


def plan_stats(plan, sp, cut):
    n = plan.n_local
    rows = np.repeat(np.arange(n), np.diff(plan.row_ptr))
    has_halo = np.zeros(n, bool)
    has_halo[rows[plan.col >= n]] = True
    sent = np.zeros(n, bool)
    sent[plan.send_ids] = True
    interior = int(np.sum(~has_halo & ~sent))
    return {"n_local": int(n), "halo_rows_in": int(plan.n_halo), "send_rows_out": int(len(plan.send_ids)),
            "send_set": int(len(np.unique(plan.send_ids))), "peers": [int(p) for p in plan.peers()],
            "workers_with_halo_column": int(has_halo.sum()), "interior": interior,
            "boundary_share": 1.0 - interior / n, "cut_edges": int(cut),
            "proxy_rows_through_exchange": int(sp.n_halo)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--config", default="c3", choices=["c3", "c4"],
                    help="c4: the 256 x 256 torus (65536 workers in all) in strips, --workers ignored")
    ap.add_argument("--workers", type=int, default=4096, help="per rank (weak) / in all (strong)")
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--fused-workers", type=int, default=4096, help="the fused leg's workers (the N = 1 line)")
    ap.add_argument("--legs", default="fused,proxy", help="legs per repetition, in order")
    ap.add_argument("--fused-steps", type=int, default=0, help="the fused leg's timed rounds (0: --steps)")
    ap.add_argument("--plan-only", action="store_true")
    ap.add_argument("--early-streams", action="store_true",
                    help="create the runners' two shared streams (distributed._stream) before any engine exists")
    ap.add_argument("--prealloc", action="store_true",
                    help="first generate (and free) a throwaway engine's shards of the fused leg's size: no rounds run "
                         "(does the first large allocation of a process behave differently?)")
    ap.add_argument("--no-force", action="store_true",
                    help="no collectives at world 1 (the halo slots are never filled): the kernels alone")
    args = ap.parse_args()

    n_global = args.workers * args.world if args.scaling == "weak" else args.workers
    if args.config == "c4":
        n_global = 65536
    t0 = time.perf_counter()
    plan, cut = rank_plan(args.world, args.rank, n_global, config=args.config)
    sp = self_plan(plan)
    out = {"world": args.world, "rank": args.rank, "config": args.config, "scaling": args.scaling, "n_global": n_global,
           "plan_s": time.perf_counter() - t0, "plan": plan_stats(plan, sp, cut)}
    if args.plan_only:
        print(json.dumps(out), flush=True)
        return 0

    os.environ["DOPT_FORCE_COLLECTIVES"] = "0" if args.no_force else "1"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import torch
    import torch.distributed as dist

    import _dopt
    import bench
    import distributed as Dm
    import topology

    torch.cuda.set_device(0)
    Dm.init_process_group("nccl", store=bench._solo_store(), rank=0, world_size=1)
    d, m, lam, eta0 = args.d, args.m, 1e-4, 0.05
    n = plan.n_local

    def barrier():
        torch.cuda.synchronize(0)

    def leg_fused():
        nf = args.fused_workers
        eng = _dopt.Engine(0, "float64", data_dtype="float32")
        try:
            eng.generate_shards("logistic", nf, d, m, seed=1000, flip=0.05)
            top = topology.random_regular(nf, 4, seed=0)
            eng.set_topology(top.row_ptr, top.col, top.w)
            return eng, (lambda k: eng.run_dsgd_pipelined(k, eta0, m, lam, lam, 0.0)), \
                (lambda: eng.run_dsgd_pipelined(0, eta0, m, lam, lam, 0.0)), {"workers": nf}
        except Exception:
            eng.close()
            raise

    def leg_proxy():
        eng = _dopt.Engine(0, "float64", data_dtype="float32")
        try:
            eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05, first_worker=plan.lo)
            run = Dm.DistributedDSGD(eng, sp, n_global, n_global * m, device=0)
            if not run._lagged_ok or (not args.no_force and (run.layout.ks == 0 or not run.exchange.collective)):
                raise SystemExit("the proxy did not take the lagged schedule with the RCCL exchange")
            info = {"workers": n, "interior_engine": eng.phase_interior_count(), "side_stream": run.side is not None,
                    "exchange_rows_out": run.layout.n_send_rows, "exchange_rows_in": run.layout.n_recv_rows}
            return eng, (lambda k: run.run_pipelined(k, eta0, m, lam, lam, 0.0)), \
                (lambda: run.run_pipelined(0, eta0, m, lam, lam, 0.0)), info
        except Exception:
            eng.close()
            raise

    if args.early_streams:
        Dm._stream(torch.device("cuda", 0), 0)
        Dm._stream(torch.device("cuda", 0), 1)
    if args.prealloc:
        tmp = _dopt.Engine(0, "float64", data_dtype="float32")
        tmp.generate_shards("logistic", args.fused_workers, d, m, seed=1000, flip=0.05)
        tmp.sync()
        tmp.close()
    legs = []
    for rep in range(args.reps):
        for name in args.legs.split(","):
            eng, rounds, flush, info = {"fused": leg_fused, "proxy": leg_proxy}[name]()
            nw = info["workers"]
            steps = args.fused_steps if (name == "fused" and args.fused_steps > 0) else args.steps
            warm = min(args.warmup, steps) if name == "fused" and args.fused_steps > 0 else args.warmup
            try:
                dt, launches, kr_ms, every, obj, cons = bench.timed_leg(eng, rounds, steps, warm, nw, d,
                                                                        barrier, 0, flush)
            finally:
                eng.close()
            legs.append({"leg": name, "rep": rep, "value": nw * steps / dt, "ms_per_round": dt / steps * 1e3,
                         "kernel_avg_ms": kr_ms / launches if launches else None, "kernel_launches": launches,
                         "final_objective": float(obj[-1]), **info})
            print(json.dumps(legs[-1]), file=sys.stderr, flush=True)
    f = [g["value"] for g in legs if g["leg"] == "fused"]
    p = [g["value"] for g in legs if g["leg"] == "proxy"]
    out.update({"steps": args.steps, "warmup": args.warmup, "legs": legs,
                "proxy_over_fused": [b / a for a, b in zip(f, p)], "kernel": bench.kernel_name()})
    print(json.dumps(out), flush=True)
    Dm.close_comms()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
