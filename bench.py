#!/usr/bin/env python3
"""Benchmark: D-SGD round throughput (worker-iterations/s) and HBM roofline on MI355X.

Workload (BASELINE.json config C3, the metric's configuration): logistic regression,
N = 4096 workers per GPU, d = 1024 (incl. bias), m = 512 rows per worker, full-shard
batches (b = m), random 4-regular topology with Metropolis-Hastings weights, fp32,
objective + consensus recorded EVERY round (as trainer.py:182-191 does).
A step = one D-SGD round over every worker (gradient, mix, step, metrics).

Multi-GPU (`--gpus N` under torch.distributed.run): ONE random 4-regular graph over
4096 x N workers (weak scaling), each rank owning a contiguous slice; halo rows of
the iterates move by grouped send/recv (RCCL) while the gradient kernel runs, and
the average model is all-reduced every round (distributed.py).

Prints ONE JSON line on rank 0 (driver contract), with `roofline` for the fused
round kernel (HIP-event timed, same timed region) and `cpu_baseline` (the oracle,
i.e. the reference's per-worker numpy round, on a bounded sample, rank 0, N=1 only).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

METRIC = "worker-iters/sec + % HBM roofline, logistic N=4096 d=1024, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def pmc_traffic(kernel_name):
    """Per-dispatch HBM bytes of `kernel_name` from the newest committed rocprofv3 PMC
    summary (profiles/<tag>_pmc.json, written by scripts/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per the gfx950 correction)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    for f in reversed(files):
        try:
            rec = json.load(open(f)).get(kernel_name)
        except Exception:
            continue
        if rec:
            return rec["hbm_bytes_per_dispatch"], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(seconds, n_workers=64, d=1024, m=512, seed=11):
    """The oracle (numpy restatement of the reference round, float64) on a bounded
    sample: n_workers workers of the C3 shape, same per-round work as the reference
    (per-worker minibatch draw + gradient, dense W @ X, objective over all sample rows,
    consensus)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import dsgd_oracle as O
    import topology

    try:
        from threadpoolctl import threadpool_info

        threads = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    rng = np.random.default_rng(seed)
    wstar = rng.standard_normal(d)
    shards = []
    for _ in range(n_workers):
        X = np.hstack([rng.standard_normal((m, d - 1)), np.ones((m, 1))])
        y = np.sign(X @ wstar)
        flip = rng.random(m) < 0.05
        y[flip] = -y[flip]
        shards.append((X, y))
    Xf = np.vstack([s[0] for s in shards])
    yf = np.concatenate([s[1] for s in shards])
    W = topology.random_regular(n_workers, 4, seed=0).dense_W()
    cfg = {"problem_type": "logistic", "local_batch_size": m, "learning_rate_eta0": 0.05,
           "l2_regularization_lambda": 1e-4, "strong_convexity_mu": 1e-4}
    O.run_decentralized(shards, W, 1, cfg, Xf, yf, 0.0)  # warm caches / BLAS threads
    t0 = time.perf_counter()
    O.run_decentralized(shards, W, 2, cfg, Xf, yf, 0.0)
    t1 = (time.perf_counter() - t0) / 2
    rounds = max(1, min(400, int(seconds / max(t1, 1e-3))))
    t0 = time.perf_counter()
    O.run_decentralized(shards, W, rounds, cfg, Xf, yf, 0.0)
    dt = time.perf_counter() - t0
    return {"value": n_workers * rounds / dt, "unit": "worker-iters/s", "cores": int(threads), "kind": "port",
            "sample": f"oracle (numpy float64 restatement of trainer.py:161-193) on {n_workers} workers x "
                      f"{m} rows x d={d}, {rounds} rounds, {dt:.1f} s, full-shard batches, metrics every round"}


def pcie_leg(eng, top, n, d, m, b, lam, eta0, steps, dt_resident):
    """Boundary cost when the caller hands over host buffers (Worker.local_data numpy arrays
    -> dopt_load_shards): the device-generated shards are copied to host memory once
    (untimed), then uploaded through the C ABI (timed: host -> HBM DMA + the convert kernel
    into the padded layout), and the same `steps` rounds run on them.  Reported as the
    PCIe-inclusive rate n*steps / (upload + rounds) next to the resident-input rate."""
    import numpy as np
    import torch

    log("pcie leg: staging shards in host memory")
    X = np.empty((n * m, d), dtype=np.float32)
    y = np.empty(n * m, dtype=np.float32)
    step = 256
    for i0 in range(0, n, step):  # pull back by worker blocks (fp64 download path)
        for i in range(i0, min(n, i0 + step)):
            Xi, yi = eng.get_shard(i)
            X[i * m:(i + 1) * m] = Xi
            y[i * m:(i + 1) * m] = yi
    off = np.arange(n + 1, dtype=np.int64) * m
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.load_shards("logistic", X, y, off)
    torch.cuda.synchronize()
    t_up = time.perf_counter() - t0
    eng.set_topology(top.row_ptr, top.col, top.w)
    eng.set_models(np.zeros((n, d)))
    eng.set_profiling(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run_dsgd(steps, eta0, b, lam, lam, 0.0)
    torch.cuda.synchronize()
    t_run = time.perf_counter() - t0
    nbytes = X.nbytes + y.nbytes
    del X, y
    return {"upload_s": t_up, "upload_GBps": nbytes / t_up / 1e9, "host_bytes": nbytes,
            "rounds_s": t_run, "rounds_s_resident": dt_resident, "steps": steps,
            "value_incl_upload": n * steps / (t_up + t_run), "unit": "worker-iters/s",
            "note": "host float32 buffers (pageable numpy) through dopt_load_shards; rounds on the "
                    "uploaded shards, same K; not the headline value (inputs resident in HBM)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300,
                    help="rounds timed (one run: the last round's metrics pass is amortised over them)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workers", type=int, default=4096, help="workers per GPU")
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--data-dtype", default=None,
                    help="shard storage (default: --dtype); float32 under --dtype float64 keeps every "
                         "operation in float64 over float32-representable rows")
    ap.add_argument("--batch", type=int, default=0,
                    help="C3 minibatch per worker (0: the full shard, the metric's configuration); b < m "
                         "draws the minibatches on the device (sampling='device', Philox + Floyd)")
    ap.add_argument("--degree", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (gloo: 1-GPU rehearsal)")
    ap.add_argument("--event-every", type=int, default=10,
                    help="bracket every k-th round kernel with a HIP event pair (0: none). A pair costs ~30 us "
                         "of round time, so the default samples 1 launch in 10 of the timed region")
    ap.add_argument("--phase", action="store_true",
                    help="drive the multi-GPU phase path even on one GPU (measures its per-rank overhead)")
    ap.add_argument("--partition", default="spectral", choices=["spectral", "ranges"],
                    help="C3 at N > 1: workers -> GPUs by graph partition (recursive spectral bisection, "
                         "computed on rank 0 and broadcast) or by contiguous id ranges")
    ap.add_argument("--pcie", action="store_true",
                    help="C3, 1 GPU: after the timed region, hand the same shards over as host buffers "
                         "(dopt_load_shards, the drop-in boundary) and report the PCIe-inclusive rate in a "
                         "'pcie' object (never 'value')")
    ap.add_argument("--config", default="c3", choices=["c3", "c4", "c5"],
                    help="c3 (default, the metric's config); c4: 256x256 torus, 65536 workers total; "
                         "c5: quadratic, d=2^20, m=b=16, 1024 workers total, complete graph")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch  # plumbing only: barrier + max-over-ranks (one HIP runtime, loaded first)
    import torch.distributed as dist

    import numpy as np

    import _dopt
    import distributed
    import topology

    dev = local % max(1, torch.cuda.device_count())
    if world > 1 or args.phase:
        torch.cuda.set_device(dev)
        if world == 1:  # --phase on one GPU: the multi-GPU code path incl. RCCL (one rank)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            distributed.init_process_group(args.backend, rank=0, world_size=1)
        else:
            distributed.init_process_group(args.backend)

    problem, mean, eta0 = "logistic", None, 0.05
    if args.config == "c3":
        n, d, m = args.workers, args.d, args.m
        n_global = n * world
        top = topology.random_regular(n_global, args.degree, seed=0)
        if world > 1 and args.partition == "spectral":  # relabel so each GPU's part is an id range
            order = [distributed.partition_order(distributed.graph_partition(top, world)) if rank == 0 else None]
            dist.broadcast_object_list(order, src=0)
            top = topology.relabel(top, order[0])
        workload = (f"C3: logistic, {n} workers/GPU, d={d}, m=b={m}, random {args.degree}-regular MH mixing, "
                    "objective+consensus every round")
    elif args.config == "c4":
        d, m, n_global = 1024, 512, 65536
        top = topology.grid(n_global)
        workload = "C4: logistic, 65536 workers total on a 256x256 torus, d=1024, m=b=512"
    else:
        problem, d, m, n_global = "quadratic", 1 << 20, 16, 1024
        eta0 = 1e-5  # L ~ d/b for N(0,1) rows of length 2^20: eta0 = 0.05 (set for d = 81) diverges
        top = topology.fully_connected(n_global)
        mean = top.uniform_offdiag()
        workload = "C5: quadratic, 1024 workers total, d=2^20, m=b=16, complete graph (column-sum mixing)"
    plan = distributed.build_plan(top, world, rank) if mean is None else None
    if plan is None:  # complete graph: contiguous slices, no halo plan needed
        bounds = distributed.partition_bounds(n_global, world)
        plan = distributed.HaloPlan(rank, world, bounds, int(bounds[rank]), int(bounds[rank + 1]),
                                    np.zeros(0, np.int64), np.zeros(world + 1, np.int64), np.zeros(0, np.int32),
                                    np.zeros(world + 1, np.int64), None, None, None)
    n = plan.n_local
    log(f"rank {rank}/{world}: generating {plan.n_local} x {m} x {d} {args.dtype} shards on device {dev}")
    eng = _dopt.Engine(dev, args.dtype, data_dtype=args.data_dtype)
    eng.generate_shards(problem, plan.n_local, d, m, seed=1000, flip=0.05, first_worker=plan.lo)
    lam = 1e-4
    b = args.batch if 0 < args.batch < m else m
    if b < m:  # minibatches drawn on the device inside the pass over all rows (the metrics need them all)
        if args.config != "c3":
            raise SystemExit("--batch < m: C3 only (device sampling)")
        eng.set_sampler("device", seed=7, first_worker=plan.lo)
        workload = workload.replace(f"m=b={m}", f"m={m}, b={b} (device-drawn minibatches)")
    if world > 1 or args.phase:
        mean_local = None if mean is None else (mean[0], mean[1][plan.lo:plan.hi])
        runner = distributed.DistributedDSGD(eng, plan, n_global, n_global * m, device=dev, mean=mean_local)
        log(f"halo: {plan.n_halo} rows in, {len(plan.send_ids)} rows out per round")

        def rounds(k):
            return runner.run(k, eta0, b, lam, lam, 0.0)
    else:
        if mean is not None:
            eng.set_mixing_mean(*mean)
        else:
            eng.set_topology(top.row_ptr, top.col, top.w)

        def rounds(k):
            obj, cons, _ = eng.run_dsgd(k, eta0, b, lam, lam, 0.0)
            return obj, cons
    log("warmup")
    if args.warmup > 0:
        rounds(args.warmup)
    eng.set_models(np.zeros((plan.n_local, d)))
    eng.kernel_stats()  # reset the event window

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    eng.set_profiling(args.event_every > 0, every=max(1, args.event_every))
    barrier()
    log(f"timing {args.steps} rounds")
    t0 = time.perf_counter()
    obj, cons = rounds(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}" if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    launches, kr_ms = eng.kernel_stats()
    if not all(map(math.isfinite, list(obj) + list(cons))):
        raise RuntimeError("non-finite metrics")

    esz = 4 if args.dtype in ("float32", "fp32", "f32") else 8
    xesz = 4 if eng.data_dtype == _dopt.F32 else 8
    tname = "float" if esz == 4 else "double"
    sname = "float" if xesz == 4 else "double"
    cpl = 1
    while cpl * 64 < (d + (16 // xesz) - 1) // (16 // xesz):
        cpl *= 2
    if cpl <= 16:
        var = 14371 | 256 if cpl <= 4 else 14371  # kernels.hip: kr_default_var<CPL>()
        if xesz != esz:
            var = 14371
        kname = (f"void dopt::k_round<{tname}, {sname}, {cpl}, {0 if problem == 'logistic' else 1}, true, true, {var}>"
                 "(dopt::RoundArgs)")
    else:
        kname = f"void dopt::k_split_step<{tname}, {4 if m <= 16 else 16}, true, true>(dopt::RoundArgs)"
    traffic, traffic_src = pmc_traffic(kname) if args.config == "c3" and n == 4096 and world == 1 else (None, None)
    bytes_per_launch = n * (xesz * (m * d + m) + esz * 2 * d)  # X_b + y_b + x read + x write
    avg_s = (kr_ms / launches) * 1e-3 if launches else float("nan")
    achieved = bytes_per_launch / avg_s / 1e9 if launches else None
    value = n_global * args.steps / dt
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "worker-iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if esz == 4 else "f64",
        "data": "synthetic (device-generated X~N(0,1)+bias, planted-w* labels, 5% flips)",
        "config": {"workload": workload,
                   "workers_per_gpu": n, "d": d, "rows_per_worker": m, "batch": b, "topology": top.name,
                   "degree": args.degree if args.config == "c3" else None,
                   "halo_rows_per_gpu": int(plan.n_halo),
                   "parallelism": (f"dp{world}: one graph of {n_global} workers, "
                                   f"{'graph-partitioned' if args.config == 'c3' and args.partition == 'spectral' else 'contiguous'} "
                                   f"slices per GPU, halo send/recv + all-reduce ({args.backend})") if world > 1
                                  else ("single GPU: the multi-GPU phase path (lagged schedule, "
                                        f"{args.backend} world 1)") if args.phase
                                  else "single GPU: fused round kernel, one launch per round"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "kernel": kname, "kernel_avg_ms": avg_s * 1e3 if launches else None,
                     "kernel_launches_timed": launches, "event_every": args.event_every,
                     "bytes_per_launch": bytes_per_launch},
        "final_objective": float(obj[-1]),
        "final_consensus": float(cons[-1]),
    }
    if args.config != "c3":
        out["metric"] = f"worker-iters/sec ({args.config.upper()}, secondary config)"
        out["scaling"] = "strong"
    if args.pcie and world == 1 and args.config == "c3":
        out["pcie"] = pcie_leg(eng, top, n, d, m, b, lam, eta0, args.steps, dt)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c3":
        log("cpu baseline")
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1 or args.phase:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
