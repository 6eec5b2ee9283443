#!/usr/bin/env python3
"""Benchmark: D-SGD round throughput (worker-iterations/s) and HBM roofline on MI355X.

Workload (BASELINE.json config C3, the metric's configuration): logistic regression,
N = 4096 workers per GPU, d = 1024 (incl. bias), m = 512 rows per worker, full-shard
batches (b = m), random 4-regular topology with Metropolis-Hastings weights,
objective + consensus recorded EVERY round (as trainer.py:182-191 does).
A step = one D-SGD round over every worker (gradient, mix, step, metrics).

Precision (the reference computes in float64, obj_problems.py / trainer.py:173): the
headline `value` runs every product, sum and transcendental in float64 with float64
iterates, over shards whose values are exactly float32-representable and are therefore
stored as float32 (dopt_set_data_dtype: the stored rows ARE the float64 rows, at half the
bytes).  Secondary legs at N=1: the same round with float64-stored rows ('f64_storage'),
the float32 engine ('f32'), the device f(x*) solver (final suboptimality, as
trainer.py:189-191 reports objective - f_opt), and the drop-in DecentralizedTrainer at C3
with the reference's legacy RNG stream ('dropin').

Multi-GPU: `python3 bench.py --gpus N` starts N ranks itself (torch.distributed.run as a
child process, before anything touches the GPU); under an external torch.distributed.run
WORLD_SIZE must equal --gpus.  `value` at every N is the metric's configuration, strong scaling:
N = 4096 workers IN TOTAL over the N ranks (4096 / N each), ONE random 4-regular graph,
graph-partitioned so each rank owns a contiguous slice; the halo rows of the iterates and every
rank's column sums (for xbar) move in ONE exchange per round (RCCL), issued beside the gradient
kernel (distributed.py's lagged schedule; C5's complete graph all-reduces the column sums
instead).  Weak scaling (`weak`, N > 1, secondary): 4096 workers PER GPU, 4096 x N in all, same
graph construction.

Prints ONE JSON line on rank 0 (driver contract), with `roofline` for the fused
round kernel (HIP-event timed, same timed region) and `cpu_baseline` (the oracle,
i.e. the reference's per-worker numpy round, on a bounded sample, rank 0, N=1 only).
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

T_START = time.time()  # process start (setup time: until the timed region begins)
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))

METRIC = "worker-iters/sec + % HBM roofline, logistic N=4096 d=1024, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def pmc_traffic(kernel_name, config="c3"):
    """Per-dispatch HBM bytes of `kernel_name` from the newest committed rocprofv3 PMC
    summary of this configuration (profiles/r<round>[_c4|_c5|_c5rs|_c5x32]_pmc.json, written by
    scripts/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled
    per the gfx950 correction).  C3 and C4 launch the same kernel instance, so the file is
    picked by configuration, not by kernel name alone."""
    import glob
    import re

    pat = {"c3": r"r\d+_pmc\.json", "c4": r"r\d+_c4_pmc\.json",
           "c5": r"r\d+_c5(rs|x32|x32direct)?_pmc\.json"}[config]
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))
                   if re.fullmatch(pat, os.path.basename(f)))
    for f in reversed(files):
        try:
            doc = json.load(open(f))
        except Exception:
            continue
        rec = doc.get(kernel_name)
        if rec:
            run = doc.get("_run") or {}
            # the profiled run itself (one box, one gpurun call): its step time and the trace's average of
            # the same kernel over that run's timed launches (scripts/pmc_summary.py)
            same = {"ms_per_step": run.get("ms_per_step"), "kernel_timed_avg_ms_trace": run.get("kernel_timed_avg_ms_trace"),
                    "kernel_avg_ms_events": run.get("kernel_avg_ms_events"), "steps": run.get("steps")} if run else None
            return rec["hbm_bytes_per_dispatch"], os.path.relpath(f, ROOT), same
    return None, None, None


# ---------------------------------------------------------------------------- CPU baseline
def _cpu_sample(n_workers, d, m, seed, seconds):
    """One process's share of the CPU baseline: the oracle's round (numpy float64 restatement
    of trainer.py:161-193) on n_workers workers of the C3 shape for about `seconds`.
    Returns (worker-iters/s, rounds, wall seconds)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import dsgd_oracle as O
    import topology

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
    return n_workers * rounds / dt, rounds, dt


def cpu_worker_main(argv):
    """`bench.py --cpu-worker SEED SECONDS`: one single-threaded sample process (BLAS threads
    set to 1 in its environment by the parent); prints its result as one JSON line."""
    seed, seconds = int(argv[0]), float(argv[1])
    rate, rounds, dt = _cpu_sample(64, 1024, 512, seed, seconds)
    print(json.dumps({"rate": rate, "rounds": rounds, "wall_s": dt}), flush=True)


def _cpu_share():
    """CPUs this process may use: the affinity mask, capped at the GPU box's CPU share per GPU
    (16: the pool grants 16 host CPUs per GPU, although nproc shows the whole machine)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    return max(1, min(avail, int(os.environ.get("DOPT_CPU_SHARE", "16"))))


def cpu_baseline(seconds, procs=None):
    """The oracle on the host cores: `procs` single-threaded processes (one per core of the
    box's CPU share), each running its own 64-worker sample of the C3 shape concurrently for
    ~`seconds`; value = the sum of their worker-iters/s.  Per-worker work is independent of N
    but for the dense W @ X (trainer.py:173), 0.08-0.14 s of a 9.25 s reference round at
    N = 4096: under 2 % of it, so per-worker extrapolation to 4096 flatters the
    CPU by at most that much."""
    procs = procs or _cpu_share()
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    env.pop("DOPT_CPU_SHARE", None)
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(11 + k), str(seconds)],
                           stdout=subprocess.PIPE, env=env) for k in range(procs)]
    res = []
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 6 + 120)
        if p.returncode != 0:
            raise RuntimeError(f"cpu baseline worker exited {p.returncode}")
        res.append(json.loads(out.decode().strip().splitlines()[-1]))
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu_model)
    except OSError:
        pass
    rates = [r["rate"] for r in res]
    return {"value": float(sum(rates)), "unit": "worker-iters/s", "cores": procs, "kind": "port",
            "cpu_model": cpu_model, "nproc": os.cpu_count(), "processes": procs, "blas_threads_per_process": 1,
            "per_process_rate": [float(r) for r in rates],
            "sample": f"oracle (numpy float64 restatement of trainer.py:161-193), {procs} concurrent single-threaded "
                      f"processes, each 64 workers x 512 rows x d=1024 ({min(r['rounds'] for r in res)}-"
                      f"{max(r['rounds'] for r in res)} rounds, ~{seconds:.0f} s), full-shard batches, metrics every "
                      f"round; aggregate per-worker rate, i.e. extrapolated per worker to C3's 4096 (the dense "
                      f"W @ X is under 2 % of a reference round at N = 4096, SURVEY.md 3.3); cores = the box's CPU "
                      f"share per GPU (affinity {len(os.sched_getaffinity(0))} CPUs, capped at 16)"}


# ---------------------------------------------------------------------------- legs
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


def _chunks_per_lane(d, xesz):
    nch = (d + (16 // xesz) - 1) // (16 // xesz)
    cpl = 1
    while cpl * 64 < nch:
        cpl *= 2
    return cpl


def kernel_name():
    """Instance name (rocprofv3's spelling) of the gradient-round kernel the runtime launched last
    (dopt_last_round_kernel: recorded by the launcher, not re-derived here)."""
    import _dopt

    return _dopt.last_round_kernel() or "unknown"


def bytes_per_round(eng, n, d, m, kname=""):
    """shard rows + labels read once, own iterate read + new iterate written
    (neighbour rows hit L2 / MALL): n * (xesz * (m*d + m) + esz * 2d).  The row-space pass
    (C5, k_rs_pass: iterates held as Z + X_i^T beta_i) reads the rows and one
    float64 coefficient per row and writes no iterate: n * m * (xesz * d + 8)."""
    import _dopt

    esz = 4 if eng.dtype == _dopt.F32 else 8
    xesz = 4 if eng.data_dtype == _dopt.F32 else 8
    if "k_rs_pass" in kname:
        return n * m * (xesz * d + 8)
    return n * (xesz * (m * d + m) + esz * 2 * d)


def timed_leg(eng, rounds, steps, warmup, n_models, d, barrier, event_every, flush=None):
    """Warmup, reset, then `steps` rounds bracketed by barrier + device sync, with HIP events
    around every `event_every`-th round kernel (at least 10 sampled launches).

    flush: the rounds are PIPELINED runs (dopt_run_dsgd_pipelined): then the warmup runs from
    the reset iterate and leaves the metrics of its last iterate owed, the timed call takes
    them in (its first pass) and leaves its own last ones owed, and flush() computes those
    after the timed region -- so the timed region holds exactly `steps` fused rounds and
    `steps` metric evaluations, the steady state of a long run (a lone dopt_run_dsgd of
    `steps` rounds adds one unfused metrics-only pass over the shards: 1/steps more work)."""
    import numpy as np

    if flush is None and warmup > 0:
        rounds(warmup)
    eng.zero_models()  # the reset iterate (Worker.x = zeros), on the device
    if flush is not None:
        rounds(max(3, warmup))  # the multi-GPU lagged schedule completes history[t] two rounds later
    eng.kernel_stats()  # reset the event window
    every = event_every if event_every > 0 else max(1, steps // 10)
    eng.set_profiling(True, every=every)
    barrier()
    t0 = time.perf_counter()
    obj, cons = rounds(steps)
    barrier()
    dt = time.perf_counter() - t0
    launches, kr_ms = eng.kernel_stats()
    eng.set_profiling(False)
    if flush is not None:
        if len(obj) != steps:
            raise RuntimeError(f"pipelined timed call wrote {len(obj)} metric entries for {steps} rounds")
        fo, fc = flush()  # the metrics of the final iterate (untimed)
        obj, cons = np.concatenate([obj, fo]), np.concatenate([cons, fc])
    if not all(map(math.isfinite, list(obj) + list(cons))):
        raise RuntimeError("non-finite metrics")
    return dt, launches, kr_ms, every, obj, cons


def secondary_leg(dev, dtype, data_dtype, top, n, d, m, steps, warmup, lam, eta0, barrier, event_every):
    """The C3 round with another storage / compute dtype on a fresh context (same generated data)."""
    import _dopt

    eng = _dopt.Engine(dev, dtype, data_dtype=data_dtype)
    try:
        eng.generate_shards("logistic", n, d, m, seed=1000, flip=0.05)
        eng.set_topology(top.row_ptr, top.col, top.w)

        def rounds(k):
            return eng.run_dsgd_pipelined(k, eta0, m, lam, lam, 0.0)

        def flush():
            return eng.run_dsgd_pipelined(0, eta0, m, lam, lam, 0.0)

        dt, launches, kr_ms, every, obj, cons = timed_leg(eng, rounds, steps, warmup, n, d, barrier, event_every,
                                                          flush)
        bpl = bytes_per_round(eng, n, d, m)
        avg = kr_ms / launches * 1e-3
        return {"value": n * steps / dt, "unit": "worker-iters/s", "ms_per_step": dt / steps * 1e3,
                "dtype": "f32" if eng.dtype == _dopt.F32 else "f64",
                "storage": "f32" if eng.data_dtype == _dopt.F32 else "f64",
                "kernel": kernel_name(), "kernel_avg_ms": avg * 1e3,
                "kernel_launches_timed": launches, "bytes_per_launch": bpl,
                "roofline_frac": bpl / avg / 1e9 / HBM_PEAK_GBS, "final_objective": float(obj[-1])}
    finally:
        eng.close()


def suboptimality(eng, lam, final_objective):
    """f_opt of the C3 problem by the device L-BFGS solver (solver.py over dopt_eval_full, one
    pass over the shards per evaluation, float64), and the reference's reported quantity
    objective - f_opt (trainer.py:189-191, f_opt from simulator.py:32-69)."""
    import solver

    t0 = time.perf_counter()
    f_opt, _, info = solver.reference_optimum(eng, lam, gtol=1e-9, max_iter=500)
    return {"f_opt": f_opt, "final_suboptimality": final_objective - f_opt, "solver_s": time.perf_counter() - t0,
            "solver_evaluations": info["evaluations"], "solver_grad_norm": info["grad_norm"],
            "note": "device L-BFGS on the full-data objective (replaces sklearn saga at sizes it cannot run)"}


def dropin_leg(eng, n, d, m, lam, eta0, rounds=128, batch=None, reps=5):
    """The drop-in DecentralizedTrainer (trainer.py API) on the same C3 shards as host arrays,
    sampling='legacy': every round draws the reference's numpy legacy-MT19937 stream
    (4096 permutations of 512 per round, worker.py:27) on the host before the device runs
    it.  Timed: `reps` interleaved pairs of run()s of `rounds` and 3 x `rounds` rounds on the
    warm engine; the per-round rate is the median over the pairs of the slope of the trainer's
    round-loop time (`loop_seconds`: the first chunk's draw before the device starts and the final
    metrics cancel in the slope).  The per-run content hash of the host shards runs before the loop;
    on the box its host-memory jitter (+-0.3 s per run) moved whole-run slopes between 0.25 and 2.1
    ms per round, so the whole-run slope is reported for reference only, like the 0-round run."""
    import numpy as np

    from trainer import DecentralizedTrainer
    from worker import Worker

    X = np.empty((n * m, d), dtype=np.float32)
    y = np.empty(n * m, dtype=np.float32)
    for i in range(n):  # the headline's shards (exactly float32)
        Xi, yi = eng.get_shard(i)
        X[i * m:(i + 1) * m] = Xi
        y[i * m:(i + 1) * m] = yi
    b = batch or m
    cfg = {"problem_type": "logistic", "local_batch_size": b, "learning_rate_eta0": eta0,
           "l2_regularization_lambda": lam, "strong_convexity_mu": lam, "dtype": "float64",
           "sampling": "legacy", "regular_degree": 4, "topology_seed": 0, "spectral_gap": False}
    ws = [Worker(i, {"X": X[i * m:(i + 1) * m], "y": y[i * m:(i + 1) * m]}, b, d, cfg) for i in range(n)]
    tr = DecentralizedTrainer(ws, "random_regular", d, cfg)
    np.random.seed(203)
    tr.run(2, X, y)  # loads the engine

    def timed(T):
        tr = DecentralizedTrainer(ws, "random_regular", d, cfg)
        t0 = time.perf_counter()
        hist, _ = tr.run(T, X, y)
        return time.perf_counter() - t0, tr.loop_seconds, hist

    zero = timed(0)[0]
    runs = []
    for _ in range(reps):
        w1, l1, _ = timed(rounds)
        w3, l3, hist = timed(3 * rounds)
        runs.append((w1, w3, l1, l3))

    def med(v):
        v = sorted(v)
        return v[len(v) // 2], v[0], v[-1]

    per_round, lo, hi = med([(l3 - l1) / (2 * rounds) for _, _, l1, l3 in runs])
    run_slope = med([(w3 - w1) / (2 * rounds) for w1, w3, _, _ in runs])
    # the fixed cost of one run() (trainer set-up, data checks, the first chunk's draw before the device
    # starts, the final metrics pass): every run's wall time less its rounds at the slope
    fixed, fixed_lo, fixed_hi = med([w - k * per_round for w1, w3, _, _ in runs for w, k in ((w1, rounds), (w3, 3 * rounds))])
    T_run = 10_000  # the reference's runs (main.py: 10^4 iterations)
    whole = n * T_run / (fixed + T_run * per_round)
    return {"value": n / per_round, "unit": "worker-iters/s",
            "basis": "measured: median over interleaved pairs of runs of the per-round slope of the trainer's "
                     "round loop",
            "value_whole_run_modelled": whole,
            "whole_run_basis": f"derived, not timed: one run({T_run}) = fixed_per_run_s + {T_run} x ms_per_round",
            "fixed_per_run_s": fixed,
            "fixed_per_run_s_range": [fixed_lo, fixed_hi], "batch": b, "rounds": [rounds, 3 * rounds],
            "reps": reps, "ms_per_round": per_round * 1e3, "ms_per_round_range": [lo * 1e3, hi * 1e3],
            "loop_s": [[r[2], r[3]] for r in runs], "run_wall_s": [[r[0], r[1]] for r in runs],
            "run_slope_ms_per_round": [x * 1e3 for x in run_slope], "zero_round_run_s": zero,
            "final_objective": float(hist["objective"][-1]),
            "note": "trainer.DecentralizedTrainer, sampling='legacy' (numpy's stream, drawn on the host one "
                    "chunk ahead of the device).  value = the measured per-round rate (median over interleaved "
                    "pairs of runs of the slope of the trainer's round-loop time, loop_seconds); "
                    "value_whole_run_modelled = a derived figure for one run(10000): the fixed cost of a run "
                    "(median over the timed runs of wall time less rounds x slope, every byte of the host "
                    "shards hashed per run) plus 10^4 rounds at the slope -- no 10^4-round run is timed"}


# ---------------------------------------------------------------------------- launch
def _solo_store():
    """Rendezvous of a one-rank process group: an in-process store (no port at all)."""
    import torch.distributed as dist

    return dist.HashStore()


def launch_ranks(n, argv, limit_s):
    """`--gpus N > 1` without an external launcher: run torch.distributed.run with N ranks on
    this node as a CHILD process (this process has not touched the GPU and never does), pass
    its output through, and return its exit code -- the worst rank's, as the launcher reports
    it.  The child gets its own process group, ended whole if it outlives `limit_s`."""
    import signal

    # --standalone: the launcher's agent binds its rendezvous store on port 0 itself and the ranks reuse that
    # store (TORCHELASTIC_USE_AGENT_STORE), so no port is picked and released before rank 0 binds it (the
    # EADDRINUSE race of a pre-picked --master-port)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--nnodes=1", f"--nproc-per-node={n}",
           "--local-addr", "127.0.0.1", os.path.abspath(__file__)] + argv
    log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    p = subprocess.Popen(cmd, start_new_session=True)
    try:
        return p.wait(timeout=limit_s)
    except subprocess.TimeoutExpired:
        log(f"ranks still running after {limit_s:.0f} s: ending the launcher's process group")
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
        return 124
    except KeyboardInterrupt:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait()
        return 130


def dry_launch(args, rank, world, local):
    """--dry-launch: the rank layout without any device work -- every rank joins a gloo
    process group (bounded by the job timeout) and rank 0 prints who came up."""
    import socket

    import torch.distributed as dist

    import distributed

    if world == 1:
        distributed.init_process_group("gloo", store=_solo_store(), rank=0, world_size=1)
    else:
        distributed.init_process_group("gloo", rank=rank, world_size=world)
    me = {"rank": rank, "local_rank": local, "pid": os.getpid(), "host": socket.gethostname()}
    every = [None] * world
    dist.all_gather_object(every, me)
    if rank == 0:
        print(json.dumps({"dry_launch": True, "n_gpus": world, "requested_backend": args.backend,
                          "comm": {"world_size": dist.get_world_size(), "backend": dist.get_backend()},
                          "ranks": every}), flush=True)
    dist.destroy_process_group()


# ---------------------------------------------------------------------------- a leg
class Setup:
    """One configuration's engine, plan and round callables on this rank."""


def setup_leg(args, config, n_global, world, rank, dev):
    import numpy as np
    import torch.distributed as dist

    import _dopt
    import distributed
    import topology

    S = Setup()
    S.problem, S.mean, S.eta0 = "logistic", None, 0.05
    if config == "c3":
        S.d, S.m = args.d, args.m
        S.top = topology.random_regular(n_global, args.degree, seed=0)
        if world > 1 and args.partition == "spectral":  # relabel so each GPU's part is an id range
            order = [distributed.partition_order(distributed.graph_partition(S.top, world)) if rank == 0 else None]
            dist.broadcast_object_list(order, src=0)
            S.top = topology.relabel(S.top, order[0])
        S.workload = (f"C3: logistic, {n_global // world if n_global % world == 0 else n_global / world} "
                      f"workers/GPU ({n_global} in all), d={S.d}, m=b={S.m}, random {args.degree}-regular MH "
                      "mixing, objective+consensus every round")
    elif config == "c4":
        S.d, S.m = 1024, 512
        S.top = topology.grid(n_global)
        S.workload = f"C4: logistic, {n_global} workers total on a 256x256 torus, d=1024, m=b=512"
    else:
        S.problem, S.d, S.m = "quadratic", 1 << 20, 16
        S.eta0 = 1e-5  # L ~ d/b for N(0,1) rows of length 2^20: eta0 = 0.05 (set for d = 81) diverges
        S.top = topology.fully_connected(n_global)
        S.mean = S.top.uniform_offdiag()
        S.workload = f"C5: quadratic, {n_global} workers total, d=2^20, m=b=16, complete graph (column-sum mixing)"
    S.n_global = n_global
    plan = distributed.build_plan(S.top, world, rank) if S.mean is None else None
    if plan is None:  # complete graph: contiguous slices, no halo plan needed
        bounds = distributed.partition_bounds(n_global, world)
        plan = distributed.HaloPlan(rank, world, bounds, int(bounds[rank]), int(bounds[rank + 1]),
                                    np.zeros(0, np.int64), np.zeros(world + 1, np.int64), np.zeros(0, np.int32),
                                    np.zeros(world + 1, np.int64), None, None, None)
    S.plan = plan
    d, m = S.d, S.m
    data_dtype = args.data_dtype
    if args.dtype in ("float32", "fp32", "f32") or (_chunks_per_lane(d, 4) > 8 and S.mean is None):
        # float32 engine, or rows beyond the mixed row-resident kernel off the complete graph: storage =
        # compute dtype (the complete graph's row-space rounds read float32 rows under float64
        # arithmetic: k_rs_pass_x32)
        data_dtype = None
    log(f"rank {rank}/{world}: generating {plan.n_local} x {m} x {d} shards ({args.dtype} arithmetic, "
        f"{data_dtype or args.dtype} storage) on device {dev}")
    eng = _dopt.Engine(dev, args.dtype, data_dtype=data_dtype)
    S.eng = eng
    eng.generate_shards(S.problem, plan.n_local, d, m, seed=1000, flip=0.05, first_worker=plan.lo)
    S.lam = lam = 1e-4
    S.b = b = args.batch if 0 < args.batch < m else m
    if b < m:  # minibatches drawn on the device inside the pass over all rows (the metrics need them all)
        if config != "c3":
            raise SystemExit("--batch < m: C3 only (device sampling)")
        eng.set_sampler("device", seed=7, first_worker=plan.lo)
        S.workload = S.workload.replace(f"m=b={m}", f"m={m}, b={b} (device-drawn minibatches)")
    S.comm = None
    eta0 = S.eta0
    if world > 1 or args.phase:
        mean_local = None if S.mean is None else (S.mean[0], S.mean[1][plan.lo:plan.hi])
        runner = distributed.DistributedDSGD(eng, plan, n_global, n_global * m, device=dev, mean=mean_local,
                                             rs_chunks=args.rs_chunks or None)
        ld, esz_state = eng.layout()
        lay = runner.layout
        S.exchange_shape = (list(lay.send_sizes), list(lay.recv_sizes), ld, esz_state)
        S.comm = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                  "halo_rows_in": int(plan.n_halo), "send_rows_out": int(len(plan.send_ids)),
                  "halo_bytes_in_per_round": int(plan.n_halo) * ld * esz_state,
                  "send_bytes_out_per_round": int(len(plan.send_ids)) * ld * esz_state,
                  "peers": [int(p) for p in runner._peers],
                  "exchange_beside_gradient": runner.side is not None,
                  "transport": ("ipc" if runner.ipc is not None else "rccl" if runner.comm is not None
                                else "process group")}
        if S.mean is None:  # the lagged schedule: the column sums ride the halo all-to-all
            S.comm.update({"collectives_per_round": 1 if world > 1 else 0,
                           "exchange": ("one k_pull launch per round reading the peers' send slots through IPC "
                                        "handles (the pull transport, dopt_lagged_ipc_*)" if runner.ipc is not None else
                                        "one RCCL group of per-peer sends / receives per round, issued by the engine "
                                        "(dopt_lagged_exchange)" if runner.comm is not None else
                                        "one all_to_all_single per round") + ": halo rows + every rank's column sums",
                           "colsum_bytes_per_peer_per_round": lay.ks * ld * esz_state,
                           "exchange_bytes_out_per_round": lay.n_send_rows * ld * esz_state})
        else:
            S.comm.update({"allreduce_bytes_per_round": ld * 8, "allreduce_chunks": runner.rs_chunks})
        log(f"comm: {S.comm}")
        if runner._lagged_ok or (S.mean is not None and runner._rowspace_ready()):
            # the lagged schedule / the row-space rounds continued across calls (as on one GPU: timed_leg)
            S.rounds = lambda k: runner.run_pipelined(k, eta0, b, lam, lam, 0.0)
            S.flush = lambda: runner.run_pipelined(0, eta0, b, lam, lam, 0.0)
        else:
            S.rounds = lambda k: runner.run(k, eta0, b, lam, lam, 0.0)
            S.flush = None
    else:
        if S.mean is not None:
            eng.set_mixing_mean(*S.mean)
        else:
            eng.set_topology(S.top.row_ptr, S.top.col, S.top.w)
        # metrics pipelined across calls (dopt_run_dsgd_pipelined; timed_leg)
        S.rounds = lambda k: eng.run_dsgd_pipelined(k, eta0, b, lam, lam, 0.0)
        S.flush = lambda: eng.run_dsgd_pipelined(0, eta0, b, lam, lam, 0.0)
    return S


def run_leg(S, args, world, barrier, dev):
    """Time the leg; returns (wall seconds max over ranks, launches, kernel ms, every, obj, cons)."""
    import torch
    import torch.distributed as dist

    log(f"warmup {args.warmup}, timing {args.steps} rounds ({S.workload})")
    dt, launches, kr_ms, every, obj, cons = timed_leg(S.eng, S.rounds, args.steps, args.warmup, S.plan.n_local,
                                                      S.d, barrier, args.event_every, S.flush)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}" if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return dt, launches, kr_ms, every, obj, cons


def per_rank(world, item):
    """item of every rank (rank order), gathered on every rank (host objects)."""
    import torch.distributed as dist

    if world == 1:
        return [item]
    out = [None] * world
    dist.all_gather_object(out, item)
    return out


def exchange_leg(args, S, world, barrier, dev, env, form):
    """N > 1, after the headline leg, on its engine and shards: the same rounds with the exchange in another
    form (`env`: the switches that select it, restored afterwards) -- not `value`.  The scaling run prices
    with real peers over xGMI what the one-GPU rank proxies cannot: the exchange serialised on the engine
    stream where the headline ran it beside the gradient kernel (or the reverse), and the other transport (the
    engine's RCCL sends / receives or its pull transport, DOPT_TRANSPORT)."""
    import torch
    import torch.distributed as dist

    import distributed

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        runner = distributed.DistributedDSGD(S.eng, S.plan, S.n_global, S.n_global * S.m, device=dev)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if not runner._lagged_ok:
        return None
    eta0, b, lam = S.eta0, S.b, S.lam
    try:
        dt, launches, kr_ms, every, obj, cons = timed_leg(
            S.eng, lambda k: runner.run_pipelined(k, eta0, b, lam, lam, 0.0), args.steps, args.warmup,
            S.plan.n_local, S.d, barrier, args.event_every, lambda: runner.run_pipelined(0, eta0, b, lam, lam, 0.0))
    finally:
        if runner.ipc is not None:
            runner.ipc.close()
    tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}" if args.backend == "nccl" else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    return {"value": S.n_global * args.steps / dt, "unit": "worker-iters/s", "ms_per_step": dt / args.steps * 1e3,
            "kernel_avg_ms": kr_ms / launches if launches else None,
            "exchange_beside_gradient": runner.side is not None,
            "transport": "ipc" if runner.ipc is not None else "rccl" if runner.comm is not None else "process group",
            "final_objective": float(obj[-1]), "form": form}


def transport_probe(args, world, dev, barrier, shape, reps=20, warm=3):
    """After the timed legs (N > 1): the round's collectives alone on this node's transport, so a scaling
    run also measures what one GPU per call cannot -- the headline leg's exchange (one all_to_all_single with
    that leg's per-peer row blocks) and C5's all-reduce of 2^20 float64 column sums (8 MiB; the chunk model
    of distributed.rs_chunks_for assumes its cost).  Each timed `reps` times back to back after `warm`,
    bracketed by barrier + sync; the max over ranks."""
    import torch
    import torch.distributed as dist

    send_sizes, recv_sizes, ld, esz = shape
    tdt = torch.float32 if esz == 4 else torch.float64
    on = f"cuda:{dev}" if args.backend == "nccl" else "cpu"
    send = torch.zeros((max(1, sum(send_sizes)), ld), dtype=tdt, device=on)
    recv = torch.zeros((max(1, sum(recv_sizes)), ld), dtype=tdt, device=on)
    sums = torch.zeros(1 << 20, dtype=torch.float64, device=on)

    def timed(fn):
        for _ in range(warm):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        barrier()
        dt = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=on)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item()) * 1e3

    a2a = timed(lambda: dist.all_to_all_single(recv[:sum(recv_sizes)], send[:sum(send_sizes)],
                                               output_split_sizes=recv_sizes, input_split_sizes=send_sizes))
    ar = timed(lambda: dist.all_reduce(sums))
    out_bytes = sum(send_sizes) * ld * esz
    return {"backend": args.backend, "world_size": world, "reps": reps,
            "alltoall_ms": a2a, "alltoall_bytes_out_per_rank": out_bytes,
            "alltoall_GBps_out_per_rank": out_bytes / (a2a * 1e-3) / 1e9 if a2a > 0 else None,
            "allreduce_8MiB_ms": ar,
            "allreduce_busbw_GBps": 2.0 * (world - 1) / world * (8 << 20) / (ar * 1e-3) / 1e9 if ar > 0 else None,
            "note": "the headline leg's exchange and C5's column-sum all-reduce alone, after the timed legs"}


def extra_leg(args, world, rank, dev, barrier, scaling):
    """The C3 leg that is not the headline at N > 1: "weak" (args.workers PER GPU, args.workers x world in
    all; --scaling weak makes it the headline instead) or "strong" (args.strong_workers = 4096 in TOTAL over
    the ranks: the metric's configuration, the headline by default) -- the same random 4-regular graph
    construction and spectral partition; every rank's kernel time and halo bytes are reported."""
    import _dopt

    n_global = args.workers * world if scaling == "weak" else args.strong_workers
    S = setup_leg(args, "c3", n_global, world, rank, dev)
    try:
        dt, launches, kr_ms, every, obj, cons = run_leg(S, args, world, barrier, dev)
        kname = kernel_name()
        bpl = bytes_per_round(S.eng, S.plan.n_local, S.d, S.m, kname)
        avg_ms = kr_ms / launches if launches else float("nan")
        mine = {"rank": rank, "workers": int(S.plan.n_local), "kernel_avg_ms": avg_ms,
                "roofline_frac": bpl / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if launches else None,
                "halo_rows_in": int(S.plan.n_halo),
                "halo_bytes_in_per_round": (S.comm or {}).get("halo_bytes_in_per_round", 0),
                "send_bytes_out_per_round": (S.comm or {}).get("send_bytes_out_per_round", 0),
                "peers": (S.comm or {}).get("peers", [])}
        ranks = per_rank(world, mine)
        return {"value": S.n_global * args.steps / dt, "unit": "worker-iters/s", "n_workers_total": S.n_global,
                "workers_per_gpu": S.n_global / world, "ms_per_step": dt / args.steps * 1e3,
                "scaling": scaling, "kernel": kname, "per_rank": ranks,
                "final_objective": float(obj[-1]), "final_consensus": float(cons[-1]),
                "dtype": "f32" if S.eng.dtype == _dopt.F32 else "f64", "workload": S.workload}
    finally:
        S.eng.close()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-worker":
        return cpu_worker_main(sys.argv[2:])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; N > 1 without an external torch.distributed.run starts "
                         "the N ranks itself.  Default: WORLD_SIZE, or 1")
    ap.add_argument("--steps", type=int, default=300,
                    help="rounds timed (one run: the last round's metrics pass is amortised over them)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workers", type=int, default=4096, help="workers per GPU (C3 weak-scaling leg)")
    ap.add_argument("--strong-workers", type=int, default=4096,
                    help="C3 strong scaling (the headline): workers in total over the N GPUs (the metric's N = 4096)")
    ap.add_argument("--scaling", default="both", choices=["weak", "strong", "both"],
                    help="C3 at N > 1: 'both' (default): value = the strong leg (the metric's 4096 workers in all), "
                         "the weak leg under 'weak'; 'strong' / 'weak': that leg alone, as value")
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--dtype", default="float64", help="iterates and arithmetic (the reference: float64)")
    ap.add_argument("--data-dtype", default="float32",
                    help="shard storage: float32 (default; the synthetic values are exactly float32, so the "
                         "float64 round reads them at half the bytes) or float64")
    ap.add_argument("--batch", type=int, default=0,
                    help="C3 minibatch per worker (0: the full shard, the metric's configuration); b < m "
                         "draws the minibatches on the device (sampling='device', Philox + Floyd)")
    ap.add_argument("--degree", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-procs", type=int, default=0, help="CPU baseline processes (0: the box's CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-alt-exchange", action="store_true",
                    help="N > 1: skip the headline leg's timings with the exchange in the other stream form and "
                         "over the other transport")
    ap.add_argument("--no-secondary", action="store_true",
                    help="N=1: skip the f64-storage / f32 legs, the f(x*) solver and the drop-in trainer leg")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (gloo: 1-GPU rehearsal)")
    ap.add_argument("--timeout", type=float, default=None,
                    help="seconds any collective may take before the job fails (default DOPT_PG_TIMEOUT or 300)")
    ap.add_argument("--launch-limit", type=float, default=1800.0,
                    help="self-launched N > 1 runs: seconds before the whole rank group is ended")
    ap.add_argument("--dry-launch", action="store_true",
                    help="start the ranks and report them (gloo process group only, no GPU work)")
    ap.add_argument("--event-every", type=int, default=0,
                    help="bracket every k-th round kernel with a HIP event pair (0: steps // 10, i.e. 10 "
                         "sampled launches whatever --steps is). A pair costs ~4-30 us of round time")
    ap.add_argument("--phase", action="store_true",
                    help="drive the multi-GPU phase path even on one GPU (measures its per-rank overhead)")
    ap.add_argument("--partition", default="spectral", choices=["spectral", "ranges"],
                    help="C3 at N > 1: workers -> GPUs by graph partition (recursive spectral bisection, "
                         "computed on rank 0 and broadcast) or by contiguous id ranges")
    ap.add_argument("--rs-chunks", type=int, default=0,
                    help="C5 across ranks (or --phase): column chunks of the row-space pass, each chunk's sums "
                         "all-reduced while the next ones stream, each chunk's average update just before the next "
                         "round's pass over it (0: distributed.rs_chunks_for -- 2 across ranks, 1 at world size 1)")
    ap.add_argument("--pcie", action="store_true",
                    help="C3, 1 GPU: after the timed region, hand the same shards over as host buffers "
                         "(dopt_load_shards, the drop-in boundary) and report the PCIe-inclusive rate in a "
                         "'pcie' object (never 'value')")
    ap.add_argument("--config", default="c3", choices=["c3", "c4", "c5"],
                    help="c3 (default, the metric's config); c4: 256x256 torus, 65536 workers total; "
                         "c5: quadratic, d=2^20, m=b=16, 1024 workers total, complete graph")
    args = ap.parse_args()
    if args.timeout is not None:
        os.environ["DOPT_PG_TIMEOUT"] = str(args.timeout)
    else:  # a bench collective never needs minutes: a stuck peer fails the run well inside the driver's limit
        os.environ.setdefault("DOPT_PG_TIMEOUT", "180")

    # ---- the rank layout, decided before anything touches the GPU
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            return launch_ranks(args.gpus, sys.argv[1:], args.launch_limit)
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            log(f"refusing: --gpus {args.gpus} but WORLD_SIZE={world} (the launcher started {world} ranks)")
            return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_launch:
        return dry_launch(args, rank, world, local)

    import torch  # plumbing only: barrier + max-over-ranks (one HIP runtime, loaded first)
    import torch.distributed as dist

    import _dopt
    import distributed

    ndev = torch.cuda.device_count()
    if world > 1 and args.backend == "nccl" and ndev < world:
        log(f"refusing: {world} ranks over RCCL need {world} GPUs, {ndev} visible (--backend gloo rehearses "
            "several ranks on one GPU)")
        return 2
    dev = local % max(1, ndev)
    if world > 1 or args.phase:
        torch.cuda.set_device(dev)
        if world == 1:  # --phase on one GPU: the multi-GPU code path incl. RCCL (one rank)
            distributed.init_process_group(args.backend, store=_solo_store(), rank=0, world_size=1)
        else:
            distributed.init_process_group(args.backend)

    def barrier():
        if world > 1:
            if args.backend == "nccl":
                dist.barrier(device_ids=[dev])  # this rank's GPU, not one guessed from the rank
            else:
                dist.barrier()
        torch.cuda.synchronize(dev)

    # C3: the headline is the strong leg (the metric's 4096 workers in all, over the N GPUs) unless --scaling weak;
    # at N = 1 the two coincide when --workers == --strong-workers (the default 4096)
    weak = args.config == "c3" and args.scaling == "weak"
    n_global = {"c3": args.workers * world if weak else args.strong_workers, "c4": 65536, "c5": 1024}[args.config]
    S = setup_leg(args, args.config, n_global, world, rank, dev)
    eng, plan, d, m, b, lam, eta0, top = S.eng, S.plan, S.d, S.m, S.b, S.lam, S.eta0, S.top
    n = plan.n_local
    setup_s = time.time() - T_START  # launch, process group, graph + partition, shard generation, plan
    dt, launches, kr_ms, every, obj, cons = run_leg(S, args, world, barrier, dev)

    esz = 4 if eng.dtype == _dopt.F32 else 8
    xesz = 4 if eng.data_dtype == _dopt.F32 else 8
    kname = kernel_name()
    full = {"c3": n == 4096, "c4": n == 65536, "c5": n == 1024}[args.config]  # the profiled shapes
    traffic, traffic_src, traffic_run = pmc_traffic(kname, args.config) if full and world == 1 else (None, None, None)
    bytes_per_launch = bytes_per_round(eng, n, d, m, kname)
    avg_s = (kr_ms / launches) * 1e-3 if launches else float("nan")
    achieved = bytes_per_launch / avg_s / 1e9 if launches else None
    value = S.n_global * args.steps / dt
    storage = ("float32 (every value exactly float32-representable; rows widened exactly to float64 as they "
               "are loaded)" if xesz == 4 and esz == 8 else ("float32" if esz == 4 else "float64"))
    mean = S.mean
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "worker-iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f32" if esz == 4 else "f64",
        "data": (f"synthetic (device-generated X~N(0,1){' rounded to float32' if xesz == 4 else ''} + bias column, "
                 "planted-w* labels, " + ("5% flips)" if S.problem == "logistic" else "noise 10)")),
        "config": {"workload": S.workload,
                   "timing": ("pipelined calls: the timed call holds exactly `steps` fused rounds and `steps` "
                              "metric evaluations (its first pass takes the warmup's last metrics, its last "
                              "metrics are taken after the timed region; DESIGN.md section 7)"
                              if S.flush is not None else "one call of `steps` rounds incl. its final metrics pass"),
                   "arithmetic": "float64" if esz == 8 else "float32",
                   "iterates": "float64" if esz == 8 else "float32", "shard_storage": storage,
                   "workers_per_gpu": n, "workers_total": S.n_global, "d": d, "rows_per_worker": m, "batch": b,
                   "topology": top.name, "degree": args.degree if args.config == "c3" else None,
                   "halo_rows_per_gpu": int(plan.n_halo),
                   "parallelism": (f"dp{world}: one graph of {S.n_global} workers, "
                                   f"{'graph-partitioned' if args.config == 'c3' and args.partition == 'spectral' else 'contiguous'} "
                                   f"slices per GPU, "
                                   f"{'all-reduce of the column sums' if mean is not None else 'one all-to-all per round (halo rows + column sums)'}"
                                   f" ({args.backend})") if world > 1
                                  else ("single GPU: the multi-GPU phase path ("
                                        f"{'row-space rounds, all-reduce of the column sums' if mean is not None else 'lagged schedule'}, "
                                        f"{args.backend} world 1)") if args.phase
                                  else ("single GPU: row-space rounds (the pass over the rows, then per-worker "
                                        "and per-column updates; DESIGN.md 6c)") if "k_rs_pass" in kname
                                  else "single GPU: fused round kernel, one launch per round"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "traffic_source_run": traffic_run,
                     "kernel": kname, "kernel_avg_ms": avg_s * 1e3 if launches else None,
                     "kernel_launches_timed": launches, "event_every": every,
                     "bytes_per_launch": bytes_per_launch},
        "final_objective": float(obj[-1]),
        "final_consensus": float(cons[-1]),
    }
    if S.comm is not None:
        out["comm"] = S.comm
    if world > 1:  # every rank's own kernel time and transfer volume
        out["per_rank"] = per_rank(world, {"rank": rank, "workers": int(n),
                                           "kernel_avg_ms": avg_s * 1e3 if launches else None,
                                           "halo_bytes_in_per_round": (S.comm or {}).get("halo_bytes_in_per_round"),
                                           "send_bytes_out_per_round": (S.comm or {}).get("send_bytes_out_per_round")})
    if args.config != "c3":
        out["metric"] = f"worker-iters/sec ({args.config.upper()}, secondary config)"
    secondary = rank == 0 and world == 1 and not args.phase and args.config == "c3" and not args.no_secondary
    if world > 1 and args.config == "c3" and S.flush is not None and not args.no_alt_exchange:
        side = "0" if S.comm.get("exchange_beside_gradient") else "1"
        legs = [("alt_exchange", {"DOPT_LAGGED_SIDE": side},
                 "the exchange on the side stream beside the gradient kernel (DOPT_LAGGED_SIDE=1)" if side == "1"
                 else "the exchange serialised on the engine stream (DOPT_LAGGED_SIDE=0)")]
        # the other transport: RCCL where the headline pulled, the pull transport where it used RCCL or the
        # process group (over gloo too: the one-GPU rehearsal's ranks share the card, as the pull tests do)
        if S.comm.get("transport") == "ipc":
            legs.append(("alt_transport", {"DOPT_TRANSPORT": "rccl"},
                         "the engine's RCCL transport: grouped ncclSend / ncclRecv (DOPT_TRANSPORT=rccl)"))
        else:
            legs.append(("alt_transport", {"DOPT_TRANSPORT": "ipc"},
                         "the pull transport: k_pull reads the peers' send slots through IPC handles "
                         "(DOPT_TRANSPORT=ipc)"))
        for key, env, form in legs:
            log(f"headline leg again, {form} (A/B with real peers)")
            try:  # diagnostic only: a failure here must not cost the line its value
                out[key] = r = exchange_leg(args, S, world, barrier, dev, env, form)
                if r is not None:  # every leg starts from zero iterates: the same bits whatever the transport
                    r["final_objective_matches_value"] = r["final_objective"] == out["final_objective"]
            except Exception as e:  # noqa: BLE001
                log(f"{key} failed: {e!r}")
                out[key] = {"error": repr(e)[:300]}
    if secondary and b == m:
        log("f(x*): device L-BFGS")
        out["suboptimality"] = suboptimality(eng, lam, float(obj[-1]))
        import contextlib

        with contextlib.redirect_stdout(sys.stderr):  # the trainers' reference prints: stdout keeps the one line
            log("drop-in trainer leg (legacy RNG stream)")
            out["dropin"] = dropin_leg(eng, n, d, m, lam, eta0)
            log("drop-in trainer leg, b = 16 (minibatch indices from the legacy stream)")
            out["dropin"]["b16"] = dropin_leg(eng, n, d, m, lam, eta0, batch=16)
    if args.pcie and world == 1 and args.config == "c3":
        out["pcie"] = pcie_leg(eng, top, n, d, m, b, lam, eta0, args.steps, dt)
    eng.close()
    if args.config == "c3" and world > 1 and args.scaling == "both":
        log(f"weak-scaling leg: {args.workers} workers per rank, {args.workers * world} over {world} ranks")
        try:  # secondary: a failure here must not cost the line its value (every rank raises alike)
            out["weak"] = extra_leg(args, world, rank, dev, barrier, "weak")
        except Exception as e:  # noqa: BLE001
            log(f"weak leg failed: {e!r}")
            out["weak"] = {"error": repr(e)[:300]}
    if world > 1 and getattr(S, "exchange_shape", None) is not None:
        log("transport probe: the headline leg's exchange and an 8 MiB all-reduce alone")
        try:  # diagnostic only, as above
            out["transport_probe"] = transport_probe(args, world, dev, barrier, S.exchange_shape)
        except Exception as e:  # noqa: BLE001
            log(f"transport_probe failed: {e!r}")
            out["transport_probe"] = {"error": repr(e)[:300]}
    if secondary and b == m:
        legs = {}
        if not (esz == 8 and xesz == 8):
            log("leg: float64 storage")
            legs["f64_storage"] = secondary_leg(dev, "float64", None, top, n, d, m, args.steps, args.warmup, lam,
                                                eta0, barrier, args.event_every)
        if esz == 8:
            log("leg: float32 engine")
            legs["f32"] = secondary_leg(dev, "float32", None, top, n, d, m, args.steps, args.warmup, lam, eta0,
                                        barrier, args.event_every)
        out["legs"] = legs
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c3":
        log("cpu baseline")
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.cpu_procs or None)
    out["setup_s"] = setup_s  # rank 0: process start -> the headline leg's warmup
    out["wall_s"] = time.time() - T_START  # rank 0: process start -> this line
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1 or args.phase:
        distributed.close_comms()  # the engine's RCCL communicators, before the process group
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
