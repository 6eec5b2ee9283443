"""The multi-GPU code path on one GPU: 2 ranks (gloo transport, both contexts on
device 0) run the phase API with the halo plan; the iterates must equal the
single-context fused run bit for bit, the metrics to rtol 1e-12 (reordered sums).
Full-shard CSR runs take the lagged schedule (distributed.py: _run_lagged; T = 1 and 2
are its edge cases), DOPT_LAGGED=0 the serial one, the complete graph the serial one."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, D, M, T = 64, 100, 32, 6


def _engine(dtype):
    """'float64/x32': float64 arithmetic over float32-stored rows (bench.py's default)."""
    import _dopt

    if dtype == "float64/x32":
        return _dopt.Engine(0, "float64", data_dtype="float32")
    return _dopt.Engine(0, dtype)


_RDV_N = 0


def _rdv(tmp_path):
    """init_method of a multi-process test: a FileStore in the test's own tmp_path.  No port is picked
    before the ranks start, so nothing on the box can take it in between (a port released
    by a pre-pick and taken before rank 0's TCPStore bound it -> EADDRINUSE)."""
    global _RDV_N
    _RDV_N += 1
    return f"file://{tmp_path}/pg_store_{os.getpid()}_{_RDV_N}"


def _rank_main(rank, world, rdv, dtype, out, mean=False, T=T, lagged="1", N=N, D=D, M=M, backend="gloo"):
    import torch  # noqa: F401  (one HIP runtime, loaded before libdopt)
    import torch.distributed as dist

    import _dopt
    import distributed as Dm
    import topology as TP

    # "1-noside": the lagged schedule on one stream; "1-pg": the exchange through the process group's
    # all-to-all-v instead of the engine's own RCCL communicator (dopt_lagged_exchange, the default);
    # "1-ipc": the engine's pull transport (dopt_lagged_ipc_*: peers' send slots read through IPC handles)
    opts = lagged.split("-")
    side = "0" if "noside" in opts else "1"
    transport = "pg" if "pg" in opts else "ipc" if "ipc" in opts else "rccl"
    lagged = opts[0]
    os.environ.update(DOPT_LAGGED=lagged, DOPT_LAGGED_SIDE=side, DOPT_TRANSPORT=transport,
                      DOPT_FORCE_COLLECTIVES="1" if backend == "nccl" else "0")
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method=rdv, rank=rank, world_size=world)
    top = _topo(mean, N, world if os.environ.get("DOPT_TEST_PARTITION") == "1" else 0)
    plan = Dm.build_plan(top, world, rank)
    if os.environ.get("DOPT_TEST_SELF_HALO") == "1":  # world 1: a third of the rows through the exchange
        plan = _self_halo_plan(top)
    eng = _engine(dtype)
    eng.generate_shards("logistic", plan.n_local, D, M, seed=9, first_worker=plan.lo)
    B = int(os.environ.get("DOPT_TEST_BATCH", M))  # B < M: device-drawn minibatches
    if B < M:
        eng.set_sampler("device", seed=31, first_worker=plan.lo)
    uni = top.uniform_offdiag() if mean is True else None
    run = Dm.DistributedDSGD(eng, plan, N, N * M, device=0,
                             mean=None if uni is None else (uni[0], uni[1][plan.lo:plan.hi]))
    info = {"interior": eng.phase_interior_count(), "n_local": plan.n_local, "n_halo": plan.n_halo,
            "send_sizes": list(run.layout.send_sizes), "recv_sizes": list(run.layout.recv_sizes),
            "ks": run.layout.ks, "side": run.side is not None, "collective": bool(run.exchange.collective),
            "native": run.comm is not None, "ipc": run.ipc is not None, "one_node": Dm._one_node(None)}
    np.save(os.path.join(out, f"info{rank}.npy"), np.array([repr(info)]))
    which = os.environ.get("DOPT_TEST_METRICS", "both")
    if os.environ.get("DOPT_TEST_PIPE") == "1":  # a chain of pipelined calls covering T rounds, then the tail
        parts, t = [], 0
        for k in [2, 1, 3, 1, T]:
            k = min(k, T - t)
            parts.append(run.run_pipelined(k, 0.05, B, 1e-3, 1e-3, 0.25, t0=t, objective=which != "cons",
                                           consensus=which != "obj"))
            t += k
        parts.append(run.run_pipelined(0, 0.05, B, 1e-3, 1e-3, 0.25, objective=which != "cons",
                                       consensus=which != "obj"))
        obj = None if which == "cons" else np.concatenate([p[0] for p in parts])
        cons = None if which == "obj" else np.concatenate([p[1] for p in parts])
    elif os.environ.get("DOPT_TEST_CHAINS"):  # several closed chains in a row on one runner (T rounds each)
        parts = [run.run(T, 0.05, B, 1e-3, 1e-3, 0.25) for _ in range(int(os.environ["DOPT_TEST_CHAINS"]))]
        obj, cons = np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])
    else:
        obj, cons = run.run(T, 0.05, B, 1e-3, 1e-3, 0.25, objective=which != "cons", consensus=which != "obj")
    obj = np.zeros(0) if obj is None else obj
    cons = np.zeros(0) if cons is None else cons
    x = run.gather_models()
    if rank == 0:
        np.savez(os.path.join(out, "dist.npz"), obj=obj, cons=cons, x=x)
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype,mean,T,lagged,world", [("float64", False, T, "1", 2), ("float32", False, T, "1", 2),
                                                      ("float64", True, T, "1", 2), ("float64", False, 1, "1", 2),
                                                      ("float64", False, 2, "1", 2), ("float32", False, T, "0", 2),
                                                      ("float64", False, 3, "1", 3),
                                                      ("float64/x32", False, T, "1", 2),
                                                      ("float64/x32", False, T, "0", 2),
                                                      ("float64/x32", True, T, "1", 2),
                                                      ("float64/x32", "csr", T, "1", 2),
                                                      ("float64/x32", False, T, "1-noside", 2),
                                                      ("float64", "torus", T, "1", 3),
                                                      ("float32", "torus", T, "1-noside", 3),
                                                      ("float64/x32", "torus", T, "1", 2),
                                                      ("float32", "csr", T, "0", 2)])
def test_ranks_match_single_context(tmp_path, dtype, mean, T, lagged, world):
    import torch.multiprocessing as mp

    mp.start_processes(_rank_main, args=(world, _rdv(tmp_path), dtype, str(tmp_path), mean, T, lagged), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == T
    _compare_single(got, dtype, mean, T)


def _topo(mean, n, parts=0):
    """The test graph (mean: the complete graph, mixed through the column sums when True and as CSR
    rows longer than the mix kernels' register-held entries when "csr"; "torus": the sqrt(n) x sqrt(n)
    torus of trainer.py:99-108, row-major ids, so contiguous slices are strips of torus rows -- config
    C4's placement); with parts > 0 relabelled by the spectral partition for that many ranks (bench.py's
    C3 placement)."""
    import distributed as Dm
    import topology as TP

    if mean == "torus":
        return TP.grid(n)
    if mean:  # True: column-sum mixing; "csr": the complete graph as CSR rows of n entries
        return TP.fully_connected(n)
    top = TP.random_regular(n, 4, seed=2)
    if parts:
        top = TP.relabel(top, Dm.partition_order(Dm.graph_partition(top, parts)))
    return top


def _compare_single(got, dtype, mean, T, N=N, D=D, M=M, exact=True, parts=0):
    import _dopt

    eng = _engine(dtype)
    eng.generate_shards("logistic", N, D, M, seed=9)
    B = int(os.environ.get("DOPT_TEST_BATCH", M))
    if B < M:
        eng.set_sampler("device", seed=31)
    top = _topo(mean, N, parts)
    if mean is True:
        eng.set_mixing_mean(*top.uniform_offdiag())
    else:
        eng.set_topology(top.row_ptr, top.col, top.w)
    obj, cons, _ = eng.run_dsgd(T, 0.05, B, 1e-3, 1e-3, 0.25)
    x = eng.get_models()
    eng.close()
    if mean is True or not exact:  # column sums / split partial dots reduced per rank then across ranks
        np.testing.assert_allclose(got["x"], x, rtol=1e-12, atol=1e-15)
    else:
        np.testing.assert_array_equal(got["x"], x)
    if len(got["obj"]):
        np.testing.assert_allclose(got["obj"], obj, rtol=1e-12 if dtype != "float32" else 1e-6)
    if len(got["cons"]):
        np.testing.assert_allclose(got["cons"], cons, rtol=1e-12 if dtype != "float32" else 1e-5)


def _self_halo_plan(top, every=3):
    """A world-1 halo plan whose exchange is not empty: every `every`-th worker's row is sent to the
    rank itself, and the OTHER workers' CSR entries of it read that copy from the halo buffer (same
    entry order and weights, so the iterates are bitwise one context's) -- on RCCL world 1 with the
    collectives forced, the mix then depends on rows the all-to-all moved."""
    import distributed as Dm

    n = top.n
    S = np.arange(0, n, every)
    pos = np.full(n, -1, np.int64)
    pos[S] = np.arange(len(S))
    rows = np.repeat(np.arange(n), np.diff(top.row_ptr))
    col = top.col.astype(np.int64).copy()
    via = (pos[col] >= 0) & (col != rows)
    col[via] = n + pos[col[via]]
    return Dm.HaloPlan(0, 1, np.array([0, n]), 0, n, S.astype(np.int64), np.array([0, len(S)]), S.astype(np.int32),
                       np.array([0, len(S)]), top.row_ptr.astype(np.int64), col.astype(np.int32), top.w.copy())


def _info(tmp_path, world):
    import ast

    return [ast.literal_eval(str(np.load(tmp_path / f"info{r}.npy")[0])) for r in range(world)]


@pytest.mark.parametrize("world,dtype,d,m,lagged", [(2, "float64", 100, 32, "1"), (8, "float64", 100, 32, "1"),
                                                    (8, "float64/x32", 1024, 16, "1"),
                                                    (8, "float64/x32", 1024, 16, "1-ipc")])
def test_torus_strips_ranks_match_single_context(tmp_path, monkeypatch, world, dtype, d, m, lagged):
    """config C4's split -- a torus (trainer.py:99-108) in strips of torus rows, one
    strip per rank (64 x 64 torus: strips of 32 rows at 2 ranks, 8 at 8 ranks, >= 256 workers per rank so
    every context launches the headline's kernel instance) -- as a chain of pipelined calls through the
    device kernels: the strip interiors stepped inside the gradient kernel (dopt_phase_interior_count =
    64 x (rows - 2)), the two boundary rows mixed in k_mixcs from the halo rows, the column sums riding
    the all-to-all to all 7 peers (or, "1-ipc", pulled by the pull transport).  Iterates bitwise one
    context's, history rtol 1e-12."""
    import torch.multiprocessing as mp

    n, t = 4096, 7
    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(world, _rdv(tmp_path), dtype, str(tmp_path), "torus", t, lagged, n, d, m),
                       nprocs=world, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == t
    info = _info(tmp_path, world)
    assert all(it["ipc"] == ("ipc" in lagged) for it in info)
    rows = 64 // world
    for r, it in enumerate(info):
        assert it["n_local"] == 64 * rows and it["n_halo"] == 2 * 64, it
        assert it["interior"] == 64 * (rows - 2), it
        assert it["ks"] > 0 and all(it["send_sizes"][p] > 0 for p in range(world) if p != r), it
        assert it["side"], it
    _compare_single(got, dtype, "torus", t, n, d, m)


def _trainer_rank(rank, world, rdv, out):
    import json

    import torch  # noqa: F401
    import torch.distributed as dist

    import data as odata
    from trainer import CentralizedTrainer, DecentralizedTrainer
    from worker import Worker

    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(G, "traj_c2.json")))
    z = np.load(os.path.join(G, "traj_c2.npz"))
    cfg = dict(meta["config"])
    shards, Xf, yf = odata.generate(cfg, order=z["order"])
    T = 300
    res = {}
    for j, label in enumerate(meta["labels"]):
        np.random.set_state(("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0))
        ws = [Worker(i, {"X": X, "y": y}, cfg["local_batch_size"], Xf.shape[1], cfg) for i, (X, y) in enumerate(shards)]
        if label == "Centralized":
            tr = CentralizedTrainer(ws, Xf.shape[1], cfg)
        else:
            topo = {"D-SGD (Ring)": "ring", "D-SGD (Fully Connected)": "fully_connected"}[label]
            tr = DecentralizedTrainer(ws, topo, Xf.shape[1], cfg)
        hist, xf = tr.run(T, Xf, yf, meta["f_opt"])
        res[f"L{j}_objective"] = np.asarray(hist["objective"])
        if "consensus_error" in hist:
            res[f"L{j}_consensus"] = np.asarray(hist["consensus_error"])
        res[f"L{j}_pos"] = np.int64(np.random.get_state()[2])
    if rank == 0:
        np.savez(os.path.join(out, "trainers.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_trainers_multiprocess_match_reference(tmp_path, world):
    """DecentralizedTrainer / CentralizedTrainer under a torch.distributed job of 2 and 8 ranks (each
    rank holds its slice of the 10 workers: 1-2 at 8 ranks) reproduce the reference's C2 trajectories."""
    import json

    import torch.multiprocessing as mp

    mp.start_processes(_trainer_rank, args=(world, _rdv(tmp_path), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(tmp_path / "trainers.npz")
    G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(G, "traj_c2.json")))
    z = np.load(os.path.join(G, "traj_c2.npz"))
    for j, label in enumerate(meta["labels"]):
        np.testing.assert_allclose(got[f"L{j}_objective"], z[f"L{j}_objective"][:300], rtol=1e-9)
        if label != "Centralized":
            np.testing.assert_allclose(got[f"L{j}_consensus"], z[f"L{j}_consensus"][:300], rtol=1e-9)


@pytest.mark.parametrize("dtype,mean,lagged", [("float64", False, "1"), ("float32", False, "1"),
                                               ("float64", True, "1"), ("float64", False, "0"),
                                               ("float64/x32", False, "1")])
def test_rccl_one_rank_matches_single_context(tmp_path, dtype, mean, lagged):
    """The RCCL code path on the one GPU this pool gives: backend "nccl", world 1, with the
    all-reduces forced (DOPT_FORCE_COLLECTIVES=1) -- async all_reduce on the engine
    stream, work.wait() ordering, object broadcast; the exchange itself has no peer here."""
    import torch.multiprocessing as mp

    mp.start_processes(_rank_main, args=(1, _rdv(tmp_path), dtype, str(tmp_path), mean, T, lagged, N, D, M, "nccl"),
                       nprocs=1, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    _compare_single(got, dtype, mean, T, exact=not mean)


@pytest.mark.parametrize("world", [2, 4])
def test_partitioned_graph_ranks_match_single_context(tmp_path, monkeypatch, world):
    """bench.py's placement: the random regular graph relabelled by the spectral partition,
    2 and 4 ranks (gloo) vs one context on the same relabelled graph -- bitwise iterates."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_PARTITION", "1")
    mp.start_processes(_rank_main, args=(world, _rdv(tmp_path), "float64", str(tmp_path), False, 5, "1"),
                       nprocs=world, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    _compare_single(got, "float64", False, 5, parts=world)


def test_eight_ranks_match_single_context(tmp_path, monkeypatch):
    """the driver's SCALE shape on the one GPU -- 8 gloo ranks x 256 workers of the
    spectrally partitioned random 4-regular graph (every rank exchanging halo rows and column sums
    with all 7 peers each round), as a chain of pipelined calls: bitwise one context's iterates."""
    import torch.multiprocessing as mp

    n, d, m, t = 2048, 100, 32, 6
    monkeypatch.setenv("DOPT_TEST_PARTITION", "1")
    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(8, _rdv(tmp_path), "float64/x32", str(tmp_path), False, t, "1", n, d, m),
                       nprocs=8, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == t
    _compare_single(got, "float64/x32", False, t, n, d, m, parts=8)


@pytest.mark.parametrize("world", [2, 4])
def test_strong_split_bench_shape_matches_single_context(tmp_path, monkeypatch, world):
    """bench.py's strong-scaling leg in miniature: a FIXED total of workers (1024, d = 1024, the
    headline's float64 arithmetic over float32 rows) split over 2 and 4 ranks by the spectral
    partition, timed as a chain of pipelined calls -- bitwise one context's iterates, history
    rtol 1e-12.  Every rank keeps >= 256 workers, so it launches the same
    round-kernel instance as the single context (the headline's: software-pipelined row loop,
    paired row-dot butterfly); below 256 workers a context takes the few-worker kernel, whose
    row dots reduce in another order."""
    import torch.multiprocessing as mp

    n, d, m, t = 1024, 1024, 16, 9
    monkeypatch.setenv("DOPT_TEST_PARTITION", "1")
    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(world, _rdv(tmp_path), "float64/x32", str(tmp_path), False, t, "1", n, d, m),
                       nprocs=world, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == t
    _compare_single(got, "float64/x32", False, t, n, d, m, parts=world)


@pytest.mark.parametrize("lagged", ["1", "0", "1-ipc"])
def test_device_sampler_ranks_match_single_context(tmp_path, monkeypatch, lagged):
    """sampling='device' across ranks: worker i's minibatch of round t depends only on
    (seed, t, global id), so 3 ranks (phase path, lagged or serial) reproduce one context's
    device-sampled run bit for bit."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_BATCH", "5")
    mp.start_processes(_rank_main, args=(3, _rdv(tmp_path), "float64", str(tmp_path), False, 5, lagged), nprocs=3,
                       join=True, start_method="spawn")
    _compare_single(np.load(tmp_path / "dist.npz"), "float64", False, 5)


@pytest.mark.parametrize("which", ["obj", "cons"])
def test_lagged_schedule_single_metric(tmp_path, monkeypatch, which):
    """The lagged schedule with only the objective or only the consensus recorded."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_METRICS", which)
    mp.start_processes(_rank_main, args=(2, _rdv(tmp_path), "float64", str(tmp_path), False, 5, "1"), nprocs=2,
                       join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == (5 if which == "obj" else 0) and len(got["cons"]) == (5 if which == "cons" else 0)
    _compare_single(got, "float64", False, 5)


@pytest.mark.parametrize("mean", [True, False])
def test_column_blocked_ranks_match_single_context(tmp_path, mean):
    """Rows too long for the row-resident kernel (fp64, d = 2100 > 2048: the column-blocked
    k_split_* path of config C5) on 2 ranks: complete graph (all-reduced column sums) and
    ring (halo rows), against one context."""
    import torch.multiprocessing as mp

    n, d, m, t = 16, 2100, 8, 4
    mp.start_processes(_rank_main, args=(2, _rdv(tmp_path), "float64", str(tmp_path), mean, t, "1", n, d, m),
                       nprocs=2, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    _compare_single(got, "float64", mean, t, n, d, m, exact=False)


@pytest.mark.parametrize("world,backend,dtype", [(2, "gloo", "float64"), (3, "gloo", "float64/x32"),
                                                 (1, "nccl", "float64")])
def test_pipelined_chain_matches_single_context(tmp_path, monkeypatch, world, backend, dtype):
    """DistributedDSGD.run_pipelined (bench.py's multi-GPU timing): a chain of calls of 2, 1,
    3, 1 and the rest of 9 rounds, then the closing call, returns exactly the history of one
    run and ends on the same iterates as one context (bitwise)."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(world, _rdv(tmp_path), dtype, str(tmp_path), False, 9, "1", N, D, M, backend),
                       nprocs=world, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == 9
    _compare_single(got, dtype, False, 9)


def _ckpt_rank(rank, world, rdv, out):
    import json

    import torch  # noqa: F401
    import torch.distributed as dist

    import data as odata
    from trainer import CentralizedTrainer, DecentralizedTrainer
    from worker import Worker

    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(G, "traj_c2.json")))
    z = np.load(os.path.join(G, "traj_c2.npz"))
    shards, Xf, yf = odata.generate(dict(meta["config"]), order=z["order"])
    res = {}
    for label in ("D-SGD (Ring)", "Centralized"):
        j = meta["labels"].index(label)
        st = ("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0)
        ck = os.path.join(out, f"ck_{j}.npz")  # every rank names the same file; rank 0 writes it

        def make(cfg):
            ws = [Worker(i, {"X": X, "y": y}, cfg["local_batch_size"], Xf.shape[1], cfg)
                  for i, (X, y) in enumerate(shards)]
            if label == "Centralized":
                return CentralizedTrainer(ws, Xf.shape[1], cfg)
            return DecentralizedTrainer(ws, "ring", Xf.shape[1], cfg)

        cfg = dict(meta["config"])
        np.random.set_state(st)
        make(dict(cfg, checkpoint_path=ck, checkpoint_every=20)).run(20, Xf, yf, meta["f_opt"])
        dist.barrier()  # the file is written before any rank resumes from it
        np.random.seed(99)
        tr = make(dict(cfg, resume_from=ck))
        h, x = tr.run(50, Xf, yf, meta["f_opt"])
        res[f"L{j}_objective"] = np.asarray(h["objective"])
        if "consensus_error" in h:
            res[f"L{j}_consensus"] = np.asarray(h["consensus_error"])
        res[f"L{j}_pos"] = np.int64(np.random.get_state()[2])
        res[f"L{j}_x"] = np.asarray(x)
    if rank == 0:
        np.savez(os.path.join(out, "ckpt.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def test_trainers_multiprocess_checkpoint_resume(tmp_path):
    """Checkpoint / resume under a 2-rank job: rank 0 writes the file after 20 rounds (the
    gathered iterates), both ranks resume from it; the 50-round history equals the
    reference's C2 trajectory (rtol 1e-9), and every rank ends on the same RNG position as
    one uninterrupted process would."""
    import json

    import torch.multiprocessing as mp

    mp.start_processes(_ckpt_rank, args=(2, _rdv(tmp_path), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    got = np.load(tmp_path / "ckpt.npz")
    G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    meta = json.load(open(os.path.join(G, "traj_c2.json")))
    z = np.load(os.path.join(G, "traj_c2.npz"))
    for label in ("D-SGD (Ring)", "Centralized"):
        j = meta["labels"].index(label)
        np.testing.assert_allclose(got[f"L{j}_objective"], z[f"L{j}_objective"][:50], rtol=1e-9)
        if label != "Centralized":
            np.testing.assert_allclose(got[f"L{j}_consensus"], z[f"L{j}_consensus"][:50], rtol=1e-9)


def _rccl_self_exchange(rank, world, rdv, out):
    """HaloExchange's all_to_all_single on an RCCL communicator of one rank, with rows sent to
    itself (a hand-made plan: rows 0..k-1 out, k halo rows in) on the engine-like side stream."""
    import torch
    import torch.distributed as dist

    import distributed as Dm

    os.environ.update(DOPT_FORCE_COLLECTIVES="1")
    torch.cuda.set_device(0)
    Dm.init_process_group("nccl", init_method=rdv, rank=0, world_size=1)
    k, ld = 37, 130
    plan = Dm.HaloPlan(0, 1, np.array([0, 64]), 0, 64, np.arange(k), np.array([0, k]), np.arange(k, dtype=np.int32),
                       np.array([0, k]), None, None, None)
    send = torch.arange((k + 3) * ld, dtype=torch.float64, device="cuda").reshape(k + 3, ld)
    halo = torch.full((k + 3, ld), -1.0, dtype=torch.float64, device="cuda")
    ex = Dm.HaloExchange(plan, send, halo, device_comm=True)
    assert ex.collective and ex.send_sizes == [k] and ex.recv_sizes == [k]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ex.finish(ex.start())
        ok = bool(torch.equal(halo[:k], send[:k])) and bool((halo[k:] == -1.0).all())
    s.synchronize()
    np.save(os.path.join(out, "ok.npy"), np.array([ok]))
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype,lagged", [("float64", "1"), ("float64/x32", "1"), ("float64", "1-noside"),
                                          ("float32", "1"), ("float64/x32", "1-noside"),
                                          ("float64", "1-pg"), ("float64/x32", "1-pg"), ("float32", "1-pg"),
                                          ("float64", "1-noside-pg")])
def test_rccl_one_rank_self_exchange_matches_single_context(tmp_path, monkeypatch, dtype, lagged):
    """the RCCL path at world 1 (collectives forced) with an exchange that moves data -- a
    third of the workers' rows and the rank's own column sums go through the all-to-all to itself (a
    self block), and the mix reads them back from the halo buffer.  With the side stream (k_mixcs_final
    and the exchange on a second stream, ProcessGroupNCCL's stream sync and work.wait() ordering them)
    or on one stream, as a pipelined chain: iterates bitwise one context's, history rtol 1e-12 -- a
    missing dependency would mix stale halo rows or column sums.  The exchange goes through the engine's
    own RCCL communicator (dopt_lagged_exchange: sends and receives on the side stream) or, "-pg", through
    the process group's all-to-all-v."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_SELF_HALO", "1")
    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(1, _rdv(tmp_path), dtype, str(tmp_path), False, 9, lagged, N, D, M, "nccl"),
                       nprocs=1, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == 9
    it = _info(tmp_path, 1)[0]
    ks = 2 if dtype == "float32" else 1
    assert it["collective"] and it["ks"] == ks and it["send_sizes"] == [len(range(0, N, 3)) + ks], it
    assert it["side"] == ("noside" not in lagged), it
    assert it["native"] == ("pg" not in lagged), it
    assert it["interior"] < N - len(range(0, N, 3)), it  # readers of the halo copies are not interior
    _compare_single(got, dtype, False, 9)


@pytest.mark.parametrize("dtype,mean,world,lagged,pipe", [("float64/x32", False, 2, "1-ipc", False),
                                                         ("float64", False, 3, "1-ipc", True),
                                                         ("float32", False, 2, "1-ipc-noside", True),
                                                         ("float64", False, 2, "1-ipc", False),
                                                         ("float64/x32", "torus", 4, "1-ipc", True)])
def test_pull_transport_matches_single_context(tmp_path, monkeypatch, dtype, mean, world, lagged, pipe):
    """DOPT_TRANSPORT=ipc (ABI 9): 2-4 processes on the one GPU, each pulling its halo rows and the peers'
    column sums out of the peers' send slots through IPC handles (k_pull after the peers' interprocess
    events, the slots alternating by round parity) -- real cross-process device traffic, no RCCL.  Side
    stream or one stream, single calls and pipelined chains (T = 1 included): iterates bitwise one
    context's, history rtol 1e-12.  A pull that ran before the peer's rows were written, or a slot reused
    while a peer still read it, would mix stale rows."""
    import torch.multiprocessing as mp

    if pipe:
        monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    for T_ in ((1, 7) if not pipe and world == 2 and dtype == "float64" else (7,)):
        sub = tmp_path / f"T{T_}"
        sub.mkdir()
        mp.start_processes(_rank_main, args=(world, _rdv(sub), dtype, str(sub), mean, T_, lagged), nprocs=world,
                           join=True, start_method="spawn")
        got = np.load(sub / "dist.npz")
        assert len(got["obj"]) == len(got["cons"]) == T_
        for r, it in enumerate(_info(sub, world)):
            assert it["ipc"] and not it["native"] and it["side"] == ("noside" not in lagged), it
        _compare_single(got, dtype, mean, T_)


@pytest.mark.parametrize("world", [2, 4])
def test_pull_transport_successive_chains(tmp_path, monkeypatch, world):
    """Three closed chains in a row on one runner (bench.py's warmup, then timed rounds): the pull transport's
    records are numbered across chains, so a rank entering the next chain never takes a peer's counter of the
    previous one for the new round.  Iterates and history bitwise those of the same schedule over the host
    transport."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_CHAINS", "3")
    got = {}
    for lagged in ("1", "1-ipc"):
        sub = tmp_path / lagged
        sub.mkdir()
        mp.start_processes(_rank_main, args=(world, _rdv(sub), "float64/x32", str(sub), False, 4, lagged), nprocs=world,
                           join=True, start_method="spawn")
        got[lagged] = np.load(sub / "dist.npz")
        assert all(it["ipc"] == (lagged == "1-ipc") for it in _info(sub, world))
    assert len(got["1"]["obj"]) == 12
    for k in ("x", "obj", "cons"):
        assert np.array_equal(got["1"][k], got["1-ipc"][k]), k


def test_pull_transport_eight_ranks_match_single_context(tmp_path, monkeypatch):
    """The pull transport at the SCALE run's rank count: 8 processes x 256 workers of the spectrally
    partitioned random 4-regular graph, every rank pulling from all 7 peers each round, pipelined chain."""
    import torch.multiprocessing as mp

    n, d, m, t = 2048, 100, 32, 6
    monkeypatch.setenv("DOPT_TEST_PARTITION", "1")
    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(8, _rdv(tmp_path), "float64/x32", str(tmp_path), False, t, "1-ipc", n, d, m),
                       nprocs=8, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    assert len(got["obj"]) == len(got["cons"]) == t
    assert all(it["ipc"] for it in _info(tmp_path, 8))
    _compare_single(got, "float64/x32", False, t, n, d, m, parts=8)


@pytest.mark.parametrize("dtype,lagged", [("float64/x32", "1-ipc"), ("float64", "1-ipc-noside")])
def test_pull_transport_one_rank_self_block(tmp_path, monkeypatch, dtype, lagged):
    """The pull transport at world 1 with a self block (collectives forced, as tools/rank_proxy.py runs a
    rank): a third of the rows and the rank's own sums pulled from its own slot into its halo."""
    import torch.multiprocessing as mp

    monkeypatch.setenv("DOPT_TEST_SELF_HALO", "1")
    monkeypatch.setenv("DOPT_TEST_PIPE", "1")
    mp.start_processes(_rank_main, args=(1, _rdv(tmp_path), dtype, str(tmp_path), False, 9, lagged, N, D, M, "nccl"),
                       nprocs=1, join=True, start_method="spawn")
    got = np.load(tmp_path / "dist.npz")
    it = _info(tmp_path, 1)[0]
    assert it["ipc"] and it["ks"] > 0 and it["one_node"], it  # (the setup's object collectives over RCCL)
    _compare_single(got, dtype, False, 9)


def _pull_stalled(rank, world, rdv, out):
    """Rank 1 sets the pull transport up and then never runs a round: rank 0's first exchange must fail
    with CollectiveError once DOPT_PG_TIMEOUT has passed."""
    import time

    import torch  # noqa: F401
    import torch.distributed as dist

    import distributed as Dm

    os.environ.update(DOPT_TRANSPORT="ipc", DOPT_PG_TIMEOUT="5")
    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    top = _topo(False, N)
    plan = Dm.build_plan(top, world, rank)
    eng = _engine("float64")
    eng.generate_shards("logistic", plan.n_local, D, M, seed=9, first_worker=plan.lo)
    run = Dm.DistributedDSGD(eng, plan, N, N * M, device=0)
    msg = ""
    if rank == 0:
        t0 = time.monotonic()
        try:
            run.run(3, 0.05, M, 1e-3, 1e-3, 0.25)
        except Dm.CollectiveError as e:
            msg = f"{time.monotonic() - t0:.1f} {e}"
        np.save(os.path.join(out, "stalled.npy"), np.array([msg]))
    dist.barrier()  # (gloo: rank 1 waits here the whole time, its context idle)
    eng.close()
    dist.destroy_process_group()


def test_pull_transport_stalled_peer_is_bounded(tmp_path):
    import torch.multiprocessing as mp

    mp.start_processes(_pull_stalled, args=(2, _rdv(tmp_path), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    msg = str(np.load(tmp_path / "stalled.npy")[0])
    assert "published" in msg and "peer 1" in msg, msg
    assert float(msg.split()[0]) < 30.0, msg


def test_rccl_alltoall_halo_exchange_one_rank(tmp_path):
    """The device halo exchange is one RCCL all_to_all_single with the plan's split sizes; at world
    1 it runs with rows sent to the rank itself, which copies them (the layout over several ranks:
    tests/test_distributed_cpu.py::test_alltoall_halo_layout, same call over gloo)."""
    import torch.multiprocessing as mp

    mp.start_processes(_rccl_self_exchange, args=(1, _rdv(tmp_path), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    assert np.load(tmp_path / "ok.npy")[0]


def _transport_errors(rank, world, rdv, out):
    """The engine-driven transport's argument and state checks (ABI 7-8), on a world-1 communicator."""
    import torch

    import _dopt

    torch.cuda.set_device(0)
    res = {"library": _dopt.comm_library()}
    eng = _dopt.Engine(0, "float64")
    eng.generate_shards("logistic", 8, 16, 4, seed=3)
    comm = _dopt.Comm(1, 0, 0, _dopt.comm_unique_id())
    res["library"] = _dopt.comm_library()

    def err(f):
        try:
            f()
        except (ValueError, RuntimeError) as e:
            return type(e).__name__ + ": " + str(e)
        return None

    res["no_transport"] = err(eng.lagged_exchange)
    res["no_buffers"] = err(lambda: eng.lagged_transport(comm, [4], [4]))  # before dopt_set_halo
    res["bad_shape"] = err(lambda: eng.lagged_transport(comm, [1, 1], [1, 1]))
    send = torch.zeros((3, 16), dtype=torch.float64, device="cuda")
    halo = torch.zeros((3, 16), dtype=torch.float64, device="cuda")
    eng.set_halo(3, halo.data_ptr(), np.array([0, 1, 2], np.int32), send.data_ptr())
    res["past_buffers"] = err(lambda: eng.lagged_transport(comm, [4], [3]))
    res["negative"] = err(lambda: eng.lagged_transport(comm, [-1], [3]))
    res["ok"] = err(lambda: eng.lagged_transport(comm, [3], [3]))
    res["detach"] = err(lambda: eng.lagged_transport(None))
    res["after_detach"] = err(eng.lagged_exchange)
    comm.check()
    comm.close()
    eng.close()
    np.save(os.path.join(out, "res.npy"), np.array([repr(res)]))


def test_engine_transport_checks(tmp_path):
    """dopt_lagged_transport / dopt_lagged_exchange refuse what they cannot do, with the reason: no transport
    attached (DOPT_ERR_STATE), blocks past the send / halo buffers or negative (ValueError), a block list of
    the wrong length; the RCCL library is the copy torch loaded (one RCCL in the process)."""
    import ast

    import torch.multiprocessing as mp

    mp.start_processes(_transport_errors, args=(1, _rdv(tmp_path), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    res = ast.literal_eval(str(np.load(tmp_path / "res.npy")[0]))
    assert "torch" in res["library"] and "rccl" in res["library"], res
    assert "no transport" in res["no_transport"], res
    assert res["no_buffers"].startswith("ValueError") and "past the buffers" in res["no_buffers"], res
    assert res["bad_shape"].startswith("ValueError"), res
    assert res["past_buffers"].startswith("ValueError") and "past the buffers" in res["past_buffers"], res
    assert res["negative"].startswith("ValueError") and "negative" in res["negative"], res
    assert res["ok"] is None and res["detach"] is None, res
    assert "no transport" in res["after_detach"], res


def _lonely_comm(rank, world, rdv, out, timeout_s):
    """Rank 0 of a world-2 engine communicator whose rank 1 never calls create (csrc/transport.cpp: the
    non-blocking setup polled under timeout_s, then aborted)."""
    import time

    import torch

    import _dopt

    torch.cuda.set_device(0)
    uid = _dopt.comm_unique_id()
    t0 = time.monotonic()
    try:
        _dopt.Comm(2, 0, 0, uid, timeout_s=timeout_s)
        msg = "created"
    except RuntimeError as e:
        msg = f"{type(e).__name__}: {e}"
    np.save(os.path.join(out, "lonely.npy"), np.array([repr({"msg": msg, "s": time.monotonic() - t0})]))


@pytest.mark.timeout(150)
def test_engine_comm_setup_without_peer_is_bounded(tmp_path):
    """dopt_comm_create is a collective; a rank whose peer never joins ends with an error
    after the timeout (the half-built communicator aborted) instead of hanging in ncclCommInitRank, and its
    process exits (no process left behind)."""
    import ast

    import torch.multiprocessing as mp

    timeout_s = 6
    ctx = mp.start_processes(_lonely_comm, args=(1, _rdv(tmp_path), str(tmp_path), timeout_s), nprocs=1,
                             join=False, start_method="spawn")
    p = ctx.processes[0]
    p.join(120)
    alive = p.is_alive()
    if alive:
        p.kill()
        p.join(10)
    assert not alive, "the lonely rank did not end within 120 s"
    assert p.exitcode == 0, p.exitcode
    res = ast.literal_eval(str(np.load(tmp_path / "lonely.npy")[0]))
    assert res["msg"].startswith("RuntimeError") and "did not complete in 6 s" in res["msg"], res
    assert timeout_s <= res["s"] < timeout_s + 30, res
