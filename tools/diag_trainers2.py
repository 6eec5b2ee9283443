#!/usr/bin/env python3
"""Diagnostic: the C2 trainers under a 2-rank gloo job on one GPU vs the reference fixture, every label
reported (max relative difference of the objective over 300 rounds), and the single-process run."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-optimization_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def run(rank, world, port, mode):
    import torch  # noqa: F401
    import torch.distributed as dist

    import data as odata
    from trainer import CentralizedTrainer, DecentralizedTrainer
    from worker import Worker

    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    meta = json.load(open(os.path.join(G, "traj_c2.json")))
    z = np.load(os.path.join(G, "traj_c2.npz"))
    cfg = dict(meta["config"])
    shards, Xf, yf = odata.generate(cfg, order=z["order"])
    res = {}
    labels = list(enumerate(meta["labels"]))
    if mode == "dsgd_first":  # the checkpoint test's order: a D-SGD run on the engine first
        labels = labels[1:2] + labels[:1]
    elif mode == "ck20":  # Centralized only, in chunks of 20 rounds (checkpoint_every)
        labels = labels[:1]
    for j, label in labels:
        if mode == "ck20":
            cfg = dict(meta["config"], checkpoint_path=f"/tmp/diag_ck_{world}.npz", checkpoint_every=20)
        else:
            cfg = dict(meta["config"])
        np.random.set_state(("MT19937", z[f"state{j}_key"], int(z[f"state{j}_pos"]), 0, 0.0))
        ws = [Worker(i, {"X": X, "y": y}, cfg["local_batch_size"], Xf.shape[1], cfg) for i, (X, y) in enumerate(shards)]
        if label == "Centralized":
            tr = CentralizedTrainer(ws, Xf.shape[1], cfg)
        else:
            topo = {"D-SGD (Ring)": "ring", "D-SGD (Fully Connected)": "fully_connected"}[label]
            tr = DecentralizedTrainer(ws, topo, Xf.shape[1], cfg)
        hist, xf = tr.run(300, Xf, yf, meta["f_opt"])
        o = np.asarray(hist["objective"])
        ref = z[f"L{j}_objective"][:300]
        res[label] = (float(np.max(np.abs(o - ref) / np.abs(ref))), o[:6].tolist(), ref[:6].tolist())
    if rank == 0:
        print(f"world {world} {mode}:", json.dumps(res, indent=1), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(run, args=(1, port, "all"), nprocs=1, join=True, start_method="spawn")
    for k, mode in enumerate(("all", "dsgd_first", "ck20")):
        mp.start_processes(run, args=(2, port + 1 + k, mode), nprocs=2, join=True, start_method="spawn")


if __name__ == "__main__":
    main()
