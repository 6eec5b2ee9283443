"""The pull transport's host setup (distributed.IpcTransport) over 2 and 3 gloo ranks on the CPU, with a
stand-in engine that records what the library would be given: every rank receives every peer's handles and
slot size in rank order, the byte offset of ITS block in each peer's send slot (the peer's send offsets, not
its own), its own receive block sizes, and the address of counters every rank sees (one shared segment);
a failure on any rank fails every rank's setup (no rank left waiting in a collective), and the segment is
removed when rank 0 closes, which also detaches the context if the transport is still its exchange."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

import distributed as D


class _Eng:
    def __init__(self, rank, fail_at=None):
        self.rank, self.fail_at, self.calls = rank, fail_at, []

    def lagged_transport(self, comm):
        self.calls.append(("detach",))

    def lagged_ipc_export(self):
        if self.fail_at == "export":
            raise RuntimeError("hipExtMallocWithFlags: out of memory")
        return bytes([self.rank]) * 64, bytes([100 + self.rank]) * 64, 4096 * (self.rank + 1)

    def lagged_ipc_check(self, step):
        if self.fail_at == f"check{step}":
            raise RuntimeError("hipStreamWaitEvent: invalid argument")
        self.calls.append(("check", step))

    def lagged_ipc_import(self, world, rank, mh, eh, slots, src_off, recv_rows, addr, timeout_s):
        if self.fail_at == "import":
            raise RuntimeError("hipIpcOpenMemHandle of peer 0: invalid argument")
        self.calls.append(("import", world, rank, list(mh), list(eh), list(slots), list(src_off), list(recv_rows),
                           addr, timeout_s))


class _Lay:
    def __init__(self, send_sizes, recv_sizes):
        self.send_sizes, self.recv_sizes = send_sizes, recv_sizes


class _Plan:
    def __init__(self, world, rank):
        self.world, self.rank = world, rank


def _rank(rank, world, rdv, out, fail_rank, fail_at):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    # rank r sends 10 * (p + 1) + r rows to peer p, and receives 10 * (r + 1) + p from p (the transpose)
    send = [10 * (p + 1) + rank if p != rank else 0 for p in range(world)]
    recv = [10 * (rank + 1) + p if p != rank else 0 for p in range(world)]
    eng = _Eng(rank, fail_at if rank == fail_rank else None)
    res = {}
    try:
        t = D.IpcTransport(eng, _Plan(world, rank), _Lay(send, recv), None, 256, 7.0)
    except D.CollectiveError as e:
        res["error"] = str(e)
    else:
        assert [c for c in eng.calls if c[0] == "check"] == [("check", 0), ("check", 1)]
        imp = [c for c in eng.calls if c[0] == "import"][0]
        res["import"] = imp[1:8] + (imp[9],)
        t._cnt[rank] = 1000 + rank  # every rank writes its own counter ...
        dist.barrier()
        res["counters"] = [int(v) for v in t._cnt]  # ... and reads every rank's
        res["segment"] = t._shm.name
        dist.barrier()
        n = len(eng.calls)
        t.close()
        res["detached_on_close"] = eng.calls[n:] == [("detach",)]
        eng._ipc_owner = None  # another transport took over: a second close leaves the context alone
        t.close()
        res["second_close_quiet"] = len(eng.calls) == n + 1
        dist.barrier()
    np.save(os.path.join(out, f"r{rank}.npy"), np.array([repr(res)]))
    dist.destroy_process_group()


def _run(tmp_path, world, fail_rank=-1, fail_at=None):
    import ast

    rdv = f"file://{tmp_path}/store"
    mp.start_processes(_rank, args=(world, rdv, str(tmp_path), fail_rank, fail_at), nprocs=world, join=True,
                       start_method="spawn")
    return [ast.literal_eval(str(np.load(tmp_path / f"r{r}.npy")[0])) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_handles_offsets_and_shared_counters(tmp_path, world):
    res = _run(tmp_path, world)
    for r, got in enumerate(res):
        w, rank, mh, eh, slots, src_off, recv_rows, timeout_s = got["import"]
        assert (w, rank, timeout_s) == (world, r, 7.0)
        assert mh == [bytes([p]) * 64 for p in range(world)] and eh == [bytes([100 + p]) * 64 for p in range(world)]
        assert slots == [4096 * (p + 1) for p in range(world)]
        # peer p's block for rank r starts after p's blocks for ranks < r: sum of 10 (q + 1) + p rows, 256 bytes each
        want = [256 * sum(10 * (q + 1) + p for q in range(r) if q != p) for p in range(world)]
        assert src_off == want, (r, src_off, want)
        assert recv_rows == [10 * (r + 1) + p if p != r else 0 for p in range(world)]
        assert got["counters"] == [1000 + p for p in range(world)]  # one segment, seen by every rank
        assert got["detached_on_close"] and got["second_close_quiet"], got
    assert len({g["segment"] for g in res}) == 1
    assert not os.path.exists("/dev/shm/" + res[0]["segment"].lstrip("/"))  # removed by rank 0's close


@pytest.mark.parametrize("fail_rank,fail_at", [(1, "export"), (0, "import"), (1, "import"), (0, "check0"),
                                               (1, "check1")])
def test_a_failure_fails_every_rank(tmp_path, fail_rank, fail_at):
    res = _run(tmp_path, 2, fail_rank, fail_at)
    for got in res:
        assert "pull transport setup failed" in got.get("error", ""), got
        assert f"rank {fail_rank}" in got["error"], got
