"""The engine-driven communicator's lifetime on the host: a Comm detaches every engine routed
through it before it is destroyed or aborted, so no context keeps a freed dopt_comm*; distributed's
close_comms / the bounded wait's timeout path close every communicator of the process.  The library calls
are recorded by a stand-in (no GPU, no RCCL)."""
import types

import numpy as np
import pytest

import _dopt
import distributed as D


class _Lib:
    def __init__(self):
        self.calls = []

    def dopt_lagged_transport(self, h, comm_h, s, r):
        self.calls.append(("transport", h.value if hasattr(h, "value") else h, comm_h))
        return 0

    def dopt_comm_destroy(self, h, abort):
        self.calls.append(("destroy", h, abort))
        return 0

    def dopt_comm_check(self, h):
        return 0


def _engine(lib, tag):
    eng = object.__new__(_dopt.Engine)
    eng._h = tag
    return eng


def _comm(tag, world=2):
    c = object.__new__(_dopt.Comm)
    c._h = tag
    c.world, c.rank, c.device = world, 0, 0
    import weakref

    c.users = weakref.WeakSet()
    return c


@pytest.fixture
def lib(monkeypatch):
    fake = _Lib()
    monkeypatch.setattr(_dopt, "lib", lambda: fake)
    return fake


def test_close_detaches_every_engine_first(lib):
    comm = _comm("C")
    a, b = _engine(lib, "A"), _engine(lib, "B")
    a.lagged_transport(comm, [0, 3], [0, 3])
    b.lagged_transport(comm, [0, 1], [0, 1])
    assert set(comm.users) == {a, b}
    comm.close(abort=True)
    kinds = [c[0] for c in lib.calls]
    # both attachments, then both detachments (NULL comm), then the abort -- never a destroy before a detach
    assert kinds[:2] == ["transport", "transport"] and kinds[-1] == "destroy"
    detached = [c for c in lib.calls[2:-1] if c[0] == "transport"]
    assert {c[1] for c in detached} == {"A", "B"} and all(c[2] is None for c in detached)
    assert lib.calls[-1] == ("destroy", "C", 1)
    assert comm.closed and not list(comm.users)
    comm.close()  # idempotent
    assert [c[0] for c in lib.calls].count("destroy") == 1
    with pytest.raises(RuntimeError, match="closed"):
        comm.check()
    with pytest.raises(ValueError, match="closed"):
        a.lagged_transport(comm, [0, 3], [0, 3])


def test_detached_or_closed_engine_leaves_the_comm(lib):
    comm = _comm("C")
    a, b = _engine(lib, "A"), _engine(lib, "B")
    a.lagged_transport(comm, [0, 3], [0, 3])
    b.lagged_transport(comm, [0, 3], [0, 3])
    a.lagged_transport(None)
    b._h = None  # as after Engine.close's dopt_destroy
    b.close()
    assert not list(comm.users)
    n = len(lib.calls)
    comm.close()
    assert lib.calls[n:] == [("destroy", "C", 0)]  # nobody left to detach


def test_timeout_path_closes_every_communicator(lib, monkeypatch):
    """_sync past DOPT_PG_TIMEOUT: the runner's communicator and every other one of the process are aborted
    (engines detached first), and the runner no longer holds one."""
    import time

    mine, other = _comm("M"), _comm("O")
    eng = _engine(lib, "E")
    eng.lagged_transport(mine, [0, 1], [0, 1])
    monkeypatch.setattr(D, "_COMMS", {("g", 0): mine, ("h", 0): other})
    clock = iter(np.arange(0.0, 1e4, 0.75))
    monkeypatch.setattr(time, "monotonic", lambda: float(next(clock)))
    monkeypatch.setattr(time, "sleep", lambda s: None)
    monkeypatch.setenv("DOPT_PG_TIMEOUT", "5")

    class _Stream:
        def query(self):
            return False

    run = types.SimpleNamespace(plan=types.SimpleNamespace(rank=1),
                                exchange=types.SimpleNamespace(what="exchange of 3 rows"), comm=mine)
    with pytest.raises(D.CollectiveError, match="did not finish in 5 s"):
        D.DistributedDSGD._sync(run, _Stream())
    assert run.comm is None and mine.closed and other.closed and not D._COMMS
    destroys = [c for c in lib.calls if c[0] == "destroy"]
    assert sorted(destroys) == [("destroy", "M", 1), ("destroy", "O", 1)]
    first_destroy = next(i for i, c in enumerate(lib.calls) if c[0] == "destroy")
    assert ("transport", "E", None) in lib.calls[:first_destroy]
