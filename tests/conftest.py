import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-optimization_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)

# one HIP runtime per process: torch first, then libdopt.so binds to it
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdopt.so on the device)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "multiproc: starts rank processes (torch.distributed); collected last")


# Files whose every test starts rank processes (their harness, not the kernels, is the fragile part):
# run after the single-process oracle-parity files, so a rendezvous failure under -x cannot hide the
# parity signal (a port race in test_gpu_distributed stopped the run before test_gpu_parity).
MULTIPROC_FILES = {"test_ipc_setup_cpu.py", "test_gpu_distributed.py", "test_distributed_cpu.py", "test_bench_launch.py"}


def _multiproc(item):
    return item.fspath.basename in MULTIPROC_FILES or item.get_closest_marker("multiproc") is not None


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_multiproc)  # stable: file and definition order kept within each group


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
