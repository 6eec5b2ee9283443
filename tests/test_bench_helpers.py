"""CPU checks of bench.py's measurement helpers (no GPU): the algorithmic bytes per launch that
roofline.achieved divides by the kernel time (C3 8.665 GB, C4 138.6 GB,
C5 direct 77.3 GB, C5 row-space 68.72 GB), and the committed PMC summary each configuration's line
reads its traffic from (profiles/), which must sit within 2 % of those bytes (no re-reads)."""
import os
import sys
import types

import pytest

import _dopt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import bench  # noqa: E402

F32, F64 = _dopt.F32, _dopt.F64
C3 = "void dopt::k_round<double, float, 4, 0, true, true, 161843>(dopt::RoundArgs)"
C5RS = "void dopt::k_rs_pass<float, true, 2, 6>(dopt::RsArgs)"
C5X32 = "void dopt::k_rs_pass_x32<true, 2, 6>(dopt::RsArgs)"
C5D = "void dopt::k_split_step<float, 4, true, true, true, 1>(dopt::RoundArgs)"  # round-2 spelling
C5DX = "void dopt::k_split_step<double, float, 4, true, true, true, 1>(dopt::RoundArgs)"


def _eng(dtype, xdtype):
    return types.SimpleNamespace(dtype=dtype, data_dtype=xdtype)


# (config, kernel, engine dtype, row storage, workers, d, m, GB in DESIGN.md, profile file)
CASES = [
    ("c3", C3, F64, F32, 4096, 1024, 512, 8.665, "profiles/r3_pmc.json"),
    ("c5", C5DX, F64, F32, 1024, 1 << 20, 16, 85.90, "profiles/r3_c5x32direct_pmc.json"),
    ("c4", C3, F64, F32, 65536, 1024, 512, 138.6, "profiles/r3_c4_pmc.json"),
    ("c5", C5D, F32, F32, 1024, 1 << 20, 16, 77.3, "profiles/r2_c5_pmc.json"),
    ("c5", C5RS, F32, F32, 1024, 1 << 20, 16, 68.72, "profiles/r2_c5rs_pmc.json"),
    ("c5", C5X32, F64, F32, 1024, 1 << 20, 16, 68.72, "profiles/r2_c5x32_pmc.json"),
]


@pytest.mark.parametrize("config,kernel,dt,xdt,n,d,m,gb,prof", CASES)
def test_bytes_and_committed_traffic(config, kernel, dt, xdt, n, d, m, gb, prof):
    b = bench.bytes_per_round(_eng(dt, xdt), n, d, m, kernel)
    assert abs(b / 1e9 - gb) < 0.01 * gb, b
    traffic, src, _ = bench.pmc_traffic(kernel, config)
    assert src == prof, src
    assert 1.0 <= traffic / b < 1.02, traffic / b


def test_traffic_lookup_is_per_configuration():
    """C3 and C4 launch the same kernel instance: each line reads its own configuration's file."""
    t3, s3, _ = bench.pmc_traffic(C3, "c3")
    t4, s4, _ = bench.pmc_traffic(C3, "c4")
    assert s3 != s4 and t4 > 10 * t3
    assert bench.pmc_traffic("void dopt::k_no_such_kernel()", "c5") == (None, None, None)
