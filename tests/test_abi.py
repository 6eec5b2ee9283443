"""C ABI: libdopt.so loads without a GPU, exports every symbol include/dopt.h declares,
and device entry points fail loudly (no CPU fallback) when no device is usable."""
import os
import re

import numpy as np
import pytest

import _dopt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "dopt.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(dopt_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    decl = declared_symbols()
    assert len(decl) >= 20
    assert sorted(_dopt.EXPORTED) == decl


def test_library_exports_everything():
    L = _dopt.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.dopt_abi_version() == 9 == _dopt.ABI_VERSION


def test_no_silent_fallback_without_gpu():
    if _dopt.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError, match="no HIP device"):
        _dopt.Engine(0, "float64")


def test_error_mapping():
    with pytest.raises(ValueError):
        _dopt.check(_dopt.ERR_INVALID)
    with pytest.raises(NotImplementedError):
        _dopt.check(_dopt.ERR_UNSUPPORTED)
    with pytest.raises(RuntimeError):
        _dopt.check(_dopt.ERR_HIP)
