"""C-ABI checks that run without a GPU: libmiba.so loads, exports exactly the
symbols include/ba.h declares, and refuses to run (loudly) with no device."""
import ctypes as C
import os
import re

import pytest

from miba import _lib
from miba.capi import BaOptions, BaProblem, BaSummary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "ba.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ba_[a-z_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def test_exports_match_header(L):
    decl = declared_functions()
    assert sorted(_lib.EXPORTS) == decl
    for name in decl:
        assert hasattr(L, name), name


def test_defaults_equal_oracle_defaults(L):
    from oracle import oracle
    a = BaOptions(); L.ba_default_options(C.byref(a))
    b = oracle.default_options()
    for name, _ in BaOptions._fields_:
        if name in ("minimizer_progress_to_stdout", "deterministic", "profile_kernels", "reserved"):
            continue
        assert getattr(a, name) == getattr(b, name), name
    assert a.minimizer_progress_to_stdout == 1  # BundleAdjustmentConfig.h:63


def test_api_version(L):
    assert L.ba_api_version() == 1
    assert b"gfx950" in L.ba_build_info()


def test_struct_layout():
    # ba_options: 4 doubles, 2 int32, 7 doubles, 2 int32, 3 doubles, 2 int32, 6 int32
    assert C.sizeof(BaOptions) == 4 * 8 + 8 + 7 * 8 + 8 + 3 * 8 + 8 + 24
    from miba.capi import BaKernelStat
    assert C.sizeof(BaKernelStat) == 32 + 8 + 3 * 8
    assert C.sizeof(BaProblem) == 16 + 8 * 8
    assert C.sizeof(BaSummary) == 8 * 2 + 4 * 8 + 8 * 7 + 160


def test_no_device_fails_loudly(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = L.ba_create(None)
    assert not h
    assert b"device" in L.ba_last_error(None)
