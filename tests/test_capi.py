"""C-ABI checks that run without a GPU: libmiba.so loads, exports exactly the
symbols include/ba.h declares, and refuses to run (loudly) with no device."""
import ctypes as C
import os
import re
import subprocess

import pytest

from miba import _lib
from miba.capi import BaOptions, BaProblem, BaSummary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("ba.h", "ba_io.h"))
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
    # and nothing else with the ba_ prefix is exported
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = sorted({l.split()[-1] for l in nm.stdout.splitlines() if l.split()[-1].startswith("ba_")})
    assert exported == decl


def test_defaults_equal_oracle_defaults(L):
    from oracle import oracle
    a = BaOptions(); L.ba_default_options(C.byref(a))
    b = oracle.default_options()
    for name, _ in BaOptions._fields_:
        if name in ("minimizer_progress_to_stdout", "deterministic", "profile_kernels", "profile_mask", "small_window",
                    "reserved"):
            continue
        assert getattr(a, name) == getattr(b, name), name
    assert a.minimizer_progress_to_stdout == 1  # BundleAdjustmentConfig.h:63


def test_api_version(L):
    assert L.ba_api_version() == 2  # ba.h version history: 2 = sized ba_summary / ba_prepare_info
    assert b"gfx950" in L.ba_build_info()


def _c_layout(struct_name, fields):
    """sizeof + offsetof of every field, from the real header compiled by gcc."""
    import subprocess
    import tempfile
    lines = [f'printf("%zu\\n", sizeof({struct_name}));']
    lines += [f'printf("%zu\\n", offsetof({struct_name}, {f}));' for f in fields]
    src = "#include <stddef.h>\n#include <stdio.h>\n#include \"ba.h\"\nint main(void){" + "".join(lines) + "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        out = [int(x) for x in subprocess.check_output([exe]).split()]
    return out[0], out[1:]


@pytest.mark.parametrize("cls,cname", [(BaOptions, "ba_options"), (BaProblem, "ba_problem"),
                                       (BaSummary, "ba_summary"), ("BaKernelStat", "ba_kernel_stat"),
                                       ("BaPrepareInfo", "ba_prepare_info")])
def test_struct_layout_matches_header(cls, cname):
    if isinstance(cls, str):
        from miba import capi
        cls = getattr(capi, cls)
    names = [n for n, _ in cls._fields_]
    size, offs = _c_layout(cname, names)
    assert C.sizeof(cls) == size
    assert [getattr(cls, n).offset for n in names] == offs


def test_no_device_fails_loudly(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = L.ba_create(None)
    assert not h
    assert b"device" in L.ba_last_error(None)
