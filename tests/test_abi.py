"""BA_API_VERSION 2: ba_summary and ba_prepare_info carry the caller's struct_size (include/ba.h), the library writes
no more than that many bytes and rejects a size below the version's minimum (VERDICT r05 weak #7 / ADVICE r05: a
caller built against an older header must not have memory past its struct overwritten). The boundary replaced is
windowOptimize's ceres::Solve (/root/reference/src/OptimizationUtils.cpp:300, headers/OptimizationUtils.h:55)."""
import ctypes as C
import os
import subprocess
import tempfile

import pytest

from miba import _lib
from miba.capi import BaPrepareInfo, BaSummary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_values(exprs):
    src = ("#include <stddef.h>\n#include <stdio.h>\n#include \"ba.h\"\nint main(void){"
           + "".join(f'printf("%ld\\n", (long)({e}));' for e in exprs) + "return 0;}\n")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "v.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "v")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        return [int(x) for x in subprocess.check_output([exe]).split()]


def test_min_sizes_and_init_macros():
    smin, pmin, ssz, psz, s_init, p_init = _c_values([
        "BA_SUMMARY_MIN_SIZE", "BA_PREPARE_INFO_MIN_SIZE", "sizeof(ba_summary)", "sizeof(ba_prepare_info)",
        "({ ba_summary s; BA_SUMMARY_INIT(s); s.struct_size; })",
        "({ ba_prepare_info i; BA_PREPARE_INFO_INIT(i); i.struct_size; })"])
    assert ssz == C.sizeof(BaSummary) and psz == C.sizeof(BaPrepareInfo)
    assert smin == BaSummary.message.offset  # every field before the message
    assert pmin == BaPrepareInfo.total_ms.offset + 8  # the round-3 layout: through total_ms
    assert s_init == ssz and p_init == psz
    assert BaSummary().struct_size == ssz and BaPrepareInfo().struct_size == psz


# ---------------------------------------------------------------------------------------------------- GPU
def _solver():
    from miba.solver import Solver
    return Solver(device=0, minimizer_progress_to_stdout=0)


def _window():
    from miba import synthetic
    return synthetic.make_problem(n_cams=8, n_points=200, obs_per_point=(2, 3), seed=4)


@pytest.mark.gpu
def test_prepare_info_round4_size_not_overwritten():
    """A caller whose ba_prepare_info ends at lin_path (the round-4 layout) gets exactly its bytes written."""
    L = _lib.lib()
    with _solver() as s:
        p = _window()
        s.prepare(p)
        size4 = BaPrepareInfo.lin_path.offset + 4  # struct_size .. lin_path
        buf = (C.c_uint8 * C.sizeof(BaPrepareInfo))(*([0xA5] * C.sizeof(BaPrepareInfo)))
        C.c_int32.from_buffer(buf, 0).value = size4
        assert L.ba_last_prepare(s._h, C.cast(buf, C.POINTER(BaPrepareInfo))) == 0
        raw = bytes(buf)
        assert all(b == 0xA5 for b in raw[size4:]), "bytes past the caller's struct_size were written"
        full = s.last_prepare()
        got = BaPrepareInfo.from_buffer_copy(raw[:size4] + bytes(C.sizeof(BaPrepareInfo) - size4))
        assert got.struct_size == size4
        for f in ("plan_reused", "obs_uploaded", "host_threads", "bcr_path", "lin_path"):
            assert getattr(got, f) == full[f], f
        # below the minimum: refused, nothing written
        buf2 = (C.c_uint8 * 64)(*([0x5A] * 64))
        C.c_int32.from_buffer(buf2, 0).value = 12
        assert L.ba_last_prepare(s._h, C.cast(buf2, C.POINTER(BaPrepareInfo))) != 0
        assert bytes(buf2)[4:] == bytes([0x5A] * 60)


@pytest.mark.gpu
def test_summary_struct_size_honoured():
    """ba_solve writes min(struct_size, sizeof) bytes of the summary and refuses struct_size 0."""
    L = _lib.lib()
    with _solver() as s:
        p = _window()
        ref = s.solve(p.copy())
        n = C.sizeof(BaSummary)
        small = BaSummary.message.offset  # a caller without the message field
        buf = (C.c_uint8 * n)(*([0xC3] * n))
        C.c_int32.from_buffer(buf, 0).value = small
        ps = p.copy()
        pst = ps.struct()
        assert L.ba_solve(s._h, C.byref(pst), C.cast(buf, C.POINTER(BaSummary))) == 0
        raw = bytes(buf)
        assert all(b == 0xC3 for b in raw[small:])
        got = BaSummary.from_buffer_copy(raw[:small] + bytes(n - small))
        assert got.struct_size == small
        assert got.num_iterations == ref["num_iterations"]
        assert abs(got.final_cost - ref["final_cost"]) <= 1e-9 * ref["final_cost"]
        # struct_size 0 (an uninitialised v1-style summary): refused before any work, untouched
        z = (C.c_uint8 * n)()
        assert L.ba_solve(s._h, C.byref(pst), C.cast(z, C.POINTER(BaSummary))) == -1
        assert bytes(z) == bytes(n)
        assert "struct_size" in s.last_error()
        assert L.ba_solve_prepared(s._h, C.byref(pst), C.cast(z, C.POINTER(BaSummary))) == -1
