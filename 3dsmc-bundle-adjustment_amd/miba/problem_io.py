"""Window-problem files through libmiba's C-ABI (include/ba_io.h): .miba window dumps
(replay of windows captured with MIBA_DUMP_DIR) and BAL text problems."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .capi import BaOptions, ProblemArrays


class ProblemFileError(RuntimeError):
    pass


def _check(L, rc: int, what: str):
    if rc != 0:
        raise ProblemFileError(f"{what} failed ({rc}): {(L.ba_last_error(None) or b'').decode()}")


def _empty(nc: int, np_: int, no: int) -> ProblemArrays:
    return ProblemArrays(np.zeros((nc, 7)), np.zeros((np_, 3)), np.zeros(4), np.zeros(4), np.zeros(no, np.int32),
                         np.zeros(no, np.int32), np.zeros((no, 2)), np.zeros(no))


def _read(path: str, dims_fn, read_fn, *extra) -> ProblemArrays:
    L = _lib.lib()
    d = [C.c_int32() for _ in range(3)]
    bpath = str(path).encode()
    _check(L, getattr(L, dims_fn)(bpath, *[C.byref(x) for x in d]), dims_fn)
    prob = _empty(*(x.value for x in d))
    ps = prob.struct()
    _check(L, getattr(L, read_fn)(bpath, C.byref(ps), *extra), read_fn)
    prob.fixed_cam = ps.fixed_cam
    return prob


def read_window(path: str) -> tuple[ProblemArrays, BaOptions]:
    """(problem, options it was captured with — ba_default_options() if the dump carries none)."""
    o = BaOptions()
    return _read(path, "ba_problem_read_dims", "ba_problem_read", C.byref(o)), o


def write_window(path: str, prob: ProblemArrays, opts: BaOptions | None = None) -> None:
    L = _lib.lib()
    ps = prob.struct()
    _check(L, L.ba_problem_write(str(path).encode(), C.byref(ps), C.byref(opts) if opts is not None else None),
           "ba_problem_write")


def read_bal(path: str) -> ProblemArrays:
    return _read(path, "ba_bal_read_dims", "ba_bal_read")


def write_bal(path: str, prob: ProblemArrays) -> None:
    L = _lib.lib()
    ps = prob.struct()
    _check(L, L.ba_bal_write(str(path).encode(), C.byref(ps)), "ba_bal_write")


def load(path: str) -> tuple[ProblemArrays, BaOptions | None]:
    """Either format, by content: a .miba dump returns its options, a BAL file returns None."""
    with open(path, "rb") as f:
        magic = f.read(8)
    if magic == b"MIBAWIN1":
        return read_window(path)
    return read_bal(path), None
