"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the CPU float64 oracle.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module. It restates the reference hot path (windowOptimize -> ceres::Solve,
/root/reference/src/OptimizationUtils.cpp:215-313) in plain C (ba_oracle.c);
parity against Ceres itself is UNPINNED (no Ceres in the image, no reference
tests on this path) — see DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(os.path.dirname(_HERE), "3dsmc-bundle-adjustment_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from miba.capi import BaOptions, BaProblem, BaSummary, ProblemArrays  # noqa: E402

_LIB_PATH = os.path.join(_HERE, "_build", "libba_oracle.so")
_lib = None


def build() -> str:
    """Compile the oracle (gcc) into oracle/_build/."""
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        deps = [os.path.join(_HERE, "ba_oracle.c"), os.path.join(_HERE, "..", "include", "ba.h")]
        if not os.path.exists(_LIB_PATH) or any(os.path.getmtime(_LIB_PATH) < os.path.getmtime(d) for d in deps):
            build()  # the oracle shares the ba_options / ba_summary layout of include/ba.h
        L = C.CDLL(_LIB_PATH)
        L.oracle_default_options.argtypes = [C.POINTER(BaOptions)]
        L.oracle_solve.argtypes = [C.POINTER(BaProblem), C.POINTER(BaOptions), C.POINTER(BaSummary)]
        L.oracle_solve.restype = C.c_int
        dp = C.POINTER(C.c_double)
        L.oracle_linearize.argtypes = [C.POINTER(BaProblem), C.POINTER(BaOptions), dp, dp, dp, dp, dp]
        L.oracle_linearize.restype = C.c_int
        L.oracle_reduced_system.argtypes = [C.POINTER(BaProblem), C.POINTER(BaOptions), C.c_double, C.c_int32,
                                            C.c_int32, C.c_int32, C.POINTER(C.c_int32), dp, dp]
        L.oracle_reduced_system.restype = C.c_int
        L.oracle_se3_plus.argtypes = [dp, dp, dp]
        L.oracle_solve_trace.argtypes = [C.POINTER(BaProblem), C.POINTER(BaOptions), C.POINTER(BaSummary), dp,
                                         C.c_int32]
        L.oracle_solve_trace.restype = C.c_int
        L.oracle_config.argtypes = [C.c_int32, C.c_int32]
        L.oracle_max_threads.restype = C.c_int32
        _lib = L
    return _lib


def default_options(**kw) -> BaOptions:
    o = BaOptions()
    lib().oracle_default_options(C.byref(o))
    o.minimizer_progress_to_stdout = 0
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def solve(prob: ProblemArrays, opts: BaOptions | None = None) -> dict:
    """Solve in place (like windowOptimize mutating its parameter blocks)."""
    opts = opts or default_options()
    s = BaSummary()
    ps = prob.struct()
    rc = lib().oracle_solve(C.byref(ps), C.byref(opts), C.byref(s))
    if rc != 0:
        raise RuntimeError(f"oracle_solve failed: {rc}")
    return s.as_dict()


TRACE_W = 8  # cost, cost_change, |gradient|, |step|, tr_ratio, tr_radius, accepted (1/0/-1), 0


def solve_trace(prob: ProblemArrays, opts: BaOptions | None = None):
    """solve() plus the per-iteration trace, rows 0..num_iterations (same layout as
    libmiba's ba_iteration_log)."""
    opts = opts or default_options()
    s = BaSummary()
    ps = prob.struct()
    rows = max(int(opts.max_num_iterations), 0) + 2
    tr = np.zeros((rows, TRACE_W))
    rc = lib().oracle_solve_trace(C.byref(ps), C.byref(opts), C.byref(s), _dptr(tr), rows)
    if rc != 0:
        raise RuntimeError(f"oracle_solve_trace failed: {rc}")
    d = s.as_dict()
    return d, tr[: d["num_iterations"] + 1].copy()


def config(threads: int = 1, profile: bool = False) -> None:
    """Execution knobs of the restatement: OpenMP threads (1 = fixed summation order, the
    checker) and the reduced-system storage (False = dense lower triangle, the checker;
    True = the co-visibility profile, the SPARSE_SCHUR stand-in timed as the CPU baseline)."""
    lib().oracle_config(int(threads), int(bool(profile)))


def max_threads() -> int:
    return int(lib().oracle_max_threads())


def linearize(prob: ProblemArrays, opts: BaOptions | None = None):
    opts = opts or default_options()
    n = prob.n_obs
    res = np.zeros((n, 3)); jc = np.zeros((n, 3, 6)); jp = np.zeros((n, 3, 3)); jk = np.zeros((n, 2, 4))
    cost = np.zeros(1)
    ps = prob.struct()
    rc = lib().oracle_linearize(C.byref(ps), C.byref(opts), _dptr(cost), _dptr(res), _dptr(jc), _dptr(jp), _dptr(jk))
    return dict(rc=rc, cost=float(cost[0]), res=res, jcam=jc, jpt=jp, jint=jk)


def reduced_system(prob: ProblemArrays, opts: BaOptions | None = None, radius: float = 0.0,
                   pt_begin: int = 0, pt_end: int | None = None, with_global: bool = True):
    opts = opts or default_options()
    ps = prob.struct()
    n = C.c_int32(0)
    lib().oracle_reduced_system(C.byref(ps), C.byref(opts), radius, 0, 0, 0, C.byref(n), None, None)
    S = np.zeros((n.value, n.value)); rhs = np.zeros(n.value)
    pe = prob.n_points if pt_end is None else pt_end
    rc = lib().oracle_reduced_system(C.byref(ps), C.byref(opts), radius, pt_begin, pe, int(with_global),
                                     C.byref(n), _dptr(S), _dptr(rhs))
    if rc != 0:
        raise RuntimeError(f"oracle_reduced_system failed: {rc}")
    return S, rhs


def se3_plus(T, delta):
    T = np.ascontiguousarray(T, dtype=np.float64)
    d = np.ascontiguousarray(delta, dtype=np.float64)
    out = np.zeros(7)
    lib().oracle_se3_plus(_dptr(T), _dptr(d), _dptr(out))
    return out
