"""Python front-end of the libmiba C-ABI (include/ba.h).

``Solver`` owns one ``ba_context`` (device buffers cached across calls, like
the reference re-optimising the same window repeatedly, main.cpp:163-168).
``Solver.solve`` is the replacement of ``ceres::Solve`` inside
``windowOptimize`` (OptimizationUtils.cpp:300): it updates the problem's
poses, points and intrinsics in place and returns the summary.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .capi import BaKernelStat, BaOptions, BaPrepareInfo, BaSummary, ProblemArrays


def default_options(**overrides) -> BaOptions:
    o = BaOptions()
    _lib.lib().ba_default_options(C.byref(o))
    for k, v in overrides.items():
        setattr(o, k, v)
    return o


class MibaError(RuntimeError):
    pass


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Solver:
    def __init__(self, options: BaOptions | None = None, **overrides):
        self._L = _lib.lib()
        self.options = options if options is not None else default_options()
        for k, v in overrides.items():
            setattr(self.options, k, v)
        h = self._L.ba_create(C.byref(self.options))
        if not h:
            raise MibaError("ba_create failed: " + (self._L.ba_last_error(None) or b"").decode())
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = (self._L.ba_last_error(self._h) or b"").decode()
            raise MibaError(f"{what} failed ({rc}): {msg}")

    def last_error(self) -> str:
        """ba_last_error() of this context: the error of the last failed call, or a note of the last solve."""
        return (self._L.ba_last_error(self._h) or b"").decode()

    def solve(self, prob: ProblemArrays) -> dict:
        s = BaSummary()
        ps = prob.struct()
        self._check(self._L.ba_solve(self._h, C.byref(ps), C.byref(s)), "ba_solve")
        return s.as_dict()

    @staticmethod
    def comm_unique_id() -> bytes:
        """RCCL unique id for ba_comm_init (rank 0 creates it, ships it to the other ranks)."""
        L = _lib.lib()
        buf = C.create_string_buffer(_lib.COMM_ID_BYTES)
        rc = L.ba_comm_unique_id(buf)
        if rc != 0:
            raise MibaError(f"ba_comm_unique_id failed ({rc}): {(L.ba_last_error(None) or b'').decode()}")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        """Make this solver one landmark shard of an nranks-way sharded window (collective)."""
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError("unique id must be BA_COMM_ID_BYTES long")
        self._check(self._L.ba_comm_init(self._h, nranks, rank, uid), "ba_comm_init")

    def comm_init_host(self, nranks: int, rank: int, allreduce) -> None:
        """Make this solver one landmark shard over a host collective instead of RCCL (ba_comm_init_host).
        ``allreduce(arr, op)`` reduces the numpy array ``arr`` (float64 or int32, a view of libmiba's
        pinned staging buffer) in place across the ranks; op is "sum", "max" or "min"."""
        ops = {0: "sum", 1: "max", 2: "min"}

        def fn(buf, count, dtype, op, user):
            try:
                ct = C.c_double if dtype == 0 else C.c_int32
                arr = np.ctypeslib.as_array((ct * int(count)).from_address(buf))
                allreduce(arr, ops[int(op)])
                return 0
            except Exception as e:  # reported through ba_last_error
                import sys
                print(f"miba host all-reduce failed: {e!r}", file=sys.stderr)
                return -1

        self._allreduce_cb = _lib.ALLREDUCE_FN(fn)  # kept alive as long as the context
        self._check(self._L.ba_comm_init_host(self._h, nranks, rank, self._allreduce_cb, None), "ba_comm_init_host")

    def iteration_log(self) -> np.ndarray:
        """Per-iteration log of the last solve (ba_iteration_log): rows 0..num_iterations of
        cost, cost_change, |gradient|, |step|, tr_ratio, tr_radius, accepted (1/0/-1), 0."""
        n = self._L.ba_iteration_log(self._h, None, 0)
        rows = np.zeros((max(n, 0), _lib.LOG_WIDTH))
        if n > 0:
            self._L.ba_iteration_log(self._h, _dptr(rows), n)
        return rows

    def set_options(self, **changes) -> None:
        for k, v in changes.items():
            setattr(self.options, k, v)
        self._check(self._L.ba_set_options(self._h, C.byref(self.options)), "ba_set_options")

    def prepare(self, prob: ProblemArrays) -> None:
        """Upload the window and build its device structure (ba_prepare)."""
        self._prepared = prob.struct()
        self._check(self._L.ba_prepare(self._h, C.byref(self._prepared)), "ba_prepare")

    def solve_prepared(self, prob: ProblemArrays) -> dict:
        """LM on the resident window from the parameters of the last prepare()."""
        s = BaSummary()
        ps = prob.struct()
        self._check(self._L.ba_solve_prepared(self._h, C.byref(ps), C.byref(s)), "ba_solve_prepared")
        return s.as_dict()

    def plan_digest(self) -> list:
        """ba_debug_plan_digest(): one FNV-1a digest per plan array of the last prepared window (as in HBM)."""
        buf = (C.c_uint64 * 64)()
        n = self._L.ba_debug_plan_digest(self._h, buf, 64)
        if n < 0:
            self._check(n, "ba_debug_plan_digest")
        return [int(buf[k]) for k in range(min(n, 64))]

    def last_prepare(self) -> dict:
        """ba_last_prepare(): whether the last prepare reused the plan, uploaded observations, its phase times and
        the reduced-solve path (bcr_path)."""
        info = BaPrepareInfo()
        self._check(self._L.ba_last_prepare(self._h, C.byref(info)), "ba_last_prepare")
        return info.as_dict()

    def kernel_stats(self) -> list:
        arr = (BaKernelStat * 32)()
        n = self._L.ba_kernel_stats(self._h, arr, 32)
        out = []
        for i in range(n):
            k = arr[i]
            out.append(dict(name=k.name.decode(), launches=k.launches, total_ms=k.total_ms,
                            bytes_per_launch=k.bytes_per_launch, flops_per_launch=k.flops_per_launch))
        return out

    def reset_kernel_stats(self) -> None:
        self._L.ba_reset_kernel_stats(self._h)

    def linearize(self, prob: ProblemArrays) -> dict:
        n = prob.n_obs
        res = np.zeros((n, 3)); jc = np.zeros((n, 3, 6)); jp = np.zeros((n, 3, 3)); jk = np.zeros((n, 2, 4))
        cost = np.zeros(1)
        ps = prob.struct()
        self._check(self._L.ba_debug_linearize(self._h, C.byref(ps), _dptr(cost), _dptr(res), _dptr(jc), _dptr(jp),
                                               _dptr(jk)), "ba_debug_linearize")
        return dict(cost=float(cost[0]), res=res, jcam=jc, jpt=jp, jint=jk)

    def camera_sums(self, prob: ProblemArrays):
        """The production camera-side pass (ba_debug_camera_sums): per active camera U (6x6), C (6x4), g (6),
        the lin record (cost, gradient norm, intrinsics block + prior) and the active camera indices."""
        ps = prob.struct()
        n = C.c_int32(0)
        self._check(self._L.ba_debug_camera_sums(self._h, C.byref(ps), C.byref(n), None, None, None),
                    "ba_debug_camera_sums")
        cd = np.zeros((max(n.value, 1), 51)); lin = np.zeros(16); ac = np.zeros(max(n.value, 1), dtype=np.int32)
        self._check(self._L.ba_debug_camera_sums(self._h, C.byref(ps), C.byref(n), _dptr(cd), _dptr(lin),
                                                 ac.ctypes.data_as(C.POINTER(C.c_int32))), "ba_debug_camera_sums")
        cd, ac = cd[: n.value], ac[: n.value]
        U = np.zeros((n.value, 6, 6))
        iu = np.triu_indices(6)
        U[:, iu[0], iu[1]] = cd[:, :21]
        U[:, iu[1], iu[0]] = cd[:, :21]
        return dict(U=U, C=cd[:, 21:45].reshape(-1, 6, 4), g=cd[:, 45:51], lin=lin, ac_cam=ac)

    def reduced_system(self, prob: ProblemArrays, radius: float = 0.0):
        ps = prob.struct()
        n = C.c_int32(0)
        self._check(self._L.ba_debug_reduced_system(self._h, C.byref(ps), radius, C.byref(n), None, None),
                    "ba_debug_reduced_system")
        S = np.zeros((n.value, n.value)); rhs = np.zeros(n.value)
        self._check(self._L.ba_debug_reduced_system(self._h, C.byref(ps), radius, C.byref(n), _dptr(S), _dptr(rhs)),
                    "ba_debug_reduced_system")
        return S, rhs
