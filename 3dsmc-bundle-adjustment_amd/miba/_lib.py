"""Loader for libmiba.so (the HIP product library). No fallback: if the
library is missing or no GPU is present, calls raise instead of silently
running something else."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from .capi import BaKernelStat, BaOptions, BaPrepareInfo, BaProblem, BaSummary

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MIBA_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libmiba.so")  # override: A/B builds

# exported symbols, exactly those declared in include/ba.h and include/ba_io.h
EXPORTS = (
    "ba_api_version", "ba_build_info", "ba_default_options", "ba_create", "ba_destroy", "ba_last_error", "ba_set_options",
    "ba_solve", "ba_prepare", "ba_solve_prepared", "ba_kernel_stats", "ba_reset_kernel_stats",
    "ba_debug_linearize", "ba_debug_reduced_system", "ba_debug_camera_sums", "ba_debug_plan_digest", "ba_comm_unique_id", "ba_comm_init", "ba_comm_init_host",
    "ba_iteration_log", "ba_last_prepare",
    "ba_problem_write", "ba_problem_read_dims", "ba_problem_read", "ba_bal_read_dims", "ba_bal_read", "ba_bal_write",
)
COMM_ID_BYTES = 128  # BA_COMM_ID_BYTES
LOG_WIDTH = 8  # BA_LOG_WIDTH
# ba_allreduce_fn: int32 (*)(void* buf, int64 count, int32 dtype, int32 op, void* user)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p)

_lib = None


def build(verbose: bool = False) -> str:
    """Compile libmiba for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    jobs = os.environ.get("MAX_JOBS", "4")
    out = subprocess.run(["make", "-C", PKG_DIR, f"-j{min(int(jobs), 16)}"], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"libmiba build failed:\n{out.stdout}\n{out.stderr}")
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libmiba.so not found at {LIB_PATH}; run __graft_entry__.build() or `make -C {PKG_DIR}`")
    L = C.CDLL(LIB_PATH)
    dp = C.POINTER(C.c_double)
    L.ba_api_version.restype = C.c_int32
    L.ba_build_info.restype = C.c_char_p
    L.ba_default_options.argtypes = [C.POINTER(BaOptions)]
    L.ba_create.argtypes = [C.POINTER(BaOptions)]
    L.ba_create.restype = C.c_void_p
    L.ba_destroy.argtypes = [C.c_void_p]
    L.ba_last_error.argtypes = [C.c_void_p]
    L.ba_last_error.restype = C.c_char_p
    L.ba_set_options.argtypes = [C.c_void_p, C.POINTER(BaOptions)]
    L.ba_set_options.restype = C.c_int32
    L.ba_solve.argtypes = [C.c_void_p, C.POINTER(BaProblem), C.POINTER(BaSummary)]
    L.ba_solve.restype = C.c_int32
    L.ba_prepare.argtypes = [C.c_void_p, C.POINTER(BaProblem)]
    L.ba_prepare.restype = C.c_int32
    L.ba_solve_prepared.argtypes = [C.c_void_p, C.POINTER(BaProblem), C.POINTER(BaSummary)]
    L.ba_solve_prepared.restype = C.c_int32
    L.ba_kernel_stats.argtypes = [C.c_void_p, C.POINTER(BaKernelStat), C.c_int32]
    L.ba_kernel_stats.restype = C.c_int32
    L.ba_reset_kernel_stats.argtypes = [C.c_void_p]
    L.ba_debug_linearize.argtypes = [C.c_void_p, C.POINTER(BaProblem), dp, dp, dp, dp, dp]
    L.ba_debug_linearize.restype = C.c_int32
    L.ba_debug_reduced_system.argtypes = [C.c_void_p, C.POINTER(BaProblem), C.c_double, C.POINTER(C.c_int32), dp, dp]
    L.ba_debug_reduced_system.restype = C.c_int32
    L.ba_debug_camera_sums.argtypes = [C.c_void_p, C.POINTER(BaProblem), C.POINTER(C.c_int32), dp, dp,
                                       C.POINTER(C.c_int32)]
    L.ba_debug_camera_sums.restype = C.c_int32
    L.ba_debug_plan_digest.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]
    L.ba_debug_plan_digest.restype = C.c_int32
    L.ba_comm_unique_id.argtypes = [C.c_char_p]
    L.ba_comm_unique_id.restype = C.c_int32
    L.ba_comm_init.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p]
    L.ba_comm_init.restype = C.c_int32
    L.ba_comm_init_host.argtypes = [C.c_void_p, C.c_int32, C.c_int32, ALLREDUCE_FN, C.c_void_p]
    L.ba_comm_init_host.restype = C.c_int32
    L.ba_iteration_log.argtypes = [C.c_void_p, dp, C.c_int32]
    L.ba_last_prepare.argtypes = [C.c_void_p, C.POINTER(BaPrepareInfo)]
    L.ba_last_prepare.restype = C.c_int32
    L.ba_iteration_log.restype = C.c_int32
    ip = C.POINTER(C.c_int32)
    L.ba_problem_write.argtypes = [C.c_char_p, C.POINTER(BaProblem), C.POINTER(BaOptions)]
    L.ba_problem_read_dims.argtypes = [C.c_char_p, ip, ip, ip]
    L.ba_problem_read.argtypes = [C.c_char_p, C.POINTER(BaProblem), C.POINTER(BaOptions)]
    L.ba_bal_read_dims.argtypes = [C.c_char_p, ip, ip, ip]
    L.ba_bal_read.argtypes = [C.c_char_p, C.POINTER(BaProblem)]
    L.ba_bal_write.argtypes = [C.c_char_p, C.POINTER(BaProblem)]
    for f in ("ba_problem_write", "ba_problem_read_dims", "ba_problem_read", "ba_bal_read_dims", "ba_bal_read",
              "ba_bal_write"):
        getattr(L, f).restype = C.c_int32
    _lib = L
    return L
