"""ctypes mirror of ``include/ba.h`` (the libmiba C-ABI).

The structures here are byte-for-byte the C structs; ``tests/test_capi.py``
checks their sizes against the compiled library. ``ProblemArrays`` keeps the
numpy buffers a ``ba_problem`` points into alive and contiguous.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

BA_OK = 0
BA_E_INVALID = -1
BA_E_DEVICE = -2
BA_E_NOMEM = -3
BA_E_COMM = -4
BA_E_INTERNAL = -5

BA_CONVERGENCE = 0
BA_NO_CONVERGENCE = 1
BA_FAILURE = 2

TERMINATION_NAMES = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE"}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class BaOptions(C.Structure):
    """Mirror of ``ba_options`` (ceresGlobalProblem, BundleAdjustmentConfig.h:44-69)."""

    _fields_ = [
        ("hub_p_repr", C.c_double),
        ("hub_p_unpr", C.c_double),
        ("weight_intrinsics", C.c_double),
        ("weight_unpr", C.c_double),
        ("max_num_iterations", C.c_int32),
        ("minimizer_progress_to_stdout", C.c_int32),
        ("eta", C.c_double),
        ("initial_trust_region_radius", C.c_double),
        ("max_trust_region_radius", C.c_double),
        ("min_trust_region_radius", C.c_double),
        ("min_relative_decrease", C.c_double),
        ("min_lm_diagonal", C.c_double),
        ("max_lm_diagonal", C.c_double),
        ("max_num_consecutive_invalid_steps", C.c_int32),
        ("jacobi_scaling", C.c_int32),
        ("function_tolerance", C.c_double),
        ("gradient_tolerance", C.c_double),
        ("parameter_tolerance", C.c_double),
        ("device", C.c_int32),
        ("deterministic", C.c_int32),
        ("profile_kernels", C.c_int32),
        ("profile_mask", C.c_int32),
        ("shard_min_obs", C.c_int32),
        ("small_window", C.c_int32),
        ("rebuild_plan", C.c_int32),
        ("reserved", C.c_int32 * 1),
    ]


class BaProblem(C.Structure):
    """Mirror of ``ba_problem`` (the flattened window of windowOptimize)."""

    _fields_ = [
        ("n_cams", C.c_int32),
        ("n_points", C.c_int32),
        ("n_obs", C.c_int32),
        ("fixed_cam", C.c_int32),
        ("cams", _dp),
        ("points", _dp),
        ("intr", _dp),
        ("intr_prior", _dp),
        ("obs_cam", _ip),
        ("obs_pt", _ip),
        ("obs_uv", _dp),
        ("obs_depth", _dp),
    ]


class BaSummary(C.Structure):
    """Mirror of ``ba_summary`` (subset of ceres::Solver::Summary). BA_API_VERSION 2: ``struct_size`` is set to
    this mirror's size on construction (the library writes no more than that)."""

    _fields_ = [
        ("struct_size", C.c_int32),
        ("reserved0", C.c_int32),
        ("initial_cost", C.c_double),
        ("final_cost", C.c_double),
        ("num_successful_steps", C.c_int32),
        ("num_unsuccessful_steps", C.c_int32),
        ("num_iterations", C.c_int32),
        ("termination_type", C.c_int32),
        ("num_obs_admissible", C.c_int32),
        ("num_active_cams", C.c_int32),
        ("num_active_points", C.c_int32),
        ("reduced_system_size", C.c_int32),
        ("linear_solver", C.c_int32),
        ("camera_band", C.c_int32),
        ("time_setup_ms", C.c_double),
        ("time_lm_ms", C.c_double),
        ("time_linearize_ms", C.c_double),
        ("time_schur_ms", C.c_double),
        ("time_factor_ms", C.c_double),
        ("time_update_ms", C.c_double),
        ("time_total_ms", C.c_double),
        ("message", C.c_char * 160),
    ]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if not self.struct_size:
            self.struct_size = C.sizeof(type(self))

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_
             if name not in ("message", "struct_size", "reserved0")}
        d["message"] = self.message.decode(errors="replace")
        d["termination"] = TERMINATION_NAMES.get(self.termination_type, str(self.termination_type))
        return d


class BaKernelStat(C.Structure):
    """Mirror of ``ba_kernel_stat``."""

    _fields_ = [
        ("name", C.c_char * 32),
        ("launches", C.c_int32),
        ("reserved", C.c_int32),
        ("total_ms", C.c_double),
        ("bytes_per_launch", C.c_double),
        ("flops_per_launch", C.c_double),
    ]


class BaPrepareInfo(C.Structure):
    """Mirror of ``ba_prepare_info`` (what the last prepare did; ba_last_prepare). ``struct_size`` is set to this
    mirror's size on construction."""

    _fields_ = [
        ("struct_size", C.c_int32),
        ("plan_reused", C.c_int32),
        ("obs_uploaded", C.c_int32),
        ("host_threads", C.c_int32),
        ("bcr_path", C.c_int32),
        ("compare_ms", C.c_double),
        ("plan_ms", C.c_double),
        ("upload_ms", C.c_double),
        ("total_ms", C.c_double),
        ("lin_path", C.c_int32),
        ("plan_device", C.c_int32),
        ("tail", C.c_int32),
        ("bsfin", C.c_int32),
    ]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if not self.struct_size:
            self.struct_size = C.sizeof(type(self))

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "struct_size"}


def default_options_py() -> BaOptions:
    """Pure-Python defaults (used only where no compiled library is loaded)."""
    o = BaOptions()
    o.hub_p_repr = 1e-3
    o.hub_p_unpr = 1e-3
    o.weight_intrinsics = 1e-6
    o.weight_unpr = 10.0
    o.max_num_iterations = 75
    o.minimizer_progress_to_stdout = 1
    o.eta = 1e-6
    o.initial_trust_region_radius = 1e4
    o.max_trust_region_radius = 1e16
    o.min_trust_region_radius = 1e-32
    o.min_relative_decrease = 1e-3
    o.min_lm_diagonal = 1e-6
    o.max_lm_diagonal = 1e32
    o.max_num_consecutive_invalid_steps = 5
    o.jacobi_scaling = 1
    o.function_tolerance = 1e-6
    o.gradient_tolerance = 1e-10
    o.parameter_tolerance = 1e-8
    o.device = -1
    o.deterministic = 0  # = ba_default_options
    o.shard_min_obs = 262144
    o.small_window = 0
    o.rebuild_plan = 0  # reuse the host plan of an unchanged window structure
    return o


@dataclass
class ProblemArrays:
    """Owning numpy view of one window problem; ``.struct()`` gives a ``BaProblem``."""

    cams: np.ndarray  # (n_cams, 7) qx qy qz qw tx ty tz
    points: np.ndarray  # (n_points, 3)
    intr: np.ndarray  # (4,)
    intr_prior: np.ndarray  # (4,)
    obs_cam: np.ndarray  # (n_obs,) int32
    obs_pt: np.ndarray  # (n_obs,) int32
    obs_uv: np.ndarray  # (n_obs, 2)
    obs_depth: np.ndarray  # (n_obs,)
    fixed_cam: int = 0
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        self.cams = np.ascontiguousarray(self.cams, dtype=np.float64).reshape(-1, 7)
        self.points = np.ascontiguousarray(self.points, dtype=np.float64).reshape(-1, 3)
        self.intr = np.ascontiguousarray(self.intr, dtype=np.float64).reshape(4)
        self.intr_prior = np.ascontiguousarray(self.intr_prior, dtype=np.float64).reshape(4)
        self.obs_cam = np.ascontiguousarray(self.obs_cam, dtype=np.int32).reshape(-1)
        self.obs_pt = np.ascontiguousarray(self.obs_pt, dtype=np.int32).reshape(-1)
        self.obs_uv = np.ascontiguousarray(self.obs_uv, dtype=np.float64).reshape(-1, 2)
        self.obs_depth = np.ascontiguousarray(self.obs_depth, dtype=np.float64).reshape(-1)

    @property
    def n_cams(self) -> int:
        return self.cams.shape[0]

    @property
    def n_points(self) -> int:
        return self.points.shape[0]

    @property
    def n_obs(self) -> int:
        return self.obs_cam.shape[0]

    def copy(self) -> "ProblemArrays":
        return ProblemArrays(
            self.cams.copy(), self.points.copy(), self.intr.copy(), self.intr_prior.copy(),
            self.obs_cam.copy(), self.obs_pt.copy(), self.obs_uv.copy(), self.obs_depth.copy(),
            int(self.fixed_cam), dict(self.meta),
        )

    def struct(self) -> BaProblem:
        p = BaProblem()
        p.n_cams = self.n_cams
        p.n_points = self.n_points
        p.n_obs = self.n_obs
        p.fixed_cam = int(self.fixed_cam)
        p.cams = self.cams.ctypes.data_as(_dp)
        p.points = self.points.ctypes.data_as(_dp)
        p.intr = self.intr.ctypes.data_as(_dp)
        p.intr_prior = self.intr_prior.ctypes.data_as(_dp)
        p.obs_cam = self.obs_cam.ctypes.data_as(_ip)
        p.obs_pt = self.obs_pt.ctypes.data_as(_ip)
        p.obs_uv = self.obs_uv.ctypes.data_as(_dp)
        p.obs_depth = self.obs_depth.ctypes.data_as(_dp)
        return p

    def save_npz(self, path) -> None:
        np.savez(path, cams=self.cams, points=self.points, intr=self.intr, intr_prior=self.intr_prior,
                 obs_cam=self.obs_cam, obs_pt=self.obs_pt, obs_uv=self.obs_uv, obs_depth=self.obs_depth,
                 fixed_cam=np.int32(self.fixed_cam))

    @staticmethod
    def load_npz(path) -> "ProblemArrays":
        z = np.load(path, allow_pickle=False)
        return ProblemArrays(z["cams"], z["points"], z["intr"], z["intr_prior"], z["obs_cam"], z["obs_pt"],
                             z["obs_uv"], z["obs_depth"], int(z["fixed_cam"]))
