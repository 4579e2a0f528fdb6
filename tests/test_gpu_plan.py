"""The device plan (csrc/ba_dplan.hip) builds exactly the host plan (csrc/ba_plan.cpp).

ba_prepare's plan passes (admissibility, point lists sorted on (active camera + 1, observation index), the camera-
major and active point orders, the Schur tiles, chunks, segments and envelope) run on the device for windows of
>= 16k observations; MIBA_DEVICE_PLAN=1 forces them on any window that fits, =0 keeps the host plan. Checked
here, on windows that exercise every branch of the plan (shuffled and duplicate observations, inadmissible depths,
non-f32 pixels, unobserved cameras and points, no gauge, long point lists that take the workgroup sort, a list too
long for it that hands the window to the host plan, an out-of-range index): ba_debug_plan_digest — one FNV-1a
digest per plan array as the kernels read it from HBM — is the same for both plans, and so is a deterministic
solve, bitwise."""
import os

import numpy as np
import pytest

from miba import synthetic
from miba.capi import ProblemArrays

pytestmark = pytest.mark.gpu

NO_TOL = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)


def _with_env(val, fn):
    old = os.environ.get("MIBA_DEVICE_PLAN")
    os.environ["MIBA_DEVICE_PLAN"] = val
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop("MIBA_DEVICE_PLAN", None)
        else:
            os.environ["MIBA_DEVICE_PLAN"] = old


def _plan(p, mode, solve_iters=0):
    from miba.solver import Solver

    def run():
        with Solver(device=0, minimizer_progress_to_stdout=0, deterministic=1, rebuild_plan=1,
                    max_num_iterations=max(solve_iters, 1), **NO_TOL) as s:
            q = p.copy()
            s.prepare(q)
            info = s.last_prepare()
            dig = s.plan_digest()
            out = None
            if solve_iters:
                sm = s.solve_prepared(q)
                out = (q.cams.copy(), q.points.copy(), q.intr.copy(), sm["final_cost"])
            return dig, info, out
    return _with_env(mode, run)


def _subset(p, keep):
    return ProblemArrays(p.cams, p.points, p.intr, p.intr_prior, p.obs_cam[keep], p.obs_pt[keep], p.obs_uv[keep],
                         p.obs_depth[keep], p.fixed_cam)


def _windows():
    w = {}
    w["c2"] = synthetic.make_config("C2")
    w["c3"] = synthetic.make_config("C3")
    w["shuffled_dup_bad"] = synthetic.make_problem(40, 3000, (2, 12), seed=3, shuffle_obs=True, dup_frac=0.05,
                                                   bad_depth_frac=0.05)
    w["long_lists"] = synthetic.make_problem(70, 400, (17, 60), seed=4, shuffle_obs=True, dup_frac=0.02,
                                             sensor_f32=True)
    p = synthetic.make_problem(30, 2000, (2, 8), seed=5, sensor_f32=True)
    keep = ~np.isin(p.obs_cam, [3, 17]) & ~np.isin(p.obs_pt, np.arange(0, 2000, 7))
    w["unobserved"] = _subset(p, keep)
    p = synthetic.make_problem(25, 1500, (2, 10), seed=6, sensor_f32=True)
    p.fixed_cam = -1
    w["no_gauge"] = p
    p = synthetic.make_problem(25, 1500, (2, 10), seed=7, sensor_f32=True)
    p.fixed_cam = 12
    w["mid_gauge"] = p
    return w


WINDOWS = _windows()


@pytest.mark.parametrize("name", sorted(WINDOWS))
def test_device_plan_matches_the_host_plan(name):
    p = WINDOWS[name]
    dh, ih, _ = _plan(p, "0")
    dd, idv, _ = _plan(p, "1")
    assert ih["plan_device"] == 0 and idv["plan_device"] == 1
    assert len(dh) == len(dd) > 0
    assert dh == dd


def test_device_plan_on_the_bench_window():
    """C4 (1M observations) takes the device plan by default; its digests are the host plan's."""
    p = synthetic.make_config("C4")
    dh, ih, _ = _plan(p, "0")
    dd, idv, _ = _plan(p, "auto")
    assert idv["plan_device"] == 1 and ih["plan_device"] == 0
    assert dh == dd


@pytest.mark.parametrize("name", ["shuffled_dup_bad", "c3"])
def test_device_plan_solve_is_bitwise_the_host_plans(name):
    p = WINDOWS[name]
    _, _, a = _plan(p, "0", solve_iters=5)
    _, _, b = _plan(p, "1", solve_iters=5)
    for x, y in zip(a[:3], b[:3]):
        np.testing.assert_array_equal(x, y)
    assert a[3] == b[3]


def test_a_list_too_long_for_the_device_sort_takes_the_host_plan():
    p = synthetic.make_problem(20, 300, (2, 6), seed=8, sensor_f32=True)
    n = 4200  # > DP_LONG_MAX links of point 0 to camera 1
    q = ProblemArrays(p.cams, p.points, p.intr, p.intr_prior, np.concatenate([p.obs_cam, np.full(n, 1)]),
                      np.concatenate([p.obs_pt, np.zeros(n, np.int32)]),
                      np.concatenate([p.obs_uv, np.tile(p.obs_uv[:1], (n, 1))]),
                      np.concatenate([p.obs_depth, np.full(n, 2.0)]), p.fixed_cam)
    dh, _, _ = _plan(q, "0")
    dd, idv, _ = _plan(q, "1")
    assert idv["plan_device"] == 0
    assert dh == dd


def test_out_of_range_index_is_rejected_by_both_plans():
    from miba.solver import MibaError, Solver
    p = synthetic.make_problem(10, 200, (2, 4), seed=9)
    p.obs_pt[17] = p.n_points + 3

    def run():
        with Solver(device=0, minimizer_progress_to_stdout=0) as s:
            with pytest.raises(MibaError, match="observation index out of range"):
                s.prepare(p.copy())
    _with_env("0", run)
    _with_env("1", run)
