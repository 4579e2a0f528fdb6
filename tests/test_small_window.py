"""The small-window path (ba_small.hip, BA_LS_SMALL): iteration 0 and the whole LM loop of
ceres::Solve (OptimizationUtils.cpp:300) in one launch of one workgroup, for the reference's own
window sizes (10-keyframe windows, BundleAdjustmentConfig.h:52-53; C1 of BASELINE.json).

Against the CPU oracle on the same seeded windows: the termination, the iteration count, the accept /
reject sequence of the iteration log (identical), the cost of every iteration (1e-9 relative for the
first three, 1e-6 after) and the final cost (<= 1e-6 relative, north_star's bound). Against the
multi-launch path (small_window = 0, the default) the same. Fixed-order reductions only: two solves of
one window are bitwise identical."""
import numpy as np
import pytest

from miba import synthetic
from oracle import oracle

pytestmark = pytest.mark.gpu

BA_LS_SMALL = 3

CASES = {
    "c1": dict(synthetic.CONFIGS["C1"]),
    "tum_like": dict(n_cams=10, n_points=300, obs_per_point=(2, 3), seed=1),
    "ten_obs": dict(n_cams=12, n_points=400, obs_per_point=(3, 10), seed=11),
    "shuffled_bad_depth": dict(n_cams=12, n_points=200, obs_per_point=(2, 6), seed=3, shuffle_obs=True,
                               bad_depth_frac=0.05),
    "no_gauge_cam_obs": dict(n_cams=8, n_points=120, obs_per_point=(2, 4), seed=4, fixed_cam=3),
    "dup_obs": dict(n_cams=10, n_points=200, obs_per_point=(2, 5), seed=6, dup_frac=0.05),
    "sixteen_cams": dict(n_cams=16, n_points=900, obs_per_point=(2, 8), seed=12),  # npad 96, the cap
    "two_cams": dict(n_cams=2, n_points=50, obs_per_point=(2, 2), seed=13),
}


def _solve(p, **opts):
    from miba.solver import Solver
    opts.setdefault("small_window", 1)
    with Solver(minimizer_progress_to_stdout=0, **opts) as s:
        sm = s.solve(p)
        log = s.iteration_log()
    return sm, log


@pytest.mark.parametrize("case", sorted(CASES))
def test_small_window_matches_oracle(case):
    p = synthetic.make_problem(**CASES[case])
    q = p.copy()
    sg, log = _solve(p)
    assert sg["linear_solver"] == BA_LS_SMALL, sg
    so, tr = oracle.solve_trace(q)
    assert sg["termination"] == so["termination"], (sg["message"], so["message"])
    assert sg["num_iterations"] == so["num_iterations"]
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert sg["num_unsuccessful_steps"] == so["num_unsuccessful_steps"]
    np.testing.assert_array_equal(log[:, 6], tr[:, 6])
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-12 * so["initial_cost"]
    np.testing.assert_allclose(log[:3, 0], tr[:3, 0], rtol=1e-9)
    np.testing.assert_allclose(log[:, 0], tr[:, 0], rtol=1e-6)
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sg, so)
    assert np.max(np.abs(p.points - q.points)) < 1e-6
    assert np.max(np.abs(p.cams - q.cams)) < 1e-6
    assert np.max(np.abs(p.intr - q.intr)) < 1e-4


@pytest.mark.parametrize("case", ["c1", "shuffled_bad_depth", "dup_obs"])
def test_small_window_matches_multi_launch(case):
    p = synthetic.make_problem(**CASES[case])
    q = p.copy()
    sa, la = _solve(p)
    sb, lb = _solve(q, small_window=0)
    assert sa["linear_solver"] == BA_LS_SMALL and sb["linear_solver"] != BA_LS_SMALL
    assert sa["num_iterations"] == sb["num_iterations"]
    np.testing.assert_array_equal(la[:, 6], lb[:, 6])
    np.testing.assert_allclose(la[:, 0], lb[:, 0], rtol=1e-9)
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-9 * sb["final_cost"]
    assert np.max(np.abs(p.points - q.points)) < 1e-8


def test_small_window_bitwise_reproducible():
    p0 = synthetic.make_problem(**CASES["ten_obs"])
    p1, p2 = p0.copy(), p0.copy()
    s1, l1 = _solve(p1)
    s2, l2 = _solve(p2)
    assert s1["linear_solver"] == BA_LS_SMALL
    assert s1["final_cost"] == s2["final_cost"]
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(p1.cams, p2.cams)
    np.testing.assert_array_equal(p1.points, p2.points)
    np.testing.assert_array_equal(p1.intr, p2.intr)


def test_small_window_prepared_resolve_and_cap():
    """ba_prepare once, ba_solve_prepared per frame (main.cpp:163-168); a window above the cap (17
    active cameras: npad 112 > 96) takes the multi-launch path."""
    from miba.solver import Solver
    p = synthetic.make_config("C1")
    with Solver(minimizer_progress_to_stdout=0, small_window=1) as s:
        s.prepare(p)
        a = s.solve_prepared(p.copy())
        b = s.solve_prepared(p.copy())
    assert a["linear_solver"] == BA_LS_SMALL and a["final_cost"] == b["final_cost"]
    big = synthetic.make_problem(n_cams=18, n_points=300, obs_per_point=(2, 4), seed=14)
    sg, _ = _solve(big)
    assert sg["linear_solver"] != BA_LS_SMALL


def test_small_window_all_inadmissible_solves_prior():
    """Every depth <= 1e-15: only the IntrinsicsPrior block remains (OptimizationUtils.cpp:236-241)."""
    p = synthetic.make_problem(**CASES["tum_like"])
    p.obs_depth[:] = 0.0
    p.intr[:] = p.intr_prior + np.array([3.0, -2.0, 1.0, 0.5])
    q = p.copy()
    sg, _ = _solve(p)
    so = oracle.solve(q)
    assert sg["termination"] == so["termination"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * max(so["final_cost"], 1e-300)
    np.testing.assert_allclose(p.intr, q.intr, rtol=1e-9)
