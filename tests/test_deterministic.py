"""ba_options.deterministic = 1: no float atomics anywhere on the LM path (the Schur tiles write
per-tile slabs that k_schur_gather sums in tile order, the overflow Schur terms run in one
workgroup in a fixed order), so two solves of the same window are bitwise identical — summary,
iteration log, cameras, points, intrinsics — as Ceres' single-threaded solve is. The result still
matches the oracle and the default (atomic) mode to rounding."""
import numpy as np
import pytest

from miba import synthetic
from oracle import oracle

pytestmark = pytest.mark.gpu

CASES = {
    "c2": None,
    "wide_overflow_dup": dict(n_cams=30, n_points=150, obs_per_point=(6, 16), seed=5, rot_noise=0.005, dup_frac=0.05),
    "shuffled_bad_depth": dict(n_cams=12, n_points=200, obs_per_point=(2, 6), seed=3, shuffle_obs=True,
                               bad_depth_frac=0.05),
}


def _prob(case):
    return synthetic.make_config("C2") if CASES[case] is None else synthetic.make_problem(**CASES[case])


def _solve(p, deterministic, iters=8):
    from miba.solver import Solver
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    q = p.copy()
    with Solver(device=0, minimizer_progress_to_stdout=0, max_num_iterations=iters, deterministic=deterministic,
                **no_tol) as s:
        sm = s.solve(q)
        log = s.iteration_log()
    return q, sm, log


@pytest.mark.parametrize("case", sorted(CASES))
def test_deterministic_solves_are_bitwise_identical(case):
    p = _prob(case)
    q1, s1, l1 = _solve(p, 1)
    q2, s2, l2 = _solve(p, 1)
    assert s1["final_cost"] == s2["final_cost"] and s1["initial_cost"] == s2["initial_cost"]
    assert s1["num_iterations"] == s2["num_iterations"] == 8
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(q1.cams, q2.cams)
    np.testing.assert_array_equal(q1.points, q2.points)
    np.testing.assert_array_equal(q1.intr, q2.intr)
    # same solve as the default mode and the oracle, to rounding
    qa, sa, _ = _solve(p, 0)
    assert abs(s1["final_cost"] - sa["final_cost"]) <= 1e-10 * sa["final_cost"]
    np.testing.assert_allclose(q1.cams, qa.cams, rtol=0, atol=1e-8)
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=8, **no_tol))
    assert abs(s1["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (s1, so)


@pytest.mark.parametrize("case", ["c2", "wide_overflow_dup_f32"])
def test_obs32_records_match_f64_arrays_bitwise(case, monkeypatch):
    """A window whose pixels / depths are all f32 values (the reference's sensor types) is streamed as 16-byte
    obs32 records; the f64 arrays (MIBA_OBS32=0) widen the same values, so the two deterministic solves agree
    bit for bit."""
    p = synthetic.make_config("C2") if case == "c2" else synthetic.make_problem(
        **CASES["wide_overflow_dup"], sensor_f32=True)
    assert np.array_equal(p.obs_uv.astype(np.float32).astype(np.float64), p.obs_uv)
    q1, s1, l1 = _solve(p, 1)
    monkeypatch.setenv("MIBA_OBS32", "0")
    q2, s2, l2 = _solve(p, 1)
    assert s1["final_cost"] == s2["final_cost"] and s1["num_iterations"] == s2["num_iterations"]
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(q1.cams, q2.cams)
    np.testing.assert_array_equal(q1.points, q2.points)
    np.testing.assert_array_equal(q1.intr, q2.intr)
