"""Plan cache of ba_prepare (ba_options.rebuild_plan = 0, the default).

The reference re-optimises the same window on every processed frame until the next keyframe arrives
(main.cpp:163-168), and windowOptimize rebuilds its ceres::Problem each time
(OptimizationUtils.cpp:218). libmiba keeps the host plan and the device structure of the last window and, when
the next window has the same structure (sizes, gauge, obs_cam, obs_pt, admissibility mask), uploads only the
parameters and the observation values that changed (ba_solver.cpp prepare_reuse).

Checked here: a reused plan gives bitwise the same deterministic solve as a fresh context; changed pixel / depth
values on the same structure are re-gathered; every structural change (one obs_pt, one admissibility flip, the
gauge, a value that is no longer an exact f32 on an obs32 plan, the deterministic option) rebuilds."""
import numpy as np
import pytest

from miba import synthetic

pytestmark = pytest.mark.gpu

NO_TOL = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)


def _solver(**kw):
    from miba.solver import Solver
    return Solver(device=0, minimizer_progress_to_stdout=0, **kw)


def _fresh(p, iters=6, **kw):
    q = p.copy()
    with _solver(max_num_iterations=iters, deterministic=1, **NO_TOL, **kw) as s:
        sm = s.solve(q)
        log = s.iteration_log()
        info = s.last_prepare()
    assert info["plan_reused"] == 0
    return q, sm, log


def _same(a, b):
    (qa, sa, la), (qb, sb, lb) = a, b
    assert sa["final_cost"] == sb["final_cost"] and sa["initial_cost"] == sb["initial_cost"]
    assert sa["num_iterations"] == sb["num_iterations"]
    np.testing.assert_array_equal(la, lb)
    np.testing.assert_array_equal(qa.cams, qb.cams)
    np.testing.assert_array_equal(qa.points, qb.points)
    np.testing.assert_array_equal(qa.intr, qb.intr)


CASES = {
    "c2": None,
    "shuffled_bad_depth": dict(n_cams=12, n_points=200, obs_per_point=(2, 6), seed=3, shuffle_obs=True,
                               bad_depth_frac=0.05, sensor_f32=True),
    "wide_overflow_dup": dict(n_cams=30, n_points=150, obs_per_point=(6, 16), seed=5, rot_noise=0.005, dup_frac=0.05),
}


def _prob(case):
    return synthetic.make_config("C2") if CASES[case] is None else synthetic.make_problem(**CASES[case])


@pytest.mark.parametrize("case", sorted(CASES))
def test_repeated_window_reuses_the_plan_bitwise(case):
    """The per-frame re-solve: the same window again (its solved parameters fed back in, as the reference's
    keyframes and map hold them after the previous call), and the original window once more."""
    p = _prob(case)
    with _solver(max_num_iterations=6, deterministic=1, **NO_TOL) as s:
        q1 = p.copy()
        s.solve(q1)
        assert s.last_prepare()["plan_reused"] == 0
        # 1) the solved window again: same structure, new parameters
        q2 = q1.copy()
        s2 = s.solve(q2)
        i2 = s.last_prepare()
        l2 = s.iteration_log()
        # 2) the original window: the same parameters as the first call
        q3 = p.copy()
        s3 = s.solve(q3)
        i3 = s.last_prepare()
        l3 = s.iteration_log()
    assert i2["plan_reused"] == 1 and i2["obs_uploaded"] == 0 and i2["plan_ms"] == 0.0, i2
    assert i3["plan_reused"] == 1 and i3["obs_uploaded"] == 0, i3
    _same((q2, s2, l2), _fresh(q1))
    _same((q3, s3, l3), _fresh(p))


def test_changed_values_on_the_same_structure_are_regathered():
    p = _prob("c2")
    rng = np.random.default_rng(7)
    r = p.copy()
    k = rng.choice(r.n_obs, size=r.n_obs // 50, replace=False)
    r.obs_uv[k] += np.float32(0.25)  # still exact f32 values (the window stays obs32)
    r.obs_uv[:] = r.obs_uv.astype(np.float32).astype(np.float64)
    r.obs_depth[k[:10]] = (r.obs_depth[k[:10]] * 1.01).astype(np.float32).astype(np.float64)
    with _solver(max_num_iterations=6, deterministic=1, **NO_TOL) as s:
        s.solve(p.copy())
        q = r.copy()
        sm = s.solve(q)
        info = s.last_prepare()
        log = s.iteration_log()
    assert info["plan_reused"] == 1 and info["obs_uploaded"] == 1, info
    _same((q, sm, log), _fresh(r))


def _mut_obs_pt(p):
    k = int(np.nonzero(p.obs_depth > 1e-15)[0][5])
    p.obs_pt[k] = (p.obs_pt[k] + 1) % p.n_points


def _mut_adm(p):
    k = int(np.nonzero(p.obs_depth > 1e-15)[0][11])
    p.obs_depth[k] = 0.0


def _mut_fixed(p):
    p.fixed_cam = 1


def _mut_not_f32(p):
    k = int(np.nonzero(p.obs_depth > 1e-15)[0][3])
    p.obs_uv[k, 0] += 1e-9  # no longer an f32 value: the obs32 plan must go


@pytest.mark.parametrize("mut", [_mut_obs_pt, _mut_adm, _mut_fixed, _mut_not_f32], ids=lambda f: f.__name__[5:])
def test_structural_change_rebuilds(mut):
    p = _prob("shuffled_bad_depth")
    r = p.copy()
    mut(r)
    with _solver(max_num_iterations=6, deterministic=1, **NO_TOL) as s:
        s.solve(p.copy())
        q = r.copy()
        sm = s.solve(q)
        info = s.last_prepare()
        log = s.iteration_log()
    assert info["plan_reused"] == 0, info
    _same((q, sm, log), _fresh(r))


def test_rebuild_plan_option_and_deterministic_switch():
    p = _prob("shuffled_bad_depth")
    with _solver(max_num_iterations=4, rebuild_plan=1, **NO_TOL) as s:
        s.solve(p.copy())
        s.solve(p.copy())
        assert s.last_prepare()["plan_reused"] == 0
        s.set_options(rebuild_plan=0)
        s.solve(p.copy())
        assert s.last_prepare()["plan_reused"] == 1
        s.set_options(deterministic=1)  # a key change: deterministic slabs need their own plan
        s.solve(p.copy())
        assert s.last_prepare()["plan_reused"] == 0
        s.solve(p.copy())
        assert s.last_prepare()["plan_reused"] == 1


def test_prepare_then_solve_prepared_on_a_reused_plan():
    """ba_prepare + ba_solve_prepared (the bench's split form) behave the same on a reused plan."""
    p = _prob("c2")
    with _solver(max_num_iterations=5, deterministic=1, **NO_TOL) as s:
        s.prepare(p.copy())
        s.solve_prepared(p.copy())
        s.prepare(p.copy())
        info = s.last_prepare()
        q = p.copy()
        sm = s.solve_prepared(q)
        log = s.iteration_log()
    assert info["plan_reused"] == 1 and info["total_ms"] > 0
    _same((q, sm, log), _fresh(p, iters=5))


@pytest.mark.parametrize("change", [dict(weight_unpr=3.0), dict(hub_p_repr=2e-3, hub_p_unpr=5e-4),
                                    dict(weight_intrinsics=1e-4), dict(min_lm_diagonal=1e-2)],
                         ids=["weight_unpr", "huber", "weight_intrinsics", "min_lm_diagonal"])
def test_changed_cost_options_on_a_reused_plan(change):
    """the plan cache keys the structure only, so the cost constants (weights, Huber scales, LM
    diagonal bounds) must follow ba_set_options on the reuse path: solve, change an option, solve the same window
    again (plan reused) and compare with a fresh context that starts with the changed options."""
    p = _prob("shuffled_bad_depth")
    with _solver(max_num_iterations=6, deterministic=1, **NO_TOL) as s:
        s.solve(p.copy())
        s.set_options(**change)
        q = p.copy()
        sm = s.solve(q)
        info = s.last_prepare()
        log = s.iteration_log()
    assert info["plan_reused"] == 1, info
    fresh = _fresh(p, **change)
    _same((q, sm, log), fresh)
    # and the change did matter (the old constants would have given another solve)
    base = _fresh(p)
    assert not np.array_equal(base[2], fresh[2]), "the option change did not change the solve"
