"""GPU parity: libmiba (HIP, gfx950) vs the CPU oracle on the same seeded
windows. Tolerances: per-observation residuals/Jacobians 1e-12 relative (same
f64 formulas, different FMA contraction); reduced camera system 1e-9 relative
(different summation order, f64 atomics); final LM cost <= 1e-6 relative
(north_star's acceptance bound)."""
import numpy as np
import pytest

from miba import synthetic
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    from miba.solver import Solver
    s = Solver(minimizer_progress_to_stdout=0)
    yield s
    s.close()


def _rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


CASES = {
    "tum_like": dict(n_cams=10, n_points=300, obs_per_point=(2, 3), seed=1),
    "banded": dict(n_cams=20, n_points=600, obs_per_point=10, seed=2),
    "shuffled_bad_depth": dict(n_cams=12, n_points=200, obs_per_point=(2, 6), seed=3, shuffle_obs=True,
                               bad_depth_frac=0.05),
    "no_gauge_cam_obs": dict(n_cams=8, n_points=120, obs_per_point=(2, 4), seed=4, fixed_cam=3),
    # points spanning > TILE_WIN cameras and repeated-camera links take the overflow (atomic) Schur path
    "wide_overflow": dict(n_cams=30, n_points=150, obs_per_point=(6, 16), seed=5, rot_noise=0.005),
    "dup_obs": dict(n_cams=10, n_points=200, obs_per_point=(2, 5), seed=6, dup_frac=0.05),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_linearize_parity(solver, case):
    p = synthetic.make_problem(**CASES[case])
    g = solver.linearize(p)
    r = oracle.linearize(p)
    assert abs(g["cost"] - r["cost"]) <= 1e-12 * r["cost"]
    for k in ("res", "jcam", "jpt", "jint"):
        assert _rel(g[k], r[k]) <= 1e-12, k


@pytest.mark.parametrize("case", sorted(CASES))
def test_camera_side_sums_parity(solver, case):
    """The production camera-side pass (k_cam_side's packed sums + k_cam_finalize, not the debug kernel):
    per active camera U = sum Jc^T Jc, C = sum Jc^T Jk, g = sum Jc^T f, and the intrinsics block with the
    IntrinsicsPrior (OptimizationUtils.cpp:117-125), against sums of the oracle's per-observation
    Jacobians; 1e-11 relative (summation order only)."""
    p = synthetic.make_problem(**CASES[case])
    g = solver.camera_sums(p)
    r = oracle.linearize(p)
    jc, jk, f = r["jcam"], r["jint"], r["res"]
    adm = p.obs_depth > 1e-15
    assert len(g["ac_cam"]) > 0
    for a, cam in enumerate(g["ac_cam"]):
        m = adm & (p.obs_cam == cam)
        U = np.einsum("nri,nrj->ij", jc[m], jc[m])
        Cc = np.einsum("nri,nrm->im", jc[m, :2], jk[m])
        gg = np.einsum("nri,nr->i", jc[m], f[m])
        assert _rel(g["U"][a], U) <= 1e-11, (case, cam)
        assert _rel(g["C"][a], Cc) <= 1e-11, (case, cam)
        assert _rel(g["g"][a], gg) <= 1e-11, (case, cam)
    w = oracle.default_options().weight_intrinsics
    Ukk = np.einsum("nrm,nrl->ml", jk[adm], jk[adm]) + w * np.eye(4)
    gk = np.einsum("nrm,nr->m", jk[adm], f[adm, :2]) - w * (p.intr_prior - p.intr)
    iu = np.triu_indices(4)
    assert _rel(g["lin"][2:12], Ukk[iu]) <= 1e-11
    assert _rel(g["lin"][12:16], gk) <= 1e-11
    assert abs(g["lin"][0] - r["cost"]) <= 1e-12 * r["cost"]


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("radius", [1e4, 3.0])
def test_reduced_system_parity(solver, case, radius):
    p = synthetic.make_problem(**CASES[case])
    S, rhs = solver.reduced_system(p, radius)
    So, ro = oracle.reduced_system(p, oracle.default_options(), radius)
    assert S.shape == So.shape
    assert _rel(S, So) <= 1e-9
    assert _rel(rhs, ro) <= 1e-9


@pytest.mark.parametrize("case", sorted(CASES))
def test_solve_parity(solver, case):
    p = synthetic.make_problem(**CASES[case])
    q = p.copy()
    sg = solver.solve(p)
    so = oracle.solve(q)
    assert sg["termination"] != "FAILURE", sg
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-12 * so["initial_cost"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sg, so)
    # converged parameters agree to the same order
    assert np.max(np.abs(p.points - q.points)) < 1e-3
    assert np.max(np.abs(p.intr - q.intr)) < 1e-2


def test_repeated_same_window(solver):
    """main.cpp:163-168 re-optimises an already-converged window every frame."""
    p = synthetic.make_problem(**CASES["tum_like"])
    s1 = solver.solve(p)
    s2 = solver.solve(p)
    assert s2["initial_cost"] <= s1["final_cost"] * (1 + 1e-9)
    assert s2["final_cost"] <= s2["initial_cost"]


def test_c2_config_final_cost():
    from miba.solver import Solver
    p = synthetic.make_config("C2")
    q = p.copy()
    with Solver(minimizer_progress_to_stdout=0) as s:
        sg = s.solve(p)
    so = oracle.solve(q)
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sg, so)
    assert sg["num_iterations"] == so["num_iterations"]


LS = {"dense": 0, "band": 1, "bcr": 2}


@pytest.mark.parametrize("ls", sorted(LS))
@pytest.mark.parametrize("case", ["banded", "tum_like", "shuffled_bad_depth", "wide_overflow"])
def test_linear_solvers_agree(case, ls, monkeypatch):
    """Dense-envelope Cholesky, banded Cholesky and block cyclic reduction solve the same
    reduced camera system: 5 LM iterations match the oracle to 1e-9 whichever runs."""
    from miba.solver import Solver
    monkeypatch.setenv("MIBA_SOLVER", ls)
    p = synthetic.make_problem(**CASES[case])
    q = p.copy()
    with Solver(minimizer_progress_to_stdout=0, max_num_iterations=5) as s:
        sg = s.solve(p)
    so = oracle.solve(q, oracle.default_options(max_num_iterations=5))
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (sg, so)
    assert sg["num_iterations"] == so["num_iterations"]
    eligible = {"dense": True, "band": sg["camera_band"] <= 6,
                "bcr": sg["camera_band"] < 10 and sg["num_active_cams"] - 1 > 10}
    if eligible[ls]:
        assert sg["linear_solver"] == LS[ls], sg


@pytest.mark.parametrize("config", ["C2", "C4"])
def test_bcr_selected_on_long_windows(config):
    """Long sliding windows (camera band < 10) take the BCR path by default."""
    from miba.solver import Solver
    p = synthetic.make_config(config)
    with Solver(minimizer_progress_to_stdout=0, max_num_iterations=2) as s:
        sg = s.solve(p)
    assert sg["linear_solver"] == LS["bcr"], sg


@pytest.mark.parametrize("case", ["tum_like", "banded", "wide_overflow", "shuffled_bad_depth"])
def test_sharded_path_single_rank(case):
    """A context with a (1-rank) RCCL communicator runs the landmark-sharded path: split
    camera-side finalisation, envelope pack / all-reduce / unpack of S, split step scalars.
    It must solve exactly the unsharded problem."""
    from miba.solver import Solver
    p = synthetic.make_problem(**CASES[case])
    q = p.copy()
    with Solver(minimizer_progress_to_stdout=0) as a:
        sa = a.solve(p)
    with Solver(minimizer_progress_to_stdout=0, shard_min_obs=0) as b:
        b.comm_init(1, 0, Solver.comm_unique_id())
        sb = b.solve(q)
    assert sb["num_obs_admissible"] == sa["num_obs_admissible"]
    assert sb["linear_solver"] == sa["linear_solver"]
    assert abs(sb["initial_cost"] - sa["initial_cost"]) <= 1e-13 * sa["initial_cost"]
    assert abs(sb["final_cost"] - sa["final_cost"]) <= 1e-10 * sa["final_cost"], (sa, sb)
    assert sb["num_iterations"] == sa["num_iterations"]
    assert np.max(np.abs(p.points - q.points)) < 1e-8
    assert np.max(np.abs(p.cams - q.cams)) < 1e-8


def test_sharded_path_matches_oracle_c2():
    from miba.solver import Solver
    p = synthetic.make_config("C2")
    q = p.copy()
    with Solver(minimizer_progress_to_stdout=0, shard_min_obs=0) as b:
        b.comm_init(1, 0, Solver.comm_unique_id())
        sb = b.solve(p)
    so = oracle.solve(q)
    assert abs(sb["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sb, so)


def test_comm_init_rejects_bad_rank():
    from miba.solver import MibaError, Solver
    with Solver(minimizer_progress_to_stdout=0) as b:
        with pytest.raises(MibaError):
            b.comm_init(2, 5, Solver.comm_unique_id())


@pytest.mark.parametrize("n_cams", [23, 64, 200, 333])
def test_bcr_persistent_matches_level_launches(n_cams, monkeypatch):
    """The persistent BCR kernels (one resident workgroup per 10-camera block; factor + one helper;
    factor + two helpers, the default where 3 workgroups per block fit) against the per-level
    launches and the oracle. The GPU paths sum the contributions in different orders and the Schur
    flush into S uses f64 atomics, so they agree to rounding: tolerances off, all run exactly 6
    iterations."""
    from miba.solver import Solver
    p = synthetic.make_problem(n_cams, 40 * n_cams, obs_per_point=(4, 9), seed=n_cams)
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=6, **no_tol))
    res = {}
    paths = {"launch": 0, "persist": 1, "split": 2, "split3": 3}
    for mode in paths:
        monkeypatch.setenv("MIBA_BCR", mode)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
            res[mode] = (s.solve(q), q)
            assert s.last_prepare()["bcr_path"] == paths[mode], mode
    sa, qa = res["launch"]
    assert sa["linear_solver"] == LS["bcr"]
    for mode in ("persist", "split", "split3"):
        sb, qb = res[mode]
        assert sb["linear_solver"] == LS["bcr"], mode
        assert sa["num_iterations"] == sb["num_iterations"] == 6, mode
        assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-10 * sa["final_cost"], mode
        np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-8, err_msg=mode)
        np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-7, err_msg=mode)
        assert abs(sb["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], mode


@pytest.mark.parametrize("n_cams,fixed", [(10, 0), (11, 0), (7, 3), (2, 0)])
def test_bcr_dense1_one_block_windows(n_cams, fixed, monkeypatch):
    """One-block windows (<= 10 active cameras; 11 cameras with the gauge camera fixed is the full 64-dof block)
    take the dense single-workgroup solve (bcr_path 4): against the split kernel and the oracle, tolerances off,
    6 iterations; a deterministic repeat is bitwise identical."""
    from miba.solver import Solver
    p = synthetic.make_problem(n_cams, 90 * n_cams, obs_per_point=(2, min(n_cams, 6)), seed=100 + n_cams,
                               fixed_cam=fixed, sensor_f32=True)
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=6, **no_tol))
    monkeypatch.setenv("MIBA_BCR_BAND", "0")  # (narrow one-block windows default to the band solve + tail)
    res = {}
    for mode, path in (("dense1", 4), ("split", 3)):
        monkeypatch.setenv("MIBA_BCR_DENSE1", "1" if mode == "dense1" else "0")
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
            res[mode] = (s.solve(q), q)
            assert s.last_prepare()["bcr_path"] == path, mode
    (sa, qa), (sb, qb) = res["dense1"], res["split"]
    assert sa["linear_solver"] == sb["linear_solver"] == LS["bcr"]
    assert sa["num_iterations"] == sb["num_iterations"] == 6
    assert sa["num_successful_steps"] == sb["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-10 * sb["final_cost"]
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-8)
    np.testing.assert_allclose(qa.intr, qb.intr, rtol=1e-9)
    np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-7)
    monkeypatch.setenv("MIBA_BCR_DENSE1", "1")
    outs = []
    for _ in range(2):
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, deterministic=1, **no_tol) as s:
            outs.append((s.solve(q)["final_cost"], q))
    assert outs[0][0] == outs[1][0]
    np.testing.assert_array_equal(outs[0][1].cams, outs[1][1].cams)


@pytest.mark.parametrize("config,iters", [("C4", 3), ("C5", 2)])
def test_large_configs_match_oracle(config, iters):
    """BASELINE.json's largest single-window configurations (C4: 200 cams / 100k points / 1M obs,
    C5: 1000 cams / 500k points / 5M obs) against the oracle for a few LM iterations (tolerances off,
    the oracle needs ~1 s (C4) / ~6 s (C5) per iteration)."""
    from miba.solver import Solver
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    p = synthetic.make_config(config)
    q = p.copy()
    with Solver(minimizer_progress_to_stdout=0, max_num_iterations=iters, **no_tol) as s:
        sg = s.solve(p)
    so = oracle.solve(q, oracle.default_options(max_num_iterations=iters, **no_tol))
    assert sg["num_iterations"] == so["num_iterations"] == iters
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (sg, so)
    np.testing.assert_allclose(p.cams, q.cams, rtol=0, atol=1e-9)
    np.testing.assert_allclose(p.intr, q.intr, rtol=1e-9)


@pytest.mark.parametrize("case", ["C1", "C3", "gauge_ovf_shuffled", "f64_layout_gauge3"])
def test_small_window_fused_schur(case, monkeypatch):
    """Small windows take the one-launch linearisation (ba_prepare_info.lin_path 1: the point side inside the Schur
    tiles, the camera side and the non-tiled points as extra workgroups of the Schur launch). Against the two-launch
    path (MIBA_SW=0) and the oracle, tolerances off, 6 iterations; gauge-only points (a single observation on the
    fixed camera), overflow points (duplicate observations), inadmissible depths, shuffled observations and the f64
    layout included."""
    from miba.solver import Solver
    if case in ("C1", "C3"):
        p = synthetic.make_config(case)
    elif case == "gauge_ovf_shuffled":
        p = synthetic.make_problem(10, 900, obs_per_point=(1, 6), seed=71, fixed_cam=0, dup_frac=0.03,
                                   bad_depth_frac=0.02, shuffle_obs=True, sensor_f32=True)
    else:
        p = synthetic.make_problem(24, 1500, obs_per_point=(1, 8), seed=72, fixed_cam=3, dup_frac=0.01)
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=6, **no_tol))
    # the default takes it for one-block windows (<= 10 active cameras) and the band tail's windows (C3); MIBA_SW=2
    # forces it on the others that fit one resident round
    on = "1" if p.n_cams <= 11 or case == "C3" else "2"
    res = {}
    for sw in (on, "0"):
        monkeypatch.setenv("MIBA_SW", sw)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
            res[sw] = (s.solve(q), q)
            assert s.last_prepare()["lin_path"] == (sw != "0"), sw
    (sa, qa), (sb, qb) = res[on], res["0"]
    assert sa["num_iterations"] == sb["num_iterations"] == 6
    assert sa["num_successful_steps"] == sb["num_successful_steps"] == so["num_successful_steps"]
    assert sa["termination_type"] == sb["termination_type"]
    assert abs(sa["initial_cost"] - sb["initial_cost"]) <= 1e-12 * sb["initial_cost"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-10 * sb["final_cost"]
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-8)
    np.testing.assert_allclose(qa.intr, qb.intr, rtol=1e-9)
    np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-7)
    # the same window again on the same context (plan cache): the same result
    monkeypatch.setenv("MIBA_SW", on)
    with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
        r1 = s.solve(p.copy())
        r2 = s.solve(p.copy())
        assert s.last_prepare()["lin_path"] == 1
    assert abs(r1["final_cost"] - r2["final_cost"]) <= 1e-12 * r1["final_cost"]


@pytest.mark.parametrize("case", ["C2", "gauge_ovf_40"])
def test_fused_point_side_larger_windows(case, monkeypatch):
    """The opt-in larger-window variant (MIBA_FPL=1: the tiled points' point side inside the Schur tiles, one
    Jacobian evaluation per observation for it and M'; k_lin_point keeps the camera side and the non-tiled points)
    against the default path and the oracle, tolerances off, 5 iterations."""
    from miba.solver import Solver
    if case == "C2":
        p = synthetic.make_config("C2")
    else:
        p = synthetic.make_problem(40, 4000, obs_per_point=(1, 9), seed=73, fixed_cam=5, dup_frac=0.02,
                                   bad_depth_frac=0.02, shuffle_obs=True, sensor_f32=True)
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=5, **no_tol))
    res = {}
    for v in ("1", "0"):
        monkeypatch.setenv("MIBA_FPL", v)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=5, **no_tol) as s:
            res[v] = (s.solve(q), q)
    (sa, qa), (sb, qb) = res["1"], res["0"]
    assert sa["num_successful_steps"] == sb["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-10 * sb["final_cost"]
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-8)
    np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-7)


BAND_CASES = {
    # the reference's sliding window: camera_band 1 (every landmark on two consecutive keyframes)
    "C3": (lambda: synthetic.make_config("C3"), 1),
    # landmark tracks of 2-3 / 2-4 keyframes: camera_band 2 / 3 (blocks of 12 / 18 dofs)
    "band2": (lambda: synthetic.make_problem(50, 4000, obs_per_point=(2, 3), seed=31, sensor_f32=True), 2),
    "band3": (lambda: synthetic.make_problem(50, 4000, obs_per_point=(2, 4), seed=32, sensor_f32=True), 3),
    # gauge in the middle, shuffled, inadmissible depths, duplicate links (overflow points), a partial last block
    "gauge_mid_dup": (lambda: synthetic.make_problem(37, 2600, obs_per_point=(1, 3), seed=33, fixed_cam=17,
                                                     dup_frac=0.02, bad_depth_frac=0.02, shuffle_obs=True,
                                                     sensor_f32=True), 2),
    # 100 keyframes: more eliminated blocks at level 0 than half-waves (two rounds), 7 levels
    "long100": (lambda: synthetic.make_problem(100, 6000, obs_per_point=(2, 2), seed=34, sensor_f32=True), 1),
    # the f64 observation layout
    "f64_band1": (lambda: synthetic.make_problem(21, 1500, obs_per_point=(2, 2), seed=35), 1),
}


@pytest.mark.parametrize("case", sorted(BAND_CASES))
def test_band_one_workgroup_solve(case, monkeypatch):
    """Narrow-band windows (camera band <= 3, more than one 64-dof BCR block) take the one-workgroup cyclic
    reduction (ba_prepare_info.bcr_path 5, ba_band.hip): against the split BCR kernel (MIBA_BCR_BAND=0) and the
    oracle, tolerances off, 6 iterations; a deterministic repeat is bitwise identical."""
    from miba.solver import Solver
    make, band = BAND_CASES[case]
    p = make()
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=6, **no_tol))
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MIBA_BCR_BAND", mode)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
            res[mode] = (s.solve(q), q)
            info = s.last_prepare()
        assert (info["bcr_path"] == 5) == (mode == "1"), (mode, info)
    (sa, qa), (sb, qb) = res["1"], res["0"]
    assert sa["camera_band"] == band, sa
    assert sa["linear_solver"] == sb["linear_solver"] == LS["bcr"]
    assert sa["num_iterations"] == sb["num_iterations"] == 6
    assert sa["num_successful_steps"] == sb["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-10 * sb["final_cost"], (sa, sb)
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (sa, so)
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-8)
    np.testing.assert_allclose(qa.intr, qb.intr, rtol=1e-9)
    np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-7)
    monkeypatch.setenv("MIBA_BCR_BAND", "1")
    outs = []
    for _ in range(2):
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, deterministic=1, **no_tol) as s:
            outs.append((s.solve(q)["final_cost"], q))
    assert outs[0][0] == outs[1][0]
    np.testing.assert_array_equal(outs[0][1].cams, outs[1][1].cams)


@pytest.mark.parametrize("case", sorted(BAND_CASES))
def test_band_tail_launch_is_the_separate_launches(case, monkeypatch):
    """The band solve's tail (ba_band.hip k_band_tail: the back-substitution chunks and the final decision as
    workgroups of the solve's launch, ba_prepare_info.tail) computes what the three launches compute: the same
    bodies, partials in the same slots (to rounding: the default mode's Schur atomics); and oracle parity."""
    from miba.solver import Solver
    make, _ = BAND_CASES[case]
    p = make()
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=6, **no_tol))
    monkeypatch.setenv("MIBA_BCR_BAND", "1")
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MIBA_TAIL", mode)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
            res[mode] = (s.solve(q), q, s.iteration_log())
            info = s.last_prepare()
        assert info["bcr_path"] == 5 and info["tail"] == (mode == "1"), (mode, info)
    (sa, qa, la), (sb, qb, lb) = res["1"], res["0"]
    # (the Schur tiles' f64 atomics make the default mode reproducible to rounding only)
    assert sa["num_successful_steps"] == sb["num_successful_steps"] and sa["num_iterations"] == sb["num_iterations"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-12 * sb["final_cost"], (sa, sb)
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-10)
    np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-9)
    np.testing.assert_allclose(la, lb, rtol=1e-6, atol=1e-14)  # (cost change and rho cancel)
    assert sa["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (sa, so)


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_backsub_final_launch_is_the_separate_launches(cfg, monkeypatch):
    """Larger windows: the point back-substitution chunks and the final reduction + LM decision in one launch
    (ba_band.hip k_backsub_final, ba_prepare_info.bsfin, opt-in MIBA_BSFIN=1; the decision workgroup waits for a
    count of the chunks, whose partials are stored past the L2) against k_backsub_chunk + k_final (the default): the same bodies, the
    same partial slots, so the same steps to rounding; and oracle parity (SPARSE_SCHUR back-substitution,
    OptimizationUtils.cpp:300)."""
    from miba.solver import Solver
    p = synthetic.make_config(cfg)
    iters = 6 if cfg == "C2" else 4
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=iters, **no_tol))
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MIBA_BSFIN", mode)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=iters, **no_tol) as s:
            res[mode] = (s.solve(q), q, s.iteration_log())
            info = s.last_prepare()
        assert info["bsfin"] == (mode == "1") and info["tail"] == 0 and info["bcr_path"] >= 2, (mode, info)
    (sa, qa, la), (sb, qb, lb) = res["1"], res["0"]
    assert sa["num_successful_steps"] == sb["num_successful_steps"] and sa["num_iterations"] == sb["num_iterations"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-12 * sb["final_cost"], (sa, sb)
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-10)
    np.testing.assert_allclose(qa.points, qb.points, rtol=0, atol=1e-9)
    np.testing.assert_allclose(la, lb, rtol=1e-6, atol=1e-14)
    assert sa["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (sa, so)


def test_band_solve_on_one_block_windows(monkeypatch):
    """The band solve (with its tail launch, the default) also on a one-block window (C1, beside the
    small-window Schur launch) against k_bcr_dense1 (MIBA_BCR_BAND=0) and the oracle."""
    from miba.solver import Solver
    p = synthetic.make_config("C1")
    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=6, **no_tol))
    res = {}
    for mode, path in (("1", 5), ("0", 4)):
        monkeypatch.setenv("MIBA_BCR_BAND", mode)
        q = p.copy()
        with Solver(minimizer_progress_to_stdout=0, max_num_iterations=6, **no_tol) as s:
            res[mode] = (s.solve(q), q)
            info = s.last_prepare()
        assert info["bcr_path"] == path and info["lin_path"] == 1, (mode, info)
    (sa, qa), (sb, qb) = res["1"], res["0"]
    assert sa["num_successful_steps"] == sb["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sa["final_cost"] - sb["final_cost"]) <= 1e-10 * sb["final_cost"]
    assert abs(sa["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]
    np.testing.assert_allclose(qa.cams, qb.cams, rtol=0, atol=1e-8)
