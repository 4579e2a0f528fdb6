"""CPU tests that pin the oracle (oracle/ba_oracle.c) against independent
restatements: finite differences of the reference cost functors, an
independent SE(3) exp, a dense Schur complement and scipy's minimiser.
Parity vs Ceres itself is unpinned (no Ceres in the image)."""
import numpy as np
import pytest

from miba import synthetic
from oracle import oracle
from refmath import huber, plus_pose, raw_residual


def small_problem(seed=11, **kw):
    base = dict(n_cams=5, n_points=40, obs_per_point=(2, 4), seed=seed)
    base.update(kw)
    return synthetic.make_problem(**base)


def test_defaults_match_reference_config():
    o = oracle.default_options()
    # ceresGlobalProblem, BundleAdjustmentConfig.h:47-50, 61-67
    assert o.hub_p_repr == 1e-3 and o.hub_p_unpr == 1e-3
    assert o.weight_intrinsics == 1e-6 and o.weight_unpr == 10
    assert o.max_num_iterations == 75 and o.eta == 1e-6
    # Ceres 2.0 defaults
    assert o.initial_trust_region_radius == 1e4 and o.min_relative_decrease == 1e-3
    assert o.function_tolerance == 1e-6 and o.gradient_tolerance == 1e-10 and o.parameter_tolerance == 1e-8


def test_residuals_match_reference_formula():
    p = small_problem()
    lin = oracle.linearize(p)
    adm = p.obs_depth > 1e-15
    N = adm.sum()
    o = oracle.default_options()
    cost = 0.0
    for k in np.nonzero(adm)[0]:
        r = raw_residual(p.cams[p.obs_cam[k]], p.points[p.obs_pt[k]], p.intr, p.obs_uv[k], p.obs_depth[k], 1 / N,
                         o.weight_unpr / N)
        rho_r, d_r = huber(r[0] ** 2 + r[1] ** 2, o.hub_p_repr)
        rho_d, d_d = huber(r[2] ** 2, o.hub_p_unpr)
        cost += 0.5 * rho_r + 0.5 * rho_d
        np.testing.assert_allclose(lin["res"][k], [np.sqrt(d_r) * r[0], np.sqrt(d_r) * r[1], np.sqrt(d_d) * r[2]],
                                   rtol=1e-12, atol=1e-15)
    cost += 0.5 * o.weight_intrinsics * np.sum((p.intr_prior - p.intr) ** 2)
    assert abs(lin["cost"] - cost) <= 1e-12 * cost


@pytest.mark.parametrize("hub", [1e3, 1e-3])
def test_jacobians_finite_difference(hub):
    """Local Jacobians vs central differences through T*exp(delta) (inlier
    regime: exact; Huber regime: the corrector's sqrt(rho') scaling)."""
    p = small_problem(seed=3, n_points=12)
    o = oracle.default_options(hub_p_repr=hub, hub_p_unpr=hub)
    lin = oracle.linearize(p, o)
    N = (p.obs_depth > 1e-15).sum()
    h = 1e-6
    for k in range(0, p.n_obs, 3):
        pose, X, K = p.cams[p.obs_cam[k]], p.points[p.obs_pt[k]], p.intr
        r0 = raw_residual(pose, X, K, p.obs_uv[k], p.obs_depth[k], 1 / N, o.weight_unpr / N)
        g_r = np.sqrt(huber(r0[0] ** 2 + r0[1] ** 2, hub)[1])
        g_d = np.sqrt(huber(r0[2] ** 2, hub)[1])
        scale = np.array([g_r, g_r, g_d])

        def f(pose_, X_, K_):
            return raw_residual(pose_, X_, K_, p.obs_uv[k], p.obs_depth[k], 1 / N, o.weight_unpr / N) * scale

        Jc = np.zeros((3, 6)); Jp = np.zeros((3, 3)); Jk = np.zeros((3, 4))
        for d in range(6):
            e = np.zeros(6); e[d] = h
            Jc[:, d] = (f(plus_pose(pose, e), X, K) - f(plus_pose(pose, -e), X, K)) / (2 * h)
        for i in range(3):
            e = np.zeros(3); e[i] = h * 10
            Jp[:, i] = (f(pose, X + e, K) - f(pose, X - e, K)) / (20 * h)
        for i in range(4):
            e = np.zeros(4); e[i] = h * 100
            Jk[:, i] = (f(pose, X, K + e) - f(pose, X, K - e)) / (200 * h)
        np.testing.assert_allclose(lin["jcam"][k], Jc, rtol=2e-5, atol=1e-7 * np.abs(Jc).max())
        np.testing.assert_allclose(lin["jpt"][k], Jp, rtol=2e-5, atol=1e-7 * np.abs(Jp).max())
        np.testing.assert_allclose(lin["jint"][k], Jk[:2], rtol=2e-5, atol=1e-7 * np.abs(Jk).max())


def test_se3_plus_matches_independent_exp():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.normal(size=4); q /= np.linalg.norm(q)
        T = np.concatenate([q, rng.normal(size=3)])
        for mag in (1e-12, 1e-6, 1e-2, 0.7):
            d = rng.normal(size=6) * mag
            a = oracle.se3_plus(T, d)
            b = plus_pose(T, d)
            if np.dot(a[:4], b[:4]) < 0:
                b[:4] = -b[:4]
            np.testing.assert_allclose(a, b, atol=1e-12)


def _dense_reference_system(p, o, radius):
    """Full dense J (scaled), damping and Schur complement in numpy."""
    lin = oracle.linearize(p, o)
    adm = np.nonzero(p.obs_depth > 1e-15)[0]
    cams_act = sorted({int(p.obs_cam[k]) for k in adm if p.obs_cam[k] != p.fixed_cam})
    pts_act = sorted({int(p.obs_pt[k]) for k in adm})
    ci = {c: i for i, c in enumerate(cams_act)}
    pi = {q: i for i, q in enumerate(pts_act)}
    nc, npt = 6 * len(cams_act), 3 * len(pts_act)
    ncol = nc + npt + 4
    rows = 3 * len(adm) + 4
    J = np.zeros((rows, ncol)); f = np.zeros(rows)
    for r, k in enumerate(adm):
        c = int(p.obs_cam[k])
        if c in ci:
            J[3 * r:3 * r + 3, 6 * ci[c]:6 * ci[c] + 6] = lin["jcam"][k]
        J[3 * r:3 * r + 3, nc + 3 * pi[int(p.obs_pt[k])]:nc + 3 * pi[int(p.obs_pt[k])] + 3] = lin["jpt"][k]
        J[3 * r:3 * r + 2, nc + npt:] = lin["jint"][k]
        f[3 * r:3 * r + 3] = lin["res"][k]
    swk = np.sqrt(o.weight_intrinsics)
    J[-4:, nc + npt:] = -swk * np.eye(4)
    f[-4:] = swk * (p.intr_prior - p.intr)
    cn = (J ** 2).sum(0)
    s = 1 / (1 + np.sqrt(cn))
    Js = J * s
    D2 = np.clip((Js ** 2).sum(0), o.min_lm_diagonal, o.max_lm_diagonal) / radius
    H = Js.T @ Js + np.diag(D2)
    g = Js.T @ f
    F = np.r_[np.arange(nc), np.arange(nc + npt, ncol)]
    E = np.arange(nc, nc + npt)
    HEE_inv = np.linalg.inv(H[np.ix_(E, E)])
    S = H[np.ix_(F, F)] - H[np.ix_(F, E)] @ HEE_inv @ H[np.ix_(E, F)]
    rhs = g[F] - H[np.ix_(F, E)] @ HEE_inv @ g[E]
    return S, rhs


@pytest.mark.parametrize("seed", [1, 2])
def test_reduced_system_matches_dense_schur(seed):
    p = small_problem(seed=seed, bad_depth_frac=0.05)
    o = oracle.default_options()
    S_ref, rhs_ref = _dense_reference_system(p, o, 1e4)
    S, rhs = oracle.reduced_system(p, o, 1e4)
    np.testing.assert_allclose(S, S_ref, rtol=1e-9, atol=1e-12 * np.abs(S_ref).max())
    np.testing.assert_allclose(rhs, rhs_ref, rtol=1e-9, atol=1e-12 * np.abs(rhs_ref).max())


def test_sharded_reduced_system_sums_to_full():
    p = small_problem(seed=5, n_points=60)
    o = oracle.default_options()
    S, rhs = oracle.reduced_system(p, o, 1e4)
    S0, r0 = oracle.reduced_system(p, o, 1e4, 0, 25, True)
    S1, r1 = oracle.reduced_system(p, o, 1e4, 25, 60, False)
    np.testing.assert_allclose(S0 + S1, S, rtol=1e-12, atol=1e-14 * np.abs(S).max())
    np.testing.assert_allclose(r0 + r1, rhs, rtol=1e-12, atol=1e-14 * np.abs(rhs).max())


def test_lm_reaches_scipy_minimum_quadratic_regime():
    """Independent minimiser cross-check: with Huber a large (all blocks in the
    quadratic zone) the objective is 0.5*|f|^2 and scipy least_squares must
    reach the same minimum as the oracle's Ceres-LM restatement."""
    from scipy.optimize import least_squares
    p = small_problem(seed=7, n_cams=4, n_points=25, obs_per_point=(3, 4))
    o = oracle.default_options(hub_p_repr=1e6, hub_p_unpr=1e6, max_num_iterations=200, function_tolerance=1e-14,
                               parameter_tolerance=1e-14, gradient_tolerance=1e-16)
    q = p.copy()
    s = oracle.solve(q, o)
    adm = np.nonzero(p.obs_depth > 1e-15)[0]
    N = len(adm)
    cams_act = [c for c in range(p.n_cams) if c != p.fixed_cam]
    from refmath import plus_pose as pp

    def unpack(z):
        cams = p.cams.copy()
        for i, c in enumerate(cams_act):
            cams[c] = pp(p.cams[c], z[6 * i:6 * i + 6])
        off = 6 * len(cams_act)
        pts = p.points + z[off:off + 3 * p.n_points].reshape(-1, 3)
        K = p.intr + z[off + 3 * p.n_points:]
        return cams, pts, K

    def fun(z):
        cams, pts, K = unpack(z)
        out = [raw_residual(cams[p.obs_cam[k]], pts[p.obs_pt[k]], K, p.obs_uv[k], p.obs_depth[k], 1 / N, 10 / N)
               for k in adm]
        return np.r_[np.concatenate(out), np.sqrt(1e-6) * (p.intr_prior - K)]

    z0 = np.zeros(6 * len(cams_act) + 3 * p.n_points + 4)
    r = least_squares(fun, z0, method="lm", xtol=1e-15, ftol=1e-15, gtol=1e-15, max_nfev=20000)
    c_scipy = 0.5 * np.sum(r.fun ** 2)
    assert abs(s["final_cost"] - c_scipy) <= 1e-6 * c_scipy, (s, c_scipy)



def test_lm_minimum_certified_by_scipy_huber_regime():
    """Independent minimiser cross-check in the regime every real window runs in: the default Huber
    a = 1e-3 with w = 1/N puts most residual blocks in the linear zone, where both LM and
    scipy converge only linearly, so the check is a certificate at the oracle's minimum: an objective
    written independently with numpy (refmath) equals the oracle's final cost there, and neither
    scipy least_squares(loss="huber", f_scale=a) nor L-BFGS-B started from it lowers the cost by more
    than 1e-6 relative. scipy's huber applies 0.5 a^2 rho(z / a^2) to each residual z = r^2; with one
    residual per block (the block norm) that is 0.5 * Ceres HuberLoss(a)(|f_b|^2), the reference's
    objective (OptimizationUtils.cpp:223-226, 279-294). Each IntrinsicsPrior row r (squared loss,
    :237-241) enters as k^2 copies of r / k, inside Huber's quadratic zone (|r| / k < a), where they sum
    to exactly 0.5 r^2."""
    from scipy.optimize import least_squares, minimize
    from refmath import plus_pose as pp, quat_R
    p = small_problem(seed=11, n_cams=3, n_points=15, obs_per_point=(2, 3))
    a = 1e-3
    o = oracle.default_options(max_num_iterations=3000, function_tolerance=1e-15, parameter_tolerance=1e-15,
                               gradient_tolerance=1e-16)
    q = p.copy()
    s = oracle.solve(q, o)
    adm = np.nonzero(p.obs_depth > 1e-15)[0]
    N = len(adm)
    cams_act = [c for c in range(p.n_cams) if c != p.fixed_cam]
    oc, op, uv, dep = p.obs_cam[adm], p.obs_pt[adm], p.obs_uv[adm], p.obs_depth[adm]
    nz = 6 * len(cams_act) + 3 * p.n_points + 4
    KSPLIT = 10

    def unpack(z):  # local perturbation of the oracle's solution q
        cams = q.cams.copy()
        for i, c in enumerate(cams_act):
            cams[c] = pp(q.cams[c], z[6 * i:6 * i + 6])
        off = 6 * len(cams_act)
        return cams, q.points + z[off:off + 3 * p.n_points].reshape(-1, 3), q.intr + z[off + 3 * p.n_points:]

    def blocks(z):  # (|f_repr|^2, |f_depth|^2) per observation, prior residual
        cams, pts, K = unpack(z)
        R = np.array([quat_R(c[:4]) for c in cams])[oc]
        pc = np.einsum("nji,nj->ni", R, pts[op] - cams[oc, 4:7])
        u = (K[0] * pc[:, 0] + K[2] * pc[:, 2]) / pc[:, 2]
        v = (K[1] * pc[:, 1] + K[3] * pc[:, 2]) / pc[:, 2]
        return ((u - uv[:, 0]) ** 2 + (v - uv[:, 1]) ** 2) / N, 10 / N * (dep - pc[:, 2]) ** 2, \
            np.sqrt(1e-6) * (p.intr_prior - K)

    def rho(x):
        return np.where(x > a * a, 2 * a * np.sqrt(x) - a * a, x)

    def F(z):
        sr, sd, fk = blocks(z)
        return 0.5 * np.sum(rho(sr)) + 0.5 * np.sum(rho(sd)) + 0.5 * np.sum(fk ** 2)

    def fun(z):
        sr, sd, fk = blocks(z)
        return np.r_[np.sqrt(sr), np.sqrt(sd), np.repeat(fk / KSPLIT, KSPLIT * KSPLIT)]

    z0 = np.zeros(nz)
    sr, sd, fk = blocks(z0)
    assert np.mean(np.r_[sr, sd] > a * a) > 0.5  # the Huber linear zone dominates
    assert np.all(np.abs(fk) / KSPLIT < a)
    assert abs(F(z0) - s["final_cost"]) <= 1e-12 * s["final_cost"]
    r = least_squares(fun, z0, method="trf", loss="huber", f_scale=a, xtol=1e-15, ftol=1e-15, gtol=1e-15,
                      max_nfev=2000)
    assert F(r.x) >= s["final_cost"] * (1 - 1e-6), (F(r.x), s["final_cost"])
    m = minimize(F, z0, method="L-BFGS-B", options=dict(maxiter=5000, ftol=1e-16, gtol=1e-14, maxcor=50))
    assert m.fun >= s["final_cost"] * (1 - 1e-6), (m.fun, s["final_cost"])
    # the reference's own stopping rule (function_tolerance 1e-6 per step) ends close to that minimum
    sd_ = oracle.solve(p.copy())
    assert s["final_cost"] <= sd_["final_cost"] <= s["final_cost"] * (1 + 1e-3)
