"""Converged-solve parity on BASELINE.json's windows against committed oracle fixtures
(tests/golden/{c3,c4,c5}_oracle.json, made by tests/golden/make_converged_golden.py).

C3 (50 cams / 4k points / 8k obs, the 50-keyframe window of configs[2]; the BCR over 5 blocks) and
C4 (200 cams / 100k points / 1M obs) run as the reference runs ceres::Solve: the default
tolerances and max_num_iterations = 75, to termination (OptimizationUtils.cpp:300,
BundleAdjustmentConfig.h:61-67). C5 (1000 cams / 500k points / 5M obs) runs 12 LM iterations with
the tolerances off. Checked: the termination, the iteration counts, the accept / reject sequence
(identical), the cost of every iteration and the final cost (<= 1e-6 relative, north_star's bound;
the first iterations to 1e-9), each step's cost change, gradient max-norm, step norm and step quality rho
(the last pins the model cost change the device forms from the normal equations), the trust-region radius sequence (C4: exact up to rounding, every
tr_ratio saturates the radius update; C5: 1e-3 relative, the late tr_ratios are ratios of cost
changes of ~1e-9 relative and carry the summation-order difference of 5M-term costs), the final
intrinsics and camera checksums."""
import json
import os

import numpy as np
import pytest

from miba import synthetic

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _gold(name):
    with open(os.path.join(GOLD, f"{name.lower()}_oracle.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name,radius_rtol", [("C3", 1e-6), ("C4", 1e-9), ("C5", 1e-3)])
def test_converged_window_matches_oracle(name, radius_rtol):
    from miba.solver import Solver
    g = _gold(name)
    p = synthetic.make_config(name)
    assert (p.n_cams, p.n_points, p.n_obs) == (g["window"]["n_cams"], g["window"]["n_points"], g["window"]["n_obs"])
    with Solver(device=0, minimizer_progress_to_stdout=0, **g["options"]) as s:
        sg = s.solve(p)
        log = s.iteration_log()
    tr = np.array(g["trace"])
    assert sg["termination"] == g["termination"], (sg["message"], g["message"])
    assert sg["num_iterations"] == g["num_iterations"]
    assert sg["num_successful_steps"] == g["num_successful_steps"]
    assert sg["num_unsuccessful_steps"] == g["num_unsuccessful_steps"]
    assert log.shape[0] == tr.shape[0]
    np.testing.assert_array_equal(log[:, 6], tr[:, 6])  # accepted / rejected / tolerance step
    assert abs(sg["initial_cost"] - g["initial_cost"]) <= 1e-12 * g["initial_cost"]
    assert abs(sg["final_cost"] - g["final_cost"]) <= 1e-6 * g["final_cost"], (sg["final_cost"], g["final_cost"])
    np.testing.assert_allclose(log[:, 0], tr[:, 0], rtol=1e-6)  # cost of every iteration
    np.testing.assert_allclose(log[:3, 0], tr[:3, 0], rtol=1e-9)
    np.testing.assert_allclose(log[:, 5], tr[:, 5], rtol=radius_rtol)
    # iteration by iteration: the cost change, the gradient max-norm, the step norm and the step quality
    # rho = cost change / model cost change. The oracle forms the model cost change as Ceres does,
    # -(J d)^T (f + J d / 2); the device from the normal equations, 0.5 (g~^T y + y^T D~ y),
    # so rho pins that identity on every step, not only through the final cost.
    scale = np.abs(tr[:, 0]).max()
    np.testing.assert_allclose(log[:, 1], tr[:, 1], rtol=radius_rtol, atol=1e-9 * scale)  # cost change
    # gradient max-norm of every linearised point (the terminal row of a solve that stops on a tolerance
    # after its last step has none: the oracle repeats the previous value, the device log leaves 0)
    np.testing.assert_allclose(log[:-1, 2], tr[:-1, 2], rtol=max(radius_rtol, 1e-6))
    np.testing.assert_allclose(log[:, 3], tr[:, 3], rtol=max(radius_rtol, 1e-6))             # |step|
    np.testing.assert_allclose(log[:, 4], tr[:, 4], rtol=max(radius_rtol, 1e-6), atol=1e-9)  # rho
    np.testing.assert_allclose(p.intr, g["final_intrinsics"], rtol=1e-6)
    cs = g["cams_checksum"]
    assert abs(np.sum(p.cams * p.cams) - cs["sum_sq"]) <= 1e-9 * cs["sum_sq"]
    ps = g["points_checksum"]
    assert abs(np.sum(p.points * p.points) - ps["sum_sq"]) <= 1e-9 * ps["sum_sq"]
