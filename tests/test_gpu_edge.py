"""Edge cases of the C-ABI on the GPU: a non-finite initial evaluation (Ceres FAILURE with
"Residual and Jacobian evaluation failed.", rc 0, no hang of the progress-word loop), windows
without any admissible observation (only the IntrinsicsPrior block, OptimizationUtils.cpp:236-241,
solved like Ceres), a forced inter-workgroup hand-off timeout of the resident BCR kernel (the
iteration is re-run with the per-level launches inside the same solve: BA_OK, oracle parity), and
two contexts solving concurrently on one GPU."""
import threading

import numpy as np
import pytest

from miba import synthetic
from oracle import oracle

pytestmark = pytest.mark.gpu


def _solver(**kw):
    from miba.solver import Solver
    return Solver(device=0, minimizer_progress_to_stdout=0, **kw)


@pytest.mark.parametrize("bad", ["nan_point", "inf_depth_point_on_camera"])
def test_non_finite_initial_evaluation_fails_like_ceres(bad):
    p = synthetic.make_problem(n_cams=10, n_points=300, obs_per_point=(2, 3), seed=1)
    if bad == "nan_point":
        p.points[17] = np.nan
    else:  # a point at a camera centre: z = 0, the projection divides by zero
        k = int(np.nonzero(p.obs_pt == 5)[0][0])
        p.points[5] = p.cams[p.obs_cam[k], 4:7]
    q = p.copy()
    with _solver() as s:
        sg = s.solve(p)  # must return (rc 0), not spin
        # the context stays usable afterwards
        ok = synthetic.make_problem(n_cams=10, n_points=300, obs_per_point=(2, 3), seed=1)
        so_ok = oracle.solve(ok.copy())
        sg_ok = s.solve(ok)
    so = oracle.solve(q)
    assert so["termination"] == "FAILURE"
    assert sg["termination"] == "FAILURE", sg
    assert sg["message"] == "Residual and Jacobian evaluation failed.", sg["message"]
    assert sg["num_iterations"] == 0
    assert abs(sg_ok["final_cost"] - so_ok["final_cost"]) <= 1e-6 * so_ok["final_cost"]


@pytest.mark.parametrize("kind", ["all_depths_zero", "no_observations"])
def test_window_without_admissible_observations_solves_the_prior(kind):
    p = synthetic.make_problem(n_cams=8, n_points=100, obs_per_point=(2, 4), seed=9)
    if kind == "all_depths_zero":
        p.obs_depth[:] = np.where(np.arange(p.n_obs) % 2 == 0, 0.0, -np.inf)
    else:
        from miba.capi import ProblemArrays
        p = ProblemArrays(p.cams, p.points[:0], p.intr, p.intr_prior, p.obs_cam[:0], p.obs_pt[:0], p.obs_uv[:0],
                          p.obs_depth[:0], p.fixed_cam)
    p.intr[:] = p.intr_prior + np.array([4.0, -3.0, 2.0, -1.0])  # intrinsics_optimized != intrinsics_initial
    q = p.copy()
    cams0 = p.cams.copy()
    with _solver() as s:
        sg = s.solve(p)
    so = oracle.solve(q)
    assert sg["num_obs_admissible"] == 0 and sg["num_active_cams"] == 0 and sg["reduced_system_size"] == 4
    assert sg["termination"] == so["termination"], (sg, so)
    assert sg["num_iterations"] == so["num_iterations"]
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-12 * so["initial_cost"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["initial_cost"], (sg, so)
    np.testing.assert_allclose(p.intr, q.intr, rtol=1e-10)
    assert np.max(np.abs(p.intr - p.intr_prior)) < 1e-2  # pulled onto the prior
    np.testing.assert_array_equal(p.cams, cams0)  # no residual on any pose


def test_bcr_handoff_timeout_reruns_the_iteration_in_the_same_solve(monkeypatch):
    p = synthetic.make_config("C2")
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=5))
    with _solver(max_num_iterations=5) as s:
        monkeypatch.setenv("MIBA_BCR_SPIN_LIMIT", "1")  # every inter-workgroup wait times out at once
        q = p.copy()
        sg = s.solve(q)  # BA_OK: the first iteration's reduced solve re-runs with the per-level launches
        note = s.last_error()
        monkeypatch.delenv("MIBA_BCR_SPIN_LIMIT")
        q2 = p.copy()
        sg2 = s.solve(q2)  # the next prepare probes the resident kernel again (no sticky fallback)
        info2 = s.last_prepare()
        note2 = s.last_error()
    assert "re-run with the per-level BCR launches" in note, note
    assert info2["bcr_path"] >= 2 and note2 == "", (info2, note2)
    for g in (sg, sg2):
        assert g["linear_solver"] == 2
        assert g["termination"] == so["termination"]
        assert g["num_iterations"] == so["num_iterations"]
        assert g["num_successful_steps"] == so["num_successful_steps"]
        assert abs(g["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (g, so)
    np.testing.assert_allclose(q.cams, q2.cams, rtol=0, atol=1e-12)
    # a fresh context uses the resident kernels again (the spin limit is back to its default)
    with _solver(max_num_iterations=5) as s2:
        sg3 = s2.solve(p.copy())
        assert s2.last_error() == ""
    assert abs(sg3["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"]


def test_one_block_window_timeout_reruns_and_restores_the_small_window_path(monkeypatch):
    """ADVICE r4 (medium / low): the default one-block path (k_bcr_dense1 + the small-window fused Schur launch,
    whose envelope tiles wait for the launch's camera side) under a forced one-poll spin bound. The wait times
    out, the iteration re-runs with the per-level launches and the two-launch linearisation inside the same
    solve (BA_OK, oracle parity); the next solve of the same window (plan cache) takes the one-block path again."""
    p = synthetic.make_config("C1")
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=8))
    monkeypatch.setenv("MIBA_BCR_BAND", "0")  # (the default one-block path is the band solve with its tail launch)
    with _solver(max_num_iterations=8) as s:
        s.solve(p.copy())
        info0 = s.last_prepare()
        assert info0["bcr_path"] == 4 and info0["lin_path"] == 1, info0
        monkeypatch.setenv("MIBA_BCR_SPIN_LIMIT", "1")
        q = p.copy()
        sg = s.solve(q)
        note = s.last_error()
        monkeypatch.delenv("MIBA_BCR_SPIN_LIMIT")
        q2 = p.copy()
        sg2 = s.solve(q2)
        info2 = s.last_prepare()
        note2 = s.last_error()
    assert "re-run with the per-level BCR launches" in note, note
    assert info2["plan_reused"] == 1 and info2["bcr_path"] == 4 and info2["lin_path"] == 1, info2
    assert note2 == "", note2
    for g in (sg, sg2):
        assert g["termination"] == so["termination"], (g, so)
        assert g["num_iterations"] == so["num_iterations"]
        assert g["num_successful_steps"] == so["num_successful_steps"]
        assert abs(g["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (g, so)
    np.testing.assert_allclose(q.cams, q2.cams, rtol=0, atol=1e-10)


def test_band_tail_timeout_reruns_with_the_separate_launches(monkeypatch):
    """The band solve's tail launch (C3: the back-substitution chunks wait for the solve, the decision for the
    chunks) under a forced one-poll spin bound: the waits time out, the decision asks for a re-run, the iteration
    re-runs with the separate launches inside the same solve (BA_OK, oracle parity), and the next solve of the
    window (plan cache) takes the tail launch again."""
    p = synthetic.make_config("C3")
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=8))
    with _solver(max_num_iterations=8) as s:
        s.solve(p.copy())
        info0 = s.last_prepare()
        assert info0["bcr_path"] == 5 and info0["tail"] == 1, info0
        monkeypatch.setenv("MIBA_BCR_SPIN_LIMIT", "1")
        q = p.copy()
        sg = s.solve(q)
        note = s.last_error()
        monkeypatch.delenv("MIBA_BCR_SPIN_LIMIT")
        q2 = p.copy()
        sg2 = s.solve(q2)
        info2 = s.last_prepare()
        note2 = s.last_error()
    assert "re-run with the per-level BCR launches" in note, note
    assert info2["plan_reused"] == 1 and info2["tail"] == 1, info2
    assert note2 == "", note2
    for g in (sg, sg2):
        assert g["termination"] == so["termination"], (g, so)
        assert g["num_iterations"] == so["num_iterations"]
        assert g["num_successful_steps"] == so["num_successful_steps"]
        assert abs(g["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (g, so)
    np.testing.assert_allclose(q.cams, q2.cams, rtol=0, atol=1e-10)


@pytest.mark.parametrize("cfg", ["C2", "C4"])
def test_backsub_final_timeout_reruns_with_the_separate_launches(cfg, monkeypatch):
    """The one-launch back-substitution + decision (k_backsub_final, larger windows) under a forced one-poll spin
    bound: the decision workgroup's wait for its chunks times out (and so do the split BCR's hand-offs), the
    iteration re-runs with the separate launches inside the same solve (BA_OK, oracle parity), and the next solve of
    the window (plan cache) takes the one-launch path again."""
    p = synthetic.make_config(cfg)
    it = 5 if cfg == "C2" else 3
    so = oracle.solve(p.copy(), oracle.default_options(max_num_iterations=it))
    monkeypatch.setenv("MIBA_BSFIN", "1")  # (opt-in: measured slower than the two launches at C4)
    with _solver(max_num_iterations=it) as s:
        s.solve(p.copy())
        assert s.last_prepare()["bsfin"] == 1
        monkeypatch.setenv("MIBA_BCR_SPIN_LIMIT", "1")
        monkeypatch.setenv("MIBA_BCR", "launch")  # (no BCR hand-off waits: the decision workgroup's is the one forced)
        q = p.copy()
        sg = s.solve(q)
        note = s.last_error()
        monkeypatch.delenv("MIBA_BCR_SPIN_LIMIT")
        monkeypatch.delenv("MIBA_BCR")
        q2 = p.copy()
        sg2 = s.solve(q2)
        info2 = s.last_prepare()
        note2 = s.last_error()
    assert "re-run with the per-level BCR launches" in note, note
    assert info2["bsfin"] == 1 and info2["bcr_path"] >= 2, info2  # (MIBA_BCR is in the plan key: a fresh plan)
    assert note2 == "", note2
    for g in (sg, sg2):
        assert g["termination"] == so["termination"], (g, so)
        assert g["num_iterations"] == so["num_iterations"]
        assert g["num_successful_steps"] == so["num_successful_steps"]
        assert abs(g["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (g, so)
    np.testing.assert_allclose(q.cams, q2.cams, rtol=0, atol=1e-10)


def test_two_contexts_solve_concurrently_on_one_gpu():
    """Two host threads, one context each, solving C2 windows at the same time on GPU 0: both resident BCR
    grids and every other launch share the device; both solves return BA_OK and match the oracle."""
    probs = [synthetic.make_config("C2"), synthetic.make_config("C2", seed=12)]
    want = [oracle.solve(p.copy()) for p in probs]
    out, errs = [None, None], []

    def run(k):
        try:
            with _solver() as s:
                for _ in range(3):  # overlapping solves, not one after the other
                    q = probs[k].copy()
                    out[k] = (s.solve(q), q)
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    hung = [k for k, t in enumerate(th) if t.is_alive()]
    assert not hung, f"solver thread(s) {hung} still running after 300 s (hang or deadlock)"
    assert not errs, errs
    assert all(o is not None for o in out), out
    for (sg, q), so in zip(out, want):
        assert sg["termination"] == so["termination"], (sg, so)
        assert sg["num_iterations"] == so["num_iterations"]
        assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sg, so)


def test_first_solves_from_two_threads_in_a_fresh_process():
    """the one-time launch setup (the 160 KB dynamic-LDS attribute of the band solve, its tail
    launch, the split BCR and the per-level kernels) is per device and thread-safe. A fresh process — nothing set
    up yet — starts four threads whose FIRST solves begin together (band + tail on C3 twice, the split BCR on C2,
    the one-block band on C1); every solve returns BA_OK and matches the oracle."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "first_solve_worker.py"), "C3,C2,C1,C3"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert not res["hung"], res
    paths = []
    for cfg, o in zip(res["configs"], res["out"]):
        assert o is not None and "error" not in o, (cfg, o)
        sg, so = o["gpu"], o["oracle"]
        paths.append(o["bcr_path"])
        assert sg["termination"] == so["termination"], (cfg, sg, so)
        assert sg["num_iterations"] == so["num_iterations"], cfg
        assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"], (cfg, sg, so)
    assert paths[0] == 5 and paths[1] >= 2, paths  # the band solve and the split BCR were both raced


def test_cooperative_bcr_launch_matches_oracle(monkeypatch):
    """MIBA_BCR_COOP=1: k_bcr_split as a cooperative launch (the runtime refuses a grid that cannot be co-resident;
    off by default, it costs ~20 us per launch on MI355X). Same arithmetic: the solve matches the oracle."""
    monkeypatch.setenv("MIBA_BCR_COOP", "1")
    p = synthetic.make_config("C2")
    so = oracle.solve(p.copy())
    with _solver() as s:
        sg = s.solve(p.copy())
        assert s.last_error() == ""
    assert sg["linear_solver"] == 2
    assert sg["num_iterations"] == so["num_iterations"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sg, so)
