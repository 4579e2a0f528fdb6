"""The reference driver's loop around the solver (main.cpp:150-195) on a synthetic TUM-like
sequence: window schedule -> windowOptimize per window -> getFirstPose/poseOffset -> TUM
trajectory text -> ATE / RPE (miba.evaluate, pinned to the reference's rgb-d-toolset in
test_trajectory.py). The GPU test is the §8 acceptance check: the GPU-solved and the
oracle-solved trajectories score within 1 mm of each other."""
import numpy as np
import pytest

from miba import evaluate, sequence, trajectory
from oracle import oracle


def _oracle_solve():
    o = oracle.default_options()
    return lambda p: oracle.solve(p, o)


def _run(solve, seed=0, **kw):
    sizes = {k: kw.pop(k) for k in ("n_keyframes", "n_landmarks") if k in kw}
    kfs, lms, K0, gt = sequence.make_tum_sequence(seed=seed, **sizes)
    txt, summ, K = sequence.run_pipeline(kfs, lms, K0, gt, solve, **kw)
    return gt, txt, summ, K


def test_pipeline_schedule_and_output_oracle():
    gt, txt, summ, K = _run(_oracle_solve())
    assert [(a, b) for a, b, _ in summ] == [(0, 9), (10, 19), (20, 29), (26, 35)]  # 3 windows + leftovers
    for _, _, s in summ:
        assert s["final_cost"] < s["initial_cost"]
    lines = txt.strip().split("\n")
    assert len(lines) == 36
    # the first pose is the nearest ground-truth record (poseOffset), to the 6 digits written
    first = [float(v) for v in lines[0].split()[1:]]
    g = trajectory.get_first_pose(lines[0].split()[0], gt)
    np.testing.assert_allclose(first, np.concatenate([g[4:], g[:4]]), rtol=1e-5, atol=1e-6)
    e = evaluate.ate(gt, txt)
    assert len(e["matches"]) == 36 and 0 < e["rmse"] < 0.05
    r = evaluate.rpe(gt, txt)
    assert r["pairs"] == 36 * 36 and r["trans_mean"] < 0.05


def test_pipeline_global_ba_schedule():
    _, txt, summ, _ = _run(_oracle_solve(), n_keyframes=14, window_size=-1)
    assert [(a, b) for a, b, _ in summ] == [(0, 13)]
    assert len(txt.strip().split("\n")) == 14


@pytest.mark.gpu
# (5, 90, 50, 10): BASELINE configs[2]'s sliding window — window_size = 50 > frame_frequency = 10
# (BundleAdjustmentConfig.h:52-53, main.cpp:163-168): windows (0,49), (10,59), ..., (40,89)
@pytest.mark.parametrize("seed,n_kf,wsize,freq", [(0, 36, 10, 10), (3, 64, 20, 10), (5, 90, 50, 10)])
def test_pipeline_gpu_matches_oracle_ate_rpe(seed, n_kf, wsize, freq):
    from miba.solver import Solver
    with Solver() as s:
        gt, txt_g, summ_g, K_g = _run(s.solve, seed=seed, n_keyframes=n_kf, window_size=wsize, frame_frequency=freq)
    _, txt_c, summ_c, K_c = _run(_oracle_solve(), seed=seed, n_keyframes=n_kf, window_size=wsize,
                                 frame_frequency=freq)
    assert [(a, b) for a, b, _ in summ_g] == [(a, b) for a, b, _ in summ_c]
    if wsize == 50:
        assert [(a, b) for a, b, _ in summ_c] == [(0, 49), (10, 59), (20, 69), (30, 79), (40, 89)]
    for (_, _, sg), (_, _, sc) in zip(summ_g, summ_c):
        assert abs(sg["final_cost"] - sc["final_cost"]) <= 1e-6 * sc["final_cost"]
    eg, ec = evaluate.ate(gt, txt_g), evaluate.ate(gt, txt_c)
    assert abs(eg["rmse"] - ec["rmse"]) <= 1e-3
    rg, rc = evaluate.rpe(gt, txt_g), evaluate.rpe(gt, txt_c)
    assert abs(rg["trans_mean"] - rc["trans_mean"]) <= 1e-3
    pg = np.array([[float(v) for v in l.split()[1:4]] for l in txt_g.strip().split("\n")])
    pc = np.array([[float(v) for v in l.split()[1:4]] for l in txt_c.strip().split("\n")])
    assert np.abs(pg - pc).max() <= 1e-3
    np.testing.assert_allclose(K_g, K_c, atol=1e-3)
