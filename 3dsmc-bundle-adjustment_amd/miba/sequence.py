"""Synthetic TUM-like keyframe sequence and the reference driver's outer loop around the solver.

``make_tum_sequence`` stands in for the tracking front-end (VirtualSensor + tracking_step,
main.cpp:150-160; no RGB-D dataset exists here): keyframes carry float32 keypoints, back-projected
local points from a noisy depth, a global_points_map in insertion order and a drifting pose
estimate, plus the TUM ground-truth text at 100 Hz. ``run_pipeline`` replays main.cpp:150-195 —
the window schedule (window.window_schedule), windowOptimize on each scheduled window with any
``ba_solve``-contract solver, then getFirstPose + poseOffset + write_keyframe_poses_to_file —
and returns the written trajectory text, ready for miba.evaluate.ate / rpe."""
from __future__ import annotations

import numpy as np

from . import trajectory, window
from .synthetic import ROS_DEFAULT_INTRINSICS, _rodrigues, quat_from_rotmat

IMAGE_W, IMAGE_H = 640, 480
TUM_FR1_INTRINSICS = np.array([517.3, 516.5, 318.6, 255.3])


def _gt_path(n: int, dt: float):
    s = np.arange(n) * dt
    pos = np.stack([0.25 * np.sin(0.6 * s), 0.08 * np.sin(0.9 * s + 0.3), 0.12 * s], 1)
    w = np.stack([0.12 * np.sin(0.5 * s), 0.25 * np.sin(0.35 * s), 0.06 * np.sin(0.8 * s)], 1)
    return _rodrigues(w), pos


def make_tum_sequence(n_keyframes: int = 36, n_landmarks: int = 1500, seed: int = 0, pixel_noise: float = 0.5,
                      depth_noise: float = 0.005, drift_rot: float = 0.002, drift_trans: float = 0.004,
                      max_obs_per_kf: int = 220, t0: float = 1305031102.175304, kf_dt: float = 0.1):
    """(keyframes, landmarks, intr_init, gt_text). Keyframe poses are tracking estimates relative to
    the first keyframe (identity), as the reference's tracker produces them."""
    rng = np.random.default_rng(seed)
    K = TUM_FR1_INTRINSICS
    K0 = ROS_DEFAULT_INTRINSICS.copy()
    # ground truth at 100 Hz; keyframes every kf_dt seconds (+ a few ms of stamp offset)
    n_gt = int(round(n_keyframes * kf_dt / 0.01)) + 20
    R_gt, t_gt = _gt_path(n_gt, 0.01)
    gt_stamps = t0 - 0.05 + np.arange(n_gt) * 0.01 + rng.uniform(-5e-4, 5e-4, n_gt)
    kf_gt = 5 + np.round(np.arange(n_keyframes) * kf_dt / 0.01).astype(int)
    kf_stamps = gt_stamps[kf_gt] + rng.uniform(-3e-3, 3e-3, n_keyframes)
    # landmarks: a textured room in front of the path
    X = np.stack([rng.uniform(-2.5, 2.5, n_landmarks), rng.uniform(-1.8, 1.8, n_landmarks),
                  rng.uniform(1.2, 5.0 + 0.12 * n_keyframes * kf_dt, n_landmarks)], 1)
    # tracking estimate: ground truth relative to the first keyframe, with a random-walk drift
    Rg, tg = R_gt[kf_gt], t_gt[kf_gt]
    R_rel = np.einsum("ji,njk->nik", Rg[0], Rg)                      # R0^T Rk
    t_rel = np.einsum("ji,nj->ni", Rg[0], tg - tg[0])                 # R0^T (tk - t0)
    dR = _rodrigues(np.cumsum(rng.normal(0, drift_rot, (n_keyframes, 3)), 0))
    dt = np.cumsum(rng.normal(0, drift_trans, (n_keyframes, 3)), 0)
    dR[0], dt[0] = np.eye(3), 0.0
    R_est, t_est = R_rel @ dR, t_rel + dt
    keyframes, landmarks = [], {}
    lm_of = {}  # ground-truth landmark index -> LandmarkId (first seen order, like the tracker's map)
    for k in range(n_keyframes):
        pc = np.einsum("ji,nj->ni", Rg[k], X - tg[k])
        z = pc[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = K[0] * pc[:, 0] / z + K[2]
            v = K[1] * pc[:, 1] / z + K[3]
        vis = np.nonzero((z > 0.3) & (u > 8) & (u < IMAGE_W - 8) & (v > 8) & (v < IMAGE_H - 8))[0]
        if len(vis) > max_obs_per_kf:
            vis = np.sort(rng.choice(vis, max_obs_per_kf, replace=False))
        uv = np.stack([u[vis], v[vis]], 1) + rng.normal(0, pixel_noise, (len(vis), 2))
        kp = uv.astype(np.float32)
        d = z[vis] * (1.0 + rng.normal(0, depth_noise, len(vis)))
        d[rng.random(len(vis)) < 0.03] = 0.0  # missing depth (VirtualSensor MINF -> skipped, :265-268)
        loc = np.stack([(kp[:, 0] - K0[2]) / K0[0] * d, (kp[:, 1] - K0[3]) / K0[1] * d, d], 1)
        T = np.concatenate([quat_from_rotmat(R_est[k]), t_est[k]])
        gpm = {}
        for local_id, g in enumerate(vis):
            if d[local_id] <= 0:
                continue
            if g not in lm_of:
                lid = len(lm_of)
                lm_of[g] = lid
                landmarks[lid] = window.se3_act(T, loc[local_id])
            gpm[local_id] = lm_of[g]
        keyframes.append(window.KeyFrame(T, kp, loc, gpm, "%.6f" % kf_stamps[k]))
    lines = ["# ground truth trajectory", "# file: 'synthetic'", "# timestamp tx ty tz qx qy qz qw"]
    q_gt = quat_from_rotmat(R_gt)
    for i in range(n_gt):
        lines.append("%.4f %.4f %.4f %.4f %.4f %.4f %.4f %.4f" % (gt_stamps[i], *t_gt[i], *q_gt[i]))
    return keyframes, landmarks, K0, "\n".join(lines) + "\n"


def run_pipeline(keyframes, landmarks, intr_init, gt_text: str, solve, frame_frequency: int = 10,
                 window_size: int = 10):
    """main.cpp:150-195 with one keyframe per frame. Returns (trajectory_text, summaries, intr_opt);
    ``keyframes`` / ``landmarks`` are updated in place."""
    intr_opt = np.array(intr_init, dtype=np.float64)
    summaries = []
    pending = list(keyframes)
    keyframes.clear()
    finished = False
    while True:
        tracked = bool(pending)  # tracking_step added a keyframe this frame
        if tracked:
            keyframes.append(pending.pop(0))
        run, a, b, fin = window.window_schedule(frame_frequency, window_size, len(keyframes), not tracked,
                                                finished, tracked)
        if run:
            summaries.append((a, b, window.window_optimize(a, b, keyframes, landmarks, intr_init, intr_opt, solve)))
        finished = finished or fin
        if not tracked:  # after the sequence ends the schedule can fire at most once
            break
    first = trajectory.get_first_pose(keyframes[0].timestamp, gt_text)
    trajectory.pose_offset(keyframes, first)
    return trajectory.format_keyframe_poses(keyframes), summaries, intr_opt
