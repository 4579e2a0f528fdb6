"""Python mirror of the reference's window handling around ceres::Solve.

``window_optimize`` restates windowOptimize (/root/reference/src/OptimizationUtils.cpp:215-313)
over plain Python keyframe / landmark containers and any solver with the
``ba_solve`` contract (e.g. ``miba.solver.Solver().solve`` or the oracle).
``window_schedule`` restates the driver's window schedule (main.cpp:132-133,
163-183). ``include/ba_window.hpp`` is the C++ adapter with the same semantics;
tests/test_window_adapter.py checks the two against each other.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .capi import ProblemArrays


# ---- SE(3) on Sophus storage [qx,qy,qz,qw,tx,ty,tz] (same operation order as ba_window.hpp)
def so3_rotate(q, v):
    qx, qy, qz, qw = q[0], q[1], q[2], q[3]
    uv0 = 2 * (qy * v[2] - qz * v[1])
    uv1 = 2 * (qz * v[0] - qx * v[2])
    uv2 = 2 * (qx * v[1] - qy * v[0])
    return np.array([v[0] + qw * uv0 + (qy * uv2 - qz * uv1),
                     v[1] + qw * uv1 + (qz * uv0 - qx * uv2),
                     v[2] + qw * uv2 + (qx * uv1 - qy * uv0)])


def se3_mul(a, b):
    t = so3_rotate(a, b[4:7])
    ax, ay, az, aw = a[0], a[1], a[2], a[3]
    bx, by, bz, bw = b[0], b[1], b[2], b[3]
    w = aw * bw - ax * bx - ay * by - az * bz
    x = aw * bx + ax * bw + ay * bz - az * by
    y = aw * by + ay * bw + az * bx - ax * bz
    z = aw * bz + az * bw + ax * by - ay * bx
    sq = x * x + y * y + z * z + w * w
    if sq != 1.0:
        f = 2.0 / (1.0 + sq)
        x, y, z, w = x * f, y * f, z * f, w * f
    return np.array([x, y, z, w, a[4] + t[0], a[5] + t[1], a[6] + t[2]])


def se3_inv(a):
    qi = np.array([-a[0], -a[1], -a[2], a[3]])
    t = so3_rotate(qi, -np.asarray(a[4:7]))
    return np.concatenate([qi, t])


def se3_act(T, p):
    return so3_rotate(T, p) + np.asarray(T[4:7])


@dataclass
class KeyFrame:
    """Mirror of CommonTypes.h:15-32 (the fields windowOptimize reads)."""

    T_w_c: np.ndarray  # (7,)
    keypoints: np.ndarray  # (K, 2) float32 pixel (cv::KeyPoint::pt)
    points3d_local: np.ndarray  # (K, 3)
    global_points_map: dict = field(default_factory=dict)  # localId -> LandmarkId (iteration order kept)
    timestamp: str = ""


def window_optimize(kf_i: int, kf_f: int, keyframes: list, landmarks: dict, intr_init, intr_opt: np.ndarray,
                    solve) -> dict:
    """windowOptimize (:215-313). ``landmarks``: LandmarkId -> (3,) point; ``intr_opt`` updated in place."""
    T0 = np.array(keyframes[kf_i].T_w_c, dtype=np.float64)
    T0inv = se3_inv(T0)
    cams = []
    obs_cam, obs_pt, uv, depth = [], [], [], []
    pt_index, ids, pts = {}, [], []
    for kf_n in range(kf_i, kf_f + 1):
        kf = keyframes[kf_n]
        kf.T_w_c = se3_mul(T0inv, kf.T_w_c)  # :248
        cams.append(kf.T_w_c.copy())
        for local_id, landmark_id in kf.global_points_map.items():  # :257
            d = float(kf.points3d_local[local_id][2])
            px, py = float(kf.keypoints[local_id][0]), float(kf.keypoints[local_id][1])
            if d <= 1e-15:  # :265-268
                continue
            if landmark_id not in pt_index:  # :271-276
                landmarks[landmark_id] = se3_act(T0inv, landmarks[landmark_id])
                pt_index[landmark_id] = len(ids)
                ids.append(landmark_id)
                pts.append(landmarks[landmark_id].copy())
            obs_cam.append(kf_n - kf_i)
            obs_pt.append(pt_index[landmark_id])
            uv.append((px, py))
            depth.append(d)
    summary = None
    try:
        # :300 — solved even when no observation is admissible: the IntrinsicsPrior block (:236-241) is always
        # added, so Ceres still pulls intr_opt toward intr_init (the poses have no residual and stay put)
        prob = ProblemArrays(np.array(cams), np.array(pts, dtype=np.float64).reshape(-1, 3),
                             np.array(intr_opt, dtype=np.float64), np.array(intr_init, dtype=np.float64),
                             np.array(obs_cam, dtype=np.int32), np.array(obs_pt, dtype=np.int32),
                             np.array(uv, dtype=np.float64).reshape(-1, 2), np.array(depth, dtype=np.float64),
                             fixed_cam=0)
        summary = solve(prob)
        intr_opt[:] = prob.intr
        for k, lid in enumerate(ids):
            landmarks[lid] = prob.points[k].copy()
        for kf_n in range(kf_i, kf_f + 1):
            keyframes[kf_n].T_w_c = prob.cams[kf_n - kf_i].copy()
    finally:
        # :303-310 map back — also when the solve raised, so the caller's window is never left re-anchored
        for kf_n in range(kf_i, kf_f + 1):
            keyframes[kf_n].T_w_c = se3_mul(T0, keyframes[kf_n].T_w_c)
        for lid in ids:
            landmarks[lid] = se3_act(T0, landmarks[lid])
    return summary


def window_schedule(frame_frequency: int, window_size: int, n_keyframes: int, tracking_finished: bool,
                    optimization_finished: bool, tracked_this_frame: bool):
    """(run, kf_i, kf_f, finishes) for main.cpp:163-183."""
    if optimization_finished:
        return (False, 0, 0, False)
    n = n_keyframes
    if window_size > 0:
        if tracked_this_frame and n % frame_frequency == 0 and n >= window_size:
            return (True, n - window_size, n - 1, False)
        if tracking_finished and n % frame_frequency != 0:
            return (True, max(n - window_size, 0), n - 1, True)
    elif window_size < 0 and tracking_finished:
        return (True, 0, n - 1, True)
    return (False, 0, 0, False)
