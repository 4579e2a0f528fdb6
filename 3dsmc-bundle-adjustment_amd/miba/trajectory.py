"""Python mirror of include/ba_trajectory.hpp: the TUM trajectory output around the solver
(getFirstPose / nearest_interp_1d / poseOffset / write_keyframe_poses_to_file,
OptimizationUtils.cpp:160-172, 323-379, nearest_interp_1d.cpp:11-78, called at main.cpp:191-195).
Same operation order as the C++ header; tests/test_trajectory_io.py checks the two match
byte for byte."""
from __future__ import annotations

import math

import numpy as np

from .window import se3_inv, se3_mul


def nearest_interp_1d(xd, yd, xi):
    """(yi, indices): first index minimising |x - xd[k]| for every x in xi."""
    yi, idx = [], []
    for x in xi:
        best, d = 0, abs(x - xd[0])
        for j in range(1, len(xd)):
            dj = abs(x - xd[j])
            if dj < d:
                best, d = j, dj
        idx.append(best)
        yi.append(yd[best])
    return yi, idx


def parse_ground_truth(text: str):
    """(timestamps, records[n,7] = tx ty tz qx qy qz qw): 3 header lines, then whitespace records."""
    body = text.split("\n", 3)[3] if text.count("\n") >= 3 else ""
    vals = [float(v) for v in body.split()]
    n = len(vals) // 8
    a = np.array(vals[:8 * n]).reshape(n, 8)
    return list(a[:, 0]), a[:, 1:]


def get_first_pose(first_timestamp: str, ground_truth_text: str) -> np.ndarray:
    """[qx,qy,qz,qw,tx,ty,tz] of the ground-truth record nearest to first_timestamp."""
    ts, rec = parse_ground_truth(ground_truth_text)
    _, idx = nearest_interp_1d(ts, ts, [float(first_timestamp)])
    tx, ty, tz, qx, qy, qz, qw = rec[idx[0]]
    n = math.sqrt(qw * qw + qx * qx + qy * qy + qz * qz)
    return np.array([qx / n, qy / n, qz / n, qw / n, tx, ty, tz])


def pose_offset(keyframes, initial_pose) -> None:
    """T <- (initial * T_0^-1) * T for every keyframe (keyframes[k].T_w_c, Sophus order)."""
    if not keyframes:
        return
    delta = se3_mul(np.asarray(initial_pose, dtype=np.float64), se3_inv(keyframes[0].T_w_c))
    for kf in keyframes:
        kf.T_w_c = se3_mul(delta, kf.T_w_c)


def _g(v: float) -> str:
    """std::ostream default floating formatting (precision 6, %g)."""
    return "%g" % v


def format_keyframe_poses(keyframes) -> str:
    """One line per keyframe: "timestamp tx ty tz qx qy qz qw"."""
    out = []
    for kf in keyframes:
        T = kf.T_w_c
        out.append(" ".join([str(kf.timestamp)] + [_g(T[i]) for i in (4, 5, 6, 0, 1, 2, 3)]))
    return "".join(line + "\n" for line in out)


def write_keyframe_poses_to_file(path: str, keyframes) -> None:
    with open(path, "w") as f:
        f.write(format_keyframe_poses(keyframes))
