"""Synthetic window generator for BASELINE.json configs C2/C4/C5
and TUM-like C1/C3 stand-ins.

The reference publishes no benchmark data and the TUM sequences are not in the
image, so every measured configuration uses synthetic windows of the stated
(cams, points, obs) shape, built like a TUM RGB-D window:

* intrinsics prior = Data/ros_default_intrinsics.txt:1 (525, 525, 319.5, 239.5),
  640x480 image; the true intrinsics are offset by a few pixels so the
  intrinsics block (IntrinsicsPrior, OptimizationUtils.cpp:110-137) has work;
* cameras on a smooth curve, ~1 cm per frame, yaw/pitch <= 0.3 rad;
* every point is observed by a contiguous band of cameras around its birth
  camera (banded co-visibility as in sequential keyframes, Map3D.cpp:7-74);
* pixel noise N(0, 0.5 px) + 2 % outliers U(+-20 px) (exercises the Huber loss,
  OptimizationUtils.cpp:223-226); depth = z (1 + N(0, 0.01))
  (points3d_local z, OptimizationUtils.cpp:261);
* initial poses perturbed by 0.01 rad / 1 cm, points by 2 cm, intrinsics at the
  prior; camera 0 is the gauge (SetParameterBlockConstant, :299);
* ``sensor_f32`` (the BASELINE configs, make_config): pixel coordinates and depths are
  float32 values, as the reference's are — cv::KeyPoint::pt is a Point2f and the depth
  comes from a float depth image (OptimizationUtils.cpp:261-262, Map3D.cpp:85-88); the
  solver widens them to f64 exactly (make_problem's default keeps full f64 values, the
  general input the C-ABI accepts).
"""
from __future__ import annotations

import numpy as np

from .capi import ProblemArrays

ROS_DEFAULT_INTRINSICS = np.array([525.0, 525.0, 319.5, 239.5])  # Data/ros_default_intrinsics.txt:1
IMAGE_W, IMAGE_H = 640, 480

# BASELINE.json configs -> (n_cams, n_points, obs_per_point, seed)
CONFIGS = {
    "C1": dict(n_cams=10, n_points=800, obs_per_point=(2, 2), seed=1),   # TUM fr1/xyz-like 10-kf window
    "C2": dict(n_cams=20, n_points=5000, obs_per_point=10, seed=2),     # 20 / 5k / 50k
    "C3": dict(n_cams=50, n_points=4000, obs_per_point=(2, 2), seed=3),  # fr2/desk-like 50-kf window
    "C4": dict(n_cams=200, n_points=100000, obs_per_point=10, seed=4),  # 200 / 100k / 1M
    "C5": dict(n_cams=1000, n_points=500000, obs_per_point=10, seed=5),  # 1000 / 500k / 5M
}


def quat_from_rotmat(R: np.ndarray) -> np.ndarray:
    """Rotation matrices (...,3,3) -> quaternions (...,4) in Sophus order x,y,z,w (w >= 0)."""
    R = np.asarray(R, dtype=np.float64)
    m = R.reshape(-1, 3, 3)
    q = np.empty((m.shape[0], 4))
    tr = m[:, 0, 0] + m[:, 1, 1] + m[:, 2, 2]
    for i in range(m.shape[0]):
        a = m[i]
        if tr[i] > 0:
            s = np.sqrt(tr[i] + 1.0) * 2
            w = 0.25 * s
            x = (a[2, 1] - a[1, 2]) / s
            y = (a[0, 2] - a[2, 0]) / s
            z = (a[1, 0] - a[0, 1]) / s
        elif a[0, 0] > a[1, 1] and a[0, 0] > a[2, 2]:
            s = np.sqrt(1.0 + a[0, 0] - a[1, 1] - a[2, 2]) * 2
            w = (a[2, 1] - a[1, 2]) / s
            x = 0.25 * s
            y = (a[0, 1] + a[1, 0]) / s
            z = (a[0, 2] + a[2, 0]) / s
        elif a[1, 1] > a[2, 2]:
            s = np.sqrt(1.0 + a[1, 1] - a[0, 0] - a[2, 2]) * 2
            w = (a[0, 2] - a[2, 0]) / s
            x = (a[0, 1] + a[1, 0]) / s
            y = 0.25 * s
            z = (a[1, 2] + a[2, 1]) / s
        else:
            s = np.sqrt(1.0 + a[2, 2] - a[0, 0] - a[1, 1]) * 2
            w = (a[1, 0] - a[0, 1]) / s
            x = (a[0, 2] + a[2, 0]) / s
            y = (a[1, 2] + a[2, 1]) / s
            z = 0.25 * s
        v = np.array([x, y, z, w])
        v /= np.linalg.norm(v)
        if v[3] < 0:
            v = -v
        q[i] = v
    return q.reshape(R.shape[:-2] + (4,))


def rotmat_from_quat(q: np.ndarray) -> np.ndarray:
    """Quaternions (...,4) x,y,z,w -> rotation matrices (Eigen toRotationMatrix formula)."""
    q = np.asarray(q, dtype=np.float64)
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    R = np.empty(q.shape[:-1] + (3, 3))
    R[..., 0, 0] = 1 - (ty * y + tz * z)
    R[..., 0, 1] = ty * x - tz * w
    R[..., 0, 2] = tz * x + ty * w
    R[..., 1, 0] = ty * x + tz * w
    R[..., 1, 1] = 1 - (tx * x + tz * z)
    R[..., 1, 2] = tz * y - tx * w
    R[..., 2, 0] = tz * x - ty * w
    R[..., 2, 1] = tz * y + tx * w
    R[..., 2, 2] = 1 - (tx * x + ty * y)
    return R


def _rodrigues(w: np.ndarray) -> np.ndarray:
    """axis-angle (...,3) -> rotation matrices (...,3,3)."""
    w = np.asarray(w, dtype=np.float64)
    th = np.linalg.norm(w, axis=-1, keepdims=True)
    k = np.where(th > 1e-15, w / np.maximum(th, 1e-300), 0.0)
    K = np.zeros(w.shape[:-1] + (3, 3))
    K[..., 0, 1], K[..., 0, 2] = -k[..., 2], k[..., 1]
    K[..., 1, 0], K[..., 1, 2] = k[..., 2], -k[..., 0]
    K[..., 2, 0], K[..., 2, 1] = -k[..., 1], k[..., 0]
    th = th[..., None]
    I = np.broadcast_to(np.eye(3), K.shape)
    return I + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def _trajectory(n_cams: int):
    t = np.arange(n_cams, dtype=np.float64)
    pos = np.stack([0.01 * t, 0.04 * np.sin(t / 35.0), 0.03 * np.sin(t / 50.0 + 0.5)], axis=1)
    yaw = 0.3 * np.sin(t / 60.0)
    pitch = 0.15 * np.sin(t / 45.0 + 1.0)
    cy, sy, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch)
    Ry = np.zeros((n_cams, 3, 3))
    Ry[:, 0, 0], Ry[:, 0, 2], Ry[:, 1, 1], Ry[:, 2, 0], Ry[:, 2, 2] = cy, sy, 1.0, -sy, cy
    Rx = np.zeros((n_cams, 3, 3))
    Rx[:, 0, 0], Rx[:, 1, 1], Rx[:, 1, 2], Rx[:, 2, 1], Rx[:, 2, 2] = 1.0, cp, -sp, sp, cp
    return Ry @ Rx, pos


def make_problem(n_cams: int, n_points: int, obs_per_point=10, seed: int = 0, pixel_noise: float = 0.5,
                 outlier_frac: float = 0.02, outlier_px: float = 20.0, depth_noise: float = 0.01,
                 rot_noise: float = 0.01, trans_noise: float = 0.01, point_noise: float = 0.02,
                 intr_offset=(2.0, -1.5, 1.0, -0.8), fixed_cam: int = 0, shuffle_obs: bool = False,
                 bad_depth_frac: float = 0.0, dup_frac: float = 0.0, cam_seed: int | None = None,
                 sensor_f32: bool = False) -> ProblemArrays:
    """Build one synthetic window. ``obs_per_point`` is an int or an inclusive (lo, hi) range.
    ``cam_seed`` draws the initial camera perturbation from its own stream, so landmark
    shards generated with different ``seed`` share identical window cameras."""
    rng = np.random.default_rng(seed)
    if isinstance(obs_per_point, (tuple, list)):
        lo, hi = int(obs_per_point[0]), int(obs_per_point[1])
    else:
        lo = hi = int(obs_per_point)
    hi = min(hi, n_cams)
    lo = min(lo, hi)
    nobs_pt = rng.integers(lo, hi + 1, size=n_points) if hi > lo else np.full(n_points, hi)
    R_wc, t_wc = _trajectory(n_cams)
    K_true = ROS_DEFAULT_INTRINSICS + np.asarray(intr_offset, dtype=np.float64)
    # band start spreads points evenly over the trajectory
    start = np.floor(np.arange(n_points) * (n_cams - nobs_pt + 1) / max(n_points, 1)).astype(np.int64)
    start = np.minimum(start, n_cams - nobs_pt)
    birth = start + nobs_pt // 2
    u = rng.uniform(60, IMAGE_W - 60, n_points)
    v = rng.uniform(50, IMAGE_H - 50, n_points)
    z = rng.uniform(0.8, 4.0, n_points)
    pc = np.stack([(u - K_true[2]) / K_true[0] * z, (v - K_true[3]) / K_true[1] * z, z], axis=1)
    X = np.einsum("nij,nj->ni", R_wc[birth], pc) + t_wc[birth]
    n_obs = int(nobs_pt.sum())
    obs_pt = np.repeat(np.arange(n_points, dtype=np.int64), nobs_pt)
    first = np.cumsum(nobs_pt) - nobs_pt
    within = np.arange(n_obs) - np.repeat(first, nobs_pt)
    obs_cam = np.repeat(start, nobs_pt) + within
    Rc = R_wc[obs_cam]
    d = X[obs_pt] - t_wc[obs_cam]
    p_c = np.einsum("nji,nj->ni", Rc, d)  # R^T (X - t)
    zc = p_c[:, 2]
    if np.any(zc <= 0.05):
        raise RuntimeError("synthetic generator produced a point behind a camera")
    uv = np.stack([K_true[0] * p_c[:, 0] / zc + K_true[2], K_true[1] * p_c[:, 1] / zc + K_true[3]], axis=1)
    uv += rng.normal(0.0, pixel_noise, uv.shape)
    out = rng.random(n_obs) < outlier_frac
    uv[out] += rng.uniform(-outlier_px, outlier_px, (int(out.sum()), 2))
    depth = zc * (1.0 + rng.normal(0.0, depth_noise, n_obs))
    if bad_depth_frac > 0:
        bad = rng.random(n_obs) < bad_depth_frac
        depth[bad] = np.where(rng.random(int(bad.sum())) < 0.5, 0.0, -np.inf)  # VirtualSensor MINF / 0
    # initial estimate
    crng = rng if cam_seed is None else np.random.default_rng(cam_seed)
    dR = _rodrigues(crng.normal(0.0, rot_noise, (n_cams, 3)))
    R0 = R_wc @ dR
    t0 = t_wc + crng.normal(0.0, trans_noise, (n_cams, 3))
    if 0 <= fixed_cam < n_cams:
        R0[fixed_cam] = R_wc[fixed_cam]
        t0[fixed_cam] = t_wc[fixed_cam]
    cams = np.concatenate([quat_from_rotmat(R0), t0], axis=1)
    pts0 = X + rng.normal(0.0, point_noise, X.shape)
    if dup_frac > 0:
        # the same landmark linked to a second keypoint of the same keyframe
        dup = np.nonzero(rng.random(n_obs) < dup_frac)[0]
        obs_cam = np.concatenate([obs_cam, obs_cam[dup]])
        obs_pt = np.concatenate([obs_pt, obs_pt[dup]])
        uv = np.concatenate([uv, uv[dup] + rng.normal(0.0, 1.0, (len(dup), 2))])
        depth = np.concatenate([depth, depth[dup] * (1.0 + rng.normal(0.0, depth_noise, len(dup)))])
        n_obs = len(obs_cam)
    if shuffle_obs:
        perm = rng.permutation(n_obs)
        obs_cam, obs_pt, uv, depth = obs_cam[perm], obs_pt[perm], uv[perm], depth[perm]
    if sensor_f32:  # keypoints and depth as the reference's sensor types hold them (float32)
        uv = uv.astype(np.float32).astype(np.float64)
        depth = depth.astype(np.float32).astype(np.float64)
    truth = dict(cams=np.concatenate([quat_from_rotmat(R_wc), t_wc], axis=1), points=X, intr=K_true)
    return ProblemArrays(cams, pts0, ROS_DEFAULT_INTRINSICS.copy(), ROS_DEFAULT_INTRINSICS.copy(), obs_cam, obs_pt,
                         uv, depth, fixed_cam, meta=dict(truth=truth, seed=seed))


def make_config(name: str, **overrides) -> ProblemArrays:
    cfg = dict(CONFIGS[name], sensor_f32=True)
    cfg.update(overrides)
    return make_problem(**cfg)


def make_landmark_shard(name: str, shard: int, **overrides) -> ProblemArrays:
    """Landmark shard ``shard`` of a window with the cameras of config ``name``: the same
    (seeded) initial cameras and intrinsics on every shard, an independent block of the
    config's size of landmarks per shard (weak scaling of ba_comm_init sharding)."""
    cfg = dict(CONFIGS[name], sensor_f32=True)
    cfg.update(overrides)
    base = cfg["seed"]
    cfg["seed"] = base + 1009 * shard
    cfg["cam_seed"] = base
    return make_problem(**cfg)
