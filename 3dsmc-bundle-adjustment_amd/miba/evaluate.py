"""ATE / RPE evaluation of TUM trajectories — a restatement of the reference's acceptance tools
(rgb-d-toolset/associate.py, evaluate_ate.py, evaluate_rpe.py) that the north_star names as the
pose-accuracy check ("pass the repo's evaluate_ate.py / evaluate_rpe.py within 1 mm").

Pinned against the reference scripts themselves: tests/golden/make_trajectory_golden.py imports
them (this container has /root/reference) and stores their outputs on fixed trajectories in
tests/golden/trajectory_golden.json; tests/test_trajectory.py checks this module against it.

Trajectory text format: ``stamp tx ty tz qx qy qz qw`` per line, '#' comments, ',' / tab
separators allowed (associate.py:58-67).
"""
from __future__ import annotations

import math
import random

import numpy as np


# ------------------------------------------------------------------ associate.py
def read_file_list(text: str) -> dict:
    """stamp -> list of data tokens (associate.py:46-67); ``text`` is the file content."""
    out = {}
    for line in text.replace(",", " ").replace("\t", " ").split("\n"):
        if not line or line[0] == "#":
            continue
        toks = [t.strip() for t in line.split(" ") if t.strip() != ""]
        if len(toks) > 1:
            out[float(toks[0])] = toks[1:]
    return out


def associate(first: dict, second: dict, offset: float = 0.0, max_difference: float = 0.02) -> list:
    """Greedy nearest-stamp matching (associate.py:69-101): candidate pairs within
    ``max_difference``, taken in increasing (|a - (b + offset)|, a, b) order, each stamp once;
    returned sorted by (a, b)."""
    cand = sorted((abs(a - (b + offset)), a, b) for a in first for b in second if abs(a - (b + offset)) < max_difference)
    used_a, used_b, matches = set(), set(), []
    for _, a, b in cand:
        if a not in used_a and b not in used_b:
            used_a.add(a)
            used_b.add(b)
            matches.append((a, b))
    matches.sort()
    return matches


# ------------------------------------------------------------------ evaluate_ate.py
def align(model: np.ndarray, data: np.ndarray):
    """Horn closed-form alignment of model (3xn) onto data (3xn) (evaluate_ate.py:51-83):
    SVD of the cross-covariance with the reflection fix. Returns rot (3x3), trans (3,),
    per-pair translational error (n,)."""
    model = np.asarray(model, dtype=np.float64)
    data = np.asarray(data, dtype=np.float64)
    mm = model.mean(axis=1, keepdims=True)
    dm = data.mean(axis=1, keepdims=True)
    W = (model - mm) @ (data - dm).T  # sum of outer(model_i, data_i)
    U, _, Vh = np.linalg.svd(W.T)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vh) < 0:
        S[2, 2] = -1.0
    rot = U @ S @ Vh
    trans = dm - rot @ mm
    err = rot @ model + trans - data
    return rot, trans[:, 0], np.sqrt(np.sum(err * err, axis=0))


def _euler_xyz_deg(quats: np.ndarray) -> np.ndarray:
    """scipy Rotation.from_quat(q).as_euler('xyz', degrees=True) (evaluate_ate.py:268-270)."""
    from scipy.spatial.transform import Rotation
    return Rotation.from_quat(quats).as_euler("xyz", degrees=True)


def _rms(v: np.ndarray) -> float:
    n = len(v)
    return float(np.sqrt(1 / n * np.sum(np.square(v))))


def ate(first_text: str, second_text: str, offset: float = 0.0, scale: float = 1.0, max_difference: float = 0.02,
        delta: int = 5, horn: bool = False) -> dict:
    """evaluate_ate.py:246-301 (first = ground truth, second = estimate): translational
    statistics after Horn alignment and the absolute / relative Euler-angle errors."""
    first = read_file_list(first_text)
    second = read_file_list(second_text)
    matches = associate(first, second, offset, max_difference)
    if len(matches) < 2:
        raise ValueError("Couldn't find matching timestamp pairs between groundtruth and estimated trajectory!")
    fx = np.array([[float(v) for v in first[a][0:3]] for a, _ in matches]).T
    sx = np.array([[float(v) * scale for v in second[b][0:3]] for _, b in matches]).T
    rot, trans, e = align(sx, fx)
    fq = np.array([[float(v) for v in first[a][3:7]] for a, _ in matches])
    sq = np.array([[float(v) for v in second[b][3:7]] for _, b in matches])
    fe = _euler_xyz_deg(fq)
    if horn:
        from scipy.spatial.transform import Rotation
        se = (Rotation.from_matrix(rot) * Rotation.from_quat(sq)).as_euler("xyz", degrees=True)
    else:
        se = _euler_xyz_deg(sq)
    d = int(delta)
    abs_err = [_rms(fe[:, k] - se[:, k]) for k in range(3)]  # AYE, APE, ARE (:168-189)
    rel_err = [_rms((fe[d:, k] - fe[:-d, k]) - (se[d:, k] - se[:-d, k])) for k in range(3)]  # RYE, RPE, RRE
    return {
        "pairs": len(e), "rmse": float(np.sqrt(np.dot(e, e) / len(e))), "mean": float(np.mean(e)),
        "median": float(np.median(e)), "std": float(np.std(e)), "min": float(np.min(e)), "max": float(np.max(e)),
        "trans_error": e, "matches": matches, "rot": rot, "trans": trans,
        "AYE": abs_err[0], "APE": abs_err[1], "ARE": abs_err[2], "RYE": rel_err[0], "RPE_pitch": rel_err[1],
        "RRE": rel_err[2],
    }


# ------------------------------------------------------------------ evaluate_rpe.py
_EPS4 = np.finfo(float).eps * 4.0


def transform44(stamp_pose) -> np.ndarray:
    """(stamp, tx, ty, tz, qx, qy, qz, qw) -> 4x4 (evaluate_rpe.py:48-75): q scaled by
    sqrt(2/|q|^2), rotation from its outer product; near-zero q -> identity rotation."""
    t = np.asarray(stamp_pose[1:4], dtype=np.float64)
    q = np.array(stamp_pose[4:8], dtype=np.float64)
    T = np.eye(4)
    T[0:3, 3] = t
    nq = float(np.dot(q, q))
    if nq < _EPS4:
        return T
    q = q * math.sqrt(2.0 / nq)
    o = np.outer(q, q)
    T[0:3, 0:3] = [[1.0 - o[1, 1] - o[2, 2], o[0, 1] - o[2, 3], o[0, 2] + o[1, 3]],
                   [o[0, 1] + o[2, 3], 1.0 - o[0, 0] - o[2, 2], o[1, 2] - o[0, 3]],
                   [o[0, 2] - o[1, 3], o[1, 2] + o[0, 3], 1.0 - o[0, 0] - o[1, 1]]]
    return T


def read_trajectory(text: str, matrix: bool = True) -> dict:
    """stamp -> 4x4 (or the 7 values) (evaluate_rpe.py:77-107); lines whose quaternion is
    exactly (0,0,0,0) or that contain a NaN are skipped."""
    rows = []
    for line in text.replace(",", " ").replace("\t", " ").split("\n"):
        if not line or line[0] == "#":
            continue
        vals = [float(t.strip()) for t in line.split(" ") if t.strip() != ""]
        if vals[4:8] == [0, 0, 0, 0] or any(math.isnan(v) for v in vals):
            continue
        rows.append(vals)
    return {r[0]: (transform44(r) if matrix else r[1:8]) for r in rows}


def find_closest_index(L, t) -> int:
    """Binary search that keeps the closest element seen along its path
    (evaluate_rpe.py:109-133) — not always the global nearest on unsorted input."""
    lo, hi = 0, len(L)
    best, diff = 0, abs(L[0] - t)
    while lo < hi:
        mid = (lo + hi) // 2
        if abs(L[mid] - t) < diff:
            diff, best = abs(L[mid] - t), mid
        if t == L[mid]:
            return mid
        if L[mid] > t:
            hi = mid
        else:
            lo = mid + 1
    return best


def ominus(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """a^-1 b (evaluate_rpe.py:135-146)."""
    return np.linalg.inv(a) @ b


def _scale_t(a: np.ndarray, s: float) -> np.ndarray:
    out = a.copy()
    out[0:3, 3] *= s
    return out


def compute_distance(T: np.ndarray) -> float:
    return float(np.linalg.norm(T[0:3, 3]))


def compute_angle(T: np.ndarray) -> float:
    return float(np.arccos(min(1, max(-1, (np.trace(T[0:3, 0:3]) - 1) / 2))))


def _along(traj: dict, fn) -> list:
    keys = sorted(traj)
    out, acc = [0], 0
    for i in range(len(keys) - 1):
        acc += fn(ominus(traj[keys[i + 1]], traj[keys[i]]))
        out.append(acc)
    return out


def evaluate_trajectory(traj_gt: dict, traj_est: dict, max_pairs: int = 10000, fixed_delta: bool = False,
                        delta: float = 1.0, delta_unit: str = "s", offset: float = 0.0, scale: float = 1.0) -> list:
    """Relative pose error pairs [stamp_est0, stamp_est1, stamp_gt0, stamp_gt1, trans, rot]
    (evaluate_rpe.py:197-286). Pair sampling draws from Python's ``random`` module exactly as
    the reference does: seed it (the reference script uses random.seed(0)) before calling."""
    sg = sorted(traj_gt)
    se = sorted(traj_est)
    back = []
    for t in se:
        tg = sg[find_closest_index(sg, t + offset)]
        tr = se[find_closest_index(se, tg - offset)]
        if tr not in back:
            back.append(tr)
    if len(back) < 2:
        raise ValueError("Number of overlap in the timestamps is too small.")
    n = len(traj_est)
    if delta_unit == "s":
        index_est = list(se)
    elif delta_unit == "m":
        index_est = _along(traj_est, compute_distance)
    elif delta_unit in ("rad", "deg"):
        k = 1.0 if delta_unit == "rad" else 180 / np.pi
        index_est = _along(traj_est, lambda T: compute_angle(T) * k)
    elif delta_unit == "f":
        index_est = list(range(n))
    else:
        raise ValueError(f"Unknown unit for delta: '{delta_unit}'")
    if not fixed_delta:
        if max_pairs == 0 or n < np.sqrt(max_pairs):
            pairs = [(i, j) for i in range(n) for j in range(n)]
        else:
            pairs = [(random.randint(0, n - 1), random.randint(0, n - 1)) for _ in range(max_pairs)]
    else:
        pairs = []
        for i in range(n):
            j = find_closest_index(index_est, index_est[i] + delta)
            if j != n - 1:
                pairs.append((i, j))
        if max_pairs != 0 and len(pairs) > max_pairs:
            pairs = random.sample(pairs, max_pairs)
    max_dt = 2 * np.median([s - t for s, t in zip(sg[1:], sg[:-1])])
    res = []
    for i, j in pairs:
        e0, e1 = se[i], se[j]
        g0 = sg[find_closest_index(sg, e0 + offset)]
        g1 = sg[find_closest_index(sg, e1 + offset)]
        if abs(g0 - (e0 + offset)) > max_dt or abs(g1 - (e1 + offset)) > max_dt:
            continue
        err = ominus(_scale_t(ominus(traj_est[e1], traj_est[e0]), scale), ominus(traj_gt[g1], traj_gt[g0]))
        res.append([e0, e1, g0, g1, compute_distance(err), compute_angle(err)])
    if len(res) < 2:
        raise ValueError("Couldn't find matching timestamp pairs between groundtruth and estimated trajectory!")
    return res


def rpe(gt_text: str, est_text: str, seed: int | None = 0, **kw) -> dict:
    """evaluate_rpe.py __main__ statistics (:335-366), with random.seed(seed) first."""
    if seed is not None:
        random.seed(seed)
    r = np.array(evaluate_trajectory(read_trajectory(gt_text), read_trajectory(est_text), **kw))
    te, re = r[:, 4], r[:, 5]
    return {"pairs": len(te), "trans_rmse": float(np.sqrt(np.dot(te, te) / len(te))), "trans_mean": float(np.mean(te)),
            "trans_median": float(np.median(te)), "trans_std": float(np.std(te)), "trans_min": float(np.min(te)),
            "trans_max": float(np.max(te)), "rot_rmse_deg": float(np.sqrt(np.dot(re, re) / len(re)) * 180 / np.pi),
            "rot_mean_deg": float(np.mean(re) * 180 / np.pi), "result": r}


def percentile(seq, q: float):
    s = sorted(seq)
    return s[int((len(s) - 1) * q)]
