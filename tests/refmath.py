"""Independent numpy restatement of the reference cost functors, used only to
pin the C oracle (finite differences, dense Schur). Written directly from
/root/reference/src/OptimizationUtils.cpp:25-49 (ReprojectionConstraint),
:72-94 (DepthPrior), :117-125 (IntrinsicsPrior) and Ceres' HuberLoss."""
import numpy as np


def quat_R(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def raw_residual(pose, X, K, uv, depth, w_r, w_d):
    """un-robustified residuals (r0, r1 | r2) of one observation"""
    R = quat_R(pose[:4])
    pc = R.T @ (np.asarray(X) - pose[4:7])
    Km = np.array([[K[0], 0, K[2]], [0, K[1], K[3]], [0, 0, 1.0]])
    pix = (Km @ pc / pc[2])[:2]
    r = np.sqrt(w_r) * (pix - np.asarray(uv))
    d = np.sqrt(w_d) * (depth - pc[2])
    return np.array([r[0], r[1], d])


def huber(s, a):
    b = a * a
    if s > b:
        r = np.sqrt(s)
        return 2 * a * r - b, max(np.finfo(float).tiny, a / r)
    return s, 1.0


def exp_se3(delta):
    """Sophus SE3::exp of [upsilon, omega] -> (R, t)"""
    ups, om = np.asarray(delta[:3]), np.asarray(delta[3:])
    th = np.linalg.norm(om)
    W = np.array([[0, -om[2], om[1]], [om[2], 0, -om[0]], [-om[1], om[0], 0]])
    if th < 1e-12:
        R = np.eye(3) + W
        V = np.eye(3) + 0.5 * W
    else:
        R = np.eye(3) + np.sin(th) / th * W + (1 - np.cos(th)) / th ** 2 * W @ W
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * W + (th - np.sin(th)) / th ** 3 * W @ W
    return R, V @ ups


def rot_to_quat(R):
    from scipy.spatial.transform import Rotation
    return Rotation.from_matrix(R).as_quat()  # x y z w


def plus_pose(pose, delta):
    """T * exp(delta) with an independent implementation"""
    R = quat_R(pose[:4]); t = pose[4:7]
    Rd, td = exp_se3(delta)
    Rn = R @ Rd
    tn = t + R @ td
    q = rot_to_quat(Rn)
    if np.dot(q, pose[:4]) < 0:
        q = -q
    return np.concatenate([q, tn])
