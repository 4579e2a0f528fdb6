"""Independent numpy restatement of include/ba_io.h (the .miba dump layout and the BAL
conversion), used only to check libmiba's C implementation (tests/test_problem_io.py)."""
import struct

import numpy as np

from miba.capi import BaOptions, ProblemArrays

MAGIC = b"MIBAWIN1"
FNV_OFFSET, FNV_PRIME = 1469598103934665603, 1099511628211


def fnv1a(data: bytes, h: int = FNV_OFFSET) -> int:
    a = np.frombuffer(data, np.uint8)
    for b in a.tolist():
        h = ((h ^ b) * FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h


def miba_bytes(p: ProblemArrays, opts: BaOptions | None = None) -> bytes:
    body = b"".join([p.cams.tobytes(), p.points.tobytes(), p.obs_uv.tobytes(), p.obs_depth.tobytes(),
                     p.obs_cam.astype("<i4").tobytes(), p.obs_pt.astype("<i4").tobytes()])
    body += b"\0" * (-len(body) % 8)
    if opts is not None:
        body += bytes(opts)
    head = MAGIC + struct.pack("<II4i8d", 1, len(bytes(opts)) if opts is not None else 0, p.n_cams, p.n_points,
                               p.n_obs, int(p.fixed_cam), *p.intr, *p.intr_prior)
    head += struct.pack("<QQ", fnv1a(body), 0)
    assert len(head) == 112
    return head + body


def quat_mul(a, b):
    return np.array([a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1],
                     a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2],
                     a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0],
                     a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2]])


def rotmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def rodrigues_R(r):
    th = np.linalg.norm(r)
    if th == 0:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def parse_bal(text: str):
    tok = text.split()
    nc, np_, no = int(tok[0]), int(tok[1]), int(tok[2])
    o = np.array(tok[3:3 + 4 * no], dtype=object).reshape(no, 4)
    cams = np.array(tok[3 + 4 * no:3 + 4 * no + 9 * nc], dtype=np.float64).reshape(nc, 9)
    pts = np.array(tok[3 + 4 * no + 9 * nc:3 + 4 * no + 9 * nc + 3 * np_], dtype=np.float64).reshape(np_, 3)
    return o[:, 0].astype(np.int64), o[:, 1].astype(np.int64), o[:, 2:].astype(np.float64), cams, pts


def bal_project(cam9, X):
    """BAL camera model (Snavely et al.): pixel of world point X."""
    P = rodrigues_R(cam9[:3]) @ X + cam9[3:6]
    p = -P[:2] / P[2]
    r2 = p @ p
    return cam9[6] * (1 + cam9[7] * r2 + cam9[8] * r2 * r2) * p


def project(T, K, X):
    """The reference's pinhole model (OptimizationUtils.cpp:36-42): pixel of world point X."""
    pc = rotmat(T[:4]).T @ (X - T[4:7])
    return np.array([K[0] * pc[0] / pc[2] + K[2], K[1] * pc[1] / pc[2] + K[3]]), pc[2]
