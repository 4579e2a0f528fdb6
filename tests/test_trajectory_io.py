"""include/ba_trajectory.hpp (getFirstPose / nearest_interp_1d / poseOffset /
write_keyframe_poses_to_file restated in C++) against its Python mirror miba/trajectory.py:
byte-identical TUM output on random keyframe sequences; plus the formatting and
nearest-neighbour rules of the reference (OptimizationUtils.cpp:160-172, 323-379)."""
import os
import subprocess

import numpy as np
import pytest

from miba import synthetic, trajectory
from miba.window import KeyFrame

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def traj_bin(tmp_path_factory):
    d = tmp_path_factory.mktemp("tr")
    exe = str(d / "trajectory_main")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "trajectory_main.cpp"), "-o", exe], check=True)
    return exe


def _gt_text(rng, n):
    lines = ["# ground truth trajectory", "# file: 'rgbd_dataset_freiburg1_xyz.bag'", "# timestamp tx ty tz qx qy qz qw"]
    t = 1305031098.6659 + np.cumsum(rng.uniform(0.009, 0.011, n))
    for k in range(n):
        q = rng.normal(size=4)
        q *= rng.uniform(0.99, 1.01) / np.linalg.norm(q)  # slightly off unit, as printed with 4 digits
        lines.append("%.4f %.4f %.4f %.4f %.4f %.4f %.4f %.4f" % (t[k], *rng.normal(size=3), *q))
    return "\n".join(lines) + "\n", t


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_cpp_matches_python_mirror(traj_bin, tmp_path, seed):
    rng = np.random.default_rng(seed)
    gt, t = _gt_text(rng, 400)
    (tmp_path / "gt.txt").write_text(gt)
    kfs, rows = [], []
    for k in range(30):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        T = np.concatenate([q, rng.normal(size=3)])
        stamp = "%.6f" % (t[5 + 9 * k] + rng.uniform(-0.004, 0.004))
        kfs.append(KeyFrame(T.copy(), np.zeros((0, 2)), np.zeros((0, 3)), {}, stamp))
        rows.append(stamp + " " + " ".join(repr(float(v)) for v in T))
    (tmp_path / "kfs.txt").write_text("\n".join(rows) + "\n")
    out = subprocess.run([traj_bin, str(tmp_path / "gt.txt"), str(tmp_path / "kfs.txt")], capture_output=True,
                         text=True, check=True).stdout
    first = trajectory.get_first_pose(kfs[0].timestamp, gt)
    trajectory.pose_offset(kfs, first)
    assert out == trajectory.format_keyframe_poses(kfs)
    # after the offset the first keyframe carries the ground-truth pose
    np.testing.assert_allclose(kfs[0].T_w_c, first, atol=1e-12)


def test_nearest_interp_first_minimum():
    _, idx = trajectory.nearest_interp_1d([0.0, 1.0, 2.0, 3.0], [0, 1, 2, 3], [1.5, -7.0, 2.6, 9.0])
    assert idx == [1, 0, 3, 3]  # ties keep the first index (strict '<')


def test_pose_line_format_is_iostream_default():
    kf = KeyFrame(np.array([0.0, 0.0, 0.70710678118, 0.70710678118, 1.23456789, -0.000012345, 1e7]),
                  np.zeros((0, 2)), np.zeros((0, 3)), {}, "1305031102.175304")
    assert trajectory.format_keyframe_poses([kf]) == "1305031102.175304 1.23457 -1.2345e-05 1e+07 0 0 0.707107 0.707107\n"
