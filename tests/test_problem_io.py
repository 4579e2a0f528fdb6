"""include/ba_io.h (libmiba's window dumps and BAL loader) against the independent numpy
restatement in tests/refio.py. The file functions are host-only, so all but the last two
tests run without a GPU."""
import ctypes as C
import os

import numpy as np
import pytest

import refio
from miba import _lib, problem_io, synthetic
from miba.capi import BaOptions


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def _small(seed=3, **kw):
    return synthetic.make_problem(8, 250, obs_per_point=(3, 6), seed=seed, **kw)


def _opts(L, **kw):
    o = BaOptions()
    L.ba_default_options(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


@pytest.mark.parametrize("with_opts", [False, True])
def test_window_dump_layout_matches_restatement(L, tmp_path, with_opts):
    p = _small()
    p.fixed_cam = 2
    o = _opts(L, max_num_iterations=17, weight_unpr=3.5) if with_opts else None
    path = tmp_path / "w.miba"
    problem_io.write_window(str(path), p, o)
    assert path.read_bytes() == refio.miba_bytes(p, o)
    q, qo = problem_io.read_window(str(path))
    for f in ("cams", "points", "intr", "intr_prior", "obs_cam", "obs_pt", "obs_uv", "obs_depth"):
        np.testing.assert_array_equal(getattr(q, f), getattr(p, f), err_msg=f)
    assert q.fixed_cam == 2
    expect = o if with_opts else _opts(L)
    assert bytes(qo) == bytes(expect)


def test_window_dump_empty_window(L, tmp_path):
    p = _small()
    e = type(p)(np.zeros((0, 7)), np.zeros((0, 3)), p.intr, p.intr_prior, [], [], np.zeros((0, 2)), [], fixed_cam=-1)
    problem_io.write_window(str(tmp_path / "e.miba"), e)
    q, _ = problem_io.read_window(str(tmp_path / "e.miba"))
    assert (q.n_cams, q.n_points, q.n_obs, q.fixed_cam) == (0, 0, 0, -1)


def test_window_dump_rejects_corruption(L, tmp_path):
    p = _small()
    good = refio.miba_bytes(p)
    cases = {
        "flip": good[:500] + bytes([good[500] ^ 1]) + good[501:],
        "trunc": good[:-8],
        "magic": b"MIBAWIN2" + good[8:],
        "header": good[:60],
    }
    bad_idx = p.copy()
    bad_idx.obs_pt[7] = p.n_points  # consistent checksum, index out of range
    cases["index"] = refio.miba_bytes(bad_idx)
    msgs = {}
    for name, data in cases.items():
        f = tmp_path / (name + ".miba")
        f.write_bytes(data)
        with pytest.raises(problem_io.ProblemFileError) as ei:
            problem_io.read_window(str(f))
        msgs[name] = str(ei.value)
    assert "checksum" in msgs["flip"]
    assert "bytes" in msgs["trunc"]
    assert "not a .miba" in msgs["magic"]
    assert "truncated header" in msgs["header"]
    assert "out of range" in msgs["index"]


def test_bal_write_uses_bal_camera_model(L, tmp_path):
    p = _small(seed=5)
    p.intr[:] = [520.0, 520.0, 321.5, 236.25]  # BAL has one focal: fx == fy
    path = tmp_path / "w.bal"
    problem_io.write_bal(str(path), p)
    oc, op, meas, cams, pts = refio.parse_bal(path.read_text())
    np.testing.assert_array_equal(oc, p.obs_cam)
    np.testing.assert_array_equal(op, p.obs_pt)
    np.testing.assert_array_equal(pts, p.points)
    np.testing.assert_array_equal(meas[:, 0], p.obs_uv[:, 0] - p.intr[2])
    np.testing.assert_array_equal(meas[:, 1], -(p.obs_uv[:, 1] - p.intr[3]))
    for k in range(0, p.n_obs, 7):
        X = p.points[p.obs_pt[k]]
        uv, _ = refio.project(p.cams[p.obs_cam[k]], p.intr, X)
        b = refio.bal_project(cams[p.obs_cam[k]], X)
        np.testing.assert_allclose(b, [uv[0] - p.intr[2], -(uv[1] - p.intr[3])], rtol=0, atol=1e-9)


def test_bal_round_trip_preserves_reprojection(L, tmp_path):
    p = _small(seed=6)
    p.intr[:] = [520.0, 520.0, 321.5, 236.25]
    path = tmp_path / "w.bal"
    problem_io.write_bal(str(path), p)
    q = problem_io.read_bal(str(path))
    assert (q.n_cams, q.n_points, q.n_obs, q.fixed_cam) == (p.n_cams, p.n_points, p.n_obs, 0)
    np.testing.assert_array_equal(q.intr, [520.0, 520.0, 0.0, 0.0])
    np.testing.assert_array_equal(q.intr_prior, q.intr)
    np.testing.assert_array_equal(q.points, p.points)
    for k in range(p.n_obs):
        X = p.points[p.obs_pt[k]]
        uv0, _ = refio.project(p.cams[p.obs_cam[k]], p.intr, X)
        uv1, z1 = refio.project(q.cams[q.obs_cam[k]], q.intr, X)
        np.testing.assert_allclose(uv1 - q.obs_uv[k], uv0 - p.obs_uv[k], rtol=0, atol=1e-8)
        assert abs(q.obs_depth[k] - z1) <= 1e-12 * max(1.0, z1)  # depth = initial-camera z
    # poses agree up to the quaternion sign
    for T0, T1 in zip(p.cams, q.cams):
        s = np.sign(T0[3]) * np.sign(T1[3])
        np.testing.assert_allclose(T1[:4] * s, T0[:4], atol=1e-12)
        np.testing.assert_allclose(T1[4:], T0[4:], atol=1e-12)


def test_bal_reader_undistorts_to_shared_focal(L, tmp_path):
    """Noise-free BAL data with per-camera focal and radial distortion: after loading, the
    reference's pinhole model at the shared focal reproduces every observation."""
    rng = np.random.default_rng(0)
    nc, np_ = 5, 40
    cams = np.zeros((nc, 9))
    cams[:, :3] = rng.normal(0, 0.1, (nc, 3))
    cams[:, 3:6] = rng.normal(0, 0.2, (nc, 3)) + [0, 0, -4.0]
    cams[:, 6] = rng.uniform(480, 560, nc)
    cams[:, 7] = rng.uniform(-0.2, 0.2, nc)
    cams[:, 8] = rng.uniform(-0.05, 0.05, nc)
    pts = rng.normal(0, 0.6, (np_, 3))
    lines, n = [], 0
    for i in range(nc):
        for j in range(np_):
            if (i + j) % 3 == 0:
                continue
            x, y = refio.bal_project(cams[i], pts[j])
            lines.append("%d %d %.17g %.17g" % (i, j, x, y))
            n += 1
    text = "%d %d %d\n" % (nc, np_, n) + "\n".join(lines) + "\n"
    text += "\n".join("%.17g" % v for v in cams.ravel()) + "\n" + "\n".join("%.17g" % v for v in pts.ravel()) + "\n"
    (tmp_path / "d.bal").write_text(text)
    q = problem_io.read_bal(str(tmp_path / "d.bal"))
    assert q.intr[0] == np.median(cams[:, 6])
    for k in range(q.n_obs):
        uv, z = refio.project(q.cams[q.obs_cam[k]], q.intr, q.points[q.obs_pt[k]])
        np.testing.assert_allclose(uv, q.obs_uv[k], rtol=0, atol=1e-8)
        assert z > 0 and abs(q.obs_depth[k] - z) <= 1e-12 * z


def test_bal_reader_rejects_bad_files(L, tmp_path):
    f = tmp_path / "b.bal"
    f.write_text("1 1 1\n0 3 1.0 2.0\n" + "0\n" * 9 + "1\n2\n3\n")
    with pytest.raises(problem_io.ProblemFileError, match="out of range"):
        problem_io.read_bal(str(f))
    f.write_text("1 1 2\n0 0 1.0 2.0\n")
    with pytest.raises(problem_io.ProblemFileError, match="malformed"):
        problem_io.read_bal(str(f))
    with pytest.raises(problem_io.ProblemFileError, match="cannot"):
        problem_io.read_bal(str(tmp_path / "missing.bal"))


@pytest.mark.gpu
def test_dump_dir_captures_and_replays(tmp_path, monkeypatch):
    """MIBA_DUMP_DIR captures the window ba_solve received; replaying the dump reproduces the solve."""
    from miba.solver import Solver
    p = synthetic.make_config("C2")
    p0 = p.copy()
    monkeypatch.setenv("MIBA_DUMP_DIR", str(tmp_path))
    with Solver(minimizer_progress_to_stdout=0, max_num_iterations=9) as s:
        s1 = s.solve(p)
    monkeypatch.delenv("MIBA_DUMP_DIR")
    files = sorted(tmp_path.glob("window_*.miba"))
    assert len(files) == 1
    q, o = problem_io.read_window(str(files[0]))
    np.testing.assert_array_equal(q.cams, p0.cams)
    np.testing.assert_array_equal(q.obs_uv, p0.obs_uv)
    assert o.max_num_iterations == 9
    with Solver(o) as s:
        s2 = s.solve(q)
    assert s2["num_iterations"] == s1["num_iterations"]
    assert abs(s2["final_cost"] - s1["final_cost"]) <= 1e-12 * s1["final_cost"]
    np.testing.assert_allclose(q.cams, p.cams, atol=1e-12)


@pytest.mark.gpu
def test_bal_problem_gpu_matches_oracle(tmp_path):
    from miba.solver import Solver
    from oracle import oracle
    p = synthetic.make_config("C2")
    p.intr[:] = p.intr_prior[:] = [525.0, 525.0, 319.5, 239.5]
    problem_io.write_bal(str(tmp_path / "c2.bal"), p)
    q = problem_io.read_bal(str(tmp_path / "c2.bal"))
    for w_unpr in (10.0, 0.0):
        a, b = q.copy(), q.copy()
        with Solver(minimizer_progress_to_stdout=0, weight_unpr=w_unpr) as s:
            sg = s.solve(a)
        sc = oracle.solve(b, oracle.default_options(weight_unpr=w_unpr))
        assert abs(sg["final_cost"] - sc["final_cost"]) <= 1e-6 * sc["final_cost"]
        assert sg["final_cost"] < sg["initial_cost"]
