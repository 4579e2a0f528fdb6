"""include/ba_window.hpp (C++ adapter of windowOptimize, OptimizationUtils.cpp:215-313)
against the independent Python mirror miba/window.py, both driving the CPU oracle
on the same dumped keyframe sequence (same global_points_map iteration order)."""
import os
import subprocess

import numpy as np
import pytest

from miba import window
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_dump(path):
    toks = open(path).read().split()
    it = iter(toks)
    assert next(it) == "K"
    kfs = []
    for _ in range(int(next(it))):
        T = np.array([float(next(it)) for _ in range(7)])
        nkp = int(next(it))
        kp = np.zeros((nkp, 2), dtype=np.float32)
        loc = np.zeros((nkp, 3))
        for i in range(nkp):
            kp[i] = [np.float32(next(it)), np.float32(next(it))]
            loc[i] = [float(next(it)) for _ in range(3)]
        gpm = {}
        for _ in range(int(next(it))):
            a = int(next(it)); b = int(next(it))
            gpm[a] = b
        kfs.append(window.KeyFrame(T, kp, loc, gpm))
    assert next(it) == "L"
    lms = {}
    for _ in range(int(next(it))):
        i = int(next(it))
        lms[i] = np.array([float(next(it)) for _ in range(3)])
    assert next(it) == "I"
    K0 = np.array([float(next(it)) for _ in range(4)])
    K = np.array([float(next(it)) for _ in range(4)])
    assert next(it) == "W"
    kf_i, kf_f = int(next(it)), int(next(it))
    summ = None
    rest = list(it)
    if rest and rest[0] == "S":
        summ = dict(initial_cost=float(rest[1]), final_cost=float(rest[2]), iters=int(rest[3]))
    return kfs, lms, K0, K, kf_i, kf_f, summ


@pytest.fixture(scope="module")
def adapter_bin(tmp_path_factory):
    oracle.lib()  # builds oracle/_build/libba_oracle.so
    d = tmp_path_factory.mktemp("wa")
    exe = str(d / "window_adapter_main")
    so = os.path.join(ROOT, "oracle", "_build", "libba_oracle.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "window_adapter_main.cpp"), so,
                    "-Wl,-rpath," + os.path.dirname(so), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("seed,kf_i,kf_f", [(7, 3, 9), (11, 0, 11), (5, 4, 5)])
def test_cpp_adapter_matches_python_mirror(adapter_bin, tmp_path, seed, kf_i, kf_f):
    fin, fout = str(tmp_path / "in.txt"), str(tmp_path / "out.txt")
    subprocess.run([adapter_bin, fin, fout, str(seed), str(kf_i), str(kf_f)], check=True)
    kfs, lms, K0, K, a, b, _ = parse_dump(fin)
    kfs_c, lms_c, _, K_c, _, _, summ_c = parse_dump(fout)
    lms_before = {k: v.copy() for k, v in lms.items()}
    T_before = [kf.T_w_c.copy() for kf in kfs]
    o = oracle.default_options()
    summ = window.window_optimize(a, b, kfs, lms, K0, K, lambda p: oracle.solve(p, o))
    assert abs(summ["final_cost"] - summ_c["final_cost"]) <= 1e-12 * summ_c["final_cost"]
    np.testing.assert_allclose(K, K_c, rtol=1e-12)
    for n, (kf, kfc) in enumerate(zip(kfs, kfs_c)):
        np.testing.assert_allclose(kf.T_w_c, kfc.T_w_c, atol=1e-12)
        if n < a or n > b:  # poses outside the window are untouched
            np.testing.assert_array_equal(kf.T_w_c, T_before[n])
    np.testing.assert_allclose(kfs[a].T_w_c, T_before[a], atol=1e-12)  # gauge keyframe
    touched = {lid for n in range(a, b + 1) for loc, lid in kfs[n].global_points_map.items()
               if kfs[n].points3d_local[loc][2] > 1e-15}
    for lid, X in lms.items():
        np.testing.assert_allclose(X, lms_c[lid], atol=1e-12)
        if lid not in touched:
            np.testing.assert_array_equal(X, lms_before[lid])


def test_window_schedule_matches_main_loop():
    # main.cpp:163-183 with frame_frequency=10, window_size=10 (the C1 configuration)
    assert window.window_schedule(10, 10, 10, False, False, True) == (True, 0, 9, False)
    assert window.window_schedule(10, 10, 11, False, False, True) == (False, 0, 0, False)
    assert window.window_schedule(10, 10, 20, False, False, True) == (True, 10, 19, False)
    assert window.window_schedule(10, 10, 23, True, False, False) == (True, 13, 22, True)   # leftovers
    assert window.window_schedule(10, 10, 20, True, False, False) == (False, 0, 0, False)
    assert window.window_schedule(10, -1, 37, True, False, False) == (True, 0, 36, True)    # global BA
    assert window.window_schedule(10, 0, 40, True, False, True) == (False, 0, 0, False)     # repo default: off
    assert window.window_schedule(10, 10, 20, False, True, True) == (False, 0, 0, False)


@pytest.mark.gpu
def test_cpp_adapter_on_gpu_matches_oracle(adapter_bin, tmp_path):
    """The same adapter driving ba_solve (libmiba on the MI355X) instead of the oracle."""
    from miba import _lib
    d = tmp_path
    exe = str(d / "window_adapter_gpu")
    so = os.path.join(ROOT, "oracle", "_build", "libba_oracle.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-DMIBA_WITH_GPU", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "window_adapter_main.cpp"), so, _lib.LIB_PATH,
                    "-Wl,-rpath," + os.path.dirname(so) + ":" + os.path.dirname(_lib.LIB_PATH), "-o", exe], check=True)
    for seed, a, b in [(7, 3, 9), (11, 0, 11)]:
        subprocess.run([adapter_bin, str(d / "i0.txt"), str(d / "o_cpu.txt"), str(seed), str(a), str(b)], check=True)
        subprocess.run([exe, str(d / "i1.txt"), str(d / "o_gpu.txt"), str(seed), str(a), str(b), "gpu"], check=True)
        *_, s_cpu = parse_dump(str(d / "o_cpu.txt"))
        *_, s_gpu = parse_dump(str(d / "o_gpu.txt"))
        assert abs(s_gpu["final_cost"] - s_cpu["final_cost"]) <= 1e-6 * s_cpu["final_cost"]
        kfs_c, lms_c, _, K_c, *_ = parse_dump(str(d / "o_cpu.txt"))
        kfs_g, lms_g, _, K_g, *_ = parse_dump(str(d / "o_gpu.txt"))
        np.testing.assert_allclose(K_g, K_c, atol=1e-3)
        for kc, kg in zip(kfs_c, kfs_g):
            np.testing.assert_allclose(kg.T_w_c[4:], kc.T_w_c[4:], atol=1e-5)


def _tiny_window(depth):
    rng = np.random.default_rng(7)
    kfs, lms = [], {}
    for l in range(6):
        lms[l] = np.array([0.1 * l - 0.2, 0.05 * l, 2.0 + 0.1 * l])
    for k in range(3):
        T = np.array([0, 0, 0, 1.0, 0.01 * k, 0.0, 0.0])
        kp = rng.uniform(100, 500, (6, 2)).astype(np.float32)
        loc = np.zeros((6, 3))
        loc[:, 2] = depth
        kfs.append(window.KeyFrame(T, kp, loc, {i: i for i in range(6)}))
    return kfs, lms


def test_all_inadmissible_window_solves_the_intrinsics_prior():
    """Every depth <= 1e-15: Ceres still solves the IntrinsicsPrior block (OptimizationUtils.cpp:236-241),
    pulling intrinsics_optimized toward intrinsics_initial; poses and landmarks are untouched."""
    kfs, lms = _tiny_window(0.0)
    T_before = [kf.T_w_c.copy() for kf in kfs]
    L_before = {k: v.copy() for k, v in lms.items()}
    K0 = np.array([525.0, 525.0, 319.5, 239.5])
    K = K0 + np.array([3.0, -2.0, 1.5, 0.5])
    summ = window.window_optimize(0, 2, kfs, lms, K0, K, lambda p: oracle.solve(p))
    assert summ["num_obs_admissible"] == 0 and summ["num_active_cams"] == 0
    assert summ["termination"] == "CONVERGENCE"
    assert np.all(np.abs(K - K0) < 1e-3 * np.abs(np.array([3.0, 2.0, 1.5, 0.5])))  # a quadratic: one step
    for kf, T in zip(kfs, T_before):
        np.testing.assert_allclose(kf.T_w_c, T, atol=1e-15)
    for k in lms:
        np.testing.assert_allclose(lms[k], L_before[k], atol=1e-15)


def test_map_back_runs_when_the_solve_raises():
    kfs, lms = _tiny_window(2.0)
    kfs[0].T_w_c = np.array([0, 0, np.sin(0.1), np.cos(0.1), 0.3, -0.2, 0.1])
    T_before = [kf.T_w_c.copy() for kf in kfs]
    L_before = {k: v.copy() for k, v in lms.items()}

    def boom(p):
        raise RuntimeError("device lost")

    with pytest.raises(RuntimeError):
        window.window_optimize(0, 2, kfs, lms, np.ones(4), np.ones(4), boom)
    for kf, T in zip(kfs, T_before):
        np.testing.assert_allclose(kf.T_w_c, T, atol=1e-12)
    for k in lms:
        np.testing.assert_allclose(lms[k], L_before[k], atol=1e-12)
