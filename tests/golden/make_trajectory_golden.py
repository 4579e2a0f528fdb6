#!/usr/bin/env python3
"""Generate tests/golden/trajectory_golden.json from the REFERENCE's own evaluators.

Run in the build container (it has /root/reference; the GPU box does not):
    python tests/golden/make_trajectory_golden.py
It imports rgb-d-toolset/associate.py, evaluate_ate.py and evaluate_rpe.py from
/root/reference unchanged, runs them on fixed synthetic TUM-format trajectories (written
here), and stores the inputs (trajectory texts) and the reference outputs: association
matches, Horn alignment, ATE statistics and Euler-angle errors (evaluate_ate.py:246-301),
RPE pairs / statistics for all-pairs, seeded random pairs (random.seed(0) as the script's
__main__ does) and fixed-delta evaluation (evaluate_rpe.py:197-366). Only data is stored.
"""
import json
import os
import random
import sys
import tempfile

import numpy as np

REF = "/root/reference/rgb-d-toolset"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "trajectory_golden.json")


def quat_xyzw(R):
    from scipy.spatial.transform import Rotation
    return Rotation.from_matrix(R).as_quat()


def make_traj(n_gt, n_est, seed, misalign=True):
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(seed)
    t0 = 1305031102.175304
    st_gt = t0 + np.arange(n_gt) / 30.0 + rng.uniform(-1e-4, 1e-4, n_gt)
    s = np.arange(n_gt) / 30.0
    pos = np.stack([0.3 * np.sin(0.7 * s), 0.2 * np.cos(0.5 * s), 0.05 * s], 1)
    rots = Rotation.from_rotvec(np.stack([0.2 * np.sin(0.3 * s), 0.4 * np.sin(0.2 * s), 0.1 * s], 1))
    gt_lines = ["# ground truth trajectory", "# file: synthetic", "# timestamp tx ty tz qx qy qz qw"]
    for k in range(n_gt):
        q = rots[k].as_quat()
        gt_lines.append("%.6f %.4f %.4f %.4f %.4f %.4f %.4f %.4f" % (st_gt[k], *pos[k], *q))
    # estimate: every other gt frame, stamp jitter < 20 ms, mm-level noise, rigidly misaligned
    idx = np.sort(rng.choice(np.arange(1, n_gt - 1), size=n_est, replace=False))
    G = Rotation.from_rotvec([0.05, -0.1, 0.3]) if misalign else Rotation.identity()
    g = np.array([0.5, -0.2, 1.0]) if misalign else np.zeros(3)
    est_lines = []
    for k in idx:
        st = st_gt[k] + rng.uniform(-0.008, 0.008)
        p = G.apply(pos[k] + rng.normal(0, 0.004, 3)) + g
        r = G * rots[k] * Rotation.from_rotvec(rng.normal(0, 0.003, 3))
        est_lines.append("%.6f %.6f %.6f %.6f %.6f %.6f %.6f %.6f" % (st, *p, *r.as_quat()))
    # a NaN line and a zero-quaternion line (skipped by evaluate_rpe.read_trajectory)
    est_lines.append("%.6f nan 0 0 0 0 0 1" % (st_gt[-1] + 0.5))
    est_lines.append("%.6f 0 0 0 0 0 0 0" % (st_gt[-1] + 0.6))
    return "\n".join(gt_lines) + "\n", "\n".join(est_lines) + "\n"


def main():
    sys.path.insert(0, REF)
    import associate  # noqa: E402
    import evaluate_ate  # noqa: E402
    import evaluate_rpe  # noqa: E402
    from scipy.spatial.transform import Rotation

    cases = {}
    for name, n_gt, n_est, seed in (("small_all_pairs", 90, 60, 1), ("large_random_pairs", 260, 150, 2)):
        gt_text, est_text = make_traj(n_gt, n_est, seed)
        d = tempfile.mkdtemp()
        fg, fe = os.path.join(d, "gt.txt"), os.path.join(d, "est.txt")
        open(fg, "w").write(gt_text)
        # ATE tools read the estimate without the NaN / zero-quat lines (associate keeps them as data)
        est_ate = "\n".join(est_text.strip().split("\n")[:-2]) + "\n"
        open(fe, "w").write(est_ate)
        first = associate.read_file_list(fg)
        second = associate.read_file_list(fe)
        matches = associate.associate(first, second, 0.0, 0.02)
        fx = np.matrix([[float(v) for v in first[a][0:3]] for a, b in matches]).transpose()
        sx = np.matrix([[float(v) for v in second[b][0:3]] for a, b in matches]).transpose()
        rot, trans, terr = evaluate_ate.align(sx, fx)
        fq = np.matrix([[float(v) for v in first[a][3:7]] for a, b in matches]).transpose()
        sq = np.matrix([[float(v) for v in second[b][3:7]] for a, b in matches]).transpose()
        fe_eu = Rotation.from_quat(fq.transpose()).as_euler("xyz", degrees=True)
        se_eu = Rotation.from_quat(sq.transpose()).as_euler("xyz", degrees=True)
        dl = 5
        ate = {
            "matches": matches, "rot": np.asarray(rot).tolist(), "trans": np.asarray(trans).ravel().tolist(),
            "trans_error": list(map(float, terr)),
            "rmse": float(np.sqrt(np.dot(terr, terr) / len(terr))),
            "AYE": float(evaluate_ate.calculateAYE(fe_eu[:, 0], se_eu[:, 0])),
            "APE": float(evaluate_ate.calculateAPE(fe_eu[:, 1], se_eu[:, 1])),
            "ARE": float(evaluate_ate.calculateARE(fe_eu[:, 2], se_eu[:, 2])),
            "RYE": float(evaluate_ate.calculateRYE(fe_eu[0:-dl, 0], fe_eu[dl:, 0], se_eu[0:-dl, 0], se_eu[dl:, 0])),
            "RPE_pitch": float(evaluate_ate.calculateRPE(fe_eu[0:-dl, 1], fe_eu[dl:, 1], se_eu[0:-dl, 1], se_eu[dl:, 1])),
            "RRE": float(evaluate_ate.calculateRRE(fe_eu[0:-dl, 2], fe_eu[dl:, 2], se_eu[0:-dl, 2], se_eu[dl:, 2])),
        }
        open(fe, "w").write(est_text)  # RPE reader skips the NaN / zero-quat lines itself
        tg, tt = evaluate_rpe.read_trajectory(fg), evaluate_rpe.read_trajectory(fe)
        rpe = {}
        for key, args in (("default", (10000, False, 1.0, "s", 0.0, 1.0)),
                          ("fixed_1s", (10000, True, 1.0, "s", 0.0, 1.0)),
                          ("fixed_5f", (10000, True, 5, "f", 0.0, 1.0)),
                          ("fixed_0.1m", (10000, True, 0.1, "m", 0.0, 1.0))):
            random.seed(0)
            res = np.array(evaluate_rpe.evaluate_trajectory(tg, tt, *args))
            te, re = res[:, 4], res[:, 5]
            rpe[key] = {"args": list(args), "n": int(len(res)), "trans_mean": float(np.mean(te)),
                        "trans_rmse": float(np.sqrt(np.dot(te, te) / len(te))), "rot_mean": float(np.mean(re)),
                        "sum_cols": res.sum(axis=0).tolist(), "rows_head": res[:25].tolist(),
                        "rows_stride97": res[::97].tolist()}
        closest = [[float(t), evaluate_rpe.find_closest_index(sorted(tg), t)] for t in
                   (sorted(tg)[0] - 1.0, sorted(tg)[7] + 0.004, sorted(tg)[-1] + 3.0, sorted(tg)[40])]
        cases[name] = {"gt_text": gt_text, "est_text": est_text, "ate": ate, "rpe": rpe, "find_closest_index": closest}
    json.dump({"generator": "tests/golden/make_trajectory_golden.py", "reference": REF, "cases": cases},
              open(OUT, "w"), indent=0)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
