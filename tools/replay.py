#!/usr/bin/env python3
"""Replay a captured window (.miba, written by libmiba under MIBA_DUMP_DIR) or a BAL problem on
the GPU, optionally beside the CPU oracle, and print both summaries.

    python tools/replay.py window_1234_000003.miba [--oracle] [--iters N] [--no-depth]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3dsmc-bundle-adjustment_amd"))
sys.path.insert(0, ROOT)

KEYS = ("initial_cost", "final_cost", "num_iterations", "num_successful_steps", "num_unsuccessful_steps",
        "termination", "num_obs_admissible", "reduced_system_size", "linear_solver", "time_setup_ms", "time_lm_ms")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--oracle", action="store_true", help="also solve on the CPU oracle and compare final costs")
    ap.add_argument("--iters", type=int, default=None, help="override max_num_iterations")
    ap.add_argument("--no-depth", action="store_true", help="weight_unpr = 0 (e.g. BAL problems)")
    ap.add_argument("--out", default=None, help="write the solved window to this .miba file")
    a = ap.parse_args()
    from miba import problem_io
    from miba.solver import Solver, default_options
    prob, opts = problem_io.load(a.path)
    opts = opts if opts is not None else default_options()
    opts.minimizer_progress_to_stdout = 0
    opts.device = -1
    if a.iters is not None:
        opts.max_num_iterations = a.iters
    if a.no_depth:
        opts.weight_unpr = 0.0
    res = {"file": a.path, "cams": prob.n_cams, "points": prob.n_points, "obs": prob.n_obs}
    q = prob.copy()
    with Solver(opts) as s:
        sg = s.solve(q)
    res["gpu"] = {k: sg[k] for k in KEYS}
    if a.oracle:
        from oracle import oracle
        o = oracle.default_options()
        for f in ("hub_p_repr", "hub_p_unpr", "weight_intrinsics", "weight_unpr", "max_num_iterations"):
            setattr(o, f, getattr(opts, f))
        sc = oracle.solve(prob.copy(), o)
        res["oracle"] = {k: sc[k] for k in KEYS}
        res["final_cost_rel_diff"] = abs(sg["final_cost"] - sc["final_cost"]) / max(sc["final_cost"], 1e-300)
    if a.out:
        problem_io.write_window(a.out, q, opts)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
