#!/usr/bin/env python3
"""Generate tests/golden/{c3,c4,c5}_oracle.json: converged-solve fixtures of the CPU oracle
(TEST INFRASTRUCTURE) on BASELINE.json's windows, for the -m gpu parity tests
(tests/test_converged_parity.py).

- C3 (50 cams / 4k points / 8k obs, synthetic.make_config("C3"), the stand-in for BASELINE
  configs[2]'s 50-keyframe fr2/desk window): the reference's solver settings, to termination
  (every point seen by 2 keyframes, so most residuals sit in the Huber linear zone and the solve
  runs to max_num_iterations = 75).
- C4 (200 cams / 100k points / 1M obs, synthetic.make_config("C4")): the reference's own
  solver settings, i.e. ceres::Solve run to termination with the default tolerances and
  max_num_iterations = 75 (/root/reference/src/OptimizationUtils.cpp:300,
  /root/reference/headers/BundleAdjustmentConfig.h:61-67).
- C5 (1000 cams / 500k points / 5M obs): 12 LM iterations with the convergence tolerances
  disabled (the oracle needs ~6 s per C5 iteration on one core).

Checker configuration of the oracle: 1 thread (fixed summation order); C4 uses the dense
reduced-camera Cholesky, C5 the co-visibility profile Cholesky (same factorisation, fill
confined to the envelope; the dense 5998^2 system is too slow to iterate on a CPU).

Run from the repository root:  python tests/golden/make_converged_golden.py [C3] [C4] [C5]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dsmc-bundle-adjustment_amd")]

from miba import synthetic  # noqa: E402
from oracle import oracle  # noqa: E402

NO_TOL = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0)
SPECS = {
    "C3": dict(profile=False, options={}),
    "C4": dict(profile=False, options={}),
    "C5": dict(profile=True, options=dict(max_num_iterations=12, **NO_TOL)),
}


def checksum(a: np.ndarray) -> dict:
    return {"sum": float(np.sum(a)), "sum_sq": float(np.sum(a * a)), "abs_max": float(np.max(np.abs(a)))}


def make(name: str) -> dict:
    spec = SPECS[name]
    p = synthetic.make_config(name)
    oracle.config(threads=1, profile=spec["profile"])
    opts = oracle.default_options(**spec["options"])
    t0 = time.perf_counter()
    summ, tr = oracle.solve_trace(p, opts)
    dt = time.perf_counter() - t0
    oracle.config(1, False)
    return {
        "config": name,
        "window": {"n_cams": p.n_cams, "n_points": p.n_points, "n_obs": p.n_obs,
                   "generator": f"miba.synthetic.make_config({name!r})"},
        "options": spec["options"],
        "oracle": {"threads": 1, "reduced_solve": "profile" if spec["profile"] else "dense", "seconds": round(dt, 1)},
        "initial_cost": summ["initial_cost"],
        "final_cost": summ["final_cost"],
        "num_iterations": summ["num_iterations"],
        "num_successful_steps": summ["num_successful_steps"],
        "num_unsuccessful_steps": summ["num_unsuccessful_steps"],
        "termination": summ["termination"],
        "message": summ["message"],
        "trace_columns": ["cost", "cost_change", "gradient_max_norm", "step_norm", "tr_ratio", "tr_radius",
                          "accepted"],
        "trace": [[float(v) for v in row[:7]] for row in tr],
        "final_intrinsics": [float(v) for v in p.intr],
        "cams_checksum": checksum(p.cams),
        "points_checksum": checksum(p.points),
    }


def main(argv):
    names = [a for a in argv if a in SPECS] or list(SPECS)
    for name in names:
        d = make(name)
        out = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{name.lower()}_oracle.json")
        with open(out, "w") as f:
            json.dump(d, f, indent=1)
        print(f"{name}: {d['num_iterations']} iterations ({d['num_successful_steps']} successful), "
              f"final cost {d['final_cost']:.15e}, {d['termination']}: {d['message']} [{d['oracle']['seconds']} s]")


if __name__ == "__main__":
    main(sys.argv[1:])
