"""Diagnostic: per-kernel time per LM iteration (libmiba HIP events around every launch) on a synthetic config.

usage: python tools/kernel_breakdown.py [C1] [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3dsmc-bundle-adjustment_amd"))
from miba import synthetic  # noqa: E402
from miba.solver import Solver  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C1"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
p = synthetic.make_config(cfg)
with Solver(minimizer_progress_to_stdout=0, max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
            parameter_tolerance=0.0) as s:
    s.solve(p.copy())
    s.set_options(profile_kernels=1, profile_mask=0)
    q = p.copy()
    s.prepare(q)
    s.reset_kernel_stats()
    sm = s.solve_prepared(q)
    st = [k for k in s.kernel_stats() if k["launches"] > 0]
    it = max(sm["num_iterations"], 1)
    print(f"{cfg}: {it} iterations, linear_solver {sm['linear_solver']}, band {sm['camera_band']}")
    for k in sorted(st, key=lambda k: -k["total_ms"]):
        print(f"  {k['name']:14s} launches {k['launches']:4d}  us/launch {1e3 * k['total_ms'] / k['launches']:8.2f}  "
              f"us/iter {1e3 * k['total_ms'] / it:8.2f}")
    s.set_options(profile_kernels=0)
    q = p.copy()
    s.prepare(q)
    t0 = time.perf_counter()
    sm = s.solve_prepared(q)
    dt = time.perf_counter() - t0
    print(f"  unprofiled: {1e3 * dt:.3f} ms for {sm['num_iterations']} iterations = {1e6 * dt / max(sm['num_iterations'], 1):.1f} us/iter")
