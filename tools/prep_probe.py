#!/usr/bin/env python3
"""New-window prepare breakdown (diagnostic): ba_prepare with rebuild_plan = 1 on a synthetic config, N times.

usage: prep_probe.py [config=C4] [reps=6]
Prints the wall time of each prepare and ba_last_prepare()'s plan / upload / total split. MIBA_PLAN_TIMES=1 in the
environment adds the host plan's per-phase times (stderr)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3dsmc-bundle-adjustment_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from miba import synthetic
    from miba.solver import Solver
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    torch.cuda.set_device(0)
    prob0 = synthetic.make_config(cfg)
    s = Solver(minimizer_progress_to_stdout=0, rebuild_plan=1, max_num_iterations=2)
    for r in range(reps):
        q = prob0.copy()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.prepare(q)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        info = s.last_prepare()
        print(f"{cfg} rep {r}: prepare {1e3 * (t1 - t0):.3f} ms (+sync {1e3 * (t2 - t1):.3f}) "
              f"plan {info['plan_ms']:.3f} upload {info['upload_ms']:.3f} total {info['total_ms']:.3f} "
              f"threads {info['host_threads']}", flush=True)


if __name__ == "__main__":
    main()
