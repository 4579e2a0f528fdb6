"""Diagnostic: per-phase cycle stamps of the hand-written kernels on a synthetic config.

usage: MIBA_BCR_STAMPS=1 | MIBA_SCHUR_STAMPS=1 | MIBA_CHOL_STAMPS=1  python tools/kernel_stamps.py [C4] [iters]
The stamped kernel variants print their phase breakdown to stderr on every launch."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3dsmc-bundle-adjustment_amd"))
from miba import synthetic  # noqa: E402
from miba.solver import Solver  # noqa: E402

p = synthetic.make_config(sys.argv[1] if len(sys.argv) > 1 else "C4")
with Solver(minimizer_progress_to_stdout=0, max_num_iterations=int(sys.argv[2]) if len(sys.argv) > 2 else 2) as s:
    print(s.solve(p))
