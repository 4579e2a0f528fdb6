"""Landmark sharding helpers on the host side of ba_comm_init.

``split_landmarks`` cuts one window into ``nranks`` shards of contiguous point ids,
balanced by admissible-observation count; every shard carries the full camera set,
intrinsics, prior and gauge (replicated), and only its own points and their
observations. ``merge_points`` puts the solved shard points back into the window.
"""
from __future__ import annotations

import numpy as np

from .capi import ProblemArrays


def shard_bounds(prob: ProblemArrays, nranks: int) -> np.ndarray:
    """Point-id boundaries [b_0 = 0, ..., b_nranks = n_points] balancing the observation count."""
    cnt = np.bincount(prob.obs_pt, minlength=prob.n_points).astype(np.int64)
    cum = np.concatenate([[0], np.cumsum(cnt)])
    total = cum[-1]
    b = [0]
    for r in range(1, nranks):
        b.append(int(np.searchsorted(cum, total * r / nranks, side="left")))
    b.append(prob.n_points)
    return np.maximum.accumulate(np.array(b, dtype=np.int64))


def split_landmarks(prob: ProblemArrays, nranks: int, rank: int) -> tuple[ProblemArrays, np.ndarray]:
    """Shard ``rank`` of ``nranks``: (problem, original point ids of its points)."""
    b = shard_bounds(prob, nranks)
    lo, hi = int(b[rank]), int(b[rank + 1])
    keep = (prob.obs_pt >= lo) & (prob.obs_pt < hi)
    ids = np.arange(lo, hi)
    sub = ProblemArrays(prob.cams.copy(), prob.points[lo:hi].copy(), prob.intr.copy(), prob.intr_prior.copy(),
                        prob.obs_cam[keep], prob.obs_pt[keep] - lo, prob.obs_uv[keep], prob.obs_depth[keep],
                        prob.fixed_cam)
    return sub, ids


def merge_points(prob: ProblemArrays, shard: ProblemArrays, ids: np.ndarray) -> None:
    """Write a solved shard's points back; cameras / intrinsics are identical on every shard."""
    prob.points[ids] = shard.points
    prob.cams[:] = shard.cams
    prob.intr[:] = shard.intr


def torch_allreduce(group=None):
    """Host collective for ``Solver.comm_init_host`` over ``torch.distributed`` (e.g. the gloo backend):
    reduces the staging array in place."""
    import torch
    import torch.distributed as dist

    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}

    def allreduce(arr, op):
        dist.all_reduce(torch.from_numpy(arr), op=ops[op], group=group)

    return allreduce
