"""Landmark sharding: host-side splitting, and the per-iteration exchange
restated on CPU with torch.distributed gloo at world_size 2 — each rank forms the reduced
camera system of its landmark block (rank 0 also the camera / intrinsics terms), the
all-reduce must give the unsharded system. The GPU side of the same path
(ba_comm_init, RCCL) is exercised by tests/test_gpu_parity.py::test_sharded_path_*."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from miba import shard, synthetic
from oracle import oracle


def _problem():
    return synthetic.make_problem(n_cams=12, n_points=90, obs_per_point=(2, 6), seed=11, bad_depth_frac=0.03)


def test_split_covers_every_observation_once():
    p = _problem()
    for nranks in (1, 2, 3, 5):
        seen = np.zeros(p.n_obs, dtype=int)
        pts = []
        for r in range(nranks):
            s, ids = shard.split_landmarks(p, nranks, r)
            assert np.array_equal(s.cams, p.cams) and np.array_equal(s.intr, p.intr) and s.fixed_cam == p.fixed_cam
            pts.append(ids)
            keep = np.isin(p.obs_pt, ids)
            seen[keep] += 1
            assert s.n_obs == int(keep.sum())
            assert np.array_equal(ids[s.obs_pt], p.obs_pt[keep])
        assert np.all(seen == 1)
        assert np.array_equal(np.concatenate(pts), np.arange(p.n_points))


def test_split_balances_observations():
    p = synthetic.make_config("C2")
    counts = [shard.split_landmarks(p, 4, r)[0].n_obs for r in range(4)]
    assert max(counts) - min(counts) <= 20  # 10 observations per point


def test_landmark_shards_share_cameras():
    a = synthetic.make_landmark_shard("C2", 0)
    b = synthetic.make_landmark_shard("C2", 1)
    assert np.array_equal(a.cams, b.cams) and np.array_equal(a.intr, b.intr)
    assert not np.array_equal(a.obs_uv[:10], b.obs_uv[:10])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, radius, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = _problem()
        b = shard.shard_bounds(p, world)
        o = oracle.default_options()
        S, rhs = oracle.reduced_system(p, o, radius, int(b[rank]), int(b[rank + 1]), rank == 0)
        tS, tr = torch.from_numpy(S), torch.from_numpy(rhs)
        dist.all_reduce(tS)
        dist.all_reduce(tr)
        if rank == 0:
            q.put((tS.numpy(), tr.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("radius", [1e4, 0.5])
def test_gloo_world2_reduced_system_allreduce(radius):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, radius, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    S2, r2 = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    S, rhs = oracle.reduced_system(_problem(), oracle.default_options(), radius)
    np.testing.assert_allclose(S2, S, rtol=1e-12, atol=1e-14 * np.abs(S).max())
    np.testing.assert_allclose(r2, rhs, rtol=1e-12, atol=1e-14 * np.abs(rhs).max())
