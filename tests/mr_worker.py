"""One rank of a multi-rank landmark-sharded libmiba solve (helper of tests/test_multirank.py).

Started as a child process per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment, before any GPU call). Every rank joins a torch.distributed gloo group, cuts its
landmark shard of the window (miba.shard.split_landmarks, or an empty shard), makes a libmiba
context that shard over the gloo host collective (ba_comm_init_host; several ranks share one GPU,
where RCCL refuses duplicate devices) and solves. It writes its summary, iteration log and
parameters to <out>/rank<r>.npz.

    python tests/mr_worker.py <out_dir> <json spec>
spec: {"problem": {"config": "C2"} | {"make_problem": {...}}, "nsplit": k (shards with points;
ranks >= k get an empty shard), "options": {...}, "env": {...}}
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3dsmc-bundle-adjustment_amd")]

import numpy as np  # noqa: E402


def build_problem(spec):
    from miba import synthetic
    pr = spec["problem"]
    if "config" in pr:
        return synthetic.make_config(pr["config"])
    return synthetic.make_problem(**pr["make_problem"])


def main():
    out_dir, spec = sys.argv[1], json.loads(sys.argv[2])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    for k, v in spec.get("env", {}).items():
        os.environ[k] = str(v)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from miba import shard
        from miba.solver import Solver

        whole = build_problem(spec)
        nsplit = int(spec.get("nsplit", world))
        if rank < nsplit:
            prob, ids = shard.split_landmarks(whole, nsplit, rank)
        else:  # an empty landmark shard: the window's cameras, no point, no observation
            from miba.capi import ProblemArrays
            prob = ProblemArrays(whole.cams.copy(), np.zeros((0, 3)), whole.intr.copy(), whole.intr_prior.copy(),
                                 np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 2)), np.zeros(0),
                                 whole.fixed_cam)
            ids = np.zeros(0, dtype=np.int64)
        opts = dict(minimizer_progress_to_stdout=0)
        opts.update(spec.get("options", {}))
        with Solver(device=0, **opts) as s:
            s.comm_init_host(world, rank, shard.torch_allreduce())
            summ = s.solve(prob)
            log = s.iteration_log()
            comm_launches = sum(k["launches"] for k in s.kernel_stats() if k["name"] == "comm")
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), cams=prob.cams, points=prob.points, intr=prob.intr,
                 ids=ids, log=log, summary=json.dumps({k: v for k, v in summ.items() if not isinstance(v, bytes)}),
                 comm_launches=comm_launches)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
