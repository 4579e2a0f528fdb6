#!/usr/bin/env python3
"""bench.py — LM iterations/s of the MI355X windowed-BA solver (libmiba).

Metric (BASELINE.json): "LM iterations/sec + ms/iter at (cams,points,obs)".
A "step" is one Levenberg-Marquardt iteration of the reference's ceres::Solve
(OptimizationUtils.cpp:300) over one resident synthetic window. Default
workload: C4 = 200 cams / 100k points / 1M obs (BASELINE.json configs[3], the
north_star's 1-GPU target window); --config C2 selects configs[1].

Timed region: ba_solve_prepared() with max_num_iterations = K and the
convergence tolerances disabled, so exactly K LM iterations run on a window
already resident in HBM (ba_prepare() is outside the timed region).
With --gpus N (torchrun, one rank per GPU) every rank solves its own window
(replicas, weak scaling); value = total iterations / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3dsmc-bundle-adjustment_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4", choices=["C1", "C2", "C3", "C4", "C5"])
    ap.add_argument("--cpu-iters", type=int, default=8, help="LM iterations of the CPU oracle sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="disable per-kernel HIP events")
    return ap.parse_args()


def load_pmc_traffic(kernel: str, config: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if present."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        rec = d.get(config, {}).get(kernel)
        if rec and rec.get("hbm_bytes_per_launch"):
            return float(rec["hbm_bytes_per_launch"])
    return None


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no HIP device visible)")
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)

    from miba import synthetic
    from miba.solver import Solver

    cfg = dict(synthetic.CONFIGS[args.config])
    cfg["seed"] = cfg["seed"] + 1000 * rank  # independent replica windows
    prob = synthetic.make_problem(**cfg)
    prob0 = prob.copy()

    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0,
                  minimizer_progress_to_stdout=0)
    solver = Solver(device=local_rank, profile_kernels=0 if args.no_profile else 1, max_num_iterations=args.warmup,
                    **no_tol)
    solver.prepare(prob)
    if args.warmup > 0:
        solver.solve_prepared(prob)
    # timed run
    prob = prob0.copy()
    solver.set_options(max_num_iterations=args.steps)
    solver.prepare(prob)
    solver.reset_kernel_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    summ = solver.solve_prepared(prob)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    iters = summ["num_iterations"]
    stats = solver.kernel_stats()
    t = torch.tensor([elapsed, float(iters)], dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed_max, iters_total = float(tmax[0]), float(tsum[1])
    else:
        elapsed_max, iters_total = elapsed, float(iters)

    if rank == 0:
        value = iters_total / elapsed_max
        ms_per_step = elapsed_max * 1e3 / max(iters, 1)
        roof = None
        kern = [k for k in stats if k["launches"] > 0]
        if kern:
            dom = max(kern, key=lambda k: k["total_ms"])
            avg_ms = dom["total_ms"] / dom["launches"]
            achieved = dom["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "kernel": dom["name"], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": load_pmc_traffic(dom["name"], args.config),
                    "avg_launch_ms": round(avg_ms, 5), "bytes_per_launch": dom["bytes_per_launch"]}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            from oracle import oracle
            q = prob0.copy()
            o = oracle.default_options(max_num_iterations=args.cpu_iters, **no_tol)
            tc0 = time.perf_counter()
            so = oracle.solve(q, o)
            tc1 = time.perf_counter()
            cpu = {"value": round(so["num_iterations"] / (so["time_lm_ms"] * 1e-3), 4),
                   "unit": "LM iterations/s", "cores": 1, "kind": "port",
                   "sample": f"{args.config} window, {so['num_iterations']} LM iterations of the f64 C oracle "
                             f"(CPU restatement, not Ceres), wall {tc1 - tc0:.1f}s incl. setup"}
        phases = {k["name"]: round(k["total_ms"] / max(iters, 1), 4) for k in stats if k["launches"] > 0}
        out = {
            "metric": "LM iterations/sec",
            "value": round(value, 3),
            "unit": "LM iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: {prob0.n_cams} cams / {prob0.n_points} points / "
                                   f"{prob0.n_obs} obs, one resident window per GPU",
                       "cams": prob0.n_cams, "points": prob0.n_points, "obs": prob0.n_obs,
                       "parallelism": f"replicas{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "lm": {"iterations": iters, "successful": summ["num_successful_steps"],
                   "unsuccessful": summ["num_unsuccessful_steps"], "initial_cost": summ["initial_cost"],
                   "final_cost": summ["final_cost"], "termination": summ["termination"]},
            "kernel_ms_per_step": phases,
        }
        print(json.dumps(out), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
