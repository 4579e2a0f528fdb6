#!/usr/bin/env python3
"""bench.py — LM iterations/s of the MI355X windowed-BA solver (libmiba).

Metric (BASELINE.json): "LM iterations/sec + ms/iter at (cams,points,obs)".
A "step" is one Levenberg-Marquardt iteration of the reference's ceres::Solve
(OptimizationUtils.cpp:300) over one resident synthetic window. Default
workload: C4 = 200 cams / 100k points / 1M obs (BASELINE.json configs[3], the
window the north_star's 1-GPU targets are stated on); --config C2 selects
configs[1].

Timed region: ba_solve_prepared() with max_num_iterations = K and the
convergence tolerances disabled, so exactly K LM iterations run on a window
already resident in HBM (ba_prepare() is outside the timed region).

--gpus N (torchrun, one rank per GPU): ONE window landmark-sharded across the N
ranks (ba_comm_init): the same 200 cameras on every rank and a
C4-size block of landmarks per rank (N x 100k points, N x 1M obs in total).
Per iteration the ranks all-reduce (RCCL over xGMI) the camera-side partials,
the packed envelope of the reduced camera system and the step scalars.
Weak scaling: value = N x LM iterations/s = landmark-shard iterations per
second (each GPU advances its C4-size shard by one LM iteration per step),
timed over the max-over-ranks wall time. --shard runs the same sharded path
with a 1-rank communicator (its overhead on one GPU).
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

HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F64_MFMA_PEAK_TF = 78.6  # MI355X FP64 matrix spec (tools/mfma_f64_rate.hip measures ~73 TF/s sustained)

# kernels whose bound is HBM bandwidth (per-observation passes) vs the f64 matrix cores
HBM_KERNELS = {"cam_side", "cam_reduce", "point_colnorm", "point_prep", "backsub_eval", "lin_finalize", "scale", "assemble",
               "update_cams", "memset_S", "obs_pairs", "final", "xnorm", "comm"}
JACOBIAN_PASS = "cam_side"  # the roofline.achieved basis (Jacobian pass, J kept in registers)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4", choices=["C1", "C2", "C3", "C4", "C5"])
    ap.add_argument("--cpu-iters", type=int, default=24, help="LM iterations of the CPU oracle sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--shard", action="store_true", help="landmark-sharded path even on one GPU")
    ap.add_argument("--problem", default=None,
                    help="bench a window file instead of a synthetic config: a .miba dump (MIBA_DUMP_DIR capture, "
                         "solved with its captured cost options) or a BAL text problem")
    return ap.parse_args()


PMC_ALIASES = {"bcr_persist": ("bcr_persist", "bcr_split")}  # profiler id -> kernel symbols it times


def load_pmc_traffic(kernel: str, config: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if present."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):  # newest first
        try:
            d = json.load(open(path))
        except Exception:
            continue
        for name in PMC_ALIASES.get(kernel, (kernel,)):
            rec = d.get(config, {}).get(name)
            if rec and rec.get("hbm_bytes_per_launch"):
                return float(rec["hbm_bytes_per_launch"])
    return None


def roofline_entry(k: dict, config: str) -> dict:
    """Roofline of one kernel from libmiba's per-launch HIP-event timing and its
    algorithmic bytes / flops per launch."""
    avg_ms = k["total_ms"] / k["launches"]
    if k["name"] in HBM_KERNELS or k["flops_per_launch"] <= 0:
        achieved = k["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9
        e = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBS, 4)}
    else:
        achieved = k["flops_per_launch"] / (avg_ms * 1e-3) / 1e12
        e = {"bound": "mfma", "achieved": round(achieved, 4), "peak": F64_MFMA_PEAK_TF, "unit": "TFLOP/s",
             "frac": round(achieved / F64_MFMA_PEAK_TF, 5)}
    e["traffic"] = load_pmc_traffic(k["name"], config)
    e.update(kernel=k["name"], avg_launch_ms=round(avg_ms, 5), launches=k["launches"],
             bytes_per_launch=k["bytes_per_launch"], flops_per_launch=k["flops_per_launch"])
    return e


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

    sharded = world > 1 or args.shard
    file_opts = None
    if args.problem:
        from miba import problem_io, shard
        whole, file_opts = problem_io.load(args.problem)
        prob = shard.split_landmarks(whole, world, rank)[0] if world > 1 else whole
        args.config = "file"
    else:
        prob = synthetic.make_landmark_shard(args.config, rank)  # shard 0 == the single-GPU window
    prob0 = prob.copy()

    no_tol = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0,
                  minimizer_progress_to_stdout=0)
    prof = 0 if args.no_profile else 1
    solver = Solver(file_opts, device=local_rank, profile_kernels=prof, max_num_iterations=max(args.warmup, 1),
                    **no_tol)
    if sharded:
        box = [Solver.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=0)
        solver.comm_init(world, rank, box[0])
    # warmup (untimed, unprofiled: first launches load the code objects)
    if args.warmup > 0:
        solver.set_options(max_num_iterations=args.warmup, profile_kernels=0)
        solver.prepare(prob)
        solver.solve_prepared(prob)
        prob = prob0.copy()
    # breakdown run: every kernel launch timed (per-iteration breakdown, dominant kernel)
    solver.set_options(max_num_iterations=5, profile_kernels=prof, profile_mask=0)
    solver.prepare(prob)
    solver.reset_kernel_stats()
    wsumm = solver.solve_prepared(prob)
    wstats = solver.kernel_stats()
    names = [k["name"] for k in wstats]
    live = [k for k in wstats if k["launches"] > 0]
    dom = max(live, key=lambda k: k["total_ms"])["name"] if live else None
    # timed run (no HIP events: event records between dependent launches cost ~5-10 us each)
    prob = prob0.copy()
    solver.set_options(max_num_iterations=args.steps, profile_kernels=0)
    solver.prepare(prob)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    summ = solver.solve_prepared(prob)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    # the same K-step region again with HIP events around the dominant kernel and the
    # Jacobian pass only: their average launch durations for the roofline
    stats = []
    if prof:
        mask = 0
        for nm in (dom, JACOBIAN_PASS):
            if nm in names:
                mask |= 1 << names.index(nm)
        solver.set_options(max_num_iterations=args.steps, profile_kernels=1, profile_mask=mask)
        solver.prepare(prob0.copy())
        solver.reset_kernel_stats()
        solver.solve_prepared(prob0.copy())
        stats = solver.kernel_stats()
    elapsed = t1 - t0
    iters = summ["num_iterations"]
    t = torch.tensor([elapsed, float(iters)], dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tmin = t.clone()
        dist.all_reduce(tmin, op=dist.ReduceOp.MIN)
        elapsed_max = float(tmax[0])
        assert float(tmin[1]) == float(tmax[1]) == float(iters), "ranks ran different iteration counts"
    else:
        elapsed_max = elapsed

    if rank == 0:
        value = world * iters / elapsed_max
        ms_per_step = elapsed_max * 1e3 / max(iters, 1)
        kern = [k for k in stats if k["launches"] > 0]
        roofs = {k["name"]: roofline_entry(k, args.config) for k in kern}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            from oracle import oracle
            q = prob0.copy()
            o = oracle.default_options(max_num_iterations=args.cpu_iters, **no_tol)
            if file_opts is not None:
                for f in ("hub_p_repr", "hub_p_unpr", "weight_intrinsics", "weight_unpr"):
                    setattr(o, f, getattr(file_opts, f))
            tc0 = time.perf_counter()
            so = oracle.solve(q, o)
            tc1 = time.perf_counter()
            cpu = {"value": round(so["num_iterations"] / (so["time_lm_ms"] * 1e-3), 4),
                   "unit": "LM iterations/s", "cores": 1, "kind": "port",
                   "sample": f"{args.config} window ({prob0.n_cams} cams / {prob0.n_points} points / {prob0.n_obs} obs), "
                             f"{so['num_iterations']} LM iterations of the f64 C oracle (CPU restatement of the "
                             f"Ceres 2.0 LM path, not Ceres; single thread), wall {tc1 - tc0:.1f}s incl. setup"}
        wit = max(wsumm["num_iterations"], 1)
        phases = {k["name"]: round(k["total_ms"] / wit, 4) for k in live}  # warmup run, every kernel timed
        if args.problem:
            workload = (f"{os.path.basename(args.problem)}: {prob0.n_cams} cams / {world}x~{prob0.n_points} points / "
                        f"{world}x~{prob0.n_obs} obs, one window from file"
                        + (f", landmark-sharded across {world} GPUs" if sharded else ""))
            par = f"landmark-shard{world}" if sharded else "single"
        elif sharded:
            workload = (f"{args.config} landmark shards: {prob0.n_cams} cams / {world}x{prob0.n_points} points / "
                        f"{world}x{prob0.n_obs} obs, one window landmark-sharded across {world} GPU(s) "
                        f"(RCCL all-reduce of the reduced camera system per LM iteration)")
            par = f"landmark-shard{world}"
        else:
            workload = f"{args.config}: {prob0.n_cams} cams / {prob0.n_points} points / {prob0.n_obs} obs, one window"
            par = "single"
        out = {
            "metric": "LM iterations/sec",
            "value": round(value, 3),
            "unit": "LM iterations/s" if world == 1 else "landmark-shard LM iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "file" if args.problem else "synthetic",
            "config": {"workload": workload, "cams": prob0.n_cams, "points": world * prob0.n_points,
                       "obs": world * prob0.n_obs, "parallelism": par},
            "roofline": roofs.get(dom),
            "roofline_source": "libmiba HIP events (solver stream) around every launch of the dominant kernel and of "
                               "the Jacobian pass, over a repeat of the timed K-step region",
            "roofline_jacobian_pass": roofs.get(JACOBIAN_PASS),
            "cpu_baseline": cpu,
            "lm": {"iterations": iters, "successful": summ["num_successful_steps"],
                   "unsuccessful": summ["num_unsuccessful_steps"], "initial_cost": summ["initial_cost"],
                   "final_cost": summ["final_cost"], "termination": summ["termination"],
                   "linear_solver": summ["linear_solver"]},
            "kernel_ms_per_step": phases,
            "kernel_ms_per_step_source": f"breakdown run after warmup ({wit} LM iterations, every launch timed with "
                                         f"HIP events)",
        }
        print(json.dumps(out), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
