#!/usr/bin/env python3
"""bench.py — LM iterations/s of the MI355X windowed-BA solver (libmiba).

Metric (BASELINE.json): "LM iterations/sec + ms/iter at (cams,points,obs)".
A "step" is one Levenberg-Marquardt iteration of the reference's ceres::Solve
(OptimizationUtils.cpp:300) over one resident synthetic window. Default
workload: C4 = synthetic.make_config("C4"), 200 cams / 100k points / 1M obs
(BASELINE.json configs[3], the window the north_star's 1-GPU targets are stated
on and the window tests/test_converged_parity.py checks); --config C2 / C5
select configs[1] / configs[4].

Timed region: ba_solve_prepared() with max_num_iterations = K and the
convergence tolerances disabled, so exactly K LM iterations run on a window
already resident in HBM (ba_prepare(), the host structure build + upload, is
timed separately as setup_ms). Five timed runs after the warmup; value is the
median (BASELINE.md's protocol). Each timed run is preceded by one untimed
re-solve of the same prepared window (identical work from the same prepared
start; MIBA_BENCH_WARM_EACH=0 turns it off): the host-side prepare leaves the
GPU idle for ~20 ms, and without it the timed solve runs ~3.5 % slower while
the clocks ramp back up (profiles/r02_bench_c4_warm_ab.txt).

--gpus N (one rank per GPU, RCCL over xGMI; under torchrun WORLD_SIZE must equal N, and without a launcher
bench.py starts the N rank processes itself, after checking that N devices are visible — it refuses, exit 2, rather
than report a smaller run as an N-GPU number): strong scaling of ONE
window: the BASELINE window's landmarks are split N ways (miba.shard.
split_landmarks, balanced by observation count), every rank holds the cameras
and its landmark block, and per LM iteration the ranks all-reduce the camera-side
partials, the packed envelope of the reduced camera system and the step scalars
(SURVEY §8e). value = LM iterations/s of the whole window over the max-over-ranks
wall time. --weak instead gives every rank a full C4-size landmark block of one
N-times larger window (same cameras), value = LM iterations/s of that window.

--config C1 / C3 (TUM-size stand-ins, ≈10 / 50 keyframes): latency of the
reference's per-frame call instead (main.cpp:163-168 re-optimises the same
window every frame): ms per full ba_solve (prepare + LM to convergence, default
tolerances) and per ba_solve_prepared re-solve of the resident window.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3dsmc-bundle-adjustment_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F64_MFMA_PEAK_TF = 78.6  # MI355X FP64 matrix spec (tools/mfma_f64_rate.hip measures ~73 TF/s sustained)
TIMED_RUNS = 5

# kernels whose bound is HBM bandwidth (per-observation passes) vs the f64 matrix cores
HBM_KERNELS = {"cam_side", "cam_reduce", "point_colnorm", "point_prep", "backsub_eval", "lin_finalize", "scale", "assemble",
               "update_cams", "memset_S", "obs_pairs", "final", "xnorm", "comm", "lin_point"}
# the roofline.achieved basis of the Jacobian pass (J kept in registers): the fused LM-loop
# linearisation launch (point side + camera side) when the window runs it, else the camera-side pass
JACOBIAN_PASSES = ("lin_point", "cam_side")
NO_TOL = dict(function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0, minimizer_progress_to_stdout=0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each). Under torchrun it must equal WORLD_SIZE; without a launcher and N > 1 "
                         "bench.py starts the N rank processes itself (one per visible device)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4", choices=["C1", "C2", "C3", "C4", "C5"])
    ap.add_argument("--weak", action="store_true", help="weak scaling: a C4-size landmark block per rank")
    ap.add_argument("--cpu-iters", type=int, default=4, help="LM iterations per timed run of the CPU oracle sample")
    ap.add_argument("--cpu-runs", type=int, default=3, help="timed runs of each CPU leg (median)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--shard", action="store_true", help="landmark-sharded path even on one GPU")
    ap.add_argument("--problem", default=None,
                    help="bench a window file instead of a synthetic config: a .miba dump (MIBA_DUMP_DIR capture, "
                         "solved with its captured cost options) or a BAL text problem")
    return ap.parse_args()


PMC_ALIASES = {"bcr_split": ("bcr_split", "bcr_persist")}  # profiler id -> kernel symbols it times


def load_pmc_traffic(kernel: str, config: str):
    """HBM bytes per launch from a committed rocprofv3 --pmc summary, if present."""
    # newest first: rNN_pmc_<config>[_sK].json (the r03_pmcfx_* diagnostic passes, e.g. the XCD map off, do not count)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        for name in PMC_ALIASES.get(kernel, (kernel,)):
            rec = d.get(config, {}).get(name)
            if rec and rec.get("hbm_bytes_per_launch"):
                return float(rec["hbm_bytes_per_launch"])
    return None


def obs_record(p) -> str:
    """How libmiba streams this window's observations (ba_plan.cpp obs32 check, DevProblem::obs32)."""
    import numpy as np
    adm = p.obs_depth > 1e-15
    f32 = all(np.array_equal(a.astype(np.float32).astype(np.float64), a) for a in (p.obs_uv[adm], p.obs_depth[adm]))
    if f32 and os.environ.get("MIBA_OBS32", "1") != "0":
        return ("obs32: 16-byte record {u, v, depth, index} per observation and sweep (pixels and depths are float32 "
                "values, as the reference's cv::KeyPoint and float depth image hold them; widened to f64 exactly)")
    return "f64 arrays: index 4 B + pixel 16 B + depth 8 B per observation and sweep"


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
    if e["traffic"]:
        e["traffic_over_algorithmic"] = round(e["traffic"] / max(k["bytes_per_launch"], 1.0), 3)
    e.update(kernel=k["name"], avg_launch_ms=round(avg_ms, 5),
             launches=k["launches"], bytes_per_launch=k["bytes_per_launch"], flops_per_launch=k["flops_per_launch"])
    return e


def host_info() -> dict:
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:
        avail = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": avail,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(prob0, args, file_opts) -> dict:
    """The oracle (CPU restatement of the Ceres 2.0 LM + SPARSE_SCHUR path, NOT Ceres) on a bounded sample
    of the same window: --cpu-runs timed runs of --cpu-iters LM iterations each (median), at 1 thread (the
    reference's num_threads default) and at the host threads this process may use."""
    from oracle import oracle
    info = host_info()
    threads_all = max(1, min(int(os.environ.get("OMP_NUM_THREADS") or info["affinity_cpus"] or 1),
                             info["affinity_cpus"] or 1, oracle.max_threads()))
    o = oracle.default_options(max_num_iterations=args.cpu_iters, **NO_TOL)
    if file_opts is not None:
        for f in ("hub_p_repr", "hub_p_unpr", "weight_intrinsics", "weight_unpr"):
            setattr(o, f, getattr(file_opts, f))
    legs = {}
    for threads in sorted({1, threads_all}):
        oracle.config(threads=threads, profile=True)
        its, setups = [], []
        for _ in range(max(args.cpu_runs, 1)):
            so = oracle.solve(prob0.copy(), o)
            its.append(so["num_iterations"] / (so["time_lm_ms"] * 1e-3))
            setups.append(so["time_setup_ms"])
        legs[threads] = {"value": round(statistics.median(its), 4), "cores": threads,
                         "setup_ms": round(statistics.median(setups), 2), "runs": [round(v, 4) for v in its]}
    oracle.config(1, False)
    one = legs[1]
    out = {"value": one["value"], "unit": "LM iterations/s", "cores": 1, "kind": "port",
           "sample": f"{args.config} window ({prob0.n_cams} cams / {prob0.n_points} points / {prob0.n_obs} obs): "
                     f"median of {max(args.cpu_runs, 1)} runs x {args.cpu_iters} LM iterations of the f64 C oracle "
                     f"(CPU restatement of the Ceres 2.0 LM + SPARSE_SCHUR path with a co-visibility profile "
                     f"Cholesky of the reduced camera system, NOT Ceres; Ceres is not installable here)",
           "setup_ms": one["setup_ms"], "runs": one["runs"], "host": info}
    if threads_all > 1:
        out["all_cores"] = legs[threads_all]
        if threads_all < (info["affinity_cpus"] or 0):
            # the GPU box shows the whole host in the affinity mask but grants one GPU's job a CPU share
            # (OMP_NUM_THREADS); more OpenMP threads than that share oversubscribe it
            out["all_cores"]["cores_reason"] = (f"OMP_NUM_THREADS={info['omp_num_threads']}: the CPU share this "
                                                f"job is granted on the GPU box ({info['affinity_cpus']} CPUs in "
                                                f"the affinity mask are the whole host)")
    return out


def time_runs(solver, prob0, steps, runs):
    """ba_prepare (setup) + ba_solve_prepared of exactly `steps` iterations, `runs` times."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    el, setup, summ = [], [], None
    # setup_ms is the cost of a NEW window: the plan is rebuilt on every prepare (rebuild_plan = 1)
    solver.set_options(max_num_iterations=steps, profile_kernels=0, rebuild_plan=1)
    for _ in range(runs):
        prob = prob0.copy()
        ts = time.perf_counter()
        solver.prepare(prob)
        setup.append((time.perf_counter() - ts) * 1e3)
        if os.environ.get("MIBA_BENCH_WARM_EACH", "1") == "1":
            # untimed re-solve of the same prepared window (identical work, from the same prepared start):
            # the host-side prepare above leaves the GPU idle for ~20 ms, and the timed solve should not
            # pay for its clocks ramping back up
            solver.solve_prepared(prob.copy())
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        summ = solver.solve_prepared(prob)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        el.append(t1 - t0)
    return el, setup, summ


def latency_bench(args):
    """TUM-size windows (C1 / C3 stand-ins): ms per full solve and per re-solve, GPU vs oracle."""
    import torch
    from miba import synthetic
    from miba.solver import Solver
    from oracle import oracle
    torch.cuda.set_device(0)
    prob0 = synthetic.make_config(args.config)
    opts = dict(minimizer_progress_to_stdout=0)
    with Solver(device=0, **opts) as s:
        for _ in range(max(args.warmup, 1)):
            s.solve(prob0.copy())
        full, repeat, resolve, its = [], [], [], []
        for rebuild, out in ((1, full), (0, repeat)):  # a new window per call / the same window again (plan cache)
            s.set_options(rebuild_plan=rebuild)
            for _ in range(max(args.steps, 5)):
                q = prob0.copy()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sm = s.solve(q)
                out.append((time.perf_counter() - t0) * 1e3)
                its.append(sm["num_iterations"])
        q = prob0.copy()
        s.prepare(q)
        for _ in range(max(args.steps, 5)):
            t0 = time.perf_counter()
            s.solve_prepared(q)
            resolve.append((time.perf_counter() - t0) * 1e3)
        # per-kernel breakdown of one profiled re-solve (HIP events around every launch; not the timed runs)
        s.set_options(profile_kernels=1, profile_mask=0)
        s.reset_kernel_stats()
        sp = s.solve_prepared(prob0.copy())
        breakdown = {k["name"]: round(k["total_ms"] * 1e3 / max(sp["num_iterations"], 1), 2)
                     for k in s.kernel_stats() if k["launches"] > 0}
        s.set_options(profile_kernels=0)
    oracle.config(1, True)
    cpu = []
    for _ in range(3):
        t0 = time.perf_counter()
        so = oracle.solve(prob0.copy())
        cpu.append((time.perf_counter() - t0) * 1e3)
    oracle.config(1, False)
    med = statistics.median
    out = {"metric": "ms per windowOptimize solve (prepare + LM to convergence)", "value": round(med(full), 4),
           "unit": "ms", "n_gpus": 1, "steps": len(full), "warmup": args.warmup, "ms_per_step": round(med(full), 4),
           "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"{args.config} TUM-size stand-in: {prob0.n_cams} cams / {prob0.n_points} points / "
                                  f"{prob0.n_obs} obs (synthetic.make_config; real TUM windows need the dataset and "
                                  f"the OpenCV/OpenGV front-end, absent offline)", "cams": prob0.n_cams,
                      "points": prob0.n_points, "obs": prob0.n_obs, "parallelism": "single"},
           "lm_iterations": its[0], "ms_per_resolve_prepared": round(med(resolve), 4),
           "ms_per_lm_iteration": round(med(full) / max(its[0], 1), 4),
           "ms_per_repeat_solve": round(med(repeat), 4),
           "kernel_us_per_lm_iteration": breakdown,
           "what": "value: ba_solve of a new window (host plan rebuilt, rebuild_plan = 1); ms_per_repeat_solve: "
                   "ba_solve of the same window again, the reference's per-frame call (main.cpp:163-168), plan cache "
                   "on; ms_per_resolve_prepared: ba_solve_prepared of the resident window",
           "cpu_baseline": {"value": round(med(cpu), 3), "unit": "ms", "cores": 1, "kind": "port",
                            "sample": f"oracle full solve of the same window ({so['num_iterations']} LM iterations), "
                                      f"median of 3", "host": host_info()}}
    print(json.dumps(out), flush=True)


def rank_plan(gpus, latency, env, n_visible, argv, port):
    """What this process does for `--gpus`: ("run", None) — this process is the one rank of a 1-GPU run or one
    rank of an outside launcher (torchrun) whose WORLD_SIZE agrees; ("spawn", [(cmd, env), ...]) — start N rank
    processes (no outside launcher, N > 1); ("error", message) — a world-size mismatch, too few visible devices or
    a config that does not shard. Decided before anything touches the GPU (the parent never initialises HIP)."""
    world = env.get("WORLD_SIZE")
    if world is not None:
        w = int(world)
        if gpus is not None and gpus != w:
            return "error", f"--gpus {gpus} disagrees with WORLD_SIZE={w} set by the launcher"
        if w > 1 and latency:
            return "error", "--config C1 / C3 is the single-GPU latency bench (TUM-size windows are never sharded)"
        return "run", None
    n = 1 if gpus is None else gpus
    if n < 1:
        return "error", f"--gpus {n}: need at least one GPU"
    if n == 1:
        return "run", None
    if latency:
        return "error", "--config C1 / C3 is the single-GPU latency bench (TUM-size windows are never sharded)"
    if n_visible < n:
        return "error", (f"--gpus {n} but only {n_visible} HIP device(s) visible (KFD topology, *_VISIBLE_DEVICES): "
                         f"refusing to report a {n}-GPU number")
    procs = []
    for r in range(n):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(([sys.executable, os.path.abspath(__file__)] + list(argv), e))
    return "spawn", procs


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def _visible_list(value: str, n: int) -> int:
    """How many of n devices a *_VISIBLE_DEVICES list keeps: distinct in-range ordinals, or UUID-style entries."""
    keep = set()
    for item in (x.strip() for x in value.split(",")):
        if not item:
            continue
        if item.isdigit():
            if int(item) >= n:
                break  # the runtimes stop at the first invalid ordinal
            keep.add(int(item))
        else:
            keep.add(item)
    return min(len(keep), n)


def visible_gpus(env=None, topology: str | None = None, dri: str | None = None) -> int:
    """HIP devices this process would see, counted WITHOUT touching HIP (no torch import, no libamdhip64, /dev/kfd
    never opened): KFD topology nodes with a non-zero gpu_id whose render node exists in /dev/dri (a container sees
    every node of the host in sysfs but only its own GPUs' render nodes), then ROCR_VISIBLE_DEVICES and
    HIP_VISIBLE_DEVICES (else CUDA_VISIBLE_DEVICES), in that order. On ROCm torch, torch.cuda.device_count() falls
    back to hipGetDeviceCount, which initialises HIP, whenever amdsmi cannot initialise; the
    parent of the rank processes must not hold the GPU when it starts them. MIBA_KFD_TOPOLOGY / MIBA_DRI_DIR point
    the count at another tree (tests)."""
    env = os.environ if env is None else env
    topology = topology or env.get("MIBA_KFD_TOPOLOGY", KFD_TOPOLOGY)
    dri = dri or env.get("MIBA_DRI_DIR", "/dev/dri")
    n = 0
    for node in sorted(glob.glob(os.path.join(topology, "*"))):
        try:
            gpu_id = int(open(os.path.join(node, "gpu_id")).read().strip() or 0)
        except (OSError, ValueError):
            continue
        if gpu_id == 0:
            continue  # a CPU node
        minor = None
        try:
            for line in open(os.path.join(node, "properties")):
                k, _, v = line.partition(" ")
                if k == "drm_render_minor":
                    minor = int(v)
        except (OSError, ValueError):
            pass
        if minor is not None and minor > 0 and os.path.isdir(dri) and \
                not os.path.exists(os.path.join(dri, f"renderD{minor}")):
            continue  # on the host, not in this container
        n += 1
    if env.get("ROCR_VISIBLE_DEVICES") is not None:
        n = _visible_list(env["ROCR_VISIBLE_DEVICES"], n)
    hip = env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES"))
    if hip is not None:
        n = _visible_list(hip, n)
    return n


def parent_gpu_state(pid: str = "self") -> list:
    """What of the GPU stack this process holds: /dev/kfd open, the HIP runtime mapped. Empty = nothing."""
    held = []
    try:
        for fd in os.listdir(f"/proc/{pid}/fd"):
            try:
                if os.readlink(f"/proc/{pid}/fd/{fd}") == "/dev/kfd":
                    held.append("/dev/kfd open")
                    break
            except OSError:
                pass
    except OSError:
        pass
    try:
        with open(f"/proc/{pid}/maps") as f:
            if any("libamdhip64" in line for line in f):
                held.append("libamdhip64 mapped")
    except OSError:
        pass
    return held


def spawn_ranks(procs) -> int:
    """Run the rank processes (rank 0's stdout is the bench line); a failed rank ends the others. The parent must
    not hold the GPU (an initialised HIP runtime in a parent of GPU processes is not safe on this pool)."""
    import subprocess
    held = parent_gpu_state()
    if held:
        print(f"bench.py: the launching process holds the GPU ({', '.join(held)}): refusing to start ranks",
              file=sys.stderr)
        return 2
    if os.environ.get("MIBA_BENCH_VERBOSE") == "1":
        print(f"bench.py: parent {os.getpid()}: /dev/kfd not open, libamdhip64 not mapped; starting {len(procs)} ranks",
              file=sys.stderr, flush=True)
    ps = [subprocess.Popen(cmd, env=env, stdout=None if r == 0 else subprocess.DEVNULL)
          for r, (cmd, env) in enumerate(procs)]
    rc = 0
    try:
        pending = set(range(len(ps)))
        while pending:
            for r in list(pending):
                c = ps[r].poll()
                if c is None:
                    continue
                pending.discard(r)
                if c != 0 and rc == 0:
                    rc = c
                    print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                    for q in pending:
                        ps[q].terminate()
            time.sleep(0.05)
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    return rc


def free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def main():
    args = parse()
    latency = args.config in ("C1", "C3") and not args.problem
    if os.environ.get("WORLD_SIZE") is None and (args.gpus or 1) > 1:
        # counted from sysfs: the parent never imports torch or loads the HIP runtime
        kind, what = rank_plan(args.gpus, latency, os.environ, visible_gpus(), sys.argv[1:], free_port())
    else:
        kind, what = rank_plan(args.gpus, latency, os.environ, 0, sys.argv[1:], 0)
    if kind == "error":
        print(f"bench.py: {what}", file=sys.stderr)
        raise SystemExit(2)
    if kind == "spawn":
        raise SystemExit(spawn_ranks(what))
    if latency:
        return latency_bench(args)
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

    from miba import shard, synthetic
    from miba.solver import Solver

    sharded = world > 1 or args.shard
    file_opts = None
    if args.problem:
        from miba import problem_io
        whole, file_opts = problem_io.load(args.problem)
        args.config = "file"
    elif args.weak:
        whole = None
        prob = synthetic.make_landmark_shard(args.config, rank)  # shard 0 == the single-GPU window's cameras
    else:
        whole = synthetic.make_config(args.config)
    if whole is not None:
        prob = shard.split_landmarks(whole, world, rank)[0] if world > 1 else whole
    prob0 = prob.copy()

    prof = 0 if args.no_profile else 1
    solver = Solver(file_opts, device=local_rank, profile_kernels=prof, max_num_iterations=max(args.warmup, 1),
                    **NO_TOL)
    if sharded:
        box = [Solver.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=0)
        solver.comm_init(world, rank, box[0])
    # warmup (untimed, unprofiled: first launches load the code objects)
    if args.warmup > 0:
        solver.set_options(max_num_iterations=args.warmup, profile_kernels=0)
        prob = prob0.copy()
        solver.prepare(prob)
        solver.solve_prepared(prob)
    # breakdown run: every kernel launch timed (per-iteration breakdown, dominant kernel)
    solver.set_options(max_num_iterations=5, profile_kernels=prof, profile_mask=0)
    prob = prob0.copy()
    solver.prepare(prob)
    solver.reset_kernel_stats()
    wsumm = solver.solve_prepared(prob)
    wstats = solver.kernel_stats()
    names = [k["name"] for k in wstats]
    live = [k for k in wstats if k["launches"] > 0]
    dom = max(live, key=lambda k: k["total_ms"])["name"] if live else None
    jac = next((nm for nm in JACOBIAN_PASSES if any(k["name"] == nm for k in live)), JACOBIAN_PASSES[-1])
    # timed runs (no HIP events: event records between dependent launches cost ~5-10 us each)
    els, setups, summ = time_runs(solver, prob0, args.steps, TIMED_RUNS)
    # the same K-step region again with HIP events around the dominant kernel and the
    # Jacobian pass only: their average launch durations for the roofline
    stats = []
    if prof:
        mask = 0
        for nm in (dom, jac):
            if nm in names:
                mask |= 1 << names.index(nm)
        solver.set_options(max_num_iterations=args.steps, profile_kernels=1, profile_mask=mask)
        solver.prepare(prob0.copy())
        solver.reset_kernel_stats()
        solver.solve_prepared(prob0.copy())
        stats = solver.kernel_stats()
    # end-to-end windowOptimize cost of this window: ba_solve = ba_prepare (host plan + upload) + the LM loop to
    # termination with the reference's own settings (tolerances on, max_num_iterations 75), median of 3 warm calls
    # new window every call (rebuild_plan = 1) and the reference's per-frame re-solve of the same window
    # (main.cpp:163-168: the plan cache reuses the structure, rebuild_plan = 0; unsharded windows only)
    def e2e_leg(rebuild):
        out, its, prep = [], 0, []
        solver.set_options(max_num_iterations=75, profile_kernels=0, function_tolerance=1e-6, gradient_tolerance=1e-10,
                           parameter_tolerance=1e-8, rebuild_plan=rebuild)
        for _ in range(4):
            q = prob0.copy()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            se = solver.solve(q)
            out.append((time.perf_counter() - t0) * 1e3)
            its = se["num_iterations"]
            prep.append(solver.last_prepare())
        return out[1:], its, prep[1:]  # the first call may grow buffers / build the plan
    e2e, e2e_it, _ = e2e_leg(1)
    e2e_rep, e2e_rep_it, rep_prep = e2e_leg(0)
    setups_rep = []
    solver.set_options(max_num_iterations=args.steps, rebuild_plan=0, **NO_TOL)
    for _ in range(TIMED_RUNS):
        q = prob0.copy()  # the caller's arrays exist before the call (as in time_runs)
        ts = time.perf_counter()
        solver.prepare(q)
        setups_rep.append((time.perf_counter() - ts) * 1e3)
    rep_info = solver.last_prepare()
    iters = summ["num_iterations"]
    elapsed = statistics.median(els)
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
        value = iters / elapsed_max
        ms_per_step = elapsed_max * 1e3 / max(iters, 1)
        kern = [k for k in stats if k["launches"] > 0]
        roofs = {k["name"]: roofline_entry(k, args.config) for k in kern}
        jr = roofs.get(jac)
        if jr is not None and jr.get("avg_launch_ms"):
            # the fused pass never writes J, so achieved / frac count only the bytes it moves
            # (bytes_per_launch, the algorithmic model; traffic = the PMC-measured HBM bytes beside it)
            us = jr["avg_launch_ms"] * 1e3
            jr["basis"] = "bytes the fused pass moves (J recomputed in registers, never written)"
            if jr.get("flops_per_launch"):
                # the pass is f64 VALU work (lin_obs + the Gram sums); same 78.6 TF/s peak as the f64 MFMA
                jr["valu_f64"] = {"achieved_tflops": round(jr["flops_per_launch"] / (us * 1e-6) / 1e12, 3),
                                  "peak_tflops": F64_MFMA_PEAK_TF,
                                  "frac": round(jr["flops_per_launch"] / (us * 1e-6) / 1e12 / F64_MFMA_PEAK_TF, 4)}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(prob0, args, file_opts)
        wit = max(wsumm["num_iterations"], 1)
        phases = {k["name"]: round(k["total_ms"] / wit, 4) for k in live}  # breakdown run, every kernel timed
        n_cams = prob0.n_cams
        n_pts = whole.n_points if whole is not None else world * prob0.n_points
        n_obs = whole.n_obs if whole is not None else world * prob0.n_obs
        if args.problem:
            workload = f"{os.path.basename(args.problem)}: {n_cams} cams / {n_pts} points / {n_obs} obs, one window"
        else:
            workload = f"{args.config}: {n_cams} cams / {n_pts} points / {n_obs} obs, one window"
        if world > 1 and not args.weak:
            workload += f", landmark-sharded across {world} GPUs (strong scaling, RCCL all-reduce per LM iteration)"
        elif args.weak:
            workload = (f"{args.config} landmark blocks: {n_cams} cams / {world}x{prob0.n_points} points / "
                        f"{world}x{prob0.n_obs} obs, one window with a C4-size landmark block per GPU (weak scaling, "
                        f"RCCL all-reduce per LM iteration)")
        elif sharded:
            workload += ", landmark-sharded path with a 1-rank RCCL communicator"
        out = {
            "metric": "LM iterations/sec",
            "value": round(value, 3),
            "unit": "LM iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "file" if args.problem else "synthetic",
            "config": {"workload": workload, "cams": n_cams, "points": n_pts, "obs": n_obs,
                       "parallelism": f"landmark-shard{world}" if sharded else "single",
                       "obs_record": obs_record(prob0)},
            "setup_ms": round(statistics.median(setups), 3),
            "end_to_end_ms": round(statistics.median(e2e), 3),
            "end_to_end": {"what": "ba_solve = ba_prepare + LM to termination with the reference settings "
                                   "(tolerances 1e-6 / 1e-10 / 1e-8, max 75 iterations), warm context, median of 3; "
                                   "a new window every call (the host plan rebuilt: rebuild_plan = 1)",
                           "lm_iterations": e2e_it, "runs_ms": [round(v, 3) for v in e2e]},
            "setup_ms_repeat": round(statistics.median(setups_rep), 3),
            "end_to_end_repeat_ms": round(statistics.median(e2e_rep), 3),
            "end_to_end_repeat": {"what": "the reference's per-frame re-solve of the same window (main.cpp:163-168): "
                                          "ba_solve of an unchanged window structure, the plan cache reuses the host "
                                          "plan and the device structure (rebuild_plan = 0) and uploads the parameters",
                                  "lm_iterations": e2e_rep_it, "runs_ms": [round(v, 3) for v in e2e_rep],
                                  "plan_reused": [int(i["plan_reused"]) for i in rep_prep],
                                  "prepare": {k: (round(v, 4) if isinstance(v, float) else v)
                                              for k, v in rep_info.items()}},
            "timed_runs": {"n": len(els), "ms_per_step": [round(e * 1e3 / max(iters, 1), 4) for e in els],
                           "statistic": "median"},
            "roofline": roofs.get(dom),
            "roofline_source": "libmiba HIP events (solver stream) around every launch of the dominant kernel and of "
                               "the Jacobian pass, over a repeat of the timed K-step region",
            "roofline_jacobian_pass": roofs.get(jac),
            "cpu_baseline": cpu,
            "lm": {"iterations": iters, "successful": summ["num_successful_steps"],
                   "note": "iterations = LM steps after iteration 0; successful counts iteration 0 (Ceres convention)",
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
