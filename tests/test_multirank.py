"""Multi-rank landmark sharding through libmiba itself: N processes, one landmark shard
each, all on GPU 0, exchanging the camera-side partials, the envelope of the reduced camera system
and the step scalars over a torch.distributed gloo host collective (ba_comm_init_host) — the same
collective sequence the RCCL backend runs across GPUs. The sharded solve must reproduce the
unsharded one (final cost 1e-10 relative, same iterations, cameras / points to rounding) and the
oracle (final cost 1e-6 relative, same iteration count), including a rank whose shard is empty.

Each rank is a child process started before it touches the GPU (tests/mr_worker.py)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from miba import synthetic
from oracle import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(tmp_path, world, spec, timeout=240):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "mr_worker.py"), str(tmp_path),
                                       json.dumps(spec)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed ({p.returncode}):\n{outs[r][-3000:]}"
    res = []
    for r in range(world):
        z = np.load(os.path.join(tmp_path, f"rank{r}.npz"))
        res.append(dict(cams=z["cams"], points=z["points"], intr=z["intr"], ids=z["ids"], log=z["log"],
                        summary=json.loads(str(z["summary"])), comm_launches=int(z["comm_launches"])))
    return res


def unsharded(prob, **opts):
    from miba.solver import Solver
    q = prob.copy()
    with Solver(device=0, minimizer_progress_to_stdout=0, **opts) as s:
        summ = s.solve(q)
        log = s.iteration_log()
    return q, summ, log


def check(res, whole, ref_q, ref_s, ref_log, so):
    s0 = res[0]["summary"]
    for r in res:
        s = r["summary"]
        # identical decisions on every rank
        assert s["num_iterations"] == s0["num_iterations"] and s["final_cost"] == s0["final_cost"], (s, s0)
        np.testing.assert_array_equal(r["cams"], res[0]["cams"])  # replicated solve: bitwise identical
        np.testing.assert_array_equal(r["log"], res[0]["log"])
    assert s0["num_obs_admissible"] == ref_s["num_obs_admissible"]
    assert s0["num_iterations"] == ref_s["num_iterations"] == so["num_iterations"], (s0, ref_s, so)
    assert s0["num_successful_steps"] == ref_s["num_successful_steps"]
    assert abs(s0["initial_cost"] - ref_s["initial_cost"]) <= 1e-12 * ref_s["initial_cost"]
    assert abs(s0["final_cost"] - ref_s["final_cost"]) <= 1e-10 * ref_s["final_cost"], (s0, ref_s)
    assert abs(s0["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (s0, so)
    np.testing.assert_array_equal(res[0]["log"][:, 6], ref_log[:, 6])  # same accept / reject sequence
    pts = whole.points.copy()
    for r in res:
        pts[r["ids"]] = r["points"]
    np.testing.assert_allclose(res[0]["cams"], ref_q.cams, rtol=0, atol=1e-8)
    np.testing.assert_allclose(pts, ref_q.points, rtol=0, atol=1e-7)
    np.testing.assert_allclose(res[0]["intr"], ref_q.intr, rtol=1e-9)


@pytest.mark.parametrize("world,nsplit,env", [(2, 2, {}), (2, 2, {"MIBA_BCR": "launch"}), (4, 3, {})])
def test_c2_sharded_ranks(tmp_path, world, nsplit, env):
    """C2 (20 cams / 5k points / 50k obs) split over 2 ranks, and over 3 ranks + one empty shard."""
    spec = {"problem": {"config": "C2"}, "nsplit": nsplit, "env": env, "options": {"shard_min_obs": 0}}
    res = run_ranks(tmp_path, world, spec)
    whole = synthetic.make_config("C2")
    ref_q, ref_s, ref_log = unsharded(whole)
    so = oracle.solve(whole.copy())
    check(res, whole, ref_q, ref_s, ref_log, so)


def test_c4_sharded_four_ranks_one_empty(tmp_path):
    """C4 (200 cams / 100k points / 1M obs, the 4-GPU headline window) on 4 ranks, one of them empty,
    to termination with the reference's default tolerances."""
    spec = {"problem": {"config": "C4"}, "nsplit": 3}
    res = run_ranks(tmp_path, 4, spec, timeout=400)
    whole = synthetic.make_config("C4")
    ref_q, ref_s, ref_log = unsharded(whole)
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_oracle.json")))
    so = dict(num_iterations=gold["num_iterations"], final_cost=gold["final_cost"])
    check(res, whole, ref_q, ref_s, ref_log, so)


def test_tum_like_two_ranks_wide_overflow(tmp_path):
    """Overflow (atomic) Schur points and repeated-camera links on both ranks."""
    mp = dict(n_cams=30, n_points=150, obs_per_point=(6, 16), seed=5, rot_noise=0.005, dup_frac=0.05)
    res = run_ranks(tmp_path, 2, {"problem": {"make_problem": mp}, "nsplit": 2, "options": {"shard_min_obs": 0}})
    whole = synthetic.make_problem(**mp)
    ref_q, ref_s, ref_log = unsharded(whole)
    so = oracle.solve(whole.copy())
    check(res, whole, ref_q, ref_s, ref_log, so)


def test_small_window_is_gathered_not_sharded(tmp_path):
    """ba_options.shard_min_obs (default 262144 admissible observations): C2's 50k observations are
    gathered onto both ranks at ba_prepare and each rank solves the whole window alone (no per-iteration
    collective), in deterministic mode, so both ranks hold bitwise the same cameras."""
    spec = {"problem": {"config": "C2"}, "nsplit": 2, "options": {"profile_kernels": 1}}
    res = run_ranks(tmp_path, 2, spec)
    whole = synthetic.make_config("C2")
    ref_q, ref_s, ref_log = unsharded(whole)
    so = oracle.solve(whole.copy())
    check(res, whole, ref_q, ref_s, ref_log, so)
    assert all(r["comm_launches"] == 0 for r in res)  # no collective inside the LM loop


def test_sharded_exchange_runs_collectives(tmp_path):
    spec = {"problem": {"config": "C2"}, "nsplit": 2, "options": {"profile_kernels": 1, "shard_min_obs": 0,
                                                                  "max_num_iterations": 4}}
    res = run_ranks(tmp_path, 2, spec)
    assert all(r["comm_launches"] > 0 for r in res)


def test_c5_sharded_two_ranks(tmp_path):
    """C5 (1000 cams / 500k points / 5M obs, BASELINE configs[4], the 8-GPU window; main.cpp:179-183's global
    BA is where windows this large come from) split over 2 ranks on GPU 0: 3 LM iterations with the tolerances
    off through the sharded exchange (the ~6 MB envelope + rhs + camera sums all-reduce of 1000 cameras).
    Cameras bitwise identical across ranks; the unsharded solve to 1e-10; the oracle fixture's first 3 trace
    rows (tests/golden/c5_oracle.json) to 1e-9."""
    opts = {"shard_min_obs": 0, "max_num_iterations": 3, "function_tolerance": 0.0, "parameter_tolerance": 0.0,
            "gradient_tolerance": 0.0}
    res = run_ranks(tmp_path, 2, {"problem": {"config": "C5"}, "nsplit": 2, "options": opts}, timeout=600)
    whole = synthetic.make_config("C5")
    ref_q, ref_s, ref_log = unsharded(whole, **{k: v for k, v in opts.items() if k != "shard_min_obs"})
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "c5_oracle.json")))
    tr = np.array(gold["trace"])[:4]
    s0 = res[0]["summary"]
    for r in res:
        assert r["summary"]["num_iterations"] == 3 and r["summary"]["final_cost"] == s0["final_cost"]
        np.testing.assert_array_equal(r["cams"], res[0]["cams"])
        np.testing.assert_array_equal(r["log"], res[0]["log"])
        assert r["comm_launches"] == 0  # unprofiled: kernel stats are not collected
    assert s0["num_obs_admissible"] == ref_s["num_obs_admissible"] == whole.n_obs
    assert abs(s0["final_cost"] - ref_s["final_cost"]) <= 1e-10 * ref_s["final_cost"], (s0, ref_s)
    np.testing.assert_array_equal(res[0]["log"][:, 6], ref_log[:, 6])
    np.testing.assert_allclose(res[0]["log"][:, 0], tr[:, 0], rtol=1e-9)  # cost of iterations 0..3
    np.testing.assert_allclose(res[0]["log"][:, 5], tr[:, 5], rtol=1e-9)  # trust-region radius
    np.testing.assert_allclose(res[0]["log"][1:, 3], tr[1:, 3], rtol=1e-6)  # |step|
    pts = whole.points.copy()
    for r in res:
        pts[r["ids"]] = r["points"]
    np.testing.assert_allclose(res[0]["cams"], ref_q.cams, rtol=0, atol=1e-8)
    np.testing.assert_allclose(pts, ref_q.points, rtol=0, atol=1e-7)


@pytest.mark.parametrize("profiled", [0, 1])
def test_bcr_timeout_rerun_in_lockstep_on_shards(tmp_path, profiled):
    """A forced hand-off timeout of the resident BCR kernel (MIBA_BCR_SPIN_LIMIT=1) on landmark shards: every
    rank sees the same decision (the timeout flag rides the step-scalar exchange), pads its enqueued iterations
    to the same count, re-runs the iteration with the per-level launches and finishes with BA_OK; the profiled
    batch loop takes the same re-run path. Same iterations on every rank, oracle parity."""
    spec = {"problem": {"config": "C2"}, "nsplit": 2, "env": {"MIBA_BCR_SPIN_LIMIT": "1"},
            "options": {"shard_min_obs": 0, "profile_kernels": profiled}}
    res = run_ranks(tmp_path, 2, spec)
    whole = synthetic.make_config("C2")
    ref_q, ref_s, ref_log = unsharded(whole)
    so = oracle.solve(whole.copy())
    check(res, whole, ref_q, ref_s, ref_log, so)
