"""bench.py --gpus N without an outside launcher: the parent plans N rank processes before
anything touches the GPU, refuses a --gpus / WORLD_SIZE mismatch and refuses to run with fewer visible devices than
asked (a 1-GPU box must not print a "2-GPU" number). CPU only: the plan is checked, no rank is started, except the
refusal, which runs bench.py for real and needs no device."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_builds_one_command_per_rank():
    argv = ["--gpus", "4", "--steps", "10", "--warmup", "2"]
    kind, procs = bench.rank_plan(4, False, {"PATH": "/usr/bin"}, 8, argv, 29511)
    assert kind == "spawn" and len(procs) == 4
    for r, (cmd, env) in enumerate(procs):
        assert cmd[0] == sys.executable and cmd[1].endswith("bench.py") and cmd[2:] == argv
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == "4" and env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/usr/bin"


@pytest.mark.parametrize("gpus,env,visible,want", [
    (None, {}, 0, "run"),                                    # default: one GPU, this process
    (1, {}, 8, "run"),
    (8, {"WORLD_SIZE": "8"}, 0, "run"),                      # under torchrun (the driver's N > 1 form)
    (None, {"WORLD_SIZE": "2"}, 0, "run"),
    (4, {"WORLD_SIZE": "8"}, 0, "error"),                    # mismatch with the launcher
    (2, {}, 1, "error"),                                     # a 1-GPU box asked for 2
    (0, {}, 8, "error"),
])
def test_plan_decisions(gpus, env, visible, want):
    assert bench.rank_plan(gpus, False, env, visible, [], 1)[0] == want


def test_latency_configs_do_not_shard():
    assert bench.rank_plan(2, True, {}, 8, [], 1)[0] == "error"
    assert bench.rank_plan(None, True, {"WORLD_SIZE": "2"}, 0, [], 1)[0] == "error"
    assert bench.rank_plan(1, True, {}, 8, [], 1)[0] == "run"


def test_too_few_devices_fails_loudly():
    """This container has no GPU: --gpus 2 must exit non-zero with a message, not print a 1-GPU line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "refusing" in r.stderr and r.stdout.strip() == ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       env=dict(env, WORLD_SIZE="4"), timeout=300)
    assert r.returncode == 2 and "disagrees with WORLD_SIZE=4" in r.stderr, (r.returncode, r.stderr)


# ---- device count without HIP ---------------------------------------------------------------
def _fake_tree(tmp_path, gpus, in_container=None, cpu_nodes=2):
    """A KFD topology like the GPU boxes': CPU nodes (gpu_id 0 or unreadable), GPU nodes with render minors; only
    the render nodes in `in_container` (default: all) exist under the fake /dev/dri."""
    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    k = 0
    for _ in range(cpu_nodes):
        d = topo / str(k); d.mkdir(parents=True); k += 1
        (d / "gpu_id").write_text("0\n")
        (d / "properties").write_text("cpu_cores_count 64\nsimd_count 0\ndrm_render_minor 0\n")
    d = topo / str(k); d.mkdir(parents=True); k += 1
    (d / "gpu_id").write_text("")  # unreadable / empty, as on the boxes
    for g in range(gpus):
        d = topo / str(k); d.mkdir(parents=True); k += 1
        minor = 128 + 8 * g
        (d / "gpu_id").write_text(f"{4000 + g}\n")
        (d / "properties").write_text(f"simd_count 1024\ndrm_render_minor {minor}\n")
        if in_container is None or g in in_container:
            (dri / f"renderD{minor}").write_text("")
    return str(topo), str(dri)


@pytest.mark.parametrize("gpus,in_container,env,want", [
    (8, None, {}, 8),
    (8, {5}, {}, 1),                                           # a 1-GPU container on an 8-GPU host
    (8, None, {"ROCR_VISIBLE_DEVICES": "0,1,2,3"}, 4),
    (8, None, {"HIP_VISIBLE_DEVICES": "2,3"}, 2),
    (8, None, {"ROCR_VISIBLE_DEVICES": "0,1", "HIP_VISIBLE_DEVICES": "1"}, 1),
    (8, None, {"CUDA_VISIBLE_DEVICES": "0,1,2"}, 3),
    (8, None, {"HIP_VISIBLE_DEVICES": ""}, 0),
    (1, None, {"ROCR_VISIBLE_DEVICES": "0", "HIP_VISIBLE_DEVICES": "0"}, 1),  # the gpurun box's settings
    (2, None, {"HIP_VISIBLE_DEVICES": "0,7"}, 1),             # stops at the first out-of-range ordinal
    (2, None, {"ROCR_VISIBLE_DEVICES": "GPU-abc,GPU-def"}, 2),
    (0, None, {}, 0),
])
def test_visible_gpus_from_sysfs(tmp_path, gpus, in_container, env, want):
    topo, dri = _fake_tree(tmp_path, gpus, in_container)
    assert bench.visible_gpus(env=env, topology=topo, dri=dri) == want


def _run_bench(tmp_path, gpus, extra_env=None, args=("--gpus", "2", "--steps", "2")):
    topo, dri = _fake_tree(tmp_path, gpus)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                        "CUDA_VISIBLE_DEVICES")}
    env.update(MIBA_KFD_TOPOLOGY=topo, MIBA_DRI_DIR=dri, MIBA_BENCH_VERBOSE="1", **(extra_env or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), capture_output=True,
                          text=True, env=env, timeout=300)


def test_one_gpu_tree_refuses_two(tmp_path):
    r = _run_bench(tmp_path, 1)
    assert r.returncode == 2 and "only 1 HIP device(s) visible" in r.stderr and r.stdout.strip() == ""


def test_parent_never_touches_the_gpu_stack(tmp_path):
    """With two (fake) devices the parent plans and starts the ranks: before Popen it has not opened /dev/kfd and
    has not mapped libamdhip64 (it never imports torch). The ranks then fail here (no GPU), which the parent
    reports with their exit code."""
    r = _run_bench(tmp_path, 2)
    assert "/dev/kfd not open, libamdhip64 not mapped; starting 2 ranks" in r.stderr, r.stderr
    assert r.returncode not in (0, 2), (r.returncode, r.stderr)  # the ranks' own failure, not a refusal


def test_parent_gpu_state_sees_the_hip_runtime():
    """The check itself: a process that has loaded torch's HIP runtime reports it."""
    code = ("import sys; sys.path.insert(0, %r); import bench; a = bench.parent_gpu_state(); import torch; "
            "b = bench.parent_gpu_state(); print(a, b)" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300).stdout
    before, after = out.strip().split("] [")
    assert "libamdhip64" not in before and "libamdhip64 mapped" in after
