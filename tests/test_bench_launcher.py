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
