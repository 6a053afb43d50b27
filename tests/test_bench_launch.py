"""bench.py starts its own ranks for --gpus N > 1 (no GPU needed).

The driver's 8-GPU run may call `python3 bench.py --gpus 8` without a launcher.  bench.py
then runs `python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1
... bench.py <same args>` as a child (before touching the GPU), relays rank 0's JSON line and
exits with the child's code; a WORLD_SIZE that disagrees with --gpus is an error, not a
warning.  (reference: coordinator.go:179-199, the coordinator starts every worker's search.)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_launch_command_for_n_gpus():
    r = run(["--gpus", "8", "--steps", "3", "--warmup", "1", "--no-probe", "--print-launch"])
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout)
    cmd = rec["launch"]
    assert rec["world_size"] == 8
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(a.startswith("--master-port=") and int(a.split("=")[1]) > 0 for a in cmd)
    i = cmd.index(os.path.abspath(BENCH))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3", "--warmup", "1", "--no-probe"]  # same args, no --print-launch


def test_one_gpu_needs_no_launcher():
    r = run(["--gpus", "1", "--print-launch"])
    assert r.returncode == 0 and json.loads(r.stdout) == {"launch": None, "world_size": 1}


def test_under_a_launcher_no_second_launch():
    r = run(["--gpus", "4", "--print-launch"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 0 and json.loads(r.stdout) == {"launch": None, "world_size": 4}


def test_world_size_mismatch_is_an_error():
    r = run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_too_few_gpus_is_an_error():
    """--gpus 2 on a host without 2 visible GPUs (this container has none) fails before
    starting any rank, unless --same-device rehearses the ranks on one card."""
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("two GPUs visible")
    r = run(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr and r.stdout == ""


def test_failing_ranks_fail_the_bench():
    """The child's exit code is bench.py's: here both ranks fail (no GPU in this container)
    and bench.py exits non-zero with no result line (on the GPU box the same command is
    the 2-rank gloo rehearsal, tools/gpu.sh check)."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("a GPU is visible: the ranks would run")
    r = run(["--gpus", "2", "--backend", "gloo", "--same-device", "--steps", "1", "--warmup", "0", "--no-probe",
             "--no-cpu-baseline", "--no-tts"])
    assert r.returncode != 0, (r.stdout, r.stderr[-2000:])
    assert r.stdout == ""
    assert "torch.distributed.run" in r.stderr  # the launcher ran


def test_node_shape_coordinator_devices():
    """bench.py's node-shape BASELINE configs put logical worker i on rank i's GPU, wrapping
    onto the GPUs the process sees, and everything on GPU 0 for --same-device rehearsals."""
    import bench
    assert bench.node_devices(8, False, 8) == list(range(8))
    assert bench.node_devices(4, False, 8) == [0, 1, 2, 3]
    assert bench.node_devices(8, False, 2) == [0, 1] * 4
    assert bench.node_devices(2, False, 0) == [0, 0]
    assert bench.node_devices(8, True, 8) == [0] * 8
