"""bench.py's launcher contract (no GPU needed): --gpus N starts N ranks
itself when no launcher did, and refuses a launcher whose WORLD_SIZE is not N
before anything touches a GPU."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr
    assert p.stdout == ""


def test_launcher_command_runs_n_ranks_of_this_script():
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "3"], port=29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3"]


def test_self_launch_only_without_a_launcher(monkeypatch):
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    monkeypatch.delenv("WORLD_SIZE", raising=False)

    class A:
        gpus = 4
    assert bench.launch_or_check(A, ["--gpus", "4"]) == 7            # the child's exit code
    assert len(calls) == 1 and "--nproc-per-node=4" in calls[0]
    A.gpus = 1
    assert bench.launch_or_check(A, ["--gpus", "1"]) is None         # one GPU: run here
    monkeypatch.setenv("WORLD_SIZE", "4")
    A.gpus = 4
    assert bench.launch_or_check(A, ["--gpus", "4"]) is None         # under torch.distributed.run
    assert len(calls) == 1
