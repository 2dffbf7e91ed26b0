"""CPU: `python3 bench.py --gpus N` starts its own N ranks when no launcher did (bench.launch_plan /
bench.run_ranks).  Nothing here touches torch or a GPU: the plan is checked as data, and run_ranks
is exercised on trivial child processes."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_single_rank_needs_no_launch():
    assert bench.launch_plan(None, [], {}) == []
    assert bench.launch_plan(1, ["--gpus", "1"], {}) == []


def test_plan_for_n_ranks():
    argv = ["--gpus", "4", "--steps", "5", "--warmup", "2"]
    plan = bench.launch_plan(4, argv, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, port=12345)
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[0] == sys.executable and cmd[1].endswith("bench.py") and cmd[2:] == argv
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "12345"
        assert env["PATH"] == "/bin" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"  # inherited


def test_free_port_chosen():
    plan = bench.launch_plan(2, ["--gpus", "2"], {})
    ports = {env["MASTER_PORT"] for _, env in plan}
    assert len(ports) == 1 and int(ports.pop()) > 0


def test_torchrun_world_must_match():
    assert bench.launch_plan(None, [], {"WORLD_SIZE": "8"}) == []  # torchrun without --gpus
    assert bench.launch_plan(8, [], {"WORLD_SIZE": "8"}) == []
    err = bench.launch_plan(8, [], {"WORLD_SIZE": "2"})
    assert isinstance(err, str) and "WORLD_SIZE=2" in err


def test_run_ranks_exit_codes(tmp_path):
    ok = [([sys.executable, "-c", f"open({str(tmp_path / str(r))!r}, 'w').write(__import__('os').environ['RANK'])"],
           {**os.environ, "RANK": str(r)}) for r in range(3)]
    assert bench.run_ranks(ok, poll_s=0.05) == 0
    assert sorted(p.read_text() for p in tmp_path.iterdir()) == ["0", "1", "2"]
    # one rank fails: its code is returned and a rank that would run on is stopped
    bad = [([sys.executable, "-c", "import sys; sys.exit(3)"], dict(os.environ)),
           ([sys.executable, "-c", "import time; time.sleep(60)"], dict(os.environ))]
    assert bench.run_ranks(bad, poll_s=0.05) == 3


def test_bench_refuses_mismatch():
    import subprocess
    env = {**os.environ, "WORLD_SIZE": "2"}
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "4"], env=env, capture_output=True, timeout=60)
    assert p.returncode == 2 and b"WORLD_SIZE=2" in p.stderr
