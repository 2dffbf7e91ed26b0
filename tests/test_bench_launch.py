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


def _args(**kw):
    import argparse
    base = {"config": 2, "no_cfg3": False, "no_gapassem": False}
    base.update(kw)
    return argparse.Namespace(**base)


@pytest.mark.parametrize("world", [1, 2, 8])
def test_cfg3_sub_object_at_every_n(world):
    """the N = 1 line carries the cfg3 sub-object too (the denominator of the 1 -> 8
    strong-scaling curve on BASELINE configs[2]); gapassem only at N = 1."""
    subs = bench.sub_objects(world, _args())
    assert "cfg3" in subs
    assert ("gapassem" in subs) == (world == 1)
    assert bench.sub_objects(world, _args(no_cfg3=True)) == (["gapassem"] if world == 1 else [])
    assert bench.sub_objects(world, _args(config=3)) == []


def test_scaling_cfg3_keys_same_at_every_n():
    """scaling_cfg3 has the same keys at N = 1 and N > 1 (speedup(N) = value(N) / value(1))."""
    def sub(v, n, e2e):
        return {"value": v, "unit": "events/s", "ms_per_step": 1.0, "e2e": e2e,
                "config": {"records_total": 10_000_000, "events_total": 208_439_620},
                "roofline": {"kernel_ms": 18.5 / n}}
    one = bench.scaling_cfg3(sub(1.1e10, 1, {"wall_s": 6.0, "events_per_s": 3.4e7}), 1)
    eight = bench.scaling_cfg3(sub(8.0e10, 8, {"wall_s": 1.2, "events_per_s": 1.7e8}), 8)
    assert one.keys() == eight.keys()
    assert one["n_gpus"] == 1 and eight["n_gpus"] == 8 and one["scaling"] == "strong"
    assert eight["value"] / one["value"] > 7 and one["e2e_wall_s"] / eight["e2e_wall_s"] == 5.0
    assert bench.CFG3_KEYS == ("value", "unit", "n_gpus", "steps", "ms_per_step", "scaling", "config", "roofline",
                               "e2e")


def test_rank_thread_share(monkeypatch):
    """Several ranks under torchrun's OMP_NUM_THREADS=1: each rank gets its share of the CPUs as
    PW_THREADS (at most 16); an explicit PW_THREADS, a chosen OMP_NUM_THREADS or one rank: untouched."""
    import os
    import bench
    ncpu = len(os.sched_getaffinity(0))
    for env, want in [({"LOCAL_WORLD_SIZE": "2", "OMP_NUM_THREADS": "1"}, str(max(1, min(16, ncpu // 2)))),
                      ({"LOCAL_WORLD_SIZE": "2", "OMP_NUM_THREADS": "4"}, None),
                      ({"LOCAL_WORLD_SIZE": "2", "OMP_NUM_THREADS": "1", "PW_THREADS": "3"}, "3"),
                      ({"WORLD_SIZE": "1", "OMP_NUM_THREADS": "1"}, None)]:
        for k in ("LOCAL_WORLD_SIZE", "WORLD_SIZE", "OMP_NUM_THREADS", "PW_THREADS"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        bench.rank_thread_share()
        assert os.environ.get("PW_THREADS") == want, env
