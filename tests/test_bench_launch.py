"""bench.py's launch contract, on CPU: ``--gpus N`` is
honoured -- under a launcher WORLD_SIZE must equal N, without one N > 1
ranks are started by bench.py itself -- decided before any GPU call."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(2, {}) == ("spawn", 2)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == ("run", 2)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", 1)
    for gpus, ws in ((1, "2"), (8, "4"), (2, "1")):
        with pytest.raises(ValueError, match="WORLD_SIZE"):
            bench.launch_plan(gpus, {"WORLD_SIZE": ws})
    with pytest.raises(ValueError):
        bench.launch_plan(0, {})


def test_launcher_cmd_is_the_drivers_form():
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-5] == os.path.join(ROOT, "bench.py")
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_world_size_mismatch_exits_nonzero_before_gpu():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE=2" in p.stderr and p.stdout == ""


def test_network_flag_needs_middlebury():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--network"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "middlebury" in p.stderr


def test_leg_watchdog_prints_the_line_and_exits_zero():
    """A config-4 side leg that does not finish (a hung exchange) must not
    cost the corr-path line: rank 0 prints it with the leg marked, every
    rank exits 0."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.leg_watchdog({'metric': 'm', 'value': 1.5}, %d, 0.5); time.sleep(30); print('late')")
    for rank in (0, 1):
        p = subprocess.run([sys.executable, "-c", code % (ROOT, rank)], capture_output=True, text=True,
                           timeout=120)
        assert p.returncode == 0, p.stderr
        assert "late" not in p.stdout
        if rank == 0:
            import json
            line = json.loads(p.stdout.strip().splitlines()[-1])
            assert line["value"] == 1.5 and "not finished" in line["config4_network"]["error"]
        else:
            assert p.stdout.strip() == ""
