"""bench.py's multi-GPU launch (BASELINE metric "at 1/2/4/8"):
`python bench.py --gpus N` with no WORLD_SIZE starts N ranks itself through
torch.distributed.run, one process per GPU, LOCAL_RANK = device ordinal.
CPU only: the argv/env of the launcher, and a real 2-rank launch in the
rank-probe mode (each rank reports its layout and exits before any GPU call)."""
import json
import re
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_launch_argv_env():
    env = {"WORLD_SIZE": "7", "PATH": "/usr/bin"}
    cmd, e = bench.rank_launch(["--gpus", "2", "--steps", "3"], 2, 29511, env=env)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))
    assert "WORLD_SIZE" not in e and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/usr/bin"


def test_two_rank_launch_probe():
    env = dict(os.environ, NT_BENCH_RANK_PROBE="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    # the two ranks share the pipe: take every JSON object, whatever the line breaks
    lines = [json.loads(x) for x in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 for x in lines)
    assert sorted(x["device"] for x in lines) == [0, 1]  # LOCAL_RANK -> device ordinal
