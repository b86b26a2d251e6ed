"""bench.py's multi-GPU launch (BASELINE metric "at 1/2/4/8"):
`python bench.py --gpus N` with no WORLD_SIZE starts N ranks itself through
torch.distributed.run, one process per GPU, LOCAL_RANK = device ordinal.
CPU only: the argv/env of the launcher, and a real 2-rank launch in the
rank-probe mode (each rank reports its layout and exits before any GPU call)."""
import json
import os
import re
import subprocess
import sys

import pytest

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


@pytest.mark.gpu
def test_two_rank_bench_on_one_gpu():
    """The driver's N>1 path end to end on the GPU box (both ranks pinned to
    device 0 by NT_BENCH_DEVICE): one JSON line with n_gpus 2, both ranks'
    verdicts checked, no mismatches."""
    env = dict(os.environ, NT_BENCH_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--sigs", "8192", "--certs", "2000", "--committee", "10", "--sha-msgs", "256",
                        "--sha-len", "20000", "--no-cpu", "--no-latency", "--no-ingest"],
                       env=env, capture_output=True, text=True, timeout=300)
    # every rank's own error lines first (the launcher's tail shows only the first rank to fail)
    errs = [x for x in r.stderr.splitlines() if "Error" in x or "error" in x][:40]
    assert r.returncode == 0, "\n".join(errs) + "\n" + r.stderr[-3000:]
    lines = [json.loads(x) for x in re.findall(r"^\{.*\}$", r.stdout, re.M)]
    assert len(lines) == 1
    d = lines[0]
    # both config-2 runs checked on both ranks: the pipelined headline and the one-stream figure
    assert d["n_gpus"] == 2 and d["parity"] == {"mismatches_vs_expected": 0, "checked": 2 * 2 * 8192}
    assert d["streams"] == 2 and d["one_stream"]["value"] > 0
    assert d["certificates"]["keyset"]["mismatches_vs_expected"] == 0
    assert d["sha512"]["spot_check_ok"]
    # the whole metric near the front of the line, and every
    # rank's share attributable (a slow rank would show in min / max)
    keys = list(d)
    assert keys.index("sha512_gbs") < 6 and keys.index("certs_per_s") < 6
    assert d["sha512_gbs"] == d["sha512"]["value"] > 0 and d["certs_per_s"] == d["certificates"]["value"] > 0
    pr = d["per_rank"]
    for cfg, size in (("cfg2", "signatures"), ("cfg3", "certificates"), ("cfg4", "messages")):
        rows = pr[cfg]["per_rank"]
        assert sorted(r["rank"] for r in rows) == [0, 1], cfg
        assert all(r["kernel_ms"] > 0 and r["rate"] > 0 for r in rows), cfg
        assert pr[cfg]["rate_min"] <= pr[cfg]["rate_mean"] <= pr[cfg]["rate_max"], cfg
        assert pr[cfg]["slowest_rank"] in (0, 1)
    assert sum(r["certificates"] for r in pr["cfg3"]["per_rank"]) == 2000
    assert sum(r["messages"] for r in pr["cfg4"]["per_rank"]) == 256
    assert all(r["signatures"] == 8192 for r in pr["cfg2"]["per_rank"])
