"""The multi-GPU bench path on the one-GPU box: torch and RCCL initialised first, the planner
library loaded after them in the same process (it binds to the HIP runtime already loaded), a plan
and the record all-gather over RCCL (tools/dist_smoke.py under torch.distributed.run, one rank)."""
import os
import socket
import subprocess
import sys

import pytest

import armour_amd as A

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torch_rccl_then_planner_one_rank():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tools", "dist_smoke.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "dist smoke ok: world_size 1, 8 records" in r.stdout


def test_copy_bandwidth():
    """the achievable-HBM reference kernel reports a plausible MI355X figure (spec 8 TB/s)"""
    gbs = A.copy_bandwidth(0, 1 << 30, 5)
    print(f"copy bandwidth {gbs:.0f} GB/s")
    assert 1000 < gbs < 8000


def _bench_two_ranks(extra):
    """bench.py under torch.distributed.run with two ranks sharing the box's one GPU (collectives on
    gloo: RCCL refuses two ranks on one device). Everything else is the N > 1 path the driver runs
    on an 8-GPU node: world sharding, barriers, max-over-ranks timing, the record all-gather and
    the argmin on rank 0."""
    import json

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--cpu-seconds", "0", "--no-extras"] + extra
    env = dict(os.environ, ARMOUR_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    return line


def test_bench_two_ranks_strong_scaling():
    """config 4's shape at N = 2: one job of 64 worlds sharded 32 + 32, every record gathered"""
    line = _bench_two_ranks(["--total-worlds", "64", "--planners", "1"])
    assert line["scaling"] == "strong" and line["total_worlds_last_step"] == 64
    assert line["config"]["worlds_per_gpu"] == 32


def test_bench_two_ranks_weak_scaling():
    """the default (weak) mode at N = 2: each rank plans its own worlds, 2 x 16 per step"""
    line = _bench_two_ranks(["--batch", "16", "--planners", "1"])
    assert line["scaling"] == "weak" and line["total_worlds_last_step"] == 32
