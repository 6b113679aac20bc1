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
