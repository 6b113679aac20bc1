"""World sharding and the record all-gather (armour_amd.dist, used by bench.py) on gloo with
world_size 2 — the same code path bench.py runs over RCCL on the GPU node."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from armour_amd import dist as D


def test_shard_covers_and_balances():
    for n in (0, 1, 7, 256, 257):
        for ws in (1, 2, 3, 8):
            parts = [list(D.shard(n, r, ws)) for r in range(ws)]
            assert sum(parts, []) == list(range(n))
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1


def test_best_picks_lowest_feasible_cost():
    rec = np.zeros((4, D.RECORD))
    rec[:, 7] = [3.0, 1.0, 0.5, 2.0]
    rec[:, 8] = [1, 1, 0, 1]
    assert D.best(rec) == 1
    rec[:, 8] = 0
    assert D.best(rec) == -1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    mine = D.shard(n, rank, ws)
    # fake per-world plan results: world i has cost (i * 7919 % 13) and is feasible when i % 3 != 0
    res = [dict(k_opt=np.full(7, i / 100), cost=float(i * 7919 % 13), feasible=i % 3 != 0, status=0) for i in mine]
    allrec, best = D.gather(D.records(res), dist, total=n)
    q.put((rank, allrec, best))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [8, 7, 256])
def test_gather_world_size_2(n):
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, n, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda t: t[0])
    ref = D.records([dict(k_opt=np.full(7, i / 100), cost=float(i * 7919 % 13), feasible=i % 3 != 0, status=0)
                     for i in range(n)])
    for rank, allrec, best in out:
        np.testing.assert_array_equal(allrec, ref)
        assert best == D.best(ref)
