"""Multi-GPU host logic: worlds shard across ranks with no data-path collective;
the only exchange is one all-gather of a fixed per-world record after the plans, followed by an
argmin over feasible worlds (the multi-start pick of the best plan).

One process per GPU under torch.distributed ("nccl" = RCCL over xGMI on the box; "gloo" in the
CPU tests). Records are [k_opt(7), cost, feasible, status] float64 (80 B per world).
"""
from __future__ import annotations

import numpy as np

RECORD = 10  # k_opt(7), cost, feasible, status


def shard(num_worlds: int, rank: int, world_size: int) -> range:
    """Contiguous block of world indices owned by `rank` (blocks differ by at most one)."""
    base, extra = divmod(num_worlds, world_size)
    lo = rank * base + min(rank, extra)
    return range(lo, lo + base + (1 if rank < extra else 0))


def records(results) -> np.ndarray:
    """Per-world records of Planner.plan() results."""
    out = np.zeros((len(results), RECORD))
    for i, r in enumerate(results):
        out[i, :7] = r["k_opt"]
        out[i, 7] = r["cost"]
        out[i, 8] = 1.0 if r["feasible"] else 0.0
        out[i, 9] = r["status"]
    return out


def best(allrec: np.ndarray) -> int:
    """Index of the lowest-cost feasible world (-1 if none); ties go to the lowest index."""
    feas = allrec[:, 8] > 0.5
    if not feas.any():
        return -1
    return int(np.argmin(np.where(feas, allrec[:, 7], np.inf)))


def gather(rec: np.ndarray, dist=None, device=None, total=None):
    """All-gather the record blocks of every rank; returns (all records in world order, best index).
    `dist` is torch.distributed (initialised) or None for a single process. With `total` (the job's
    world count, sharded by shard()) the blocks may differ by one row: each is padded to the largest
    for the collective and trimmed after."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return rec, best(rec)
    import torch

    ws = dist.get_world_size()
    sizes = [len(shard(total, r, ws)) for r in range(ws)] if total is not None else [len(rec)] * ws
    rows = max(sizes)
    padded = np.zeros((rows, RECORD))
    padded[:len(rec)] = rec
    t = torch.from_numpy(padded)
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    allrec = np.concatenate([o.cpu().numpy()[:n] for o, n in zip(out, sizes)])
    return allrec, best(allrec)
