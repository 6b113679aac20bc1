"""The multi-GPU bench path on one GPU: torch + RCCL initialised first (as bench.py --gpus N does),
then the planner library in the same process (it binds to the HIP runtime already loaded), a plan
and the record all-gather over RCCL. Run under torch.distributed.run (any nproc)."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))

rank, ws, lr = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
torch.cuda.set_device(lr)
dist.init_process_group("nccl", rank=rank, world_size=ws)
t = torch.ones(4, device="cuda") * rank
out = [torch.empty_like(t) for _ in range(ws)]
dist.all_gather(out, t)
import armour_amd as A  # noqa: E402
from armour_amd import dist as D  # noqa: E402

worlds = [A.make_world(100 + rank * 8 + i, 10, profile="survey") for i in range(8)]
P = A.Planner(T=40, max_obstacles=10, max_worlds=8, device=lr)
res, tm = P.plan(worlds)
allrec, best = D.gather(D.records(res), dist, device="cuda", total=8 * ws)
y = (torch.arange(10, device="cuda") * 2).sum().item()
if rank == 0:
    print(f"dist smoke ok: world_size {ws}, {allrec.shape[0]} records, best {best}, reach {tm['reach_ms']:.1f} ms, "
          f"torch after planner: {y}", flush=True)
dist.barrier()
dist.destroy_process_group()
