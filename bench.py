#!/usr/bin/env python3
"""Benchmark: ARMOUR planning iterations/sec (Kinova 7-DOF, 100 time steps, 20 obstacles).

Metric (BASELINE.json): planning iterations/sec at 1/2/4/8 GPUs. One planning iteration = one
complete plan of KPR/armour_main.cu (JRS -> PZ FK/RNEA -> torque radius -> hyperplanes -> NLP to
termination -> feasibility re-check). A step = one batch of `--batch` synthetic random-obstacle
worlds planned on each GPU (default: two whole waves of 64-job reach bundles) (weak scaling: every rank plans its own worlds); after each step the
per-world records (k_opt, cost, feasible) are all-gathered over RCCL and rank 0 takes the argmin
over feasible worlds (the only collective on this path).

Usage: python bench.py [--gpus N --steps K --warmup W --batch B]
       (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0,
                    help="worlds per GPU per step (0: two whole bundle waves of the device, floor(2 * CUs * 64 / T): "
                         "327 on MI355X at T=100)")
    ap.add_argument("--planners", type=int, default=2,
                    help="planners per GPU planning their own --batch concurrently (one HIP stream each, "
                         "one host thread each); 2 overlaps one planner's solver with the other's reach")
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--O", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0: skip)")
    ap.add_argument("--robot", default="kinova", choices=["kinova", "fetch"],
                    help="kinova: built-in Gen3 tables (configs 1-4); fetch: tests/golden/robot_fetch.json, the "
                         "Fetch arm from its URDF (config 5, at fp64)")
    return ap.parse_args()


def cpu_baseline(worlds, T, seconds, robot=None):
    """Oracle (CPU restatement of the reference path, oracle/) on the host cores: whole plans of
    the same worlds until `seconds` of work, OpenMP threads = the box's CPU share (<= 16)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OraclePlanner  # test/baseline infrastructure only

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    done, t0 = 0, time.perf_counter()
    for w in worlds:
        P = OraclePlanner(*w, T=T, threads=threads, robot=robot)
        P.reach()
        P.plan()
        done += 1
        if time.perf_counter() - t0 > seconds and done >= 2:
            break
    dt = time.perf_counter() - t0
    return dict(value=done / dt, unit="plans/s", cores=threads, kind="port",
                sample=f"{done} full plans (oracle C++ restatement, T={T}, O={len(worlds[0][4])}) in {dt:.1f}s")


def lib_digest():
    import hashlib

    from armour_amd import LIB_PATH

    return hashlib.sha1(open(LIB_PATH, "rb").read()).hexdigest()[:16]


def traffic_record(T, O, batch):
    """HBM traffic per reach_kernel launch from the newest committed PMC summary of the same
    workload AND the same library build (profiles/r*_reach_traffic.json, made by tools/gpu_prof.sh
    + tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected); None if
    there is none."""
    import glob

    best = None
    digest = lib_digest()
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_reach_traffic.json"))):
        rec = json.load(open(fn))
        if rec.get("config") == dict(T=T, O=O, batch=batch) and rec.get("lib_sha1") == digest:
            best = (fn, rec)
    return best


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != a.gpus and a.gpus > 1:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world_size}", file=sys.stderr)
    dist = None
    if world_size > 1:
        import torch
        import torch.distributed as dist_mod

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist_mod.init_process_group("nccl", rank=rank, world_size=world_size)
        dist = dist_mod

    import armour_amd as A
    from armour_amd import dist as D

    if a.batch <= 0:
        a.batch = A.default_batch(a.T, local_rank)

    # weak scaling: rank r plans worlds r*batch .. r*batch+batch-1 (armour_amd.dist.shard of the whole job)
    robot, geo, robot_name = None, A.KINOVA, "Kinova Gen3 7-DOF"
    if a.robot == "fetch":
        from armour_amd import robot_tables as RT
        robot = RT.load_json(os.path.join(ROOT, "tests", "golden", "robot_fetch.json"))
        geo = RT.geometry(robot)
        robot_name = "Fetch arm (URDF, 7 actuated + fixed gripper)"
    # a.planners planners per GPU (one HIP stream each) plan their own batch concurrently from host
    # threads (ctypes releases the GIL in armour_plan_batch); the GPU overlaps one planner's solver
    # iterations with another's reach. The rank's worlds are split between them.
    P = a.planners
    worlds_all = [A.make_world(i, a.O, robot=geo) for i in D.shard(a.batch * P * world_size, rank, world_size)]
    subs = [worlds_all[p * a.batch:(p + 1) * a.batch] for p in range(P)]
    worlds = subs[0]
    planners = [A.Planner(T=a.T, max_obstacles=a.O, max_worlds=a.batch, device=local_rank, robot=robot)
                for _ in range(P)]
    planner = planners[0]

    def plan_all():
        # one step: every planner plans its batch; the collective below stays on this thread, so
        # every rank issues it in the same order
        if P == 1:
            res, tm = planner.plan(worlds)
            return res, [tm]
        out = [None] * P

        def work(p):
            out[p] = planners[p].plan(subs[p])

        ths = [threading.Thread(target=work, args=(p,)) for p in range(P)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if any(o is None for o in out):
            raise RuntimeError("a planner thread failed")
        return [r for o in out for r in o[0]], [o[1] for o in out]

    def gather(res):
        return D.gather(D.records(res), dist, device="cuda" if dist is not None else None)

    def barrier():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        # untimed: planners one after another, so first-launch costs do not pile up on one kernel
        res = [r for p in range(P) for r in planners[p].plan(subs[p])[0]]
        gather(res)
    barrier()
    t0 = time.perf_counter()
    tms = []
    for _ in range(a.steps):
        res, tm = plan_all()
        allrec, best = gather(res)
        tms.extend(tm)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank != 0:
        dist.destroy_process_group()
        return
    total_plans = a.steps * a.batch * P * world_size
    # roofline of the dominant kernel (reach_kernel): algorithmic bytes = monomial bytes read and
    # written by the PZ operators, timed with HIP events on the planner stream
    rk_ms = float(np.mean([t["reach_kernel_ms"] for t in tms]))
    rk_bytes = float(np.mean([t["reach_bytes"] for t in tms]))
    achieved = rk_bytes / (rk_ms * 1e-3) / 1e9
    n_feas = int(allrec[:, 8].sum())
    line = {
        "metric": "planning iterations/sec (7-DOF, 100 t-steps, 20 obs)",
        "value": total_plans / elapsed,
        "unit": "plans/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic random-obstacle worlds (armour_amd.worlds, seeds rank*batch+i)",
        "config": {"workload": f"{robot_name}, T={a.T}, O={a.O} box obstacles, "
                               + (f"{a.batch} worlds/GPU/step" if P == 1 else
                                  f"{P} concurrent planners x {a.batch} worlds/GPU/step"),
                   "num_time_steps": a.T, "obstacles": a.O, "worlds_per_gpu": a.batch * P,
                   "planners_per_gpu": P, "worlds_per_planner": a.batch,
                   "parallelism": f"world-sharded x{world_size}, RCCL all_gather of per-world records"},
        "breakdown_ms": {"reach": float(np.mean([t["reach_ms"] for t in tms])),
                         "nlp": float(np.mean([t["nlp_ms"] for t in tms])),
                         "reach_kernel": rk_ms},
        "feasible_worlds": n_feas,
        "total_worlds_last_step": int(allrec.shape[0]),
        "roofline": {"kernel": "reach_kernel", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes_per_launch": rk_bytes, "launch_ms": rk_ms},
        "cpu_baseline": None,
    }
    tr = traffic_record(a.T, a.O, a.batch) if a.robot == "kinova" else None
    if tr is not None:
        line["roofline"]["traffic"] = tr[1]["traffic_bytes_per_launch"]
        line["roofline"]["traffic_source"] = os.path.relpath(tr[0], ROOT)
    if a.cpu_seconds > 0 and world_size == 1:   # the CPU baseline is an N = 1 figure (rank 0 only)
        rs = None
        if robot is not None:
            from armour_amd import robot_tables as RT
            rs = RT.to_struct(robot)
        line["cpu_baseline"] = cpu_baseline(worlds, a.T, a.cpu_seconds, robot=rs)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
