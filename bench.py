#!/usr/bin/env python3
"""Benchmark: ARMOUR planning iterations/sec (Kinova 7-DOF, 100 time steps, 20 obstacles).

Metric (BASELINE.json): planning iterations/sec at 1/2/4/8 GPUs. One planning iteration = one
complete plan of KPR/armour_main.cu (JRS -> PZ FK/RNEA -> torque radius -> hyperplanes -> NLP to
termination -> feasibility re-check). Worlds: SURVEY.md §8(d)'s synthetic generator as written
(armour_amd.worlds, profile "survey": full start-state ranges, obstacles rejected only when they
intersect the start configuration), so a share of the worlds is infeasible and the solver works
against active constraints; the line reports the feasible fraction.

Modes
  weak (default): every rank plans its own --batch worlds per planner per step (default: eight
      whole waves of 64-job reach bundles); `value` = all ranks' worlds / max-over-ranks step time.
  strong (--total-worlds N, config 4): one fixed job of N worlds sharded over the ranks
      (armour_amd.dist.shard), each rank's shard split over its planners.
After each step the per-world records are all-gathered over RCCL and rank 0 takes the argmin over
feasible worlds (the only collective on this path).

Rank 0 at N = 1 also reports: the roofline of the reach kernel (its timed-region launches'
device-clock spans; HIP events under load and the kernel alone beside them) and SURVEY §8(d)'s per-plan byte count B_plan = B_setup + E * B_eval; the measured copy peak;
single-plan latency (the drop-in's use: one world per call) at T = 100 and 128 and the wall time of
the armour_main process; the CPU baseline (the oracle on config 1, 1 thread and the box's share).

Usage: python bench.py [--gpus N --steps K --warmup W --batch B --planners P --total-worlds N]
       (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
C_PAIRS = 36           # generator pairs of a buffered obstacle (KPR/CollisionChecking.cu:26-39)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0,
                    help="worlds per planner per step (0: four two-wave batches, 4 * floor(2 * CUs * 64 / T), about eight "
                         "bundle waves of the device: 1308 on MI355X at T=100; one two-wave batch where T * O > 2000 "
                         "(device memory; T=200, O=40: 163); DESIGN.md section 6: 5 %% more plans/s than two waves, 327)")
    ap.add_argument("--planners", type=int, default=0,
                    help="planners per GPU planning their own batch concurrently (one HIP stream and one host thread "
                         "each): one planner's solver fills the GPU around the others'. 0 (default): 3 in weak mode "
                         "(DESIGN.md section 6: measured best, 2 about 2.5 %% behind, 4 behind); in strong mode each "
                         "rank times 1, 2 and 3 planners on its own share during warmup and keeps the fastest "
                         "(DESIGN.md section 7: the best count depends on the share size)")
    ap.add_argument("--total-worlds", type=int, default=0,
                    help="strong scaling (config 4): one job of this many worlds sharded over the ranks")
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--O", type=int, default=20)
    ap.add_argument("--profile", default="survey", choices=["survey", "default"],
                    help="world generator: survey = SURVEY §8(d) as written; default = half start-state ranges and "
                         "5 cm start clearance (the round-1 workload, every world feasible)")
    ap.add_argument("--robot", default="kinova", choices=["kinova", "fetch"],
                    help="kinova: built-in Gen3 tables (configs 1-4); fetch: tests/golden/robot_fetch.json, the "
                         "Fetch arm from its URDF (config 5, at fp64)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="per CPU-baseline leg (0: skip)")
    ap.add_argument("--no-extras", action="store_true", help="skip the N=1 extras (latency, copy peak, roofline)")
    ap.add_argument("--dump-records", default="",
                    help="rank 0 saves the last step's gathered per-world records (armour_amd.dist.RECORD layout, "
                         "world order) to this .npy file (tests/test_gpu_dist.py compares them with the oracle)")
    return ap.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, robot=None, geo=None):
    """The oracle (CPU restatement of the reference path, oracle/) planning BASELINE config 1
    (Kinova, T=100, O=10, one plan at a time) from the same generator: one leg on 1 thread, one on
    the box's CPU share (<= 16 threads; the reference runs 32 OpenMP threads, Parameters.h:35)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import armour_amd as A
    from oracle import OraclePlanner  # test/baseline infrastructure only

    share = max(1, min(16, len(os.sched_getaffinity(0))))
    legs = {}
    seed = 10_000
    for threads in (1, share):
        done, t0 = 0, time.perf_counter()
        while True:
            w = A.make_world(seed, 10, robot=geo, profile="survey")
            seed += 1
            P = OraclePlanner(*w, T=100, threads=threads, robot=robot)
            P.reach()
            P.plan()
            done += 1
            if time.perf_counter() - t0 > seconds and done >= 1:
                break
        dt = time.perf_counter() - t0
        legs[threads] = (done / dt, done, dt)
    v, done, dt = legs[share]
    v1, done1, dt1 = legs[1]
    return dict(value=v, unit="plans/s", cores=share, kind="port", cpu_model=cpu_model(),
                sample=f"config 1 (Kinova, T=100, O=10): {done} full plans of the oracle C++ restatement in {dt:.1f}s on "
                       f"{share} threads",
                one_thread=dict(value=v1, unit="plans/s", sample=f"{done1} plans in {dt1:.1f}s"))


def lib_digest():
    import hashlib

    from armour_amd import LIB_PATH

    return hashlib.sha1(open(LIB_PATH, "rb").read()).hexdigest()[:16]


def traffic_record(T, O, batch, profile):
    """HBM traffic per reach-kernel launch from the newest committed PMC summary of the same
    workload AND library build (profiles/r*_reach_traffic.json, tools/pmc_traffic.py: separate
    FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected); None if there is none."""
    import glob

    best = None
    digest = lib_digest()
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_reach_traffic.json"))):
        rec = json.load(open(fn))
        if (rec.get("config") == dict(T=T, O=O, batch=batch) and rec.get("lib_sha1") == digest
                and rec.get("profile", "default") == profile):
            best = (fn, rec)
    return best


def rocprof_record(kernel="lane_reach_kernel", solo=False):
    """The kernel's rocprofv3 --kernel-trace --stats line from the newest committed summary of the
    same library build (profiles/r*_kernel_stats*.txt written by tools/gpu.sh stats, whose header
    names the command and the library's SHA-1): (file, calls, average ns, min ns), or None.
    solo: a summary of `bench.py --planners 1` (every launch alone on the GPU, as the roofline's
    `achieved` is timed); else one of the default bench (three planners)."""
    import glob

    digest, best = lib_digest(), None
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_kernel_stats*.txt"))):
        lines = open(fn).read().splitlines()
        if not any(ln.startswith("# lib_sha1 ") and ln.split()[2] == digest for ln in lines):
            continue
        if any(ln.startswith("# stats ") and "--planners 1" in ln for ln in lines) != solo:
            continue
        for ln in lines:
            if kernel in ln and not ln.startswith("#"):
                f = ln[72:].split()
                best = (fn, int(f[0]), float(f[2]), float(f[3]))
                break
    return best


def io_lower_bound(P, W, nsample=16):
    """Design-independent lower bound of the reach phase's HBM bytes per launch: every job reads its
    7 JRS joint records (reach.h JrsJoint, 13 doubles) and writes only what the solver consumes — per
    link the centre, radius and 3 x 6 generators and its k-only monomials (u16 hash + 3 doubles), per
    joint the torque centre, radius and monomials (u16 + double) and the torque radius
    (KPR/armour_main.cu:114-211). Intermediates kept on chip cost nothing here."""
    T, NJ = P.T, P.NJ
    tot = 0.0
    n = min(nsample, W)
    for w in range(n):
        lk, tq = P.monomial_counts(w)
        tot += T * (7 * 13 * 8 + NJ * 24 * 8 + 7 * 3 * 8) + 26 * float(lk.sum()) + 10 * float(tq.sum())
    return tot / n * W


def latency(A, O, robot, geo):
    """the drop-in's use: one world per call (KSI/uarmtd_planner.m runs one armour_main per plan)"""
    out = {}
    for T in (100, 128):
        P = A.Planner(T=T, max_obstacles=O, max_worlds=1, robot=robot)
        ws = [[A.make_world(50_000 + s, O, robot=geo, profile="survey")] for s in range(8)]
        P.plan(ws[0])
        ms = []
        for w in ws:
            t0 = time.perf_counter()
            P.plan(w)
            ms.append((time.perf_counter() - t0) * 1e3)
        out[f"T{T}_ms_per_plan"] = float(np.median(ms))
        out[f"T{T}_ms_max"] = float(np.max(ms))
        P.close()
    exe = os.path.join(ROOT, "armour-dev_amd", "armour_amd", "armour_main")
    if robot is None and os.path.exists(exe):
        q0, qd0, qdd0, qdes, obs = A.make_world(50_000, O, geo, profile="survey")
        with tempfile.TemporaryDirectory() as d:
            with open(os.path.join(d, "armour.in"), "w") as f:
                for v in (q0, qd0, qdd0, qdes):
                    f.write(" ".join(f"{x:.10f}" for x in v) + "\n")
                f.write(f"{len(obs)}\n")
                for o in obs:
                    f.write(" ".join(f"{x:.10f}" for x in o) + "\n")
            walls = []
            for _ in range(3):
                t0 = time.perf_counter()
                r = subprocess.run([exe, d], capture_output=True, text=True, timeout=120)
                walls.append((time.perf_counter() - t0) * 1e3)
                if r.returncode != 0:
                    walls = None
                    break
            if walls:
                rep = open(os.path.join(d, "armour.out")).read().split()
                out["armour_main_wall_ms"] = float(np.median(walls))
                out["armour_main_reported_ms"] = float(rep[-1])
                out["armour_main_T"] = 128
            # served mode: one `armour_main --serve` keeps the planner warm; each replan is a plain
            # armour_main process that forwards the buffer directory (armour_main.cpp)
            srv = subprocess.Popen([exe, "--serve", d], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            try:
                for _ in range(600):
                    if os.path.exists(os.path.join(d, "armour.sock")) or srv.poll() is not None:
                        break
                    time.sleep(0.1)
                served = []
                for _ in range(6):
                    t0 = time.perf_counter()
                    r = subprocess.run([exe, d], capture_output=True, text=True, timeout=120)
                    served.append((time.perf_counter() - t0) * 1e3)
                    if r.returncode != 0:
                        served = None
                        break
                if served:
                    out["armour_main_served_wall_ms"] = float(np.median(served[1:]))
            finally:
                srv.terminate()
                srv.wait(timeout=30)
    return out


def per_plan_bytes(P, res, T, O, NJ, reach_bytes, nsample=8):
    """B_plan = B_setup + E * B_eval with E the constraint + Jacobian evaluations of
    the solver (recorded per world), M_links / M_tau the k-only monomials kept per world"""
    m = 7 * T + NJ * T * O + 28
    ml, mt = [], []
    for w in range(min(nsample, len(res))):
        lk, tq = P.monomial_counts(w)
        ml.append(int(lk.sum()))
        mt.append(int(tq.sum()))
    M_links, M_tau = float(np.mean(ml)), float(np.mean(mt))
    hyper = 40.0 * T * NJ * O * C_PAIRS
    B_eval = hyper + (24 + 8) * M_links * 2 + (8 + 8) * M_tau * 2 + 8.0 * m * (1 + 7)
    B_setup = hyper + 8.0 * T * NJ * 18 + reach_bytes
    E = float(np.mean([r["evaluations"] for r in res]))
    return dict(B_setup=B_setup, B_eval=B_eval, E=E, B_plan=B_setup + E * B_eval, M_links=M_links, M_tau=M_tau)


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != a.gpus and a.gpus > 1:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world_size}", file=sys.stderr)
    dist = None
    # collective backend: "nccl" (= RCCL over xGMI, one rank per GPU); ARMOUR_DIST_BACKEND=gloo runs
    # the same path with host-side collectives (tests/test_gpu_dist.py: two ranks sharing one GPU)
    backend = os.environ.get("ARMOUR_DIST_BACKEND", "nccl")
    coll_device = "cuda" if backend == "nccl" else None
    if world_size > 1:
        import torch
        import torch.distributed as dist_mod

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local_rank = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        dist_mod.init_process_group(backend, rank=rank, world_size=world_size)
        dist = dist_mod

    import armour_amd as A
    from armour_amd import dist as D

    robot, geo, robot_name = None, A.KINOVA, "Kinova Gen3 7-DOF"
    if a.robot == "fetch":
        from armour_amd import robot_tables as RT
        robot = RT.load_json(os.path.join(ROOT, "tests", "golden", "robot_fetch.json"))
        geo = RT.geometry(robot)
        robot_name = "Fetch arm (URDF, 7 actuated + fixed gripper)"

    strong = a.total_worlds > 0
    auto_planners = strong and a.planners <= 0
    if a.planners <= 0:
        a.planners = 3
    if strong:
        mine = list(D.shard(a.total_worlds, rank, world_size))
        worlds_mine = {i: A.make_world(i, a.O, robot=geo, profile=a.profile) for i in mine}
    else:
        if a.batch <= 0:
            # four two-wave batches (4 x 327 at T = 100: 2044 bundles, 8 waves) where three planners'
            # plane caches, arenas and scratch fit the device's memory with it; one where T * O is
            # larger (config 3, T = 200 and O = 40: ~4x the per-world memory, and three planners of
            # 4 x 163 worlds run out of device memory)
            a.batch = (4 if a.T * a.O <= 100 * 20 else 1) * A.default_batch(a.T, local_rank)
        mine = list(D.shard(a.batch * a.planners * world_size, rank, world_size))

    def setup(nplan):
        """this rank's worlds split over nplan planners: (sub-batches of world indices, worlds, planners)"""
        if strong:
            per = -(-len(mine) // nplan)
            si = [mine[p * per:(p + 1) * per] for p in range(nplan)]
            si = [x for x in si if x]
            sw = [[worlds_mine[i] for i in x] for x in si]
        else:
            si = [mine[p * a.batch:(p + 1) * a.batch] for p in range(nplan)]
            sw = [[A.make_world(i, a.O, robot=geo, profile=a.profile) for i in x] for x in si]
        pl = []
        try:
            for x in sw:
                pl.append(A.Planner(T=a.T, max_obstacles=a.O, max_worlds=len(x), device=local_rank, robot=robot))
        except BaseException:
            for q in pl:
                q.close()
            raise
        return si, sw, pl

    P = a.planners
    subs_idx, subs, planners = setup(P)
    P = len(planners)
    if strong:
        a.batch = max(len(x) for x in subs)
    n_rank = sum(len(x) for x in subs)
    total_job = a.total_worlds if strong else a.batch * P * world_size

    def fail(exc):
        print(f"bench: rank {rank}: {exc!r}", file=sys.stderr, flush=True)
        if dist is not None:
            os._exit(1)  # the other ranks' collectives cannot complete; end this rank at once
        raise exc

    def plan_all():
        # one step: every planner plans its batch from its own host thread (ctypes releases the GIL
        # in armour_plan_batch); the collective below stays on this thread
        P = len(planners)
        if P == 1:
            res, tm = planners[0].plan(subs[0])
            return res, [tm]
        out, errs = [None] * P, [None] * P

        def work(p):
            try:
                out[p] = planners[p].plan(subs[p])
            except BaseException as e:  # re-raised on the main thread
                errs[p] = e

        ths = [threading.Thread(target=work, args=(p,)) for p in range(P)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        for e in errs:
            if e is not None:
                fail(e)
        return [r for o in out for r in o[0]], [o[1] for o in out]

    def gather(res):
        return D.gather(D.records(res), dist, device=coll_device if dist is not None else None,
                        total=total_job if strong else None)

    def barrier():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    calib = None
    try:
        if auto_planners:
            # strong mode: this rank's share is planned with 1, 2 and 3 concurrent planners (one
            # untimed step, then the best of two timed steps each), and the fastest count is kept.
            # Untimed for the bench line (warmup); the counts per share are in the line's config.
            calib = {}
            for cand in (1, 2, 3):
                if cand > len(mine):
                    continue
                if cand != P:
                    for pl in planners:
                        pl.close()
                    subs_idx, subs, planners = setup(cand)
                    P = len(planners)
                for pl, sw in zip(planners, subs):
                    pl.plan(sw)
                best_ms = float("inf")
                for _ in range(2):
                    t1 = time.perf_counter()
                    plan_all()
                    best_ms = min(best_ms, (time.perf_counter() - t1) * 1e3)
                calib[str(cand)] = round(best_ms, 3)
            keep = int(min(calib, key=calib.get))
            if keep != P:
                for pl in planners:
                    pl.close()
                subs_idx, subs, planners = setup(keep)
                P = len(planners)
            a.batch = max(len(x) for x in subs)
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
    except Exception as e:  # noqa: BLE001
        fail(e)
    if dist is not None:
        import torch

        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_device or "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank != 0:
        dist.destroy_process_group()
        return
    if a.dump_records:
        np.save(a.dump_records, allrec)
    total_plans = a.steps * total_job
    value = total_plans / elapsed
    n_feas = int(allrec[:, 8].sum())
    iters = [r["iterations"] for r in res]
    line = {
        "metric": "planning iterations/sec (7-DOF, 100 t-steps, 20 obs)",
        "value": value,
        "unit": "plans/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic random-obstacle worlds (armour_amd.worlds profile '{a.profile}', "
                + ("seeds 0..total_worlds-1 sharded over ranks)" if strong else
                   "seeds rank*batch*planners + i: every rank its own worlds)"),
        "config": {"workload": f"{robot_name}, T={a.T}, O={a.O} box obstacles, "
                               + (f"one job of {a.total_worlds} worlds over {world_size} GPU(s)" if strong else
                                  f"{P} concurrent planner(s) x {a.batch} worlds/GPU/step"),
                   "num_time_steps": a.T, "obstacles": a.O, "worlds_per_gpu": n_rank,
                   "planners_per_gpu": P, "worlds_per_planner": a.batch, "world_profile": a.profile,
                   "planner_calibration_ms": calib,
                   "parallelism": f"world-sharded x{world_size}, RCCL all_gather of per-world records"},
        "breakdown_ms": {"reach": float(np.mean([t["reach_ms"] for t in tms])),
                         "nlp": float(np.mean([t["nlp_ms"] for t in tms])),
                         "reach_kernel": float(np.mean([t["reach_kernel_ms"] for t in tms]))},
        "feasible_worlds": n_feas,
        "total_worlds_last_step": int(allrec.shape[0]),
        "feasible_fraction": n_feas / max(1, int(allrec.shape[0])),
        "solver": {"mean_iterations": float(np.mean(iters)), "max_iterations": int(np.max(iters)),
                   "mean_evaluations": float(np.mean([r["evaluations"] for r in res])),
                   "iteration_limit": 100,
                   "status_counts": {k: int(sum(r["status"] == c for r in res))
                                     for k, c in (("converged", 0), ("iteration_limit", 1), ("line_search_failure", 2),
                                                  ("local_infeasibility", 4))}},
        "roofline": None,
        "cpu_baseline": None,
    }
    if world_size == 1 and not a.no_extras:
        # Roofline of the dominant kernel (the bundle reach kernel) over the timed region's own
        # launches: its algorithmic bytes per launch over the mean execution span of those launches
        # on the device clock (first workgroup start to last workgroup end, armour_get_reach_span:
        # the duration rocprofv3 --kernel-trace --stats reports for the kernel). HIP events around
        # the launch also count the time it waits for CUs the other planners' kernels hold; they
        # are reported beside it, as is the kernel alone on the GPU.
        solo, tm_solo = planners[0].plan(subs[0])
        rk_ms, rk_bytes = tm_solo["reach_kernel_ms"], tm_solo["reach_bytes"]
        spans = [t["reach_span_ms"] for t in tms if t.get("reach_span_ms", -1) > 0]
        rk_span = float(np.mean(spans)) if spans else float("nan")
        rk_load_ms = float(np.mean([t["reach_kernel_ms"] for t in tms]))
        achieved = rk_bytes / (rk_span * 1e-3) / 1e9
        line["roofline"] = {
            "kernel": "lane_reach_kernel", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_launch": rk_bytes,
            "launch_ms": rk_span, "launches": len(spans), "worlds_per_launch": len(subs[0]),
            "timing": f"device clock span (armour_get_reach_span), mean over the timed region's {len(spans)} launches "
                      f"({P} planners sharing the GPU): the kernel duration rocprofv3 reports",
            "hip_events_under_load": {"launch_ms": rk_load_ms, "frac": rk_bytes / (rk_load_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                      "timing": "HIP events around each launch in the timed region (includes the wait "
                                                "for CUs other planners' kernels hold)"},
            "solo": {"launch_ms": rk_ms, "span_ms": tm_solo.get("reach_span_ms"),
                     "achieved": rk_bytes / (rk_ms * 1e-3) / 1e9, "frac": rk_bytes / (rk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "timing": "HIP events, the planner alone on the GPU after the timed region"},
            "limiter": "memory latency: dependent load rounds per simplify step, not bandwidth (DESIGN.md §4)",
        }
        # SURVEY §8(d)'s per-plan byte model prices the reference's design (hyperplanes stored and
        # re-read every evaluation), which this build does not move: a reference-design figure, not
        # a roofline of this build
        pp = per_plan_bytes(planners[0], solo, a.T, a.O, planners[0].NJ, rk_bytes / len(subs[0]))
        line["reference_design_bytes"] = {**pp, "at_this_rate_GBps": pp["B_plan"] * value / 1e9,
                                          "note": "SURVEY §8(d) B_plan of the reference's design x this build's plans/s; "
                                                  "this build forms the hyperplanes in registers and moves ~3.5 MB per "
                                                  "evaluation, not B_eval (DESIGN.md §6)"}
        # the worlds of the last step that ended at the 100-iteration limit, planned again with
        # Ipopt's default limit of 3000 (KPR/armour_main.cu:256-261 sets none)
        capped = [i for i, r in enumerate(res) if r["status"] == 1]
        if capped:
            flat = [w for s in subs for w in s]
            L = A.Planner(T=a.T, max_obstacles=a.O, max_worlds=len(capped), device=local_rank, robot=robot,
                          max_iter=3000)
            long_res, _ = L.plan([flat[i] for i in capped])
            L.close()
            f100 = [int(i) for i in capped if res[i]["feasible"]]
            f3000 = [int(i) for r, i in zip(long_res, capped) if r["feasible"]]
            line["solver"]["iteration_limit_study"] = {
                "worlds": len(capped), "feasible_at_100": len(f100), "feasible_at_3000": len(f3000),
                # which capped worlds are feasible (step indices), not only how many: the verdicts
                # agree world by world when the two lists are equal
                "feasible_worlds_at_100": f100, "feasible_worlds_at_3000": f3000,
                "same_worlds_feasible": f100 == f3000,
                "iterations_at_3000": [int(r["iterations"]) for r in long_res],
                "status_at_3000": [int(r["status"]) for r in long_res],
                "cost_delta": [float(r["cost"] - res[i]["cost"]) for r, i in zip(long_res, capped)]}
        lb = io_lower_bound(planners[0], len(subs[0]))
        line["roofline"]["io_lower_bound"] = {
            "bytes_per_launch": lb, "frac": lb / (rk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": "design-independent: JRS scalars in, link and torque tables out (bench.py io_lower_bound); "
                    "the kernel's own arena traffic is the algorithmic figure above"}
        for solo_rec, key, note in (
                (True, "rocprof", "rocprofv3 --kernel-trace --stats of bench.py --planners 1 on the same library build: "
                                  "every launch alone on the GPU, as `solo` above"),
                (False, "rocprof_under_load", "rocprofv3 --kernel-trace --stats of this bench command on the same library "
                                              "build: the average spans the timed region's launches under three planners "
                                              "and the solo launch, as `launch_ms` above")):
            rp = rocprof_record(solo=solo_rec) if a.robot == "kinova" else None
            if rp is not None:
                fn, calls, avg_ns, min_ns = rp
                line["roofline"][key] = {
                    "source": os.path.relpath(fn, ROOT), "calls": calls, "avg_ms": avg_ns * 1e-6,
                    "min_ms": min_ns * 1e-6, "frac_avg": rk_bytes / (avg_ns * 1e-9) / 1e9 / HBM_PEAK_GBS,
                    "frac_min": rk_bytes / (min_ns * 1e-9) / 1e9 / HBM_PEAK_GBS, "note": note}
        tr = traffic_record(a.T, a.O, len(subs[0]), a.profile) if a.robot == "kinova" else None
        if tr is not None:
            line["roofline"]["traffic"] = tr[1]["traffic_bytes_per_launch"]
            line["roofline"]["traffic_source"] = os.path.relpath(tr[0], ROOT)
        try:
            line["copy_peak_GBps"] = A.copy_bandwidth(local_rank)  # 2 x 2 GiB, 16 B/lane copy kernel
        except Exception as e:  # noqa: BLE001
            line["copy_peak_GBps"] = None
            print(f"copy peak not measured: {e!r}", file=sys.stderr)
        for p in planners[1:]:
            p.close()
        line["latency"] = latency(A, a.O, robot, geo)
    if a.cpu_seconds > 0 and world_size == 1:   # the CPU baseline is an N = 1 figure (rank 0 only)
        rs = None
        if robot is not None:
            from armour_amd import robot_tables as RT
            rs = RT.to_struct(robot)
        line["cpu_baseline"] = cpu_baseline(a.cpu_seconds, robot=rs, geo=geo)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
