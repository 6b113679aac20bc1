"""Throughput of P planners planning concurrently from P host threads (one HIP stream each) on one
GPU, against one planner (development tool). ctypes releases the GIL during armour_plan_batch.
usage: python tools/concurrent_planners.py [worlds_per_planner] [planners] [steps]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 164
NP = int(sys.argv[2]) if len(sys.argv) > 2 else 2
STEPS = int(sys.argv[3]) if len(sys.argv) > 3 else 6
T, O = 100, 20

planners = [A.Planner(T=T, max_obstacles=O, max_worlds=W) for _ in range(NP)]
worlds = [[A.make_world(p * W + s, O) for s in range(W)] for p in range(NP)]
for p in range(NP):
    planners[p].plan(worlds[p])   # warm-up


def worker(p, out):
    for _ in range(STEPS):
        res, _ = planners[p].plan(worlds[p])
    out[p] = sum(r["feasible"] for r in res)


out = [0] * NP
threads = [threading.Thread(target=worker, args=(p, out)) for p in range(NP)]
t0 = time.perf_counter()
for th in threads:
    th.start()
for th in threads:
    th.join()
dt = time.perf_counter() - t0
print(f"{NP} planners x {W} worlds, {STEPS} steps each: {NP * W * STEPS / dt:.0f} plans/s "
      f"({dt / STEPS * 1e3:.1f} ms per round of {NP} batches)", flush=True)
