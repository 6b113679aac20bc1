"""Generate tests/golden/bench_survey_T100_O20.npz: the oracle's plan of every world the default
bench step plans (build container, repo root):

    python tests/golden/make_bench_worlds.py            # 981 worlds, ~3 min on 8 cores
    python tests/golden/make_bench_worlds.py --extend 3924   # seeds 981..3923 (_ext.npz), ~11 min

bench.py's default step at N = 1 on an MI355X (256 CUs, T = 100) is three concurrent planners x
327 worlds = seeds 0..980 of armour_amd.make_world(seed, 20, profile="survey") (SURVEY.md §8(d)'s
generator as written). Per world the fixture freezes the oracle's (CPU restatement's) result:
feasible, status, iterations, evaluations, k_opt, cost, the KKT error at the last iterate, and a
SHA-1 of the world's inputs (so a changed generator fails the tests instead of comparing other
worlds). tests/test_bench_worlds.py checks the fixture against the generator and a sample against
a fresh oracle; tests/test_gpu_bench_worlds.py plans all of them on the GPU in the bench's
3 x 327 concurrent batches. Parity with the reference itself stays unpinned.

Optional: --cap-study re-plans the worlds that end at the 100-iteration cap with Ipopt's default
iteration limit (3000, KPR/armour_main.cu:256-261 sets none) and writes
tests/golden/bench_cap_study.json.
"""
from __future__ import annotations

import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

OUT = os.path.dirname(os.path.abspath(__file__))
NAME = "bench_survey_T100_O20"
T, O, N_WORLDS, PROFILE = 100, 20, 981, "survey"


def world_digest(world) -> bytes:
    h = hashlib.sha1()
    for a in world:
        h.update(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes())
    return h.digest()


def plan_one(args):
    seed, max_iter = args
    import armour_amd as A
    from oracle import OraclePlanner

    w = A.make_world(seed, O, profile=PROFILE)
    R = OraclePlanner(*w, T=T, threads=1)
    R.reach()
    r = R.plan(max_iter=max_iter)
    return seed, world_digest(w), r


def main():
    cap_study = "--cap-study" in sys.argv
    if "--extend" in sys.argv:
        return extend(int(sys.argv[sys.argv.index("--extend") + 1]))
    t0 = time.time()
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        out = pool.map(plan_one, [(s, 0) for s in range(N_WORLDS)], chunksize=4)
    out.sort(key=lambda t: t[0])
    rec = dict(
        seed=np.array([s for s, _, _ in out], dtype=np.int64),
        digest=np.array([np.frombuffer(d, dtype=np.uint8) for _, d, _ in out]),
        feasible=np.array([r["feasible"] for _, _, r in out]),
        status=np.array([r["status"] for _, _, r in out], dtype=np.int32),
        iterations=np.array([r["iterations"] for _, _, r in out], dtype=np.int32),
        evaluations=np.array([r["evaluations"] for _, _, r in out], dtype=np.int32),
        k_opt=np.array([r["k_opt"] for _, _, r in out]),
        cost=np.array([r["cost"] for _, _, r in out]),
        kkt=np.array([r["kkt"] for _, _, r in out]),
        T=np.int64(T), O=np.int64(O),
    )
    np.savez_compressed(os.path.join(OUT, NAME + ".npz"), **rec)
    st = rec["status"]
    summary = dict(worlds=N_WORLDS, T=T, O=O, profile=PROFILE, feasible=int(rec["feasible"].sum()),
                   converged=int((st == 0).sum()), iteration_cap=int((st == 1).sum()),
                   line_search_failure=int((st == 2).sum()), local_infeasibility=int((st == 4).sum()),
                   mean_iterations=float(rec["iterations"].mean()),
                   seconds=round(time.time() - t0, 1))
    print(json.dumps(summary), flush=True)
    if cap_study:
        capped = [int(s) for s in rec["seed"][st == 1]]
        with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
            long = pool.map(plan_one, [(s, 3000) for s in capped], chunksize=1)
        rows = []
        for (s, _, r) in long:
            i = s
            rows.append(dict(seed=s, cap100=dict(feasible=bool(rec["feasible"][i]), cost=float(rec["cost"][i]),
                                                 kkt=float(rec["kkt"][i])),
                             cap3000=dict(feasible=r["feasible"], status=r["status"], iterations=r["iterations"],
                                          cost=r["cost"], kkt=r["kkt"],
                                          dk=float(np.abs(r["k_opt"] - rec["k_opt"][i]).max()))))
        json.dump(dict(generator="tests/golden/make_bench_worlds.py --cap-study", summary=summary, worlds=rows),
                  open(os.path.join(OUT, "bench_cap_study.json"), "w"), indent=1)
        print(json.dumps(rows, indent=1))


def extend(total):
    """seeds N_WORLDS .. total-1 into bench_survey_T100_O20_ext.npz: with the base fixture, the worlds
    of bench.py's default step from round 5 on (three planners x 1308 worlds = seeds 0..3923;
    tests/test_gpu_bench_worlds.py). The base fixture (seeds 0..980) stays what the phase-1 and
    fidelity studies cover."""
    t0 = time.time()
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        out = pool.map(plan_one, [(s, 0) for s in range(N_WORLDS, total)], chunksize=4)
    out.sort(key=lambda t: t[0])
    rec = dict(
        seed=np.array([s for s, _, _ in out], dtype=np.int64),
        digest=np.array([np.frombuffer(d, dtype=np.uint8) for _, d, _ in out]),
        feasible=np.array([r["feasible"] for _, _, r in out]),
        status=np.array([r["status"] for _, _, r in out], dtype=np.int32),
        iterations=np.array([r["iterations"] for _, _, r in out], dtype=np.int32),
        evaluations=np.array([r["evaluations"] for _, _, r in out], dtype=np.int32),
        k_opt=np.array([r["k_opt"] for _, _, r in out]),
        cost=np.array([r["cost"] for _, _, r in out]),
        kkt=np.array([r["kkt"] for _, _, r in out]),
        T=np.int64(T), O=np.int64(O),
    )
    np.savez_compressed(os.path.join(OUT, NAME + "_ext.npz"), **rec)
    st = rec["status"]
    print(json.dumps(dict(worlds=len(out), first_seed=N_WORLDS, feasible=int(rec["feasible"].sum()),
                          converged=int((st == 0).sum()), iteration_cap=int((st == 1).sum()),
                          local_infeasibility=int((st == 4).sum()), seconds=round(time.time() - t0, 1))), flush=True)


if __name__ == "__main__":
    main()
