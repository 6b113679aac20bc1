"""Workload probe: per world profile, one planner, default batch: reach / NLP ms, iteration and status
histograms, feasible fraction; single-world latency with each reach engine. JSON lines."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402


def main():
    T, O = 100, 20
    B = A.default_batch(T)
    P = A.Planner(T=T, max_obstacles=O, max_worlds=B)
    for prof in ("default", "survey"):
        worlds = [A.make_world(s, O, profile=prof) for s in range(B)]
        P.plan(worlds)
        res, tm = P.plan(worlds)
        it = np.array([r["iterations"] for r in res])
        st = np.array([r["status"] for r in res])
        print(json.dumps(dict(profile=prof, W=B, reach_ms=tm["reach_ms"], nlp_ms=tm["nlp_ms"],
                              feasible=float(np.mean([r["feasible"] for r in res])),
                              it_mean=float(it.mean()), it_p50=int(np.median(it)), it_p90=int(np.percentile(it, 90)),
                              it_max=int(it.max()), status_counts=np.bincount(st, minlength=4).tolist())), flush=True)
    P.close()
    # reach time of each engine by batch size (jobs = W x T), T = 100
    for W in (1, 4, 10, 20, 41, 82, 164):
        for eng in ("lane", "job"):
            os.environ["ARMOUR_ENGINE"] = eng
            P = A.Planner(T=100, max_obstacles=O, max_worlds=W)
            ws = [A.make_world(s, O) for s in range(W)]
            P.reach(ws)
            ms = sorted(P.reach(ws)["reach_ms"] for _ in range(3))[1]
            print(json.dumps(dict(sweep=eng, W=W, jobs=W * 100, reach_ms=ms)), flush=True)
            P.close()
    os.environ.pop("ARMOUR_ENGINE", None)
    for eng in ("lane", "job"):
        os.environ["ARMOUR_ENGINE"] = eng
        for T1 in (100, 128):
            P = A.Planner(T=T1, max_obstacles=O, max_worlds=1)
            w = [A.make_world(7, O)]
            P.plan(w)
            ms = []
            for _ in range(5):
                t0 = time.perf_counter()
                res, tm = P.plan(w)
                ms.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps(dict(engine=eng, T=T1, wall_ms=float(np.median(ms)), reach_ms=tm["reach_ms"],
                                  nlp_ms=tm["nlp_ms"], iterations=res[0]["iterations"])), flush=True)
            P.close()
        os.environ.pop("ARMOUR_ENGINE", None)


if __name__ == "__main__":
    main()
