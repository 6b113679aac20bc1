"""Barrier-strategy study: the oracle's solver with the build's monotone barrier
against an adaptive one (Ipopt's mu_strategy "adaptive", KPR/Parameters.h:57: LOQO mu oracle,
kkt-error globalisation; oracle/src/ipm.cpp mu_strategy 1) on the reference's 100 saved worlds
(first replans, tests/golden/saved_worlds_T100.npz) and the first 300 headline-workload worlds
(survey profile, T = 100, O = 20). Writes profiles/r03_mu_study.json. CPU only (oracle).

usage: python tools/mu_study.py"""
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("armour-dev_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))


def saved_worlds():
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "saved_worlds_T100.npz"), allow_pickle=False))
    return fx


def job(args):
    kind, i = args
    import armour_amd as A
    from oracle import OraclePlanner
    if kind == "saved":
        r = saved_worlds()["rows"][i]
        n = int(np.max(np.nonzero(~np.all(np.isnan(r), axis=1))[0])) + 1  # drop the padding rows
        w = A.csv_world(r[:n])
    else:
        w = A.make_world(i, 20, profile="survey")
    R = OraclePlanner(*w, T=100, threads=1)
    R.reach()
    out = {}
    for name, ms in (("monotone", 0), ("adaptive", 1)):
        r = R.plan(mu_strategy=ms)
        out[name] = dict(feasible=r["feasible"], status=r["status"], iterations=r["iterations"],
                         evaluations=r["evaluations"], cost=r["cost"])
    return kind, i, out


def summary(rows):
    s = {}
    for name in ("monotone", "adaptive"):
        s[name] = dict(feasible=sum(r[name]["feasible"] for r in rows),
                       converged=sum(r[name]["status"] == 0 for r in rows),
                       iteration_limit=sum(r[name]["status"] == 1 for r in rows),
                       mean_iterations=float(np.mean([r[name]["iterations"] for r in rows])),
                       mean_evaluations=float(np.mean([r[name]["evaluations"] for r in rows])))
    both = [r for r in rows if r["monotone"]["feasible"] and r["adaptive"]["feasible"]]
    d = np.array([r["adaptive"]["cost"] - r["monotone"]["cost"] for r in both])
    s["both_feasible"] = len(both)
    s["cost_adaptive_minus_monotone"] = dict(mean=float(d.mean()) if len(d) else None,
                                             min=float(d.min()) if len(d) else None,
                                             max=float(d.max()) if len(d) else None)
    s["decision_differs"] = sum(r["monotone"]["feasible"] != r["adaptive"]["feasible"] for r in rows)
    return s


def main():
    fx = saved_worlds()
    jobs = [("saved", i) for i in range(len(fx["rows"]))] + [("survey", i) for i in range(300)]
    with mp.get_context("fork").Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(job, jobs, chunksize=2)
    out = {"generator": "tools/mu_study.py", "sets": {}}
    for kind in ("saved", "survey"):
        rows = [o for k, i, o in res if k == kind]
        out["sets"][kind] = summary(rows)
        out["sets"][kind]["worlds"] = len(rows)
        out["sets"][kind]["differing_worlds"] = [dict(world=i, **o) for k, i, o in res
                                                 if k == kind and o["monotone"]["feasible"] != o["adaptive"]["feasible"]]
    path = os.path.join(ROOT, "profiles", "r03_mu_study.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "differing_worlds"} for k, v in out["sets"].items()},
                     indent=1))


if __name__ == "__main__":
    main()
