"""Phase-1 study of the headline workload's infeasible verdicts (VERDICT r03 "Next round" 1a).

For every world the solver declares infeasible (tests/golden/bench_survey_T100_O20.npz, feasible
false), minimise the largest constraint violation with scipy's SLSQP — min t s.t. c(x) + t >= 0,
x in the box [-1, 1]^7 (the reference's bounds, NLPclass.cu:87-165; constraints :272-396 as the
oracle evaluates them) — from x = 0, from the solver's last iterate and from 3 random starts. A world
whose best point passes finalize_solution's re-check (NLPclass.cu:449-538, the reference's verdict:
KPR/armour_main.cu:295-316 writes the plan iff that check passes) is a false -1 of the solver.

    python tools/phase1_study.py [--procs 7] [--out tests/golden/phase1_study.json] [--fixture NAME]

The oracle (test infrastructure) evaluates the NLP; nothing here touches the product.
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

FIX = None


def _init(name):
    global FIX
    FIX = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz")))


def study(i):
    from scipy.optimize import minimize
    import armour_amd as A
    from oracle import OraclePlanner

    fx = FIX
    world = A.make_world(int(fx["seed"][i]), int(fx["O"]), profile="survey")
    R = OraclePlanner(*world, T=int(fx["T"]), threads=1)
    R.reach()
    gl, gu = R.bounds()
    lo, hi = np.abs(gl) < 1e19, np.abs(gu) < 1e19
    memo = {}

    def ev(x):
        k = x.tobytes()
        if k not in memo:
            memo.clear()
            memo[k] = R.eval(x)
        return memo[k]

    def cons(x):
        g = ev(np.ascontiguousarray(x))[0]
        return np.concatenate([g[lo] - gl[lo], gu[hi] - g[hi]])

    def jac(x):
        J = ev(np.ascontiguousarray(x))[1]
        return np.concatenate([J[lo], -J[hi]])

    n = cons(np.zeros(7)).size
    # finalize_solution's own region (NLPclass.cu:449-538): torque rows within the bounds widened by
    # TORQUE_INPUT_CONSTRAINT_VIOLATION_THRESHOLD 1e-2, collision rows below 1e-4
    # (KPR/Parameters.h:38,41), the other rows exact
    T, O, NJ = int(fx["T"]), int(fx["O"]), R.NJ
    nt, nc = T * 7, T * NJ * O
    relax = np.zeros(R.m)
    relax[:nt] = 1e-2
    relax[nt:nt + nc] = 1e-4
    relax = np.concatenate([relax[lo], relax[hi]])
    rng = np.random.default_rng(1000 + i)
    starts = [("zero", np.zeros(7)), ("last_iterate", np.clip(fx["k_opt"][i], -1, 1))]
    starts += [(f"random{q}", rng.uniform(-1, 1, 7)) for q in range(3)]
    runs = []
    best = None
    t0 = time.time()
    for name, x0 in starts:
        tt = max(0.0, -cons(x0).min())
        r = minimize(lambda z: z[7], np.append(x0, tt), jac=lambda z: np.eye(8)[7],
                     bounds=[(-1, 1)] * 7 + [(0, None)],
                     constraints=[dict(type="ineq", fun=lambda z: cons(z[:7]) + z[7],
                                       jac=lambda z: np.hstack([jac(z[:7]), np.ones((n, 1))]))],
                     method="SLSQP", options=dict(maxiter=300, ftol=1e-12))
        x = np.clip(r.x[:7], -1, 1)
        viol = float(max(0.0, -cons(x).min()))
        feas = R.feasible(R.eval(x, jac=False))
        runs.append(dict(start=name, max_violation=viol, finalize_feasible=bool(feas), nit=int(r.nit)))
        if best is None or viol < best[0]:
            best = (viol, x, feas)
    # phase 1 on the re-check's region, from x = 0 and the best strict point
    rbest = None
    for name, x0 in [("zero", np.zeros(7)), ("strict_best", best[1])]:
        tt = max(0.0, -(cons(x0) + relax).min())
        r = minimize(lambda z: z[7], np.append(x0, tt), jac=lambda z: np.eye(8)[7],
                     bounds=[(-1, 1)] * 7 + [(0, None)],
                     constraints=[dict(type="ineq", fun=lambda z: cons(z[:7]) + relax + z[7],
                                       jac=lambda z: np.hstack([jac(z[:7]), np.ones((n, 1))]))],
                     method="SLSQP", options=dict(maxiter=300, ftol=1e-12))
        x = np.clip(r.x[:7], -1, 1)
        viol = float(max(0.0, -(cons(x) + relax).min()))
        feas = R.feasible(R.eval(x, jac=False))
        runs.append(dict(start="relaxed_" + name, max_violation=viol, finalize_feasible=bool(feas), nit=int(r.nit)))
        if rbest is None or viol < rbest:
            rbest = viol
    return dict(world=int(i), relaxed_least_violation=rbest, seed=int(fx["seed"][i]), status=int(fx["status"][i]),
                least_violation=best[0], false_infeasible=bool(any(r["finalize_feasible"] for r in runs)),
                x_best=[float(v) for v in best[1]], runs=runs, seconds=round(time.time() - t0, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=7)
    ap.add_argument("--fixture", default="bench_survey_T100_O20")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "phase1_study.json"))
    ap.add_argument("--limit", type=int, default=0)
    a = ap.parse_args()
    _init(a.fixture)
    worlds = [int(i) for i in np.nonzero(~FIX["feasible"])[0]]
    if a.limit:
        worlds = worlds[:a.limit]
    out = []
    t0 = time.time()
    with Pool(a.procs, initializer=_init, initargs=(a.fixture,)) as p:
        for k, r in enumerate(p.imap_unordered(study, worlds)):
            out.append(r)
            if r["false_infeasible"]:
                print(f"world {r['world']}: FEASIBLE point found (violation {r['least_violation']:.2e})", flush=True)
            if (k + 1) % 20 == 0:
                print(f"{k + 1}/{len(worlds)} worlds, {time.time() - t0:.0f} s", flush=True)
    out.sort(key=lambda r: r["world"])
    false = [r["world"] for r in out if r["false_infeasible"]]
    viol = np.array([r["least_violation"] for r in out])
    rec = dict(fixture=a.fixture, method="SLSQP phase 1: min t s.t. c(x) + t >= 0, |x| <= 1; "
               "starts x=0, the solver's last iterate, 3 uniform random; then the same on the re-check's region "
               "(torque bounds widened by 1e-2, collision rows <= 1e-4) from x=0 and the best strict point",
               infeasible_worlds=len(out), false_infeasible=false, n_false_infeasible=len(false),
               relaxed_least_violation_quantiles={q: float(np.quantile([r["relaxed_least_violation"] for r in out], q)) for q in (0, 0.1, 0.5)} if out else {},
               least_violation_quantiles={q: float(np.quantile(viol, q)) for q in (0, 0.1, 0.5, 0.9, 1)} if len(viol) else {},
               worlds=out)
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in rec.items() if k != "worlds"}))


if __name__ == "__main__":
    main()
