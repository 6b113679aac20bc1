"""Pricing study: Ipopt's default adaptive pair — mu_oracle quality-function with
adaptive_mu_globalization obj-constr-filter (oracle/src/ipm.cpp mu_strategy 2, restated from Ipopt's
published algorithm; the reference sets only IPOPT_MU_STRATEGY "adaptive", KPR/Parameters.h:57) —
against the product's LOQO / kkt-error rule (mu_strategy 1, the frozen fixture
tests/golden/bench_survey_T100_O20.npz) on every headline world (seeds 0..980 of
make_world(seed, 20, profile="survey"), T = 100). Oracle only; nothing runs on the device.

Writes profiles/r05_mu_pair_study.json: verdict (feasibility) changes, status changes, k_opt deltas of
worlds converged under both, iteration and evaluation counts.

usage: python tools/mu_pair_study.py [N_WORLDS]   (~5 min on 8 cores for 981)"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


STRATEGY = int(os.environ.get("MU_STRATEGY", "2"))
QF_GRID = int(os.environ.get("QF_GRID", "0"))  # > 0: sigma from a fixed log grid (the device-friendly form)


def plan(seed):
    import armour_amd as A
    from oracle import OraclePlanner

    R = OraclePlanner(*A.make_world(seed, 20, profile="survey"), T=100, threads=1)
    R.reach()
    r = R.plan(mu_strategy=STRATEGY, flags=QF_GRID << 8)
    return seed, r["feasible"], r["status"], r["iterations"], r["evaluations"], r["k_opt"], r["cost"]


def _cost_delta(c, c0, both):
    """ipopt_default_pair cost - product cost over the worlds converged under both"""
    d = (c - c0)[both]
    rel = d / np.maximum(np.abs(c0[both]), 1e-12)
    return {"mean": float(d.mean()), "min": float(d.min()), "max": float(d.max()),
            "relative_median": float(np.median(rel)), "relative_max_abs": float(np.abs(rel).max()),
            "lower_under_ipopt_pair": int((d < 0).sum()), "higher_under_ipopt_pair": int((d > 0).sum())}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 981
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "bench_survey_T100_O20.npz")))
    t0 = time.time()
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        res = sorted(pool.map(plan, range(n), chunksize=4))
    feas = np.array([r[1] for r in res], bool)
    st = np.array([r[2] for r in res])
    it = np.array([r[3] for r in res])
    ev = np.array([r[4] for r in res])
    k = np.array([r[5] for r in res])
    f0, s0, i0, e0, k0 = fx["feasible"][:n].astype(bool), fx["status"][:n], fx["iterations"][:n], \
        fx["evaluations"][:n], fx["k_opt"][:n]
    both = (s0 == 0) & (st == 0)
    dk = np.abs(k - k0).max(axis=1)
    names = {0: "converged", 1: "iteration_limit", 2: "line_search_failure", 4: "local_infeasibility"}
    out = {
        "worlds": n,
        "strategies": {"product": "adaptive: mu_oracle loqo + adaptive_mu_globalization kkt-error, mu on a 2^(1/8) "
                                  "grid, floor tol/10 (mu_strategy 1; the fixture)",
                       "ipopt_default_pair": "adaptive: mu_oracle quality-function + adaptive_mu_globalization "
                                             "obj-constr-filter, mu_min 1e-11 (mu_strategy 2)"},
        "verdict_changes": {"feasible_to_infeasible": [int(i) for i in np.where(f0 & ~feas)[0]],
                            "infeasible_to_feasible": [int(i) for i in np.where(~f0 & feas)[0]]},
        "feasible": {"product": int(f0.sum()), "ipopt_default_pair": int(feas.sum())},
        "status_counts": {"product": {names[c]: int((s0 == c).sum()) for c in names},
                          "ipopt_default_pair": {names[c]: int((st == c).sum()) for c in names}},
        "status_changes": int((s0 != st).sum()),
        "converged_both": int(both.sum()),
        "k_opt_delta_converged_both": {"max": float(dk[both].max()) if both.any() else None,
                                       "median": float(np.median(dk[both])) if both.any() else None,
                                       "p99": float(np.quantile(dk[both], 0.99)) if both.any() else None,
                                       "over_1e-4": int((dk[both] > 1e-4).sum()),
                                       "over_1e-2": int((dk[both] > 1e-2).sum())},
        "iterations_mean": {"product": float(i0.mean()), "ipopt_default_pair": float(it.mean())},
        "evaluations_mean": {"product": float(e0.mean()), "ipopt_default_pair": float(ev.mean())},
        "cost_delta_converged_both": _cost_delta(np.array([r[6] for r in res]), fx["cost"][:n], both),
        "seconds": round(time.time() - t0, 1),
    }
    out["mu_strategy"] = STRATEGY
    out["qf_grid"] = QF_GRID
    tag = "" if STRATEGY == 2 else f"_s{STRATEGY}"
    tag += f"_g{QF_GRID}" if QF_GRID else ""
    path = os.path.join(ROOT, "profiles", f"r05_mu_pair_study{tag}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
