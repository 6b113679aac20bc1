"""Pricing study: Ipopt's limited-memory BFGS (hessian_approximation
limited-memory, KPR/armour_main.cu:259; history 6, Ipopt's default, restated in oracle/src/ipm.cpp
IpmOptions::lbfgs_hist) against the product's damped full BFGS matrix, on every world of the first
headline batch (seeds 0..980 of make_world(seed, 20, profile="survey"), T = 100), the set of
tools/mu_pair_study.py. Oracle only; nothing runs on the device.

Three solver configurations against the product's (mu_strategy 1 + damped BFGS, the frozen fixture
tests/golden/bench_survey_T100_O20.npz):
  lbfgs6             the product's barrier rule with L-BFGS(6)
  ipopt_pair         Ipopt's default adaptive pair (quality function + obj-constr-filter, mu_min
                     1e-11) with the damped BFGS (the round-5 study, re-run for the same table)
  reference_config   Ipopt's default adaptive pair with L-BFGS(6): the closest restatement here of
                     the reference's Ipopt options (KPR/armour_main.cu:256-261, KPR/Parameters.h:50-59)

Writes profiles/r06_lbfgs_study.json: verdict (feasibility) and status changes, k_opt deltas of the
worlds converged under both, cost deltas, iteration and evaluation counts.

usage: python tools/lbfgs_study.py [N_WORLDS] [CONFIG ...]   (~5 min per configuration on 8 cores)"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

CONFIGS = {  # name: (mu_strategy, L-BFGS history)
    "lbfgs6": (1, 6),
    "ipopt_pair": (2, 0),
    "reference_config": (2, 6),
}


def plan(args):
    seed, mu, hist = args
    import armour_amd as A
    from oracle import OraclePlanner

    R = OraclePlanner(*A.make_world(seed, 20, profile="survey"), T=100, threads=1)
    R.reach()
    r = R.plan(mu_strategy=mu, flags=hist << 16)
    return seed, r["feasible"], r["status"], r["iterations"], r["evaluations"], r["k_opt"], r["cost"]


NAMES = {0: "converged", 1: "iteration_limit", 2: "line_search_failure", 4: "local_infeasibility"}


def compare(res, fx, n):
    feas = np.array([r[1] for r in res], bool)
    st = np.array([r[2] for r in res])
    it = np.array([r[3] for r in res])
    ev = np.array([r[4] for r in res])
    k = np.array([r[5] for r in res])
    c = np.array([r[6] for r in res])
    f0, s0, i0, e0, k0, c0 = fx["feasible"][:n].astype(bool), fx["status"][:n], fx["iterations"][:n], \
        fx["evaluations"][:n], fx["k_opt"][:n], fx["cost"][:n]
    both = (s0 == 0) & (st == 0)
    dk = np.abs(k - k0).max(axis=1)
    d = (c - c0)[both]
    return {
        "verdict_changes": {"feasible_to_infeasible": [int(i) for i in np.where(f0 & ~feas)[0]],
                            "infeasible_to_feasible": [int(i) for i in np.where(~f0 & feas)[0]]},
        "feasible": int(feas.sum()),
        "status_counts": {NAMES[q]: int((st == q).sum()) for q in NAMES},
        "status_changes": int((s0 != st).sum()),
        "converged_both": int(both.sum()),
        "k_opt_delta_converged_both": {"max": float(dk[both].max()), "median": float(np.median(dk[both])),
                                       "p90": float(np.quantile(dk[both], 0.9)),
                                       "over_1e-4": int((dk[both] > 1e-4).sum()),
                                       "over_1e-2": int((dk[both] > 1e-2).sum())},
        "cost_delta_converged_both": {"mean": float(d.mean()), "lower": int((d < 0).sum()),
                                      "higher": int((d > 0).sum())},
        "iterations_mean": float(it.mean()),
        "evaluations_mean": float(ev.mean()),
        "_k": k, "_st": st, "_feas": feas,
    }


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 981
    names = sys.argv[2:] or list(CONFIGS)
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "bench_survey_T100_O20.npz")))
    out = {"worlds": n,
           "product": {"solver": "mu_strategy 1 (LOQO / kkt-error, floor tol/10, 2^(1/8) grid) + damped full BFGS",
                       "feasible": int(fx["feasible"][:n].sum()),
                       "status_counts": {NAMES[q]: int((fx["status"][:n] == q).sum()) for q in NAMES},
                       "iterations_mean": float(fx["iterations"][:n].mean()),
                       "evaluations_mean": float(fx["evaluations"][:n].mean())},
           "configs": {}}
    ks = {}
    t0 = time.time()
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        for nm in names:
            mu, hist = CONFIGS[nm]
            t1 = time.time()
            res = sorted(pool.map(plan, [(s, mu, hist) for s in range(n)], chunksize=4))
            cmp = compare(res, fx, n)
            ks[nm] = (cmp.pop("_k"), cmp.pop("_st"), cmp.pop("_feas"))
            cmp["mu_strategy"], cmp["lbfgs_history"] = mu, hist
            cmp["seconds"] = round(time.time() - t1, 1)
            out["configs"][nm] = cmp
            print(nm, json.dumps(cmp), flush=True)
    # the L-BFGS change alone, with the barrier rule fixed: ipopt_pair vs reference_config
    if "ipopt_pair" in ks and "reference_config" in ks:
        (ka, sa, fa), (kb, sb, fb) = ks["ipopt_pair"], ks["reference_config"]
        both = (sa == 0) & (sb == 0)
        dk = np.abs(ka - kb).max(axis=1)
        out["lbfgs_under_ipopt_pair"] = {"verdict_changes": int((fa != fb).sum()), "status_changes": int((sa != sb).sum()),
                                         "converged_both": int(both.sum()),
                                         "k_opt_delta_median": float(np.median(dk[both])),
                                         "k_opt_delta_max": float(dk[both].max())}
    out["seconds"] = round(time.time() - t0, 1)
    path = os.path.join(ROOT, "profiles", "r06_lbfgs_study.json")
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
