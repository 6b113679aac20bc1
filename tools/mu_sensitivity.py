"""Sensitivity of the barrier strategies to rounding-level differences.

The GPU solver and the oracle see constraint values that differ at rounding level (~1e-15
relative: block-order sums, device math library). This plans headline-workload worlds on the
oracle twice per strategy — clean, and with every g / J value scaled by 1 + 1e-15 u (u uniform,
oracle_plan_ex's noise hook) — and reports how far the two plans drift apart: status, iteration
count and the largest |k_opt difference| over plans feasible in both runs.

usage: python tools/mu_sensitivity.py [N worlds] [out.json]"""
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("armour-dev_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

# (mu_strategy, IpmOptions::mu_study): the product's adaptive rule is (1, 0); bit 0 drops its
# 2^(1/8) grid, bit 1 its tol / 10 floor (Ipopt's mu_min 1e-11)
VARIANTS = {"monotone": (0, 0), "adaptive_ipopt_floor": (1, 3), "adaptive_floor": (1, 1), "adaptive": (1, 0)}
# round 6: the candidate device rules — the product's rule with L-BFGS(6)
# (flags bits 16-23), Ipopt's quality-function pair with the product's floor and grid on a 16-point
# sigma grid (mu_strategy 3, flags bits 8-15), the same with L-BFGS(6), and Ipopt's pair as Ipopt
# sets it with L-BFGS(6) (the reference's configuration); MU_VARIANTS=r06 selects them
if os.environ.get("MU_VARIANTS") == "r06":
    VARIANTS = {"adaptive": (1, 0), "adaptive_lbfgs6": (1, 6 << 16), "qf_s3_g16": (3, 16 << 8),
                "qf_s3_g16_lbfgs6": (3, (16 << 8) | (6 << 16)), "reference_config": (2, 6 << 16)}
NOISE = 1e-15


def job(i):
    import armour_amd as A
    from oracle import OraclePlanner
    R = OraclePlanner(*A.make_world(i, 20, profile="survey"), T=100, threads=1)
    R.reach()
    out = {}
    for name, (ms, fl) in VARIANTS.items():
        a = R.plan(mu_strategy=ms, flags=fl)
        b = R.plan(mu_strategy=ms, flags=fl, noise=NOISE)
        out[name] = dict(feasible=[a["feasible"], b["feasible"]], status=[a["status"], b["status"]],
                         iterations=[a["iterations"], b["iterations"]],
                         dk=float(np.abs(a["k_opt"] - b["k_opt"]).max()))
    return i, out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r04_mu_sensitivity.json")
    with mp.get_context("fork").Pool(7) as pool:
        res = pool.map(job, range(n), chunksize=2)
    summ = {}
    for name in VARIANTS:
        rows = [o[name] for _, o in res]
        conv = [r for r in rows if r["status"][0] == 0 and r["status"][1] == 0]
        dk = np.array([r["dk"] for r in conv])
        summ[name] = dict(worlds=len(rows),
                          status_differs=sum(r["status"][0] != r["status"][1] for r in rows),
                          iterations_differ=sum(r["iterations"][0] != r["iterations"][1] for r in rows),
                          decision_differs=sum(r["feasible"][0] != r["feasible"][1] for r in rows),
                          converged_both=len(conv),
                          dk_converged_max=float(dk.max()) if len(dk) else None,
                          dk_converged_median=float(np.median(dk)) if len(dk) else None,
                          converged_dk_over_1e8=int((dk > 1e-8).sum()),
                          feasible=sum(r["feasible"][0] for r in rows),
                          mean_iterations=float(np.mean([r["iterations"][0] for r in rows])))
    rec = dict(generator="tools/mu_sensitivity.py", noise=NOISE, summary=summ,
               worlds={i: o for i, o in res})
    json.dump(rec, open(path, "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
