"""Quick GPU parity + timing probe (development tool; the judged tests live in tests/)."""
import sys, time, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd')); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import armour_amd as A
from oracle import OraclePlanner

T, O = 100, 20
worlds = [A.make_world(s, O) for s in range(2)]
t0 = time.time(); P = A.Planner(T=T, max_obstacles=O, max_worlds=64); print('create', time.time() - t0, flush=True)
t0 = time.time(); tm = P.reach(worlds); print('reach', tm, time.time() - t0, flush=True)
for w in range(2):
    Ok = OraclePlanner(*worlds[w], T=T, threads=16); Ok.reach()
    lg = P.link_generators(w); lg_o = Ok.link_gens().reshape(T, 7, 3, 6) if False else Ok.get(0).reshape(T, 7, 6, 3).transpose(0, 1, 3, 2)
    tr = P.torque_radius(w); tr_o = Ok.torque_radius()
    print(f'w{w} link_gens maxdiff {np.abs(lg - lg_o).max():.3e}  torque_radius maxdiff {np.abs(tr - tr_o).max():.3e}', flush=True)
    for x in [np.zeros(7), np.array([0.5, 0.6, 0.7, 0.0, -0.5, -0.6, -0.7])]:
        g, J = P.eval_constraints(w, x)
        go, Jo = Ok.eval(x)
        print(f'   x={x[:2]} g maxdiff {np.abs(g - go).max():.3e} J maxdiff {np.abs(J - Jo).max():.3e}  (max|g| {np.abs(go).max():.2f}) decisions equal {np.array_equal(g[7*T:7*T+7*T*O] > 1e-4, go[7*T:7*T+7*T*O] > 1e-4)}', flush=True)
t0 = time.time(); res, tm = P.plan(worlds); print('plan', tm, time.time() - t0, flush=True)
for w in range(2):
    Ok = OraclePlanner(*worlds[w], T=T, threads=16); Ok.reach(); ro = Ok.plan()
    r = res[w]
    print(f'w{w} gpu k {np.round(r["k_opt"], 5)} feas {r["feasible"]} st {r["status"]} it {r["iterations"]} ev {r["evaluations"]} cost {r["cost"]:.6f}', flush=True)
    print(f'    cpu k {np.round(ro["k_opt"], 5)} feas {ro["feasible"]} st {ro["status"]} it {ro["iterations"]} ev {ro["evaluations"]} cost {ro["cost"]:.6f}  |dk| {np.abs(r["k_opt"] - ro["k_opt"]).max():.2e}', flush=True)
for W in [8, 64]:
    ws = [A.make_world(100 + s, O) for s in range(W)]
    P.plan(ws)
    t0 = time.time(); res, tm = P.plan(ws); dt = time.time() - t0
    print(f'W={W}: {dt*1e3:.1f} ms wall, {W/dt:.1f} plans/s, timing {tm}, feasible {sum(r["feasible"] for r in res)}/{W}, iters {[r["iterations"] for r in res[:8]]}', flush=True)
# per-op profile of the reach program (one reach of 64 worlds)
if os.environ.get('ARMOUR_PROFILE_OPS') == '2':
    P2 = A.Planner(T=T, max_obstacles=O, max_worlds=64)
    ws = [A.make_world(100 + s, O) for s in range(64)]
    tm = P2.reach(ws)
    prof, phase = P2.reach_profile()
    ph = (phase.astype(np.float64) / (64 * T)).round(0)
    print('reach', tm)
    print('big-path phases cycles/job [-, order, pass1, scan+alloc, pass2, blocksum, stage, -]:', ph[:8])
    print('small-path phases cycles/job [load, sort, groups, keep+write, reduce+finish]:', ph[8:13], 'between ops', ph[13], 'headers', ph[14])
elif os.environ.get('ARMOUR_PROFILE_OPS'):
    names = ['JRS', 'MAKE1D', 'MAKEROT', 'MAKEBOX', 'CONST', 'ZERO', 'VIEW', 'TRANSPOSE', 'MUL', 'ADD', 'STACK3', 'ADD1D',
             'EMIT_LINK', 'EMIT_TORQUE', 'TORQUE_RADIUS', 'CROSS_C', 'CROSS_PP']
    P2 = A.Planner(T=T, max_obstacles=O, max_worlds=64)
    ws = [A.make_world(100 + s, O) for s in range(64)]
    P2.reach(ws)
    prof, phase = P2.reach_profile()
    prof = prof.astype(np.float64)
    codes = P2.reach_program()
    jobs = 64 * T
    tot = prof[:, 0].sum()
    print(f'profile: {len(codes)} ops, {tot / jobs:.3e} cycles/job (thread-0 view)')
    for c in range(len(names)):
        m = codes == c
        if m.any():
            print(f'  {names[c]:14s} n={m.sum():4d} cycles/job {prof[m, 0].sum() / jobs:10.0f} ({100 * prof[m, 0].sum() / tot:5.1f}%) terms/job {prof[m, 1].sum() / jobs:9.0f}')
    terms = prof[:, 1] / jobs
    for lo, hi in [(0, 64), (64, 256), (256, 1024), (1024, 4096), (4096, 1 << 30)]:
        m = (((codes >= 8) & (codes <= 11)) | (codes >= 15)) & (terms > lo) & (terms <= hi)
        print(f'  terms in ({lo},{hi}]: ops {m.sum():4d} cycles/job {prof[m, 0].sum() / jobs:10.0f} terms/job {prof[m, 1].sum() / jobs:9.0f}')
    order = np.argsort(-prof[:, 0])[:10]
    for k in order:
        print(f'  op {k:4d} {names[codes[k]]:8s} cycles/job {prof[k, 0] / jobs:9.0f} terms/job {prof[k, 1] / jobs:8.1f}')
    np.save(os.path.join(ROOT, 'gpurun_out', 'reach_profile.npy'), np.concatenate([codes[:, None].astype(np.float64), prof], 1))
