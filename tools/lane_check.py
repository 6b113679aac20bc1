"""Bundle engine (ARMOUR_ENGINE=lane, lane_kernel.hip) vs the per-job engine (ARMOUR_ENGINE=job):
reach outputs, constraints/Jacobians at fixed x, op-by-op dumps of job 0, and reach timing.
Development tool (the judged tests live in tests/)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
import armour_amd as A

T, O = int(os.environ.get('LC_T', 100)), 20
W = int(os.environ.get('LC_W', 4))
worlds = [A.make_world(s, O) for s in range(W)]


def planner(engine, dump=False, mw=W):
    os.environ['ARMOUR_ENGINE'] = engine
    if dump:
        os.environ['ARMOUR_DUMP_OPS'] = '1'
    else:
        os.environ.pop('ARMOUR_DUMP_OPS', None)
    return A.Planner(T=T, max_obstacles=O, max_worlds=mw)


Pj = planner('job', dump=True)
Pl = planner('lane', dump=True)
tj = Pj.reach(worlds)
tl = Pl.reach(worlds)
print('job ', tj, flush=True)
print('lane', tl, flush=True)
dj, dl = Pj.reach_dump(), Pl.reach_dump()
codes = Pj.reach_program()
bad = np.where(np.abs(dj - dl).max(axis=1) > 1e-12)[0]
print('dump: ops differing', len(bad), 'first', bad[:10], flush=True)
for k in bad[:6]:
    print('  op', k, 'code', codes[k], '\n    job ', dj[k], '\n    lane', dl[k], flush=True)
worst = 0.0
for w in range(W):
    a, b = Pj.link_generators(w), Pl.link_generators(w)
    tr1, tr2 = Pj.torque_radius(w), Pl.torque_radius(w)
    d1, d2 = np.abs(a - b).max(), np.abs(tr1 - tr2).max()
    line = f'w{w} link_gens {d1:.3e} torque_radius {d2:.3e}'
    for x in [np.zeros(7), np.linspace(-0.7, 0.7, 7)]:
        g1, J1 = Pj.eval_constraints(w, x)
        g2, J2 = Pl.eval_constraints(w, x)
        line += f' | g {np.abs(g1 - g2).max():.3e} J {np.abs(J1 - J2).max():.3e} bitwise {np.array_equal(g1, g2) and np.array_equal(J1, J2)}'
        worst = max(worst, np.abs(g1 - g2).max(), np.abs(J1 - J2).max())
    worst = max(worst, d1, d2)
    print(line, flush=True)
print('WORST', worst, flush=True)
if os.environ.get('LC_TIME'):
    del Pj, Pl
    WB = 256
    ws = [A.make_world(100 + s, O) for s in range(WB)]
    for eng in ['lane', 'job']:
        P = planner(eng, mw=WB)
        P.reach(ws)
        t0 = time.time()
        tm = P.reach(ws)
        print(f'{eng}: reach W={WB} {tm["reach_kernel_ms"]:.2f} ms kernel, {tm["reach_ms"]:.2f} ms reach, bytes {tm.get("reach_bytes", 0):.3e}, wall {1e3*(time.time()-t0):.1f} ms', flush=True)
        del P
