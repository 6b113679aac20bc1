"""Per-op and per-phase cycles of the bundle reach engine (ARMOUR_PROFILE_OPS=1). Development tool."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
os.environ['ARMOUR_PROFILE_OPS'] = '1'
os.environ['ARMOUR_ENGINE'] = 'lane'
import armour_amd as A
T, O, W = 100, 20, int(os.environ.get('LP_W', 256))
names = ['JRS', 'MAKE1D', 'MAKEROT', 'MAKEBOX', 'CONST', 'ZERO', 'VIEW', 'TRANSPOSE', 'MUL', 'ADD', 'STACK3', 'ADD1D',
         'EMIT_LINK', 'EMIT_TORQUE', 'TORQUE_RADIUS', 'CROSS_C', 'CROSS_PP']
P = A.Planner(T=T, max_obstacles=O, max_worlds=W)
ws = [A.make_world(100 + s, O, profile=os.environ.get('LP_PROFILE', 'survey')) for s in range(W)]
tm = P.reach(ws)
print('reach', tm)
import ctypes
n = A.lib().armour_get_reach_profile(P.h, None, 0)
buf = (ctypes.c_ulonglong * (2 * n + 16 + 8 * 17))()
A.lib().armour_get_reach_profile(P.h, buf, n + 8 + 4 * 17)
arr = np.array(buf[:], dtype=np.uint64)
prof, phase, pcode = arr[:2 * n].reshape(n, 2), arr[2 * n:2 * n + 16], arr[2 * n + 16:].reshape(17, 8)
codes = P.reach_program()
nb = (W * T + 63) // 64
cyc = prof[:, 0].astype(np.float64) / nb
terms = prof[:, 1].astype(np.float64) / nb
print(f'bundles {nb}; cycles per bundle {cyc.sum():.3e} ({cyc.sum() / 2.4e3:.0f} us at 2.4 GHz)')
tot = {}
for k in range(len(codes)):
    tot.setdefault(names[codes[k]], [0, 0.0, 0.0])
    tot[names[codes[k]]][0] += 1
    tot[names[codes[k]]][1] += cyc[k]
    tot[names[codes[k]]][2] += terms[k]
for nm, (c, cy, te) in sorted(tot.items(), key=lambda z: -z[1][1]):
    print(f'  {nm:14s} ops {c:4d} cycles {cy:11.0f} ({100 * cy / cyc.sum():5.1f} %)  terms/op {te / max(c, 1):8.1f}')
ph = pcode.astype(np.float64).sum(axis=0) / nb
print('simplify phases per bundle [header+stage, order, heads+scan, alloc, rounds, tail, combine+finish]:')
print('   ', np.round(ph[:7]).astype(np.int64), 'sum', int(ph[:7].sum()))
for c in range(17):
    if pcode[c].sum():
        cnt = tot[names[c]][0]
        print(f'   {names[c]:10s} per op:', np.round(pcode[c, :7].astype(np.float64) / nb / cnt).astype(np.int64))
pr = phase.astype(np.float64) / nb
print(f'round sub-phases per bundle: index {pr[0]:.0f}, terms+decide {pr[1]:.0f}, barrier {pr[2]:.0f}, stores {pr[3]:.0f}, loop {pr[7]:.0f}; rounds {pr[5]:.0f}, member steps {pr[6]:.0f}')
print(f'   per round: index {pr[0]/pr[5]:.0f} terms+decide {pr[1]/pr[5]:.0f} barrier {pr[2]/pr[5]:.0f} stores {pr[3]/pr[5]:.0f}; per member step {pr[1]/pr[6]:.0f}')
top = np.argsort(-cyc)[:15]
for k in top:
    print(f'  op {k:4d} {names[codes[k]]:10s} cycles {cyc[k]:9.0f} terms {terms[k]:8.1f}')
