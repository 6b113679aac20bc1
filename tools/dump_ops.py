"""Diagnostics: op-by-op state of reach job 0 (world 0, t=0) on the GPU (ARMOUR_DUMP_OPS) and,
when the CPU emulation library is present, the first op where the two diverge."""
import os, sys, ctypes
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'armour-dev_amd'))
out = os.path.join(ROOT, 'gpurun_out')
os.makedirs(out, exist_ok=True)
import armour_amd as A
w = A.make_world(0, 20)
if sys.argv[1:] == ['gpu']:
    os.environ['ARMOUR_DUMP_OPS'] = '1'
    P = A.Planner(T=100, max_obstacles=20, max_worlds=1)
    P.reach([w])
    np.save(os.path.join(out, 'dump_gpu.npy'), P.reach_dump())
    np.save(os.path.join(out, 'codes.npy'), P.reach_program())
    print('saved')
else:
    L = ctypes.CDLL(os.path.join(ROOT, 'tests/emu/libreach_emu.so'))
    codes = np.load(os.path.join(out, 'codes.npy'))
    d = np.zeros((len(codes), 8))
    L.emu_set_dump(d.ctypes.data_as(ctypes.c_void_p))
    NJ = 7
    bufs = [np.zeros(NJ * 18), np.zeros(NJ * 3), np.zeros(NJ * 3), np.zeros(NJ, np.int32), np.zeros(NJ * 64, np.uint16),
            np.zeros(NJ * 64 * 3), np.zeros(7), np.zeros(7), np.zeros(7, np.int32), np.zeros(7 * 256, np.uint16), np.zeros(7 * 256), np.zeros(7)]
    q0, qd0, qdd0 = [np.ascontiguousarray(a) for a in w[:3]]
    used = ctypes.c_long(); bts = ctypes.c_double(); nops = ctypes.c_int(); nsl = ctypes.c_int()
    L.emu_reach(100, 0, *[a.ctypes.data_as(ctypes.c_void_p) for a in (q0, qd0, qdd0)], *[b.ctypes.data_as(ctypes.c_void_p) for b in bufs],
                ctypes.byref(used), ctypes.byref(bts), ctypes.byref(nops), ctypes.byref(nsl))
    g = np.load(os.path.join(out, 'dump_gpu.npy'))
    names = ['JRS', 'MAKE1D', 'MAKEROT', 'MAKEBOX', 'CONST', 'ZERO', 'VIEW', 'TRANSPOSE', 'MUL', 'ADD', 'STACK3', 'ADD1D', 'EMIT_LINK', 'EMIT_TORQUE', 'TORQUE_RADIUS', 'CROSS_C', 'CROSS_PP']
    bad = np.where(np.abs(g - d).max(1) > 1e-12 * (1 + np.abs(d).max(1)))[0]
    print('diverging ops:', len(bad))
    for k in bad[:12]:
        print(k, names[codes[k]], 'gpu', np.round(g[k], 6), '\n      cpu', np.round(d[k], 6))
