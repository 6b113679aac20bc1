"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/liboracle.so, the CPU restatement of the reference hot path
(oracle/src/*). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline — never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_dp = ctypes.POINTER(ctypes.c_double)


def _ptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        L.oracle_create.restype = ctypes.c_void_p
        L.oracle_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int] + [_dp] * 5 + [ctypes.c_int]
        L.oracle_create_robot.restype = ctypes.c_void_p
        L.oracle_create_robot.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + [_dp] * 5 + [ctypes.c_int]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_create_armtd.restype = ctypes.c_void_p
        L.oracle_create_armtd.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + [_dp] * 6 + [ctypes.c_int]
        L.oracle_reach.restype = ctypes.c_double
        L.oracle_reach.argtypes = [ctypes.c_void_p]
        L.oracle_num_constraints.argtypes = [ctypes.c_void_p]
        L.oracle_set_obstacles.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp]
        L.oracle_bounds.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.oracle_eval.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp]
        L.oracle_cost.restype = ctypes.c_double
        L.oracle_cost.argtypes = [ctypes.c_void_p, _dp, _dp]
        L.oracle_feasible.argtypes = [ctypes.c_void_p, _dp]
        L.oracle_get.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp]
        L.oracle_pz.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                ctypes.POINTER(ctypes.c_ulonglong), _dp, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_plan.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, ctypes.c_int]
        L.oracle_plan_mu.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int]
        L.oracle_plan_ex.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double]
        _LIB = L
    return _LIB


class OraclePlanner:
    """One planning problem on the CPU oracle (KPR/armour_main.cu semantics)."""

    def __init__(self, q0, qd0, qdd0, q_des, obstacles, T=100, threads=1, robot_id=0, num_joints=7, robot=None):
        """robot: None (Kinova tables) or a ctypes structure in the armour_robot layout
        (include/armour_hip.h; armour_amd.robot_tables.to_struct builds one)"""
        self.T = T
        self.NJ = int(robot.num_joints) if robot is not None else num_joints
        obstacles = np.ascontiguousarray(np.asarray(obstacles, dtype=np.float64).reshape(-1, 12))
        self.O = obstacles.shape[0]
        arrs = [np.ascontiguousarray(np.asarray(a, dtype=np.float64)) for a in (q0, qd0, qdd0, q_des)]
        obs = obstacles if self.O > 0 else np.zeros((1, 12))
        if robot is None:
            self.h = lib().oracle_create(robot_id, T, self.O, *[_ptr(a) for a in arrs], _ptr(obs), threads)
        else:
            self._robot = robot
            self.h = lib().oracle_create_robot(ctypes.byref(robot), T, self.O, *[_ptr(a) for a in arrs], _ptr(obs),
                                               threads)
        if not self.h:
            raise ValueError("oracle_create failed")
        self.m = lib().oracle_num_constraints(self.h)
        self.reach_ms = None

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_free(self.h)
            self.h = None

    def reach(self):
        self.reach_ms = lib().oracle_reach(self.h)
        if self.reach_ms < 0:
            raise RuntimeError("oracle reach failed")
        return self.reach_ms

    def set_obstacles(self, obstacles):
        """replace the obstacle set after reach() (the reach sets do not depend on it; only the
        buffered-obstacle hyperplanes are recomputed) — fixture tooling"""
        obstacles = np.ascontiguousarray(np.asarray(obstacles, dtype=np.float64).reshape(-1, 12))
        self.O = obstacles.shape[0]
        self._obs = obstacles if self.O > 0 else np.zeros((1, 12))
        if lib().oracle_set_obstacles(self.h, self.O, _ptr(self._obs)) != 0:
            raise ValueError("oracle_set_obstacles failed")
        self.m = lib().oracle_num_constraints(self.h)

    def bounds(self):
        gl = np.zeros(self.m)
        gu = np.zeros(self.m)
        lib().oracle_bounds(self.h, _ptr(gl), _ptr(gu))
        return gl, gu

    def eval(self, x, jac=True, centers=False):
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
        g = np.zeros(self.m)
        J = np.zeros((self.m, 7)) if jac else None
        lc = np.zeros((self.T, self.NJ, 3)) if centers else None
        lib().oracle_eval(self.h, _ptr(x), _ptr(g), _ptr(J), _ptr(lc))
        out = [g]
        if jac:
            out.append(J)
        if centers:
            out.append(lc)
        return out[0] if len(out) == 1 else tuple(out)

    def cost(self, x):
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
        grad = np.zeros(7)
        f = lib().oracle_cost(self.h, _ptr(x), _ptr(grad))
        return f, grad

    def feasible(self, g):
        return bool(lib().oracle_feasible(self.h, _ptr(np.ascontiguousarray(g))))

    def get(self, what):
        sizes = {0: self.T * self.NJ * 18, 1: self.T * 7, 2: self.T * self.NJ * self.O * 36 * 3,
                 3: self.T * self.NJ * self.O * 36, 4: self.T * self.NJ * self.O * 36}
        out = np.zeros(max(1, sizes[what]))
        lib().oracle_get(self.h, what, _ptr(out))
        return out[:sizes[what]]

    def link_gens(self):
        """[T, NJ, 3, 6] residual generators (KPR/armour_main.cu:114,125)"""
        return self.get(0).reshape(self.T, self.NJ, 6, 3).transpose(0, 1, 3, 2)

    def torque_radius(self):
        """[T, 7] (KPR/armour_main.cu:173-211)"""
        return self.get(1).reshape(self.T, 7)

    def pz(self, kind, idx, cap=4096):
        c = np.zeros(9)
        ind = np.zeros(9)
        hs = np.zeros(cap, dtype=np.uint64)
        co = np.zeros((cap, 9))
        r = ctypes.c_int()
        cl = ctypes.c_int()
        n = lib().oracle_pz(self.h, kind, idx, _ptr(c), _ptr(ind),
                            hs.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), _ptr(co), cap,
                            ctypes.byref(r), ctypes.byref(cl))
        k = r.value * cl.value
        return dict(rows=r.value, cols=cl.value, center=c[:k], indep=ind[:k], hashes=hs[:n],
                    coeffs=co[:n, :k])

    def plan(self, max_iter=0, mu_strategy=1, flags=0, noise=0.0):
        """mu_strategy 1: adaptive barrier (the default, KPR/Parameters.h:57's strategy); 0: monotone
        (an option: DESIGN.md §5). flags / noise: oracle_plan_ex (capi.cpp), studies only"""
        k = np.zeros(7)
        g = np.zeros(self.m)
        stats = np.zeros(8)
        feas = lib().oracle_plan_ex(self.h, _ptr(k), _ptr(g), _ptr(stats), max_iter, mu_strategy, flags, noise)
        if feas < 0:
            raise RuntimeError("oracle plan failed")
        return dict(k_opt=k, feasible=bool(feas), g=g, reach_ms=stats[0], nlp_ms=stats[1],
                    iterations=int(stats[2]), evaluations=int(stats[3]), status=int(stats[4]),
                    cost=stats[5], kkt=stats[6], restart_iter=int(stats[7]))


class OracleArmtd(OraclePlanner):
    """The ARMTD comparison planner (oracle/src/armtd.h) on one problem: the content of armtd.in
    (ACMP/armtd_main.cu:37-102). tables: [7][6][T] = c_cos, g_cos, r_cos, c_sin, g_sin, r_sin."""

    def __init__(self, q0, qd0, q_des, tables, k_range, obstacles, T=100, threads=1):
        self.T = T
        self.NJ = 7
        obstacles = np.ascontiguousarray(np.asarray(obstacles, dtype=np.float64).reshape(-1, 12))
        self.O = obstacles.shape[0]
        arrs = [np.ascontiguousarray(np.asarray(a, dtype=np.float64)) for a in (q0, qd0, q_des)]
        tab = np.ascontiguousarray(np.asarray(tables, dtype=np.float64).reshape(7, 6, T))
        kr = np.ascontiguousarray(np.asarray(k_range, dtype=np.float64))
        obs = obstacles if self.O > 0 else np.zeros((1, 12))
        self._keep = (arrs, tab, kr, obs)
        self.h = lib().oracle_create_armtd(None, T, self.O, *[_ptr(a) for a in arrs], _ptr(tab), _ptr(kr), _ptr(obs),
                                           threads)
        if not self.h:
            raise ValueError("oracle_create_armtd failed")
        self.m = lib().oracle_num_constraints(self.h)
        self.reach_ms = None
