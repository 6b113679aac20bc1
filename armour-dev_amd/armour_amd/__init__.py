"""armour_amd — Python binding of the MI355X-native ARMOUR planner (libarmour_hip.so).

The product is the C ABI in include/armour_hip.h; this module is a thin ctypes layer over it,
used by tests/, bench.py and __graft_entry__.py. It loads the in-tree library and raises if the
library or a GPU is missing — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .robots import KINOVA
from .worlds import csv_world, example_world, make_world, straight_line_waypoint

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ARMOUR_LIB") or os.path.join(_HERE, "libarmour_hip.so")  # ARMOUR_LIB: diagnostics builds
NF = 7
_LIB = None
_dp = ctypes.POINTER(ctypes.c_double)


ARMOUR_E_ARG, ARMOUR_E_HIP, ARMOUR_E_CAPACITY, ARMOUR_E_STATE, ARMOUR_E_INTERNAL = -1, -2, -3, -4, -5  # include/armour_hip.h


class ArmourError(RuntimeError):
    pass


class Config(ctypes.Structure):
    _fields_ = [("robot", ctypes.c_int), ("num_time_steps", ctypes.c_int), ("max_obstacles", ctypes.c_int),
                ("max_worlds", ctypes.c_int), ("device", ctypes.c_int), ("max_iter", ctypes.c_int)]


class World(ctypes.Structure):
    _fields_ = [("q0", ctypes.c_double * NF), ("qd0", ctypes.c_double * NF), ("qdd0", ctypes.c_double * NF),
                ("q_des", ctypes.c_double * NF), ("num_obstacles", ctypes.c_int), ("obstacles", _dp)]


_WORLD_DTYPE = np.dtype({"names": ["q0", "qd0", "qdd0", "q_des", "num_obstacles", "obstacles"],
                         "formats": [(np.float64, NF)] * 4 + [np.int32, np.uintp],
                         "offsets": [World.q0.offset, World.qd0.offset, World.qdd0.offset, World.q_des.offset,
                                     World.num_obstacles.offset, World.obstacles.offset],
                         "itemsize": ctypes.sizeof(World)})


class ArmtdWorld(ctypes.Structure):
    _fields_ = [("q0", ctypes.c_double * NF), ("qd0", ctypes.c_double * NF), ("q_des", ctypes.c_double * NF),
                ("jrs_tables", _dp), ("k_range", ctypes.c_double * NF), ("num_obstacles", ctypes.c_int),
                ("obstacles", _dp)]


class Result(ctypes.Structure):
    _fields_ = [("k_opt", ctypes.c_double * NF), ("feasible", ctypes.c_int), ("solver_status", ctypes.c_int),
                ("iterations", ctypes.c_int), ("evaluations", ctypes.c_int), ("cost", ctypes.c_double),
                ("kkt_error", ctypes.c_double), ("error", ctypes.c_int)]


class Timing(ctypes.Structure):
    _fields_ = [("reach_ms", ctypes.c_double), ("nlp_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("reach_kernel_ms", ctypes.c_double), ("reach_bytes", ctypes.c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class PlanOutput(ctypes.Structure):
    """armour_plan_output (include/armour_hip.h): the single-world entry's result and the caller's
    output arrays (null: skipped)"""
    _fields_ = [("result", Result), ("timing", Timing), ("constraints", _dp), ("joint_bounds", _dp),
                ("link_centers", _dp), ("link_generators", _dp), ("torque_radius", _dp)]


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ArmourError(f"HIP planner library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.armour_create.restype = ctypes.c_void_p
        L.armour_create.argtypes = [ctypes.POINTER(Config)]
        L.armour_create_robot.restype = ctypes.c_void_p
        L.armour_create_robot.argtypes = [ctypes.POINTER(Config), ctypes.c_void_p]
        L.armour_robot_builtin.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.armour_device_compute_units.argtypes = [ctypes.c_int]
        L.armour_copy_bandwidth.restype = ctypes.c_double
        L.armour_copy_bandwidth.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
        L.armour_destroy.argtypes = [ctypes.c_void_p]
        L.armour_last_error.restype = ctypes.c_char_p
        L.armour_num_constraints.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.armour_num_joints.argtypes = [ctypes.c_void_p]
        L.armour_create_armtd.restype = ctypes.c_void_p
        L.armour_create_armtd.argtypes = [ctypes.POINTER(Config)]
        L.armour_plan_armtd_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ArmtdWorld),
                                              ctypes.POINTER(Result), ctypes.POINTER(Timing)]
        L.armour_reach_armtd_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ArmtdWorld),
                                               ctypes.POINTER(Timing)]
        L.armour_plan_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(World), ctypes.POINTER(Result),
                                        ctypes.POINTER(Timing)]
        L.armour_reach_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(World), ctypes.POINTER(Timing)]
        L.armour_plan.argtypes = [ctypes.c_void_p, ctypes.POINTER(World), ctypes.POINTER(PlanOutput)]
        L.armour_eval_constraints.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp, _dp]
        L.armour_get_reach_program.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.armour_get_monomial_counts.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                 ctypes.POINTER(ctypes.c_int)]
        L.armour_get_reach_occupancy.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong),
                                                 ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
        L.armour_get_joint_bounds.argtypes = [ctypes.c_void_p, _dp]
        L.armour_get_plane_cache_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
        L.armour_get_reach_span.argtypes = [ctypes.c_void_p, _dp]
        L.armour_get_reach_dump.argtypes = [ctypes.c_void_p, _dp, ctypes.c_int]
        L.armour_get_reach_profile.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        for name in ("armour_get_constraints", "armour_get_link_centers", "armour_get_link_generators",
                     "armour_get_torque_radius"):
            getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_int, _dp]
        _LIB = L
    return _LIB


# every symbol include/armour_hip.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = ["armour_copy_bandwidth", "armour_create", "armour_create_robot", "armour_robot_builtin", "armour_device_compute_units", "armour_destroy", "armour_last_error", "armour_num_constraints",
               "armour_plan_batch", "armour_reach_batch", "armour_eval_constraints", "armour_get_constraints",
               "armour_get_link_centers", "armour_get_link_generators", "armour_get_torque_radius",
               "armour_num_joints", "armour_get_joint_bounds", "armour_get_reach_program", "armour_get_reach_profile",
               "armour_get_reach_dump", "armour_get_reach_occupancy", "armour_get_monomial_counts",
               "armour_create_armtd", "armour_plan_armtd_batch", "armour_reach_armtd_batch",
               "armour_get_plane_cache_stats", "armour_plan", "armour_get_reach_span"]


def default_batch(T: int, device: int = 0, waves: int = 2) -> int:
    """worlds per step that fill `waves` whole bundle waves of the device (lane_kernel.hip runs one
    64-job bundle per CU at a time): floor(waves * CUs * 64 / T)"""
    n = lib().armour_device_compute_units(device)
    _check(min(0, n))
    return max(1, (waves * n * 64) // T)


def copy_bandwidth(device: int = 0, nbytes: int = 2 << 30, reps: int = 10) -> float:
    """device-to-device copy bandwidth in GB/s (read + write bytes / time) of a 16 B-per-lane
    streaming copy kernel (armour_copy_bandwidth): the achievable HBM figure for roofline fractions"""
    v = lib().armour_copy_bandwidth(device, nbytes, reps)
    if v < 0:
        raise ArmourError(f"armour_copy_bandwidth: {lib().armour_last_error().decode()}")
    return v


def _check(rc):
    if rc != 0:
        raise ArmourError(f"armour error {rc}: {lib().armour_last_error().decode()}")


def _ptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


class Planner:
    """Batched MI355X planner. A world is (q0, qd0, qdd0, q_des, obstacles[O, 12])."""

    def __init__(self, T=100, max_obstacles=20, max_worlds=1, device=0, max_iter=0, robot=None, _armtd=False):
        """robot: None (built-in Kinova Gen3 tables) or a robot-table dict (armour_amd.robot_tables)"""
        cfg = Config(0, T, max_obstacles, max_worlds, device, max_iter)
        if _armtd:
            self.h = lib().armour_create_armtd(ctypes.byref(cfg))
        elif robot is None:
            self.h = lib().armour_create(ctypes.byref(cfg))
        else:
            from .robot_tables import to_struct
            self._robot = to_struct(robot)
            self.h = lib().armour_create_robot(ctypes.byref(cfg), ctypes.byref(self._robot))
        if not self.h:
            raise ArmourError(f"armour_create failed: {lib().armour_last_error().decode()}")
        self.T = T
        self.NJ = lib().armour_num_joints(self.h)
        self.max_worlds = max_worlds
        self._keep = []
        self.O = 0

    def close(self):
        if getattr(self, "h", None) and _LIB is not None:  # (module teardown may have cleared _LIB)
            _LIB.armour_destroy(self.h)
        self.h = None

    def __del__(self):
        self.close()

    def num_constraints(self, O):
        return lib().armour_num_constraints(self.h, O)

    def _worlds(self, worlds):
        # the armour_world array filled through a NumPy view of its fields (one vectorised store
        # per field instead of a ctypes assignment per element); obstacles in one contiguous block
        n = len(worlds)
        arr = (World * n)()
        view = np.frombuffer(arr, dtype=_WORLD_DTYPE)
        for k, f in enumerate(("q0", "qd0", "qdd0", "q_des")):
            view[f] = np.asarray([w[k] for w in worlds], dtype=np.float64).reshape(n, NF)
        obs = [np.asarray(w[4], dtype=np.float64).reshape(-1, 12) for w in worlds]
        counts = np.array([o.shape[0] for o in obs], dtype=np.int64)
        block = np.ascontiguousarray(np.concatenate(obs) if counts.sum() else np.zeros((0, 12)))
        self._keep = [block]
        view["num_obstacles"] = counts
        starts = np.concatenate([[0], np.cumsum(counts)[:-1]]) * 12 * 8
        view["obstacles"] = np.where(counts > 0, block.ctypes.data + starts, 0)
        self.O = int(counts[0]) if n else 0
        return arr

    def plan_one(self, world):
        """armour_plan (the single-world entry): (result dict, timing dict, outputs dict) with the
        payloads of the five .out files"""
        arr = self._worlds([world])
        m = self.num_constraints(np.asarray(world[4]).reshape(-1, 12).shape[0])
        outs = dict(constraints=np.zeros(m), joint_bounds=np.zeros(28), link_centers=np.zeros((self.T, self.NJ, 3)),
                    link_generators=np.zeros((self.T, self.NJ, 3, 6)), torque_radius=np.zeros((self.T, NF)))
        po = PlanOutput()
        for k, v in outs.items():
            setattr(po, k, v.ctypes.data_as(_dp))
        _check(lib().armour_plan(self.h, arr, ctypes.byref(po)))
        r = po.result
        res = dict(k_opt=np.array(r.k_opt[:]), feasible=bool(r.feasible), status=r.solver_status,
                   iterations=r.iterations, evaluations=r.evaluations, cost=r.cost, kkt=r.kkt_error, error=r.error)
        return res, po.timing.as_dict(), outs

    def plan(self, worlds):
        arr = self._worlds(worlds)
        res = (Result * len(worlds))()
        tm = Timing()
        _check(self._plan_call(self.h, len(worlds), arr, res, ctypes.byref(tm)))
        return self._results(res), self._span(tm.as_dict())

    def _plan_call(self, *a):
        return lib().armour_plan_batch(*a)

    @staticmethod
    def _results(res):
        out = []
        for r in res:
            out.append(dict(k_opt=np.array(r.k_opt[:]), feasible=bool(r.feasible), status=r.solver_status,
                            iterations=r.iterations, evaluations=r.evaluations, cost=r.cost, kkt=r.kkt_error,
                            error=r.error))
        return out

    def reach(self, worlds):
        arr = self._worlds(worlds)
        tm = Timing()
        _check(self._reach_call(self.h, len(worlds), arr, ctypes.byref(tm)))
        return self._span(tm.as_dict())

    def _span(self, tm):
        # the reach launch's device-clock execution span (armour_get_reach_span; -1 when unknown)
        v = ctypes.c_double(-1.0)
        rc = lib().armour_get_reach_span(self.h, ctypes.byref(v))
        tm["reach_span_ms"] = v.value if rc == 0 else -1.0
        return tm

    def _reach_call(self, *a):
        return lib().armour_reach_batch(*a)

    def eval_constraints(self, w, x, jac=True):
        m = self.num_constraints(self.O)
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
        g = np.zeros(m)
        J = np.zeros((m, NF)) if jac else None
        _check(lib().armour_eval_constraints(self.h, w, _ptr(x), _ptr(g), _ptr(J)))
        return (g, J) if jac else g

    def constraints(self, w):
        g = np.zeros(self.num_constraints(self.O))
        _check(lib().armour_get_constraints(self.h, w, _ptr(g)))
        return g

    def link_centers(self, w):
        c = np.zeros((self.T, self.NJ, 3))
        _check(lib().armour_get_link_centers(self.h, w, _ptr(c)))
        return c

    def link_generators(self, w):
        """[T, NJ, 3, 6] (the armour_joint_position_radius.out payload)"""
        g = np.zeros((self.T, self.NJ, 3, 6))
        _check(lib().armour_get_link_generators(self.h, w, _ptr(g)))
        return g

    def joint_bounds(self):
        """the 28 trailing values of armour_constraints.out: per joint [lb + qe, ub - qe], then
        per joint [-v + qde, v - qde]"""
        b = np.zeros(28)
        _check(lib().armour_get_joint_bounds(self.h, _ptr(b)))
        return b

    def reach_program(self):
        """op codes of the reach kernel's program (diagnostics)"""
        n = lib().armour_get_reach_program(self.h, None, 0)
        codes = (ctypes.c_int * n)()
        lib().armour_get_reach_program(self.h, codes, n)
        return np.array(codes[:])

    def reach_dump(self):
        """[nops, 8] op-by-op state of job 0; needs ARMOUR_DUMP_OPS at creation"""
        n = lib().armour_get_reach_dump(self.h, None, 0)
        if n < 0:
            _check(n)
        d = np.zeros((n, 8))
        _check(min(0, lib().armour_get_reach_dump(self.h, _ptr(d), n)))
        return d

    def reach_profile(self):
        """([nops, 2] accumulated (cycles, terms) per op, [16] phase cycles);
        needs ARMOUR_PROFILE_OPS at creation"""
        n = lib().armour_get_reach_profile(self.h, None, 0)
        if n < 0:
            _check(n)
        buf = (ctypes.c_ulonglong * (2 * n + 16))()
        _check(min(0, lib().armour_get_reach_profile(self.h, buf, n + 8)))
        a = np.array(buf[:], dtype=np.uint64)
        return a[:2 * n].reshape(n, 2), a[2 * n:]

    def monomial_counts(self, w):
        """(link [T, NJ], torque [T, 7]) k-only monomial counts of world w"""
        lk = np.zeros((self.T, self.NJ), dtype=np.int32)
        tq = np.zeros((self.T, NF), dtype=np.int32)
        _check(lib().armour_get_monomial_counts(self.h, w, lk.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                                tq.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return lk, tq

    OCCUPANCY = ("arena_hashes", "arena_rows", "operator_terms", "link_monomials", "torque_monomials",
                 "worlds_retried", "worlds_failed")

    def occupancy(self):
        """{name: (largest use in the last reach, capacity)} (armour_get_reach_occupancy)"""
        n = len(self.OCCUPANCY)
        used = (ctypes.c_longlong * n)()
        caps = (ctypes.c_longlong * n)()
        rc = lib().armour_get_reach_occupancy(self.h, used, caps, n)
        _check(min(0, rc))
        return {k: (int(used[i]), int(caps[i])) for i, k in enumerate(self.OCCUPANCY)}

    def reach_span_ms(self):
        """device-clock execution span of the last reach launch, ms (armour_get_reach_span)"""
        v = ctypes.c_double()
        _check(lib().armour_get_reach_span(self.h, ctypes.byref(v)))
        return v.value

    def plane_cache_stats(self):
        """certified plane cache of the current reach sets (armour_get_plane_cache_stats)"""
        keys = ("planes_kept", "pairs", "blocks_cached", "blocks", "max_per_pair", "pool_records", "box_misses")
        out = (ctypes.c_longlong * len(keys))()
        _check(min(0, lib().armour_get_plane_cache_stats(self.h, out, len(keys))))
        return {k: int(out[i]) for i, k in enumerate(keys)}

    def torque_radius(self, w):
        r = np.zeros((self.T, NF))
        _check(lib().armour_get_torque_radius(self.h, w, _ptr(r)))
        return r


class ArmtdPlanner(Planner):
    """The ARMTD comparison planner (armour_create_armtd). A world is the content of one armtd.in:
    (q0, qd0, q_des, jrs_tables[7, 6, T], k_range[7], obstacles[O, 12]) with the tables per joint
    c_cos, g_cos, r_cos, c_sin, g_sin, r_sin (ACMP/armtd_main.cu:37-102)."""

    def __init__(self, T=100, max_obstacles=20, max_worlds=1, device=0, max_iter=0):
        super().__init__(T=T, max_obstacles=max_obstacles, max_worlds=max_worlds, device=device, max_iter=max_iter,
                         _armtd=True)

    def _worlds(self, worlds):
        n = len(worlds)
        arr = (ArmtdWorld * n)()
        keep = []
        for k, (q0, qd0, q_des, tab, kr, obs) in enumerate(worlds):
            a = arr[k]
            a.q0[:] = [float(v) for v in q0]
            a.qd0[:] = [float(v) for v in qd0]
            a.q_des[:] = [float(v) for v in q_des]
            a.k_range[:] = [float(v) for v in kr]
            t = np.ascontiguousarray(np.asarray(tab, dtype=np.float64).reshape(NF, 6, self.T))
            o = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, 12))
            keep += [t, o]
            a.jrs_tables = _ptr(t)
            a.num_obstacles = o.shape[0]
            a.obstacles = _ptr(o) if o.shape[0] else None
        self._keep = keep
        self.O = arr[0].num_obstacles if n else 0
        return arr

    def _plan_call(self, *a):
        return lib().armour_plan_armtd_batch(*a)

    def _reach_call(self, *a):
        return lib().armour_reach_armtd_batch(*a)


__all__ = ["ArmtdPlanner", "Planner", "ArmourError", "ARMOUR_E_CAPACITY", "ARMOUR_E_INTERNAL", "copy_bandwidth", "default_batch", "make_world", "example_world", "csv_world", "straight_line_waypoint", "KINOVA", "LIB_PATH", "ABI_SYMBOLS"]
