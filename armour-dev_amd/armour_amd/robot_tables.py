"""Robot tables from a URDF and its meshes.

The reference compiles each robot in as a hand-written header (KPR/KinovaWithoutGripperInfo.h,
ACMP/FetchInfo.h). Here a robot is data: the plain-C `armour_robot` of include/armour_hip.h, filled
either from the built-in Kinova tables (`builtin()`) or from a URDF (`from_urdf()`):

  * joint i of the serial chain from the root link: axis (URDF `<axis>`, +-1/2/3 = x/y/z, 0 for a
    fixed joint), frame offset `trans[i]` / `rots[i]` = the joint `<origin>` xyz / rpy;
  * link i = the child of joint i: mass, centre of mass (`<inertial><origin>` xyz) and inertia
    (row-major [ixx ixy ixz; ixy iyy iyz; ixz iyz izz]);
  * link zonotope = the axis-aligned bounding box of the link's first visual mesh, centre and half
    extents, exactly the rule of polynomial_zonotope_matlab/create_pz_bounding_boxes.m (raw mesh
    points; a 10 cm cube when the link has no mesh or an empty one);
  * joint limits of the actuated joints: `<limit>` lower / upper (continuous joints: +-1000, the
    reference's convention), velocity, effort;
  * what a URDF does not hold (uncertainties, friction / damping / armature, the robust
    controller's ultimate-bound constants, torque warning limits) comes from `extras`.

Checked against the reference's own headers (tests/test_robot_tables.py): from
urdfs/kinova_arm/kinova_without_gripper.urdf this reproduces every URDF-derived table of
KinovaWithoutGripperInfo.h, the link zonotopes included; from urdfs/fetch_arm/fetch_arm_7DOF.urdf (7
actuated joints and the fixed gripper: 8 joints, config 5's "Fetch 8-DOF arm") the axes, offsets,
masses, centres of mass and inertias of the first 8 joints of FetchInfo.h.
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
import xml.etree.ElementTree as ET

import numpy as np

MAXJ = 9
NF = 7


class ArmourRobot(ctypes.Structure):
    """ctypes mirror of armour_robot (include/armour_hip.h)"""
    _fields_ = [
        ("num_joints", ctypes.c_int),
        ("axes", ctypes.c_int * MAXJ),
        ("wrap", ctypes.c_int * NF),
        ("trans", ctypes.c_double * ((MAXJ + 1) * 3)),
        ("rots", ctypes.c_double * (MAXJ * 3)),
        ("mass", ctypes.c_double * MAXJ),
        ("com", ctypes.c_double * (MAXJ * 3)),
        ("inertia", ctypes.c_double * (MAXJ * 9)),
        ("mass_uncertainty", ctypes.c_double),
        ("inertia_uncertainty", ctypes.c_double),
        ("friction", ctypes.c_double * MAXJ),
        ("damping", ctypes.c_double * MAXJ),
        ("armature", ctypes.c_double * MAXJ),
        ("state_lb", ctypes.c_double * NF),
        ("state_ub", ctypes.c_double * NF),
        ("speed_limits", ctypes.c_double * NF),
        ("torque_limits", ctypes.c_double * NF),
        ("gravity", ctypes.c_double),
        ("link_center", ctypes.c_double * (MAXJ * 3)),
        ("link_generators", ctypes.c_double * (MAXJ * 3)),
        ("alpha", ctypes.c_double),
        ("V_m", ctypes.c_double),
        ("M_max", ctypes.c_double),
        ("M_min", ctypes.c_double),
        ("K", ctypes.c_double),
    ]


_ARRAY_LEN = {name: t._length_ for name, t in ArmourRobot._fields_ if hasattr(t, "_length_")}


def to_struct(tables: dict) -> ArmourRobot:
    s = ArmourRobot()
    for name, t in ArmourRobot._fields_:
        if name not in tables:
            continue
        v = tables[name]
        if name in _ARRAY_LEN:
            a = np.zeros(_ARRAY_LEN[name])
            flat = np.asarray(v, dtype=np.float64).ravel()
            a[:flat.size] = flat
            arr = getattr(s, name)
            for i in range(_ARRAY_LEN[name]):
                arr[i] = int(a[i]) if t._type_ is ctypes.c_int else float(a[i])
        else:
            setattr(s, name, int(v) if t is ctypes.c_int else float(v))
    return s


def from_struct(s: ArmourRobot) -> dict:
    out = {}
    for name, t in ArmourRobot._fields_:
        v = getattr(s, name)
        out[name] = list(v) if hasattr(t, "_length_") else v
    return _shaped(out)


def _shaped(d: dict) -> dict:
    """numpy arrays shaped per joint (trans [NJ+1, 3], inertia [NJ, 3, 3], ...), trimmed to NJ"""
    nj = int(d["num_joints"])
    r = dict(d)
    r["axes"] = np.asarray(d["axes"], dtype=np.int64)[:nj]
    r["wrap"] = np.asarray(d["wrap"], dtype=np.int64)[:NF]
    r["trans"] = np.asarray(d["trans"], dtype=np.float64).reshape(-1, 3)[:nj + 1]
    for k in ("rots", "com", "link_center", "link_generators"):
        r[k] = np.asarray(d[k], dtype=np.float64).reshape(-1, 3)[:nj]
    r["inertia"] = np.asarray(d["inertia"], dtype=np.float64).reshape(-1, 3, 3)[:nj]
    for k in ("mass", "friction", "damping", "armature"):
        r[k] = np.asarray(d[k], dtype=np.float64)[:nj]
    for k in ("state_lb", "state_ub", "speed_limits", "torque_limits"):
        r[k] = np.asarray(d[k], dtype=np.float64)[:NF]
    return r


def builtin(robot_id: int = 0) -> dict:
    """the product's built-in tables (robot 0: KPR/KinovaWithoutGripperInfo.h) through the C ABI"""
    from . import lib, _check
    s = ArmourRobot()
    _check(lib().armour_robot_builtin(robot_id, ctypes.byref(s)))
    return from_struct(s)


# ---- URDF + meshes -------------------------------------------------------------------------------
def stl_points(path: str):
    """vertices of a binary or ASCII STL (None for an empty / header-only file)"""
    with open(path, "rb") as f:
        b = f.read()
    if len(b) < 84:
        return None
    if b[:5] == b"solid" and b"facet" in b[:4096]:
        pts = [list(map(float, ln.split()[1:4])) for ln in b.decode(errors="ignore").splitlines()
               if ln.strip().startswith("vertex")]
        return np.array(pts, dtype=np.float64) if pts else None
    n = struct.unpack("<I", b[80:84])[0]
    if n == 0 or len(b) < 84 + 50 * n:
        return None
    rec = np.frombuffer(b[84:84 + 50 * n], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    return rec["v"].reshape(-1, 3).astype(np.float64)


def mesh_box(path: str | None):
    """(centre, half extents) of create_pz_bounding_boxes.m: raw mesh bounds, else a 10 cm cube"""
    pts = stl_points(path) if path and os.path.exists(path) else None
    if pts is None:
        lo, hi = np.full(3, -0.05), np.full(3, 0.05)
    else:
        lo, hi = pts.min(axis=0), pts.max(axis=0)
    return (lo + hi) / 2, (hi - lo) / 2


def _vec(el, attr, default="0 0 0"):
    return np.array([float(v) for v in (el.get(attr) if el is not None and el.get(attr) else default).split()])


def _axis_code(joint) -> int:
    if joint.get("type") == "fixed":
        return 0
    ax = _vec(joint.find("axis"), "xyz", "1 0 0")
    k = int(np.argmax(np.abs(ax)))
    if np.count_nonzero(np.abs(ax) > 1e-12) != 1:
        raise ValueError(f"joint {joint.get('name')}: only axis-aligned joint axes are supported")
    return int(np.sign(ax[k])) * (k + 1)


def from_urdf(urdf_path: str, num_joints: int, extras: dict | None = None, mesh_root: str | None = None) -> dict:
    """tables of the first `num_joints` joints of the URDF's serial chain from its root link"""
    root = ET.parse(urdf_path).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = [j for j in root.findall("joint")]
    children = {j.find("child").get("link") for j in joints}
    base = [n for n in links if n not in children]
    if len(base) != 1:
        raise ValueError(f"expected one root link, found {base}")
    mesh_root = mesh_root or os.path.dirname(os.path.abspath(urdf_path))
    chain, cur = [], base[0]
    while len(chain) < num_joints:
        nxt = [j for j in joints if j.find("parent").get("link") == cur]
        if not nxt:
            raise ValueError(f"chain ends after {len(chain)} joints at link {cur}")
        chain.append(nxt[0])  # serial chain: the first child joint in document order
        cur = nxt[0].find("child").get("link")
    nj = num_joints
    t = dict(num_joints=nj, axes=[], trans=[], rots=[], mass=[], com=[], inertia=[], link_center=[],
             link_generators=[], state_lb=[], state_ub=[], speed_limits=[], torque_limits=[], wrap=[])
    for i, j in enumerate(chain):
        t["axes"].append(_axis_code(j))
        org = j.find("origin")
        t["trans"].append(_vec(org, "xyz"))
        t["rots"].append(_vec(org, "rpy"))
        link = links[j.find("child").get("link")]
        inr = link.find("inertial")
        if inr is not None:
            t["mass"].append(float(inr.find("mass").get("value")))
            t["com"].append(_vec(inr.find("origin"), "xyz"))
            I = inr.find("inertia")
            g = {k: float(I.get(k, 0)) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")}
            t["inertia"].append([[g["ixx"], g["ixy"], g["ixz"]], [g["ixy"], g["iyy"], g["iyz"]], [g["ixz"], g["iyz"], g["izz"]]])
        else:
            t["mass"].append(0.0)
            t["com"].append(np.zeros(3))
            t["inertia"].append(np.zeros((3, 3)))
        vis = link.find("visual")
        mesh = vis.find("geometry/mesh") if vis is not None else None
        path = os.path.join(mesh_root, mesh.get("filename").replace("package://", "")) if mesh is not None else None
        c, g = mesh_box(path)
        t["link_center"].append(c)
        t["link_generators"].append(g)
        if i < NF:
            lim = j.find("limit")
            cont = j.get("type") == "continuous"
            t["state_lb"].append(-1000.0 if cont else float(lim.get("lower")))
            t["state_ub"].append(1000.0 if cont else float(lim.get("upper")))
            t["speed_limits"].append(float(lim.get("velocity")) if lim is not None else 0.0)
            t["torque_limits"].append(float(lim.get("effort")) if lim is not None else 0.0)
            t["wrap"].append(1 if cont else 0)
    t["trans"].append(np.zeros(3))  # the frame after the last joint (the headers' trailing row)
    out = dict(mass_uncertainty=0.0, inertia_uncertainty=0.0, friction=np.zeros(nj), damping=np.zeros(nj),
               armature=np.zeros(nj), gravity=9.81, alpha=1.0, V_m=0.0, M_max=1.0, M_min=1.0, K=1.0)
    out.update({k: np.asarray(v, dtype=np.float64) if k != "num_joints" else v for k, v in t.items()})
    out["axes"] = np.asarray(t["axes"], dtype=np.int64)
    out["wrap"] = np.asarray(t["wrap"], dtype=np.int64)
    for k, v in (extras or {}).items():
        out[k] = np.asarray(v, dtype=np.float64) if isinstance(v, (list, tuple, np.ndarray)) else v
    return out


# What the URDFs do not hold, from the reference's headers.
KINOVA_EXTRAS = dict(  # KPR/KinovaWithoutGripperInfo.h:40-112
    mass_uncertainty=0.03, inertia_uncertainty=0.03,
    armature=[8.03, 11.9962024615303644, 9.0025427861751517, 11.5806439316706360,
              8.4665040917914123, 8.8537069373742430, 8.8587303664685315],
    torque_limits=[56.7, 56.7, 56.7, 56.7, 29.4, 29.4, 29.4],  # the header's warning limits
    alpha=10.0, V_m=1e-2, M_max=15.79635774, M_min=5.095620491878957, K=5.0, gravity=9.81)
FETCH_EXTRAS = dict(  # ACMP/FetchInfo.h:45-97; FetchInfo.h has no M_max: its M_min is Kinova's
    mass_uncertainty=0.03, inertia_uncertainty=0.03,   # copied, and M_max is taken the same way
    # the URDF's wrist_roll_joint carries no <limit>; FetchInfo.h:88-90 lists all seven
    speed_limits=[1.256, 1.454, 1.571, 1.521, 1.571, 2.268, 2.268],
    torque_limits=[33.82, 131.76, 76.94, 66.18, 29.35, 25.7, 7.36],
    alpha=1.0, V_m=1e-7, M_max=15.79635774, M_min=5.09562049, K=5.0, gravity=9.81)


def save_json(tables: dict, path: str):
    def conv(v):
        return v.tolist() if isinstance(v, np.ndarray) else v
    with open(path, "w") as f:
        json.dump({k: conv(v) for k, v in tables.items()}, f, indent=1)


def load_json(path: str) -> dict:
    with open(path) as f:
        d = json.load(f)
    return _shaped(from_struct(to_struct(d)))


def geometry(tables: dict):
    """the world generator's view (armour_amd.robots.Robot) of a table set"""
    from .robots import Robot
    tb = _shaped(from_struct(to_struct(tables))) if not isinstance(tables.get("trans"), np.ndarray) or \
        np.asarray(tables["trans"]).ndim != 2 else tables
    return Robot(num_joints=int(tb["num_joints"]), axes=np.asarray(tb["axes"]), trans=np.asarray(tb["trans"]),
                 rots=np.asarray(tb["rots"]), link_c=np.asarray(tb["link_center"]),
                 link_g=np.asarray(tb["link_generators"]), state_lb=np.asarray(tb["state_lb"]),
                 state_ub=np.asarray(tb["state_ub"]), speed_limits=np.asarray(tb["speed_limits"]),
                 torque_limits=np.asarray(tb["torque_limits"]))
