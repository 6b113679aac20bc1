"""Point models of the reference's definitions — TEST INFRASTRUCTURE, independent of the oracle.

The oracle (oracle/src) restates the reference's set arithmetic (PZsparse, the JRS, PZ FK and PZ
RNEA); the HIP path computes the same sets. Both could share a wrong reading of the reference.
These numpy models evaluate the *definitions* the sets must enclose, at points, with no PZ code:

  * the degree-5 Bezier desired trajectory (KPR/Trajectory.cu:542-599: control points
    q0, q0 + T qd0 / 5, q0 + 2 T qd0 / 5 + T^2 qdd0 / 20, then three times q0 + k; DURATION = 1,
    KPR/Parameters.h:14), its derivatives by the Bezier difference rule;
  * forward kinematics of the link boxes (KPR/Dynamics.cu:69-81: p += R trans_i, R = R R_i,
    link_i = R box_i + p, with R_i = RPY_i Rot_axis(q_i) as KPR/Trajectory.cu:136-142 and the
    reference's RPY matrix Rx(roll) Ry(pitch) Rz(yaw), KPR/PZsparse.cu:160-176);
  * the passivity-based RNEA with an auxiliary velocity (KPR/Dynamics.cu:83-181, the same
    recursion as the MATLAB rnea the reference checks against in KPR/debug_script.m:98-107),
    plus armature * qdda_a + damping * qd (Dynamics.cu:172-176).

tests/test_oracle_containment.py samples these at random times inside each interval, parameters
k and tracking errors within the reference's ultimate bounds (qe, qde, qdae, qddae,
KPR/KinovaWithoutGripperInfo.h:102-112), and checks that the oracle's (and, in the -m gpu test, the
HIP path's) sliced reachable sets contain every sample: SURVEY.md §7 step 1's soundness properties.
"""
from __future__ import annotations

import itertools
from math import comb

import numpy as np

GRAVITY_AXIS = 2


# ---- trajectory ---------------------------------------------------------------------------------
def control_points(q0, qd0, qdd0, k, duration=1.0):
    """[..., 6] Bezier control points of KPR/Trajectory.cu:554-559 (k in radians)"""
    q0, qd0, qdd0, k = np.broadcast_arrays(*(np.asarray(v, dtype=np.float64) for v in (q0, qd0, qdd0, k)))
    Tqd0, TTqdd0 = qd0 * duration, qdd0 * duration ** 2
    return np.stack([q0, q0 + Tqd0 / 5, q0 + 2 * Tqd0 / 5 + TTqdd0 / 20, q0 + k, q0 + k, q0 + k], axis=-1)


def _bernstein(n, t):
    t = np.asarray(t, dtype=np.float64)[..., None]
    i = np.arange(n + 1)
    return np.array([comb(n, j) for j in i]) * t ** i * (1 - t) ** (n - i)


def bezier(beta, t, duration=1.0):
    """(q, qd, qdd) of the degree-5 curve with control points beta [..., 6] at s = t in [0, 1]"""
    beta = np.asarray(beta)
    d1 = 5 * np.diff(beta, axis=-1)
    d2 = 4 * np.diff(d1, axis=-1)
    q = np.sum(_bernstein(5, t) * beta, axis=-1)
    qd = np.sum(_bernstein(4, t) * d1, axis=-1) / duration
    qdd = np.sum(_bernstein(3, t) * d2, axis=-1) / duration ** 2
    return q, qd, qdd


# ---- rotations ----------------------------------------------------------------------------------
def rot_axis(axis, q):
    """[N, 3, 3] rotation about x / y / z (axis 1 / 2 / 3; 0: identity, a fixed joint)"""
    q = np.asarray(q, dtype=np.float64)
    R = np.zeros(q.shape + (3, 3))
    R[...] = np.eye(3)
    if axis == 0:
        return R
    a, b = [(1, 2), (2, 0), (0, 1)][abs(axis) - 1]
    c, s = np.cos(q), np.sin(q)
    R[..., a, a] = c
    R[..., b, b] = c
    R[..., a, b] = -s
    R[..., b, a] = s
    return R


def rpy(roll, pitch, yaw):
    """Rx(roll) Ry(pitch) Rz(yaw), the reference's fixed-frame rotation (KPR/PZsparse.cu:160-176)"""
    return (rot_axis(1, np.array(roll)) @ rot_axis(2, np.array(pitch)) @ rot_axis(3, np.array(yaw)))


def joint_rotations(robot, q):
    """[NJ, N, 3, 3]: R_i = RPY_i Rot_axis_i(q_i) for the actuated joints, RPY_i for the fixed ones"""
    q = np.atleast_2d(q)
    out = []
    for i in range(int(robot["num_joints"])):
        R = np.broadcast_to(rpy(*robot["rots"][i]), (q.shape[0], 3, 3))
        ax = int(robot["axes"][i])
        if ax != 0 and i < q.shape[1]:
            R = R @ rot_axis(ax, q[:, i])
        out.append(np.array(R))
    return out


# ---- forward kinematics -------------------------------------------------------------------------
BOX_CORNERS = np.array(list(itertools.product((-1.0, 1.0), repeat=3)))  # [8, 3]


def link_points(robot, q, box_coords=BOX_CORNERS):
    """[NJ, N, P, 3] world points of each link box (centre + diag(generators) * box_coords) at the
    joint angles q [N, nq] (KPR/Dynamics.cu:69-81, link boxes :48-66)"""
    q = np.atleast_2d(q)
    N = q.shape[0]
    Rs = joint_rotations(robot, q)
    R = np.broadcast_to(np.eye(3), (N, 3, 3))
    p = np.zeros((N, 3))
    out = []
    for i in range(int(robot["num_joints"])):
        p = p + R @ robot["trans"][i]
        R = R @ Rs[i]
        local = robot["link_center"][i] + box_coords * robot["link_generators"][i]  # [P, 3]
        out.append(p[:, None, :] + np.einsum("nij,pj->npi", R, local))
    return np.array(out)


# ---- dynamics -----------------------------------------------------------------------------------
def rnea(robot, q, qd, qda, qdda, mass=None, inertia=None):
    """[N, nq] joint torques of the passivity-based RNEA with auxiliary velocity qda
    (KPR/Dynamics.cu:83-181) with gravity, plus armature * qdda + damping * qd.
    mass [N, NJ], inertia [N, NJ, 3, 3] (default: the nominal tables)."""
    q, qd, qda, qdda = (np.atleast_2d(np.asarray(v, dtype=np.float64)) for v in (q, qd, qda, qdda))
    N, nq = q.shape
    NJ = int(robot["num_joints"])
    m = np.broadcast_to(robot["mass"], (N, NJ)) if mass is None else mass
    I = np.broadcast_to(robot["inertia"], (N, NJ, 3, 3)) if inertia is None else inertia
    Rs = joint_rotations(robot, q)
    trans = robot["trans"]
    com = robot["com"]
    w = np.zeros((N, 3))
    wa = np.zeros((N, 3))
    wd = np.zeros((N, 3))
    acc = np.zeros((N, 3))
    acc[:, GRAVITY_AXIS] = robot["gravity"]
    F, Nm = [], []
    for i in range(NJ):
        Rt = np.swapaxes(Rs[i], 1, 2)
        p = trans[i]
        acc = np.einsum("nij,nj->ni", Rt, acc + np.cross(wd, p) + np.cross(w, np.cross(wa, p)))
        w = np.einsum("nij,nj->ni", Rt, w)
        wa = np.einsum("nij,nj->ni", Rt, wa)
        wd = np.einsum("nij,nj->ni", Rt, wd)
        ax = int(robot["axes"][i])
        if ax != 0:
            z = np.zeros(3)
            z[abs(ax) - 1] = 1.0
            w = w + qd[:, i, None] * z
            wd = wd + np.cross(wa, qd[:, i, None] * z) + qdda[:, i, None] * z
            wa = wa + qda[:, i, None] * z
        c = com[i]
        F.append(m[:, i, None] * (acc + np.cross(wd, c) + np.cross(w, np.cross(wa, c))))
        Iw = np.einsum("nij,nj->ni", I[:, i], w)
        Nm.append(np.einsum("nij,nj->ni", I[:, i], wd) + np.cross(wa, Iw))
    f = np.zeros((N, 3))
    n = np.zeros((N, 3))
    u = np.zeros((N, nq))
    for i in range(NJ - 1, -1, -1):
        R1 = Rs[i + 1] if i + 1 < NJ else np.broadcast_to(np.eye(3), (N, 3, 3))
        Rf = np.einsum("nij,nj->ni", R1, f)
        n = Nm[i] + np.einsum("nij,nj->ni", R1, n) + np.cross(com[i], F[i]) + np.cross(trans[i + 1], Rf)
        f = Rf + F[i]
        ax = int(robot["axes"][i])
        if ax != 0 and i < nq:
            u[:, i] = n[:, abs(ax) - 1] + robot["armature"][i] * qdda[:, i] + robot["damping"][i] * qd[:, i]
    return u


def ultimate_bounds(robot):
    """(qe, qde, qdae, qddae) of KPR/KinovaWithoutGripperInfo.h:102-112"""
    eps = np.sqrt(2 * robot["V_m"] / robot["M_min"])
    K = robot["K"]
    return eps / K, 2 * eps, eps, 2 * K * eps


def robust_term(robot):
    """alpha (M_max - M_min) eps, the robust-input part of the torque radius (KPR/armour_main.cu:186)"""
    eps = np.sqrt(2 * robot["V_m"] / robot["M_min"])
    return robot["alpha"] * (robot["M_max"] - robot["M_min"]) * eps


# ---- zonotope membership ------------------------------------------------------------------------
def zonotope_excess(c, G, p):
    """max over facet normals of |n . (p - c)| - sum_i |n . g_i| for the 3-D zonotope c + G [-1,1]^k
    (G [..., 3, k], c [..., 3], p [..., P, 3]); <= 0 iff p lies in the zonotope. The facet normals of
    a 3-D zonotope are the cross products of generator pairs; the coordinate axes are added (valid
    support directions for any set) so that a degenerate G still bounds every direction."""
    G = np.asarray(G)
    k = G.shape[-1]
    normals = [np.cross(G[..., :, a], G[..., :, b]) for a in range(k) for b in range(a + 1, k)]
    eye = np.broadcast_to(np.eye(3), G.shape[:-2] + (3, 3))
    normals += [eye[..., j, :] for j in range(3)]
    Nn = np.stack(normals, axis=-2)                                   # [..., M, 3]
    norm = np.linalg.norm(Nn, axis=-1, keepdims=True)
    ok = norm[..., 0] > 1e-12                                         # parallel pairs span no facet
    Nn = Nn / np.where(ok[..., None], norm, 1.0)
    h = np.abs(np.einsum("...mj,...jk->...mk", Nn, G)).sum(-1)       # [..., M] support half-widths
    d = np.einsum("...mj,...pj->...pm", Nn, p - c[..., None, :])     # [..., P, M]
    return np.where(ok[..., None, :], np.abs(d) - h[..., None, :], -np.inf).max(-1)  # [..., P]
