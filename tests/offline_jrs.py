"""Offline JRS tables of the ARMTD comparison planner — TEST INFRASTRUCTURE (fixture generation).

The reference ships its precomputed joint reachable sets as MATLAB files
(ACMP/offline_jrs/orig_parameterization/JRS_<c_kvi>.mat, made by ACMP/offline_jrs/
create_orig_offline_jrs.m with CORA): a cell JRS{1..100} of CORA zonotope objects over the state
[cos q, sin q, q, dq, k_a, k_v]. The objects are MATLAB class instances, so their property values
sit in the file's MCOS subsystem; scipy.io reads that subsystem as plain data (no code runs) and the
100 Z = [centre, generators] matrices (6 rows) appear there in cell order.

armtd_input() slices them as the MATLAB caller does (KSI/uarmtd_planner.m:260-318): per joint the
file whose c_kvi is closest to qd0_i, then per interval Z(1,1), Z(1,2), sum|Z(1,3:end)|, Z(2,1),
Z(2,2), sum|Z(2,3:end)| and k_range_i = JRS{1}.Z(5,2).
"""
from __future__ import annotations

import io
import os

import numpy as np

JRS_DIR = "/root/reference/kinova_src/kinova_simulator_interfaces/kinova_planner_realtime_armtd_comparison/" \
          "offline_jrs/orig_parameterization"
C_KVI = np.linspace(-np.pi, np.pi, 401)  # create_orig_offline_jrs.m:23-24


def load_jrs(c_kvi, jrs_dir=JRS_DIR):
    """the 100 Z matrices (6 x n) of JRS_<c_kvi>.mat, in time order"""
    import scipy.io as sio
    from scipy.io.matlab._mio5 import MatFile5Reader

    fn = os.path.join(jrs_dir, "JRS_%0.3f.mat" % c_kvi)
    d = sio.loadmat(fn)
    ws = d["__function_workspace__"].tobytes()
    hdr = open(fn, "rb").read(128)
    r = MatFile5Reader(io.BytesIO(hdr + ws[8:]), struct_as_record=True, squeeze_me=False)
    r.initialize_read()
    r.mat_stream.seek(128)
    h, _ = r.read_var_header()
    v = r.read_var_array(h, process=False)
    arr = v[0, 0]["MCOS"][0]["arr"]
    Z = [a for a in arr.ravel() if isinstance(a, np.ndarray) and a.dtype == np.float64 and a.ndim == 2 and a.shape[0] == 6]
    if len(Z) != 100:
        raise ValueError(f"{fn}: expected 100 zonotopes, found {len(Z)}")
    kv = float(np.asarray(d["current_c_kvi"]).ravel()[0])
    for z in Z:  # sanity: the k_v centre is the file's, the first generator spans k_a only at t = 0
        if abs(z[5, 0] - kv) > 1e-9:
            raise ValueError(f"{fn}: k_v centre {z[5, 0]} != {kv}")
    return Z


def tables_from(Z):
    """[6][T] = c_cos, g_cos, r_cos, c_sin, g_sin, r_sin (uarmtd_planner.m:288-314) and k_range"""
    T = len(Z)
    tab = np.zeros((6, T))
    for i, z in enumerate(Z):
        tab[0, i], tab[1, i], tab[2, i] = z[0, 0], z[0, 1], np.abs(z[0, 2:]).sum()
        tab[3, i], tab[4, i], tab[5, i] = z[1, 0], z[1, 1], np.abs(z[1, 2:]).sum()
    return tab, float(Z[0][4, 1])


def armtd_input(qd0, jrs_dir=JRS_DIR):
    """(tables [7][6][100], k_range [7]) for the start velocities qd0"""
    tabs, kr = [], []
    for v in qd0:
        c = C_KVI[int(np.argmin(np.abs(v - C_KVI)))]
        tab, k = tables_from(load_jrs(c, jrs_dir))
        tabs.append(tab)
        kr.append(k)
    return np.array(tabs), np.array(kr)
