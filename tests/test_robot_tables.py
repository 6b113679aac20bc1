"""Robot tables as data: the URDF + mesh generator (armour_amd.robot_tables)
pinned against the reference's hand-written robot headers, and the C ABI's table round trip.

Pins (reference data, copied as values):
  * KPR/KinovaWithoutGripperInfo.h:10-100 — the product's built-in tables (armour_robot_builtin(0))
    must equal the tables generated from urdfs/kinova_arm/kinova_without_gripper.urdf and its STLs
    (link zonotopes to the header's 6 printed decimals);
  * ACMP/FetchInfo.h:17-58 — axes, joint offsets, masses, centres of mass and inertias of the first 8
    joints must equal the tables generated from urdfs/fetch_arm/fetch_arm_7DOF.urdf.
"""
import os

import numpy as np
import pytest

import armour_amd as A
from armour_amd import robot_tables as RT

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = "/root/reference"

# ACMP/FetchInfo.h:17-58, first 8 of its 9 joints (the 9th is a fixed payload link)
FETCH_INFO = dict(
    axes=[3, 2, 1, 2, 1, 2, 1, 0],
    trans=[[-0.0326, 0, 0.726], [0.117, 0, 0.06], [0.219, 0, 0], [0.133, 0, 0], [0.197, 0, 0], [0.1245, 0, 0],
           [0.1385, 0, 0], [0.16645, 0, 0]],
    mass=[2.5587, 2.6615, 2.3311, 2.1299, 1.6563, 1.725, 0.1354, 1.5175],
    com=[[0.0927, -0.0056, 0.0564], [0.1432, 0.0072, -0.0001], [0.1165, 0.0014, 0], [0.1279, 0.0073, 0],
         [0.1097, -0.0266, 0], [0.0882, 0.0009, -0.0001], [0.0095, 0.0004, -0.0002], [-0.09, -0.0001, -0.0017]],
    inertia=[[0.0043, -0.0001, 0.001, -0.0001, 0.0087, -0.0001, 0.001, -0.0001, 0.0087],
             [0.0028, -0.0021, 0, -0.0021, 0.0111, 0, 0, 0, 0.0112],
             [0.0019, -0.0001, 0, -0.0001, 0.0045, 0, 0, 0, 0.0047],
             [0.0024, -0.0016, 0, -0.0016, 0.0082, 0, 0, 0, 0.0084],
             [0.0016, -0.0003, 0, -0.0003, 0.003, 0, 0, 0, 0.0035],
             [0.0018, -0.0001, 0, -0.0001, 0.0042, 0, 0, 0, 0.0042],
             [0.0001, 0, 0, 0, 0.0001, 0, 0, 0, 0.0001],
             [0.0013, 0, 0, 0, 0.0019, 0, 0, 0, 0.0024]],
    state_lb=[-1.6056, -1.221, -1000.0, -2.251, -1000.0, -2.16, -1000.0],
    state_ub=[1.6056, 1.518, 1000.0, 2.251, 1000.0, 2.16, 1000.0],
    speed_limits=[1.256, 1.454, 1.571, 1.521, 1.571, 2.268, 2.268],
    torque_limits=[33.82, 131.76, 76.94, 66.18, 29.35, 25.7, 7.36],
)


def test_kinova_urdf_tables_equal_the_reference_header():
    built = RT.builtin(0)   # the product's copy of KinovaWithoutGripperInfo.h
    gen = RT.load_json(os.path.join(GOLD, "robot_kinova_urdf.json"))
    assert int(gen["num_joints"]) == int(built["num_joints"]) == 7
    for k in ("axes", "wrap"):
        assert np.array_equal(gen[k], built[k]), k
    for k in ("trans", "mass", "com", "inertia", "state_lb", "state_ub", "speed_limits", "torque_limits",
              "armature", "friction", "damping"):
        assert np.allclose(gen[k], built[k], rtol=0, atol=1e-12), k
    assert np.allclose(gen["rots"], built["rots"], rtol=0, atol=1e-12)   # URDF pi to 33 digits vs M_PI
    # create_pz_bounding_boxes.m on the STLs; the header prints 6 decimals
    assert np.allclose(gen["link_center"], built["link_center"], rtol=0, atol=5.1e-7)
    assert np.allclose(gen["link_generators"], built["link_generators"], rtol=0, atol=5.1e-7)
    for k in ("alpha", "V_m", "M_max", "M_min", "K", "gravity", "mass_uncertainty", "inertia_uncertainty"):
        assert gen[k] == built[k], k


def test_fetch_urdf_tables_equal_fetch_info():
    gen = RT.load_json(os.path.join(GOLD, "robot_fetch.json"))
    assert int(gen["num_joints"]) == 8
    assert list(gen["axes"]) == FETCH_INFO["axes"]
    assert np.allclose(gen["trans"][:8], FETCH_INFO["trans"], rtol=0, atol=1e-12)
    assert np.allclose(gen["rots"], 0.0)
    for k in ("mass", "com"):
        assert np.allclose(gen[k], FETCH_INFO[k], rtol=0, atol=1e-12), k
    assert np.allclose(gen["inertia"].reshape(8, 9), FETCH_INFO["inertia"], rtol=0, atol=1e-12)
    for k in ("state_lb", "state_ub", "speed_limits", "torque_limits"):
        assert np.allclose(gen[k], FETCH_INFO[k], rtol=0, atol=1e-12), k
    assert list(gen["wrap"]) == [0, 0, 1, 0, 1, 0, 1]   # the continuous joints
    # every link has a mesh box (no 10 cm default cube)
    assert not np.any(np.all(np.isclose(gen["link_generators"], 0.05), axis=1))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_fixtures_regenerate_from_the_reference():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_robots", os.path.join(GOLD, "make_robots.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for name, tables in mod.generate(REF).items():
        saved = RT.load_json(os.path.join(GOLD, name))
        fresh = RT._shaped(RT.from_struct(RT.to_struct(tables)))
        for k, v in saved.items():
            assert np.allclose(np.asarray(fresh[k], dtype=float), np.asarray(v, dtype=float), rtol=0, atol=0), (name, k)


def test_stl_box_rule():
    # create_pz_bounding_boxes.m: bounds of the raw points; no / empty mesh -> 10 cm cube
    c, g = RT.mesh_box(None)
    assert np.allclose(c, 0) and np.allclose(g, 0.05)


def test_table_struct_round_trip():
    built = RT.builtin(0)
    again = RT.from_struct(RT.to_struct(built))
    for k, v in built.items():
        assert np.array_equal(np.asarray(again[k]), np.asarray(v)), k


def test_geometry_view_for_worlds():
    fetch = RT.load_json(os.path.join(GOLD, "robot_fetch.json"))
    geo = RT.geometry(fetch)
    w = A.make_world(0, 6, robot=geo)
    assert w[4].shape == (6, 12)
    assert np.all(w[0] >= np.where(geo.state_lb < -100, -np.pi, geo.state_lb))
