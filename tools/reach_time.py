"""Diagnostics: bundle-engine reach kernel time (HIP events, planner alone) on the bench's survey
worlds (T=100, O=20) at the given world counts. ARMOUR_LIB selects a variant build
(make -C armour-dev_amd/csrc lane_variant ...); ARMOUR_ENGINE=lane|job forces an engine (default: the
planner's choice by batch size).

usage: python tools/reach_time.py [W ...]   (default: 327 491 654 981)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

sizes = [int(v) for v in sys.argv[1:]] or [327, 491, 654, 981]
lib = os.path.basename(os.environ.get("ARMOUR_LIB", "libarmour_hip.so"))
for W in sizes:
    P = A.Planner(T=100, max_obstacles=20, max_worlds=W)
    worlds = [A.make_world(s, 20, profile="survey") for s in range(W)]
    P.reach(worlds)
    ts = [P.reach(worlds)["reach_kernel_ms"] for _ in range(3)]
    print(f"{lib} W={W}: reach kernel {min(ts):.2f} ms ({min(ts) / W * 1e3:.1f} us/world)", flush=True)
    P.close()
