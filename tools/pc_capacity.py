"""Certified plane cache region use on the headline workload (981 survey worlds, T = 100, O = 20, in
the bench's 3 x 327 batches): (world, t) blocks whose kept planes fit the region of ARMOUR_PC_K records
per pair (the rest fall back to the full scan, bitwise the same). Development tool.
usage: ARMOUR_PC_K=k python tools/pc_capacity.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "armour-dev_amd"))
import armour_amd as A  # noqa: E402

tot = {"planes_kept": 0, "pairs": 0, "blocks_cached": 0, "blocks": 0, "max_per_pair": 0}
P = A.Planner(T=100, max_obstacles=20, max_worlds=327)
for b in range(3):
    P.reach([A.make_world(s, 20, profile="survey") for s in range(327 * b, 327 * (b + 1))])
    st = P.plane_cache_stats()
    for k in tot:
        tot[k] = max(tot[k], st[k]) if k == "max_per_pair" else tot[k] + st[k]
print(f"ARMOUR_PC_K={os.environ.get('ARMOUR_PC_K', 'default')}: {tot}, pool records {st['pool_records']}, "
      f"planes per pair {tot['planes_kept'] / tot['pairs']:.2f}, blocks overflowing {tot['blocks'] - tot['blocks_cached']}", flush=True)
