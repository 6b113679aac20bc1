"""Regenerate the robot-table fixtures from the reference's URDFs and meshes (run in the build
container, where /root/reference exists; the GPU box has only the JSON):

  robot_kinova_urdf.json  urdfs/kinova_arm/kinova_without_gripper.urdf, 7 joints, + KINOVA_EXTRAS
  robot_fetch.json        urdfs/fetch_arm/fetch_arm_7DOF.urdf, 8 joints (7 actuated + gripper), + FETCH_EXTRAS

usage: python tests/golden/make_robots.py [reference root]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "armour-dev_amd"))
from armour_amd import robot_tables as RT  # noqa: E402

SOURCES = {
    "robot_kinova_urdf.json": ("urdfs/kinova_arm/kinova_without_gripper.urdf", 7, RT.KINOVA_EXTRAS),
    "robot_fetch.json": ("urdfs/fetch_arm/fetch_arm_7DOF.urdf", 8, RT.FETCH_EXTRAS),
}


def generate(ref_root):
    return {name: RT.from_urdf(os.path.join(ref_root, urdf), nj, extras) for name, (urdf, nj, extras) in SOURCES.items()}


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    for name, tables in generate(ref).items():
        RT.save_json(tables, os.path.join(HERE, name))
        print("wrote", name)
