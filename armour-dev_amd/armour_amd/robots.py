"""Robot tables as data (KPR/KinovaWithoutGripperInfo.h:10-112).

The product's C++ runtime carries the same tables (armour-dev_amd/csrc/robots.cpp); this module
is what the Python side (world generator, tests) uses for geometry.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Robot:
    num_joints: int
    axes: np.ndarray
    trans: np.ndarray      # [(NJ+1), 3]
    rots: np.ndarray       # [NJ, 3]  roll pitch yaw
    link_c: np.ndarray     # [NJ, 3]
    link_g: np.ndarray     # [NJ, 3]
    state_lb: np.ndarray
    state_ub: np.ndarray
    speed_limits: np.ndarray
    torque_limits: np.ndarray


KINOVA = Robot(
    num_joints=7,
    axes=np.array([3, 3, 3, 3, 3, 3, 3]),
    trans=np.array([
        [0, 0, 0.15643], [0, 0.005375, -0.12838], [0, -0.21038, -0.006375],
        [0, 0.006375, -0.21038], [0, -0.20843, -0.006375], [0, 0.00017505, -0.10593],
        [0, -0.10593, -0.00017505], [0, 0, 0]]),
    rots=np.array([[np.pi, 0, 0], [np.pi / 2, 0, 0], [-np.pi / 2, 0, 0], [np.pi / 2, 0, 0],
                   [-np.pi / 2, 0, 0], [np.pi / 2, 0, 0], [-np.pi / 2, 0, 0]]),
    link_c=np.array([
        [0.000000, -0.001297, -0.088375], [0.000000, -0.089400, -0.007877],
        [0.000000, -0.001502, -0.129375], [0.000000, -0.087450, -0.013648],
        [0.000001, -0.009023, -0.071752], [0.000000, -0.041661, -0.009251],
        [0.000000, -0.018585, -0.033462]]),
    link_g=np.array([
        [0.046358, 0.047354, 0.086000], [0.046000, 0.135400, 0.047501],
        [0.046000, 0.047501, 0.127000], [0.046000, 0.133450, 0.042293],
        [0.034999, 0.044023, 0.069252], [0.035000, 0.076739, 0.044076],
        [0.045500, 0.056085, 0.030963]]),
    state_lb=np.array([-1000.0, -2.41, -1000.0, -2.66, -1000.0, -2.23, -1000.0]),
    state_ub=np.array([1000.0, 2.41, 1000.0, 2.66, 1000.0, 2.23, 1000.0]),
    speed_limits=np.array([1.3963, 1.3963, 1.3963, 1.3963, 1.2218, 1.2218, 1.2218]),
    torque_limits=np.array([56.7, 56.7, 56.7, 56.7, 29.4, 29.4, 29.4]),
)
