// armour-mi355x — robot tables (host side)
#pragma once
#include "common.h"
#include "../../include/armour_hip.h"

namespace armour {
void kinova_gen3(RobotParams& r);       // KPR/KinovaWithoutGripperInfo.h + KPR/Parameters.h
void finalize_params(RobotParams& r);   // derived tables (RPY matrices)
void planner_defaults(RobotParams& r);  // KPR/Parameters.h planner parameters
// RobotParams from plain C robot tables (armour_robot of include/armour_hip.h); false if invalid
bool robot_from_tables(const ::armour_robot& t, RobotParams& r);
void robot_to_tables(const RobotParams& r, ::armour_robot& t);
}  // namespace armour
