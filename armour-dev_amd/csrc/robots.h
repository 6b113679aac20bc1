// armour-mi355x — robot tables (host side)
#pragma once
#include "common.h"

namespace armour {
void kinova_gen3(RobotParams& r);       // KPR/KinovaWithoutGripperInfo.h + KPR/Parameters.h
void finalize_params(RobotParams& r);   // derived tables (RPY matrices)
}  // namespace armour
