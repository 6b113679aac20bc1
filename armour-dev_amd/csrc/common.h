// armour-mi355x — shared definitions for the HIP (gfx950) planner.
//
// Sizes that the reference fixes at compile time (KPR/Parameters.h:17-29) are runtime values
// here: time steps T, obstacles O, joints NJ. NUM_FACTORS stays 7 because the 63-bit monomial
// hash (KPR/PZsparse.h:23-40) is laid out for 7 factors.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#define AD __host__ __device__ inline

namespace armour {

constexpr int NF = 7;          // trajectory parameters / actuated joints (NUM_FACTORS)
constexpr int MAX_J = 9;       // largest NUM_JOINTS supported
constexpr int OBS_GEN = 3;     // MAX_OBSTACLE_GENERATOR_NUM
constexpr int MAX_OBS = 40;    // MAX_OBSTACLE_NUM (KPR/Parameters.h:26)
constexpr int BUF_GEN = OBS_GEN + 6;
constexpr int COMB = BUF_GEN * (BUF_GEN - 1) / 2;  // 36 generator pairs
constexpr int LL_PLANES = 15;  // planes spanned by two link generators (6 choose 2)
constexpr int OO_PLANES = OBS_GEN * (OBS_GEN - 1) / 2;  // planes spanned by two obstacle generators

// monomial hash layout (KPR/PZsparse.h:23-40): k (7 x 2 bit) | qde | qdae | qddae (7 x 1 bit) |
// cosqe | sinqe (7 x 2 bit)
constexpr int SLOT_K = 0, SLOT_QDE = NF, SLOT_QDAE = 2 * NF, SLOT_QDDAE = 3 * NF, SLOT_COS = 4 * NF, SLOT_SIN = 5 * NF;
constexpr uint64_t HASH_K_ONLY = (uint64_t)1 << (2 * NF);
constexpr uint64_t HASH_K_LINKS_ONLY = (uint64_t)1 << (5 * NF);
constexpr uint64_t K_MASK = HASH_K_ONLY - 1;

AD int slot_bit(int slot) {
    // bit position of a degree slot: 2-bit k slots, 1-bit qde/qdae/qddae, 2-bit cos/sin
    return slot < SLOT_QDE ? 2 * slot : slot < SLOT_COS ? 2 * NF + (slot - SLOT_QDE) : 5 * NF + 2 * (slot - SLOT_COS);
}
AD uint64_t slot_hash(int slot) { return (uint64_t)1 << slot_bit(slot); }

// Robot + planner parameters, a POD copied to the device once (KPR/KinovaWithoutGripperInfo.h,
// KPR/Parameters.h).
struct RobotParams {
    int num_joints;
    int axes[MAX_J];
    double trans[(MAX_J + 1) * 3];
    double rots[MAX_J * 3];
    double mass[MAX_J];
    double mass_uncertainty;
    double com[MAX_J * 3];
    double inertia[MAX_J * 9];
    double inertia_uncertainty;
    double friction[MAX_J];
    double damping[MAX_J];
    double armature[MAX_J];
    double state_lb[NF], state_ub[NF];
    double speed_limits[NF];
    double torque_limits[NF];
    double gravity;
    double link_c[MAX_J][3];
    double link_g[MAX_J][3];
    double alpha, V_m, M_max, M_min, eps, K, qe, qde, qdae, qddae;
    int wrap_mask[NF];
    // planner parameters
    double duration;
    double simplify_threshold;
    double k_range[NF];
    double collision_violation;
    double torque_violation;
    double cost_scale;
    double t_plan;
    // pre-computed RPY rotation matrices of each joint (column-major) and their transposes
    double rpy[MAX_J + 1][9];
};

}  // namespace armour
