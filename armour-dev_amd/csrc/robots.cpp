// armour-mi355x — robot tables and planner parameters (host side).
// Kinova Gen3 without gripper: KPR/KinovaWithoutGripperInfo.h:10-112; parameters:
// KPR/Parameters.h:10-59. RPY rotation matrices are pre-computed here with the reference's own
// closed form (PZsparse.cu:160-176) so device code needs no trigonometry for them.
#include "robots.h"
#include "../../include/armour_hip.h"
#include <cmath>
#include <cstring>

namespace armour {

static void rpy_matrix(double roll, double pitch, double yaw, double* c) {
    c[0 + 0] = std::cos(pitch) * std::cos(yaw);
    c[0 + 3] = -std::cos(pitch) * std::sin(yaw);
    c[0 + 6] = std::sin(pitch);
    c[1 + 0] = std::cos(roll) * std::sin(yaw) + std::cos(yaw) * std::sin(pitch) * std::sin(roll);
    c[1 + 3] = std::cos(roll) * std::cos(yaw) - std::sin(pitch) * std::sin(roll) * std::sin(yaw);
    c[1 + 6] = -std::cos(pitch) * std::sin(roll);
    c[2 + 0] = std::sin(roll) * std::sin(yaw) - std::cos(roll) * std::cos(yaw) * std::sin(pitch);
    c[2 + 3] = std::cos(yaw) * std::sin(roll) + std::cos(roll) * std::sin(pitch) * std::sin(yaw);
    c[2 + 6] = std::cos(pitch) * std::cos(roll);
}

void finalize_params(RobotParams& r) {
    for (int i = 0; i < r.num_joints; i++) rpy_matrix(r.rots[3 * i], r.rots[3 * i + 1], r.rots[3 * i + 2], r.rpy[i]);
    rpy_matrix(0, 0, 0, r.rpy[MAX_J]);
}

void kinova_gen3(RobotParams& r) {
    std::memset(&r, 0, sizeof(r));
    r.num_joints = 7;
    for (int i = 0; i < 7; i++) r.axes[i] = 3;
    const double trans[] = {0, 0, 0.15643, 0, 0.005375, -0.12838, 0, -0.21038, -0.006375,
                            0, 0.006375, -0.21038, 0, -0.20843, -0.006375, 0, 0.00017505, -0.10593,
                            0, -0.10593, -0.00017505, 0, 0, 0};
    std::memcpy(r.trans, trans, sizeof(trans));
    const double rots[] = {M_PI, 0, 0, M_PI * 0.5, 0, 0, -M_PI * 0.5, 0, 0, M_PI * 0.5, 0, 0,
                           -M_PI * 0.5, 0, 0, M_PI * 0.5, 0, 0, -M_PI * 0.5, 0, 0};
    std::memcpy(r.rots, rots, sizeof(rots));
    const double mass[] = {1.3773, 1.1636, 1.1636, 0.9302, 0.6781, 0.6781, 0.5};
    std::memcpy(r.mass, mass, sizeof(mass));
    r.mass_uncertainty = 0.03;
    const double com[] = {-0.000023, -0.010364, -0.07336, -0.000044, -0.09958, -0.013278,
                          -0.000044, -0.006641, -0.117892, -0.000018, -0.075478, -0.015006,
                          0.000001, -0.009432, -0.063883, 0.000001, -0.045483, -0.00965,
                          0.000281, 0.011402, -0.029798};
    std::memcpy(r.com, com, sizeof(com));
    const double inertia[] = {
        0.00457, 0.000001, 0.000002, 0.000001, 0.004831, 0.000448, 0.000002, 0.000448, 0.001409,
        0.011088, 0.000005, 0, 0.000005, 0.001072, -0.000691, 0, -0.000691, 0.011255,
        0.010932, 0, -0.000007, 0, 0.011127, 0.000606, -0.000007, 0.000606, 0.001043,
        0.008147, -0.000001, 0, -0.000001, 0.000631, -0.0005, 0, -0.0005, 0.008316,
        0.001596, 0, 0, 0, 0.001607, 0.000256, 0, 0.000256, 0.000399,
        0.001641, 0, 0, 0, 0.00041, -0.000278, 0, -0.000278, 0.001641,
        0.000587, 0.000003, 0.000003, 0.000003, 0.000369, -0.000118, 0.000003, -0.000118, 0.000609};
    std::memcpy(r.inertia, inertia, sizeof(inertia));
    r.inertia_uncertainty = 0.03;
    const double arm[] = {8.03, 11.9962024615303644, 9.0025427861751517, 11.5806439316706360,
                          8.4665040917914123, 8.8537069373742430, 8.8587303664685315};
    std::memcpy(r.armature, arm, sizeof(arm));
    const double lb[] = {-1000.0, -2.41, -1000.0, -2.66, -1000.0, -2.23, -1000.0};
    const double ub[] = {1000.0, 2.41, 1000.0, 2.66, 1000.0, 2.23, 1000.0};
    const double sp[] = {1.3963, 1.3963, 1.3963, 1.3963, 1.2218, 1.2218, 1.2218};
    const double tq[] = {56.7, 56.7, 56.7, 56.7, 29.4, 29.4, 29.4};
    for (int i = 0; i < 7; i++) {
        r.state_lb[i] = lb[i]; r.state_ub[i] = ub[i]; r.speed_limits[i] = sp[i]; r.torque_limits[i] = tq[i];
        r.wrap_mask[i] = (i % 2 == 0) ? 1 : 0;  // NLPclass.cu:225-231 (continuous joints 0,2,4,6)
    }
    r.gravity = 9.81;
    const double lc[7][3] = {{0.000000, -0.001297, -0.088375}, {0.000000, -0.089400, -0.007877},
                             {0.000000, -0.001502, -0.129375}, {0.000000, -0.087450, -0.013648},
                             {0.000001, -0.009023, -0.071752}, {0.000000, -0.041661, -0.009251},
                             {0.000000, -0.018585, -0.033462}};
    const double lg[7][3] = {{0.046358, 0.047354, 0.086000}, {0.046000, 0.135400, 0.047501},
                             {0.046000, 0.047501, 0.127000}, {0.046000, 0.133450, 0.042293},
                             {0.034999, 0.044023, 0.069252}, {0.035000, 0.076739, 0.044076},
                             {0.045500, 0.056085, 0.030963}};
    std::memcpy(r.link_c, lc, sizeof(lc));
    std::memcpy(r.link_g, lg, sizeof(lg));
    r.alpha = 10.0;
    r.V_m = 1e-2;
    r.M_max = 15.79635774;
    r.M_min = 5.095620491878957;
    r.eps = std::sqrt(2 * r.V_m / r.M_min);
    r.K = 5.0;
    r.qe = r.eps / r.K;
    r.qde = 2 * r.eps;
    r.qdae = r.eps;
    r.qddae = 2 * r.K * r.eps;
    planner_defaults(r);
    finalize_params(r);
}

void planner_defaults(RobotParams& r) {
    // planner parameters (Parameters.h)
    r.duration = 1.0;
    r.simplify_threshold = 5e-4;
    for (int i = 0; i < NF; i++) r.k_range[i] = M_PI / 48;
    r.collision_violation = 1e-4;
    r.torque_violation = 1e-2;
    r.cost_scale = 10.0;
    r.t_plan = 0.5;
}

bool robot_from_tables(const armour_robot& t, RobotParams& r) {
    if (t.num_joints < NF || t.num_joints > MAX_J) return false;
    std::memset(&r, 0, sizeof(r));
    r.num_joints = t.num_joints;
    for (int i = 0; i < t.num_joints; i++) {
        if (t.axes[i] < -3 || t.axes[i] > 3) return false;
        if (i < NF && t.axes[i] == 0) return false;  // the actuated joints come first
        r.axes[i] = t.axes[i];
    }
    std::memcpy(r.trans, t.trans, sizeof(r.trans));
    std::memcpy(r.rots, t.rots, sizeof(r.rots));
    std::memcpy(r.mass, t.mass, sizeof(r.mass));
    std::memcpy(r.com, t.com, sizeof(r.com));
    std::memcpy(r.inertia, t.inertia, sizeof(r.inertia));
    r.mass_uncertainty = t.mass_uncertainty;
    r.inertia_uncertainty = t.inertia_uncertainty;
    std::memcpy(r.friction, t.friction, sizeof(r.friction));
    std::memcpy(r.damping, t.damping, sizeof(r.damping));
    std::memcpy(r.armature, t.armature, sizeof(r.armature));
    for (int i = 0; i < NF; i++) {
        r.state_lb[i] = t.state_lb[i];
        r.state_ub[i] = t.state_ub[i];
        r.speed_limits[i] = t.speed_limits[i];
        r.torque_limits[i] = t.torque_limits[i];
        r.wrap_mask[i] = t.wrap[i] ? 1 : 0;
    }
    r.gravity = t.gravity;
    for (int i = 0; i < MAX_J; i++)
        for (int e = 0; e < 3; e++) {
            r.link_c[i][e] = t.link_center[3 * i + e];
            r.link_g[i][e] = t.link_generators[3 * i + e];
        }
    r.alpha = t.alpha;
    r.V_m = t.V_m;
    r.M_max = t.M_max;
    r.M_min = t.M_min;
    r.K = t.K;
    if (!(r.M_min > 0) || !(r.K > 0) || !(r.V_m >= 0)) return false;
    // derived bounds as the reference's header computes them (KinovaWithoutGripperInfo.h:102-112)
    r.eps = std::sqrt(2 * r.V_m / r.M_min);
    r.qe = r.eps / r.K;
    r.qde = 2 * r.eps;
    r.qdae = r.eps;
    r.qddae = 2 * r.K * r.eps;
    planner_defaults(r);
    finalize_params(r);
    return true;
}

void robot_to_tables(const RobotParams& r, armour_robot& t) {
    std::memset(&t, 0, sizeof(t));
    t.num_joints = r.num_joints;
    for (int i = 0; i < MAX_J; i++) t.axes[i] = r.axes[i];
    std::memcpy(t.trans, r.trans, sizeof(t.trans));
    std::memcpy(t.rots, r.rots, sizeof(t.rots));
    std::memcpy(t.mass, r.mass, sizeof(t.mass));
    std::memcpy(t.com, r.com, sizeof(t.com));
    std::memcpy(t.inertia, r.inertia, sizeof(t.inertia));
    t.mass_uncertainty = r.mass_uncertainty;
    t.inertia_uncertainty = r.inertia_uncertainty;
    std::memcpy(t.friction, r.friction, sizeof(t.friction));
    std::memcpy(t.damping, r.damping, sizeof(t.damping));
    std::memcpy(t.armature, r.armature, sizeof(t.armature));
    for (int i = 0; i < NF; i++) {
        t.state_lb[i] = r.state_lb[i];
        t.state_ub[i] = r.state_ub[i];
        t.speed_limits[i] = r.speed_limits[i];
        t.torque_limits[i] = r.torque_limits[i];
        t.wrap[i] = r.wrap_mask[i];
    }
    t.gravity = r.gravity;
    for (int i = 0; i < MAX_J; i++)
        for (int e = 0; e < 3; e++) {
            t.link_center[3 * i + e] = r.link_c[i][e];
            t.link_generators[3 * i + e] = r.link_g[i][e];
        }
    t.alpha = r.alpha;
    t.V_m = r.V_m;
    t.M_max = r.M_max;
    t.M_min = r.M_min;
    t.K = r.K;
}

}  // namespace armour
