// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
//
// Robot tables and planner parameters, restated as runtime data instead of the reference's
// compile-time #defines:
//   KPR/KinovaWithoutGripperInfo.h:10-112  (robot)
//   KPR/Parameters.h:10-59                  (planner parameters)
// NUM_FACTORS (= 7) stays a compile-time constant because the 63-bit monomial hash layout
// (KPR/PZsparse.h:23-40) is built on it; NUM_JOINTS and NUM_TIME_STEPS become runtime values.
#pragma once
#include <cmath>
#include <cstdint>

namespace oracle {

constexpr int NF = 7;          // NUM_FACTORS
constexpr int MAX_J = 9;       // largest NUM_JOINTS supported (Fetch arm: 9)
constexpr int MAX_OBS = 64;    // obstacle cap (reference MAX_OBSTACLE_NUM = 40)
constexpr int OBS_GEN = 3;     // MAX_OBSTACLE_GENERATOR_NUM
constexpr int BUF_GEN = OBS_GEN + 6;                 // BUFFER_OBSTACLE_GENERATOR_NUM
constexpr int COMB = BUF_GEN * (BUF_GEN - 1) / 2;    // COMB_NUM = 36

struct Robot {
    int num_joints = 7;
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
    // ultimate bound (KinovaWithoutGripperInfo.h:102-112)
    double alpha, V_m, M_max, M_min, eps, K, qe, qde, qdae, qddae;
    // joints whose cost term is wrapped to [-pi, pi] (NLPclass.cu:225-231 hard-codes 0,2,4,6)
    int wrap_mask[NF];
};

struct Params {
    int T = 128;                          // NUM_TIME_STEPS (Parameters.h:17)
    double duration = 1.0;                // DURATION (Parameters.h:14)
    double simplify_threshold = 5e-4;     // SIMPLIFY_THRESHOLD (Parameters.h:10)
    double k_range[NF];                   // Parameters.h:21
    double collision_violation = 1e-4;    // Parameters.h:38
    double torque_violation = 1e-2;       // Parameters.h:41
    double cost_scale = 10.0;             // Parameters.h:44
    double t_plan = 0.5;                  // armour_main.cu:81
};

inline Robot kinova_without_gripper() {
    Robot r{};
    r.num_joints = 7;
    for (int i = 0; i < 7; i++) r.axes[i] = 3;
    const double trans[] = {0, 0, 0.15643,  0, 0.005375, -0.12838,  0, -0.21038, -0.006375,
                            0, 0.006375, -0.21038,  0, -0.20843, -0.006375,  0, 0.00017505, -0.10593,
                            0, -0.10593, -0.00017505,  0, 0, 0};
    for (int i = 0; i < 24; i++) r.trans[i] = trans[i];
    const double rots[] = {M_PI, 0, 0,  M_PI * 0.5, 0, 0,  -M_PI * 0.5, 0, 0,  M_PI * 0.5, 0, 0,
                           -M_PI * 0.5, 0, 0,  M_PI * 0.5, 0, 0,  -M_PI * 0.5, 0, 0};
    for (int i = 0; i < 21; i++) r.rots[i] = rots[i];
    const double mass[] = {1.3773, 1.1636, 1.1636, 0.9302, 0.6781, 0.6781, 0.5};
    for (int i = 0; i < 7; i++) r.mass[i] = mass[i];
    r.mass_uncertainty = 0.03;
    const double com[] = {-0.000023, -0.010364, -0.07336,  -0.000044, -0.09958, -0.013278,
                          -0.000044, -0.006641, -0.117892,  -0.000018, -0.075478, -0.015006,
                          0.000001, -0.009432, -0.063883,  0.000001, -0.045483, -0.00965,
                          0.000281, 0.011402, -0.029798};
    for (int i = 0; i < 21; i++) r.com[i] = com[i];
    const double inertia[] = {
        0.00457, 0.000001, 0.000002, 0.000001, 0.004831, 0.000448, 0.000002, 0.000448, 0.001409,
        0.011088, 0.000005, 0, 0.000005, 0.001072, -0.000691, 0, -0.000691, 0.011255,
        0.010932, 0, -0.000007, 0, 0.011127, 0.000606, -0.000007, 0.000606, 0.001043,
        0.008147, -0.000001, 0, -0.000001, 0.000631, -0.0005, 0, -0.0005, 0.008316,
        0.001596, 0, 0, 0, 0.001607, 0.000256, 0, 0.000256, 0.000399,
        0.001641, 0, 0, 0, 0.00041, -0.000278, 0, -0.000278, 0.001641,
        0.000587, 0.000003, 0.000003, 0.000003, 0.000369, -0.000118, 0.000003, -0.000118, 0.000609};
    for (int i = 0; i < 63; i++) r.inertia[i] = inertia[i];
    r.inertia_uncertainty = 0.03;
    for (int i = 0; i < 7; i++) { r.friction[i] = 0.0; r.damping[i] = 0.0; }
    const double arm[] = {8.03, 11.9962024615303644, 9.0025427861751517, 11.5806439316706360,
                          8.4665040917914123, 8.8537069373742430, 8.8587303664685315};
    for (int i = 0; i < 7; i++) r.armature[i] = arm[i];
    const double lb[] = {-1000.0, -2.41, -1000.0, -2.66, -1000.0, -2.23, -1000.0};
    const double ub[] = {1000.0, 2.41, 1000.0, 2.66, 1000.0, 2.23, 1000.0};
    const double sp[] = {1.3963, 1.3963, 1.3963, 1.3963, 1.2218, 1.2218, 1.2218};
    const double tq[] = {56.7, 56.7, 56.7, 56.7, 29.4, 29.4, 29.4};
    for (int i = 0; i < 7; i++) {
        r.state_lb[i] = lb[i]; r.state_ub[i] = ub[i]; r.speed_limits[i] = sp[i]; r.torque_limits[i] = tq[i];
        r.wrap_mask[i] = (i % 2 == 0) ? 1 : 0;
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
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 3; j++) { r.link_c[i][j] = lc[i][j]; r.link_g[i][j] = lg[i][j]; }
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
    return r;
}

inline Params default_params(int T) {
    Params p;
    p.T = T;
    for (int i = 0; i < NF; i++) p.k_range[i] = M_PI / 48;
    return p;
}

}  // namespace oracle
