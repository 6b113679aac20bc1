// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
//
// The ARMTD comparison planner (kinova_planner_realtime_armtd_comparison/, "ACMP/" below), restated
// on top of the ARMOUR oracle: its reach set is ARMOUR's forward kinematics over joint rotations
// built from offline JRS tables instead of the Bernstein trajectory, and its NLP keeps only the
// collision rows and the constant-acceleration joint extrema (no RNEA, no torque rows):
//   input          ACMP/armtd_main.cu:37-102 (q0, qd0, q_des; per joint the cos/sin centre,
//                  k-generator and radius of every interval, then k_range; obstacles)
//   JRS            ACMP/Trajectory.cu:29-81 (tables rotated by q0; radius x 5)
//   FK             ACMP/Dynamics.cu:6-57 (= KPR/Dynamics.cu fk), reduce_link_PZ, hyperplanes
//   NLP            ACMP/NLPclass.cu: m = NJ*T*O + 28 (:45-46), bounds (:75-140), cost (:186-216,
//                  q_plan = q0 + 0.5 qd0 + k/8), collision rows then extrema (:221-330)
//   extrema        ACMP/Trajectory.cu:83-383 (braking at t_move = 0.5). The reference's gradient
//                  is taken with respect to k_actual = k_range * x, not x: kept as is.
//   finalize       ACMP/NLPclass.cu:358-452: the collision check covers links 0 .. NUM_FACTORS-2
//                  only (the loop bound of :375): kept as is.
//   solver         tolerance 1e-7 (ACMP/Parameters.h:42)
#pragma once
#include <vector>
#include "planner.h"

namespace oracle {

struct ArmtdPlanner : Planner {
    std::vector<double> tab;   // [joint][6][T]: c_cos, g_cos, r_cos, c_sin, g_sin, r_sin (armtd_main.cu:70-90)
    double kr[NF];             // k_range per joint (armtd_main.cu:89)

    ArmtdPlanner(const Robot& r, const Params& p, const double* q0, const double* qd0, const double* q_des,
                 const double* tables, const double* k_range, int num_obstacles, const double* obs);

    void reach() override;
    int m() const override { return NJ * T * O + NF * 4; }
    void bounds(double* g_l, double* g_u) const override;
    double eval_f(const double* x) const override;
    void eval_grad_f(const double* x, double* grad) const override;
    void eval_g_jac(const double* x, double* g, double* jac, double* link_center = nullptr) const override;
    bool feasible(const double* g) const override;

    void poly_zono(int t);                                         // Trajectory.cu:29-81
    void extremum(const double* k, double* ext, double* grad) const;  // Trajectory.cu:83-383 (grad: 28 x NF)
};

}  // namespace oracle
