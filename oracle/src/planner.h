// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
//
// One ARMOUR planning iteration restated on the CPU:
//   reach():  JRS (Trajectory.cu:63-254) -> FK + reduce_link_PZ + RNEA nominal/interval +
//             disturbance + reduce (armour_main.cu:97-143) -> torque radius (:173-211) ->
//             buffered-obstacle hyperplanes (CollisionChecking.cu:136-228, as CPU loops)
//   eval_*(): the armtd_NLP callbacks (NLPclass.cu:62-417), with the GPU collision kernel
//             (CollisionChecking.cu:230-299) as CPU loops
//   feasible(): finalize_solution's re-check (NLPclass.cu:422-538)
#pragma once
#include <vector>
#include "dyn.h"

namespace oracle {

struct Planner {
    Robot robot;
    Params prm;
    int T, NJ, O;
    double q0[NF], qd0[NF], qdd0[NF], q_des[NF];
    std::vector<double> obstacles;   // O * 12 : center, g1, g2, g3 (armour_main.cu:73-77)
    Bezier* traj = nullptr;
    KinDyn* kd = nullptr;
    std::vector<double> link_gens;   // [(t*NJ + l) * 18], Eigen 3x6 column-major (armour_main.cu:114)
    std::vector<double> torque_radius;  // [t * NF + j]  (== Eigen (NF x T) column-major)
    std::vector<double> hA, hd, hdelta;  // hyperplanes [((t*NJ + l)*O + o)*COMB + p] (CollisionChecking.cu:283-295)
    int num_threads = 1;

    double tol = 1e-4;                // the solver's tolerance (IPOPT_OPTIMIZATION_TOLERANCE, Parameters.h:50)

    Planner(const Robot& r, const Params& p, const double* q0, const double* qd0, const double* qdd0,
            const double* q_des, int num_obstacles, const double* obs);
    virtual ~Planner();

    virtual void reach();             // armour_main.cu:97-222
    void buffer_obstacles();          // CollisionChecking.cu:136-228 (part of reach())
    // test tooling: replace the obstacle set after reach() (the reach sets do not depend on it)
    void set_obstacles(int num_obstacles, const double* obs);
    virtual int m() const { return NF * T + NJ * T * O + NF * 4; }  // NLPclass.cu:47-49
    virtual void bounds(double* g_l, double* g_u) const;              // NLPclass.cu:87-165
    virtual double eval_f(const double* x) const;                     // :207-236
    virtual void eval_grad_f(const double* x, double* grad) const;    // :241-267
    // eval_g and eval_jac_g (:272-396); jac may be null; also returns sliced link centres
    virtual void eval_g_jac(const double* x, double* g, double* jac, double* link_center = nullptr) const;
    virtual bool feasible(const double* g) const;                     // :449-538

    // pieces exposed for parity tests
    void link_slice(int t, int l, const double* x, double* c3, double* grad21) const;
    void torque_slice(int t, int j, const double* x, double* val, double* grad7) const;
    void collision_row(int t, int l, int o, const double* c3, const double* dc21, double* g, double* grad7) const;
};

}  // namespace oracle
