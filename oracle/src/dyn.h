// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// Restatement of class KinematicsDynamics (KPR/Dynamics.h:6-48, KPR/Dynamics.cu:6-181).
#pragma once
#include <vector>
#include "traj.h"

namespace oracle {

struct KinDyn {
    Bezier* traj;
    const Robot* robot;
    double thr;
    int T, NJ;
    double trans[(MAX_J + 1) * 3];
    double com[MAX_J * 3];
    std::vector<PZ> mass_nom, mass_unc, I_nom, I_unc;  // [joint]
    std::vector<PZ> links;                             // [joint * T + t]
    std::vector<PZ> u_nom, u_nom_int;                  // [factor * T + t]

    explicit KinDyn(Bezier* traj);                     // Dynamics.cu:6-67
    void fk(int t);                                    // :69-81
    void rnea(int t, const std::vector<PZ>& mass_arr, const std::vector<PZ>& I_arr,
              std::vector<PZ>& u, bool setGravity = true);  // :83-181
    void rnea_nominal(int t) { rnea(t, mass_nom, I_nom, u_nom); }
    void rnea_interval(int t) { rnea(t, mass_unc, I_unc, u_nom_int); }
};

}  // namespace oracle
