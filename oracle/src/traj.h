// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// Restatement of class BezierCurve (KPR/Trajectory.h:32-95, KPR/Trajectory.cu:15-822).
#pragma once
#include <vector>
#include "pz.h"

namespace oracle {

double q_des_func(double q0, double Tqd0, double TTqdd0, double k, double t);      // Trajectory.cu:542
double qd_des_func(double q0, double Tqd0, double TTqdd0, double k, double t);     // :558
double qdd_des_func(double q0, double Tqd0, double TTqdd0, double k, double t);    // :574
double q_des_extrema2_k_derivative(double q0, double Tqd0, double TTqdd0, double k);   // :601
double q_des_extrema3_k_derivative(double q0, double Tqd0, double TTqdd0, double k);   // :644
double qd_des_extrema2_k_derivative(double q0, double Tqd0, double TTqdd0, double k);  // :687
double qd_des_extrema3_k_derivative(double q0, double Tqd0, double TTqdd0, double k);  // :749
double q_des_k_indep(double q0, double Tqd0, double TTqdd0, double s);    // :812
double qd_des_k_indep(double q0, double Tqd0, double TTqdd0, double s, double duration);   // :816
double qdd_des_k_indep(double q0, double Tqd0, double TTqdd0, double s, double duration);  // :820

struct Bezier {
    const Robot* robot;
    const Params* prm;
    int T;
    double q0[NF], qd0[NF], qdd0[NF], Tqd0[NF], TTqdd0[NF];
    double q_ext1[NF], q_ext2[NF], q_extv1[NF], q_extv2[NF];
    double qd_ext1[NF], qd_ext2[NF], qd_extv1[NF], qd_extv2[NF];
    double qdd_ext1[NF], qdd_ext2[NF], qdd_extv1[NF], qdd_extv2[NF];
    double ds;
    // PZ arrays indexed [joint * T + t]
    std::vector<PZ> cos_q_des, sin_q_des, R, R_t, qd_des, qda_des, qdda_des;

    Bezier(const Robot& r, const Params& p, const double* q0, const double* qd0, const double* qdd0);  // :15-61
    void makePolyZono(int s_ind);                                                   // :63-254
    PZ& Rz(int i, int t) { return R[i * T + t]; }
    void returnJointPositionExtremum(double* ext, const double* k) const;           // :256-288
    void returnJointPositionExtremumGradient(double* g, const double* k) const;     // :290-397
    void returnJointVelocityExtremum(double* ext, const double* k) const;           // :399-431
    void returnJointVelocityExtremumGradient(double* g, const double* k) const;     // :433-540
};

}  // namespace oracle
