// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// Restatement of KPR/Trajectory.cu. The degree-5 Bernstein trajectory with control points
// (q0, q0+Tqd0/5, q0+2Tqd0/5+TTqdd0/20, q0+k, q0+k, q0+k) is written in Bernstein form; the
// reference writes the same polynomials in expanded (MATLAB-codegen) form, so values agree to
// rounding. The k-derivatives of the interior extremum values (Trajectory.cu:601-810, MATLAB
// codegen) are restated through the envelope theorem: at an interior root t* of dq/dt,
// d/dk q(t*(k), k) = dq/dk(t*) = t*^3 (6 t*^2 - 15 t* + 10); at a root of d2q/dt2,
// d/dk qd(t*(k), k) = 30 t*^2 (t* - 1)^2. tests/test_oracle_properties.py checks both against
// finite differences (test_jacobian_matches_finite_differences, whose rows include the 28 extremum
// rows), and tests/test_oracle_containment.py checks the extremum values against a dense sampling
// of an independent Bezier point model (test_oracle_extremum_rows_bracket_the_trajectory).
#include "traj.h"
#include <algorithm>
#include <cmath>
#include <cstring>

namespace oracle {

// --- Bernstein trajectory (Trajectory.cu:542-599) ---
static inline void ctrl(double q0, double Tqd0, double TTqdd0, double k, double* b) {
    b[0] = q0;
    b[1] = q0 + Tqd0 / 5;
    b[2] = q0 + (2 * Tqd0) / 5 + TTqdd0 / 20;
    b[3] = q0 + k;
}

double q_des_func(double q0, double Tqd0, double TTqdd0, double k, double t) {
    double b[4];
    ctrl(q0, Tqd0, TTqdd0, k, b);
    const double u = 1.0 - t;
    const double u2 = u * u, t2 = t * t;
    const double B0 = u2 * u2 * u, B1 = 5 * t * u2 * u2, B2 = 10 * t2 * u2 * u;
    const double B345 = t2 * t * (10 * u2 + 5 * t * u + t2);
    return B0 * b[0] + B1 * b[1] + B2 * b[2] + B345 * b[3];
}

double qd_des_func(double q0, double Tqd0, double TTqdd0, double k, double t) {
    double b[4];
    ctrl(q0, Tqd0, TTqdd0, k, b);
    const double u = 1.0 - t;
    const double u2 = u * u;
    return 5 * (u2 * u2 * (b[1] - b[0]) + 4 * t * u2 * u * (b[2] - b[1]) + 6 * t * t * u2 * (b[3] - b[2]));
}

double qdd_des_func(double q0, double Tqd0, double TTqdd0, double k, double t) {
    double b[4];
    ctrl(q0, Tqd0, TTqdd0, k, b);
    const double u = 1.0 - t;
    return 20 * (u * u * u * (b[2] - 2 * b[1] + b[0]) + 3 * t * u * u * (b[3] - 2 * b[2] + b[1]) +
                 3 * t * t * u * (b[2] - b[3]));
}

// interior critical points of q(t) (roots of dq/dt besides t = 1), Trajectory.cu:263-264
static inline void q_roots(double Tqd0, double TTqdd0, double k, double* r2, double* r3) {
    const double disc = std::sqrt(64 * Tqd0 * Tqd0 + 14 * Tqd0 * TTqdd0 - 120 * k * Tqd0 + TTqdd0 * TTqdd0);
    const double den = 5 * (6 * Tqd0 - 12 * k + TTqdd0);
    *r2 = (2 * Tqd0 + TTqdd0 + disc) / den;
    *r3 = (2 * Tqd0 + TTqdd0 - disc) / den;
}
// interior critical points of qd(t) (roots of d2q/dt2), Trajectory.cu:406-407
static inline void qd_roots(double Tqd0, double TTqdd0, double k, double* r2, double* r3) {
    const double disc = std::sqrt(6 * (150 * k * k - 180 * k * Tqd0 - 20 * k * TTqdd0 + 54 * Tqd0 * Tqd0 +
                                       14 * Tqd0 * TTqdd0 + TTqdd0 * TTqdd0));
    const double den = 10 * (6 * Tqd0 - 12 * k + TTqdd0);
    *r2 = (18 * Tqd0 - 30 * k + 4 * TTqdd0 + disc) / den;
    *r3 = (18 * Tqd0 - 30 * k + 4 * TTqdd0 - disc) / den;
}
// interior critical points of qdd(t) at k = 0 (Trajectory.cu:54-55)
static inline void qdd_roots_k0(double Tqd0, double TTqdd0, double* r1, double* r2) {
    const double disc = std::sqrt(2 * (152 * Tqd0 * Tqd0 + 42 * Tqd0 * TTqdd0 + 3 * TTqdd0 * TTqdd0));
    const double den = 10 * (6 * Tqd0 + TTqdd0);
    *r1 = (32 * Tqd0 + 6 * TTqdd0 + disc) / den;
    *r2 = (32 * Tqd0 + 6 * TTqdd0 - disc) / den;
}

double q_des_extrema2_k_derivative(double q0, double Tqd0, double TTqdd0, double k) {
    double r2, r3;
    q_roots(Tqd0, TTqdd0, k, &r2, &r3);
    return r2 * r2 * r2 * (6 * r2 * r2 - 15 * r2 + 10);
}
double q_des_extrema3_k_derivative(double q0, double Tqd0, double TTqdd0, double k) {
    double r2, r3;
    q_roots(Tqd0, TTqdd0, k, &r2, &r3);
    return r3 * r3 * r3 * (6 * r3 * r3 - 15 * r3 + 10);
}
double qd_des_extrema2_k_derivative(double q0, double Tqd0, double TTqdd0, double k) {
    double r2, r3;
    qd_roots(Tqd0, TTqdd0, k, &r2, &r3);
    return 30 * r2 * r2 * (r2 - 1) * (r2 - 1);
}
double qd_des_extrema3_k_derivative(double q0, double Tqd0, double TTqdd0, double k) {
    double r2, r3;
    qd_roots(Tqd0, TTqdd0, k, &r2, &r3);
    return 30 * r3 * r3 * (r3 - 1) * (r3 - 1);
}

double q_des_k_indep(double q0, double Tqd0, double TTqdd0, double s) { return q_des_func(q0, Tqd0, TTqdd0, 0.0, s); }
double qd_des_k_indep(double q0, double Tqd0, double TTqdd0, double s, double D) { return qd_des_func(q0, Tqd0, TTqdd0, 0.0, s) / D; }
double qdd_des_k_indep(double q0, double Tqd0, double TTqdd0, double s, double D) { return qdd_des_func(q0, Tqd0, TTqdd0, 0.0, s) / (D * D); }

// Trajectory.cu:15-61
Bezier::Bezier(const Robot& r, const Params& p, const double* q0_, const double* qd0_, const double* qdd0_)
    : robot(&r), prm(&p), T(p.T) {
    for (int i = 0; i < NF; i++) {
        q0[i] = q0_[i]; qd0[i] = qd0_[i]; qdd0[i] = qdd0_[i];
        Tqd0[i] = qd0[i] * p.duration;
        TTqdd0[i] = qdd0[i] * p.duration * p.duration;
    }
    const int NJ = r.num_joints;
    cos_q_des.assign(NF * T, PZ());
    sin_q_des.assign(NF * T, PZ());
    R.assign((NJ + 1) * T, PZ());
    R_t.assign(NJ * T, PZ());
    qd_des.assign(NF * T, PZ());
    qda_des.assign(NF * T, PZ());
    qdda_des.assign(NF * T, PZ());
    const double D = p.duration;
    for (int i = 0; i < NF; i++) {
        q_roots(Tqd0[i], TTqdd0[i], 0.0, &q_ext1[i], &q_ext2[i]);
        q_extv1[i] = q_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], q_ext1[i]);
        q_extv2[i] = q_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], q_ext2[i]);
        qd_roots(Tqd0[i], TTqdd0[i], 0.0, &qd_ext1[i], &qd_ext2[i]);
        qd_extv1[i] = qd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], qd_ext1[i], D);
        qd_extv2[i] = qd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], qd_ext2[i], D);
        qdd_roots_k0(Tqd0[i], TTqdd0[i], &qdd_ext1[i], &qdd_ext2[i]);
        qdd_extv1[i] = qdd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], qdd_ext1[i], D);
        qdd_extv2[i] = qdd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], qdd_ext2[i], D);
    }
    ds = 1.0 / T;
}

// bound of a k-independent part over [s_lb, s_ub] given its two interior extrema
static inline void bound_k_indep(double vlb, double vub, double s_lb, double s_ub, double e1, double v1,
                                 double e2, double v2, double* lo, double* hi) {
    if (vlb > vub) std::swap(vlb, vub);
    if (s_lb < e1 && e1 < s_ub) { vlb = std::min(vlb, v1); vub = std::max(vub, v1); }
    if (s_lb < e2 && e2 < s_ub) { vlb = std::min(vlb, v2); vub = std::max(vub, v2); }
    *lo = vlb;
    *hi = vub;
}

// Trajectory.cu:63-254
void Bezier::makePolyZono(int s_ind) {
    const Robot& r = *robot;
    const double thr = prm->simplify_threshold;
    const double D = prm->duration;
    const double s_lb = s_ind * ds;
    const double s_ub = (s_ind + 1) * ds;
    const int t = s_ind;

    for (int i = 0; i < NF; i++) {
        const double kr = prm->k_range[i];

        // Part 1: q_des
        double kc_lb = s_lb * s_lb * s_lb * (6 * s_lb * s_lb - 15 * s_lb + 10);
        double kc_ub = s_ub * s_ub * s_ub * (6 * s_ub * s_ub - 15 * s_ub + 10);
        double kdc = (kc_ub + kc_lb) * 0.5;
        double kdr = (kc_ub - kc_lb) * 0.5 * kr;
        double ki_lb, ki_ub;
        bound_k_indep(q_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], s_lb), q_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], s_ub),
                      s_lb, s_ub, q_ext1[i], q_extv1[i], q_ext2[i], q_extv2[i], &ki_lb, &ki_ub);
        double kir = (ki_ub - ki_lb) * 0.5;
        const double qc = (ki_lb + ki_ub) * 0.5;
        const Interval qri(-kdr - kir - r.qe, kdr + kir + r.qe);
        const Interval kI(-kr, kr);

        // Part 1.a: cos(q_des), 2nd-order Taylor with interval remainder (:103-117)
        double cos_c = std::cos(qc);
        Interval cos_ri = (-qri) * std::sin(qc) - 0.5 * cos(qc + kdc * kI + qri) * pow(qri + kdc * kI, 2);
        cos_c += getCenter(cos_ri);
        cos_ri = cos_ri - getCenter(cos_ri);
        double cos_coeff[2] = {-kdc * kr * std::sin(qc), getRadius(cos_ri)};
        uint64_t cos_deg[2][NF * 6] = {{0}};
        cos_deg[0][i] = 1;
        cos_deg[1][i + NF * 4] = 1;
        cos_q_des[i * T + t] = PZ(cos_c, cos_coeff, cos_deg, 2, thr);

        // Part 1.b: sin(q_des) (:120-134)
        double sin_c = std::sin(qc);
        Interval sin_ri = qri * std::cos(qc) - 0.5 * sin(qc + kdc * kI + qri) * pow(qri + kdc * kI, 2);
        sin_c += getCenter(sin_ri);
        sin_ri = sin_ri - getCenter(sin_ri);
        double sin_coeff[2] = {kdc * kr * std::cos(qc), getRadius(sin_ri)};
        uint64_t sin_deg[2][NF * 6] = {{0}};
        sin_deg[0][i] = 1;
        sin_deg[1][i + NF * 5] = 1;
        sin_q_des[i * T + t] = PZ(sin_c, sin_coeff, sin_deg, 2, thr);

        PZ Ri = PZ::rpy(r.rots[i * 3], r.rots[i * 3 + 1], r.rots[i * 3 + 2]);
        if (r.axes[i] != 0) {
            PZ rz = PZ::rot(cos_c, cos_coeff, cos_deg, 2, sin_c, sin_coeff, sin_deg, 2, r.axes[i], thr);
            Ri = mul(Ri, rz, thr);
        }
        R[i * T + t] = Ri;
        R_t[i * T + t] = Ri.transpose();

        // Part 2: qd_des (:151-192); even-T bounding trick of the reference kept as is
        kc_lb = (30 * s_lb * s_lb * (s_lb - 1) * (s_lb - 1)) / D;
        kc_ub = (30 * s_ub * s_ub * (s_ub - 1) * (s_ub - 1)) / D;
        if (kc_ub < kc_lb) std::swap(kc_lb, kc_ub);
        kdc = (kc_ub + kc_lb) * 0.5 * kr;
        kdr = (kc_ub - kc_lb) * 0.5 * kr;
        bound_k_indep(qd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], s_lb, D), qd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], s_ub, D),
                      s_lb, s_ub, qd_ext1[i], qd_extv1[i], qd_ext2[i], qd_extv2[i], &ki_lb, &ki_ub);
        kir = (ki_ub - ki_lb) * 0.5;
        const double qdc = (ki_lb + ki_ub) * 0.5;
        double qd_coeff[2] = {kdc, kdr + kir + r.qde};
        uint64_t qd_deg[2][NF * 6] = {{0}};
        qd_deg[0][i] = 1;
        qd_deg[1][i + NF * 1] = 1;
        qd_des[i * T + t] = PZ(qdc, qd_coeff, qd_deg, 2, thr);
        double qda_coeff[2] = {kdc, kdr + kir + r.qdae};
        uint64_t qda_deg[2][NF * 6] = {{0}};
        qda_deg[0][i] = 1;
        qda_deg[1][i + NF * 2] = 1;
        qda_des[i * T + t] = PZ(qdc, qda_coeff, qda_deg, 2, thr);

        // Part 3: qdd_des (:195-244)
        const double MAXIMA = 0.5 - std::sqrt(3.0) / 6;
        const double MINIMA = 0.5 + std::sqrt(3.0) / 6;
        const double tmp_lb = (60 * s_lb * (2 * s_lb * s_lb - 3 * s_lb + 1)) / D / D;
        const double tmp_ub = (60 * s_ub * (2 * s_ub * s_ub - 3 * s_ub + 1)) / D / D;
        if (s_ub <= MAXIMA) { kc_lb = tmp_lb; kc_ub = tmp_ub; }
        else if (s_lb <= MAXIMA) { kc_lb = std::min(tmp_lb, tmp_ub); kc_ub = (60 * MAXIMA * (2 * MAXIMA * MAXIMA - 3 * MAXIMA + 1)) / D / D; }
        else if (s_ub <= MINIMA) { kc_lb = tmp_ub; kc_ub = tmp_lb; }
        else if (s_lb <= MINIMA) { kc_lb = (60 * MINIMA * (2 * MINIMA * MINIMA - 3 * MINIMA + 1)) / D / D; kc_ub = std::max(tmp_lb, tmp_ub); }
        else { kc_lb = tmp_lb; kc_ub = tmp_ub; }
        kdc = (kc_ub + kc_lb) * 0.5 * kr;
        kdr = (kc_ub - kc_lb) * 0.5 * kr;
        bound_k_indep(qdd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], s_lb, D), qdd_des_k_indep(q0[i], Tqd0[i], TTqdd0[i], s_ub, D),
                      s_lb, s_ub, qdd_ext1[i], qdd_extv1[i], qdd_ext2[i], qdd_extv2[i], &ki_lb, &ki_ub);
        kir = (ki_ub - ki_lb) * 0.5;
        const double qddc = (ki_lb + ki_ub) * 0.5;
        double qdd_coeff[2] = {kdc, kdr + kir + r.qddae};
        uint64_t qdd_deg[2][NF * 6] = {{0}};
        qdd_deg[0][i] = 1;
        qdd_deg[1][i + NF * 3] = 1;
        qdda_des[i * T + t] = PZ(qddc, qdd_coeff, qdd_deg, 2, thr);
    }

    // fixed joints at the end of the chain (:248-251)
    for (int i = NF; i < r.num_joints; i++) {
        R[i * T + t] = PZ::rpy(r.rots[i * 3], r.rots[i * 3 + 1], r.rots[i * 3 + 2]);
        R_t[i * T + t] = R[i * T + t].transpose();
    }
    R[r.num_joints * T + t] = PZ::rpy(0, 0, 0);
}

// extremum candidates: t = 0, two interior roots (if in [0,1]), t = 1
template <typename F>
static inline void extremum(F f, double e2, double e3, double* mn, double* mx, int* mnid, int* mxid) {
    const double v1 = f(0.0), v2 = f(e2), v3 = f(e3), v4 = f(1.0);
    if (v1 < v4) { *mn = v1; *mnid = 1; *mx = v4; *mxid = 4; }
    else { *mn = v4; *mnid = 4; *mx = v1; *mxid = 1; }
    if (0 <= e2 && e2 <= 1) {
        if (v2 < *mn) { *mn = v2; *mnid = 2; }
        if (*mx < v2) { *mx = v2; *mxid = 2; }
    }
    if (0 <= e3 && e3 <= 1) {
        if (v3 < *mn) { *mn = v3; *mnid = 3; }
        if (*mx < v3) { *mx = v3; *mxid = 3; }
    }
}

// Trajectory.cu:256-288 (min/max via std::min/max: identical values to the id-tracking form)
void Bezier::returnJointPositionExtremum(double* ext, const double* k) const {
    for (int i = 0; i < NF; i++) {
        const double ka = prm->k_range[i] * k[i];
        double e2, e3;
        q_roots(Tqd0[i], TTqdd0[i], ka, &e2, &e3);
        auto f = [&](double t) { return q_des_func(q0[i], Tqd0[i], TTqdd0[i], ka, t); };
        double mn, mx; int a, b;
        extremum(f, e2, e3, &mn, &mx, &a, &b);
        ext[i] = mn;
        ext[i + NF] = mx;
    }
}

// Trajectory.cu:290-397
void Bezier::returnJointPositionExtremumGradient(double* g, const double* k) const {
    for (int i = 0; i < NF; i++) {
        const double ka = prm->k_range[i] * k[i];
        double e2, e3;
        q_roots(Tqd0[i], TTqdd0[i], ka, &e2, &e3);
        auto f = [&](double t) { return q_des_func(q0[i], Tqd0[i], TTqdd0[i], ka, t); };
        double mn, mx; int mnid, mxid;
        extremum(f, e2, e3, &mn, &mx, &mnid, &mxid);
        auto grad = [&](int id) {
            switch (id) {
                case 1: return 0.0;
                case 2: return q_des_extrema2_k_derivative(q0[i], Tqd0[i], TTqdd0[i], ka);
                case 3: return q_des_extrema3_k_derivative(q0[i], Tqd0[i], TTqdd0[i], ka);
                default: return 1.0;
            }
        };
        const double gmn = grad(mnid), gmx = grad(mxid);
        for (int j = 0; j < NF; j++) {
            g[i * NF + j] = (i == j) ? gmn * prm->k_range[i] : 0.0;
            g[(i + NF) * NF + j] = (i == j) ? gmx * prm->k_range[i] : 0.0;
        }
    }
}

// Trajectory.cu:399-431
void Bezier::returnJointVelocityExtremum(double* ext, const double* k) const {
    for (int i = 0; i < NF; i++) {
        const double ka = prm->k_range[i] * k[i];
        double e2, e3;
        qd_roots(Tqd0[i], TTqdd0[i], ka, &e2, &e3);
        auto f = [&](double t) { return qd_des_func(q0[i], Tqd0[i], TTqdd0[i], ka, t); };
        double mn, mx; int a, b;
        extremum(f, e2, e3, &mn, &mx, &a, &b);
        ext[i] = mn / prm->duration;
        ext[i + NF] = mx / prm->duration;
    }
}

// Trajectory.cu:433-540
void Bezier::returnJointVelocityExtremumGradient(double* g, const double* k) const {
    for (int i = 0; i < NF; i++) {
        const double ka = prm->k_range[i] * k[i];
        double e2, e3;
        qd_roots(Tqd0[i], TTqdd0[i], ka, &e2, &e3);
        auto f = [&](double t) { return qd_des_func(q0[i], Tqd0[i], TTqdd0[i], ka, t); };
        double mn, mx; int mnid, mxid;
        extremum(f, e2, e3, &mn, &mx, &mnid, &mxid);
        auto grad = [&](int id) {
            switch (id) {
                case 1: return 0.0;
                case 2: return qd_des_extrema2_k_derivative(q0[i], Tqd0[i], TTqdd0[i], ka);
                case 3: return qd_des_extrema3_k_derivative(q0[i], Tqd0[i], TTqdd0[i], ka);
                default: return 1.0;
            }
        };
        const double gmn = grad(mnid), gmx = grad(mxid);
        for (int j = 0; j < NF; j++) {
            g[i * NF + j] = (i == j) ? gmn * prm->k_range[i] / prm->duration : 0.0;
            g[(i + NF) * NF + j] = (i == j) ? gmx * prm->k_range[i] / prm->duration : 0.0;
        }
    }
}

}  // namespace oracle
