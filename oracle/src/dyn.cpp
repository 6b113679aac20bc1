// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// Restatement of KPR/Dynamics.cu. Operation order (and therefore every simplify() point) is
// the reference's: left-to-right evaluation of each '+' chain, cross() products through stack().
#include "dyn.h"
#include <cstdlib>

namespace oracle {

KinDyn::KinDyn(Bezier* tr) : traj(tr), robot(tr->robot), thr(tr->prm->simplify_threshold), T(tr->T), NJ(tr->robot->num_joints) {
    const Robot& r = *robot;
    for (int i = 0; i < (NJ + 1) * 3; i++) trans[i] = r.trans[i];
    for (int i = 0; i < NJ * 3; i++) com[i] = r.com[i];
    mass_nom.resize(NJ); mass_unc.resize(NJ); I_nom.resize(NJ); I_unc.resize(NJ);
    for (int i = 0; i < NJ; i++) {
        double m = r.mass[i];
        mass_nom[i] = PZ(1, 1, &m);
        mass_unc[i] = PZ(1, 1, &m, r.mass_uncertainty);
        // Dynamics.cu:85-88 fills a column-major Matrix3d linearly from inertia[i*9 + j]
        I_nom[i] = PZ(3, 3, &r.inertia[i * 9]);
        I_unc[i] = PZ(3, 3, &r.inertia[i * 9], r.inertia_uncertainty);
    }
    u_nom.assign(NF * T, PZ());
    u_nom_int.assign(NF * T, PZ());
    // link box PZs: generators on the qde_0 / qdae_0 / qddae_0 slots (Dynamics.cu:98-116)
    links.assign(NJ * T, PZ());
    for (int i = 0; i < NJ; i++) {
        PZ comp[3];
        for (int j = 0; j < 3; j++) {
            uint64_t degree[1][NF * 6] = {{0}};
            degree[0][NF * (j + 1)] = 1;
            double g = r.link_g[i][j];
            comp[j] = PZ(r.link_c[i][j], &g, degree, 1, thr);
        }
        PZ box = stack3(comp[0], comp[1], comp[2], thr);
        for (int t = 0; t < T; t++) links[i * T + t] = box;
    }
}

// Dynamics.cu:69-81
void KinDyn::fk(int t) {
    PZ FK_R = PZ::rpy(0, 0, 0);
    PZ FK_T(3, 1);
    for (int i = 0; i < NJ; i++) {
        PZ P(3, 1, &trans[3 * i]);
        FK_T = add(FK_T, mul(FK_R, P, thr), thr);
        FK_R = mul(FK_R, traj->R[i * T + t], thr);
        links[i * T + t] = add(mul(FK_R, links[i * T + t], thr), FK_T, thr);
    }
}

// Dynamics.cu:83-181
void KinDyn::rnea(int t, const std::vector<PZ>& mass_arr, const std::vector<PZ>& I_arr, std::vector<PZ>& u, bool setGravity) {
    const Robot& r = *robot;
    PZ w(3, 1), wdot(3, 1), w_aux(3, 1), linear_acc(3, 1);
    std::vector<PZ> F(NJ), N(NJ);
    if (setGravity) linear_acc.center[2] = r.gravity;

    for (int i = 0; i < NJ; i++) {
        const PZ& Rt = traj->R_t[i * T + t];
        const double* p = &trans[3 * i];
        // line 16: linear_acc = R_t * (linear_acc + cross(wdot, p) + cross(w, cross(w_aux, p)))
        PZ s1 = add(linear_acc, cross_pm(wdot, p, thr), thr);
        PZ s2 = add(s1, cross_pp(w, cross_pm(w_aux, p, thr), thr), thr);
        linear_acc = mul(Rt, s2, thr);
        // line 13
        w = mul(Rt, w, thr);
        if (r.axes[i] != 0) {
            const int ax = std::abs(r.axes[i]) - 1;
            w.addOneDimPZ(traj->qd_des[i * T + t], ax, 0, thr);
            // line 14
            w_aux = mul(Rt, w_aux, thr);
            // line 15
            wdot = mul(Rt, wdot, thr);
            PZ temp(3, 1);
            temp.addOneDimPZ(traj->qd_des[i * T + t], ax, 0, thr);
            wdot = add(wdot, cross_pp(w_aux, temp, thr), thr);
            wdot.addOneDimPZ(traj->qdda_des[i * T + t], ax, 0, thr);
            w_aux.addOneDimPZ(traj->qda_des[i * T + t], ax, 0, thr);
        } else {
            w_aux = mul(Rt, w_aux, thr);
            wdot = mul(Rt, wdot, thr);
        }
        // line 23 & 27
        const double* c = &com[3 * i];
        PZ f1 = add(linear_acc, cross_pm(wdot, c, thr), thr);
        PZ f2 = add(f1, cross_pp(w, cross_pm(w_aux, c, thr), thr), thr);
        F[i] = mul(mass_arr[i], f2, thr);
        // line 29
        N[i] = add(mul(I_arr[i], wdot, thr), cross_pp(w_aux, mul(I_arr[i], w, thr), thr), thr);
    }

    PZ f(3, 1), n(3, 1);
    for (int i = NJ - 1; i >= 0; i--) {
        const PZ& R1 = traj->R[(i + 1) * T + t];
        const double* p1 = &trans[3 * (i + 1)];
        // line 29: n = N + R*n + cross(com, F) + cross(p_{i+1}, R*f)
        PZ n1 = add(N[i], mul(R1, n, thr), thr);
        PZ n2 = add(n1, cross_mp(&com[3 * i], F[i], thr), thr);
        n = add(n2, cross_mp(p1, mul(R1, f, thr), thr), thr);
        // line 28
        f = add(mul(R1, f, thr), F[i], thr);
        if (r.axes[i] != 0) {
            PZ ui = n.elem(std::abs(r.axes[i]) - 1, 0);
            ui = add(ui, scale(r.armature[i], traj->qdda_des[i * T + t]), thr);
            ui = add(ui, scale(r.damping[i], traj->qd_des[i * T + t]), thr);
            u[i * T + t] = ui;
        }
    }
}

}  // namespace oracle
