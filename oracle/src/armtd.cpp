// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// Restatement of the ARMTD comparison planner (ACMP/ = kinova_planner_realtime_armtd_comparison/),
// see armtd.h for the map of what follows which reference lines.
#include "armtd.h"
#include <cmath>
#include <cstring>
#include <stdexcept>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle {

static const double ZERO7[NF] = {0, 0, 0, 0, 0, 0, 0};

ArmtdPlanner::ArmtdPlanner(const Robot& r, const Params& p, const double* q0_, const double* qd0_, const double* q_des_,
                           const double* tables, const double* k_range, int num_obstacles, const double* obs)
    : Planner(r, p, q0_, qd0_, ZERO7, q_des_, num_obstacles, obs) {
    tab.assign(tables, tables + (size_t)NF * 6 * T);
    for (int i = 0; i < NF; i++) kr[i] = k_range[i];
    tol = 1e-7;  // IPOPT_OPTIMIZATION_TOLERANCE (ACMP/Parameters.h:42)
}

// ACMP/Trajectory.cu:29-81: the offline JRS of cos / sin of the relative joint angle, rotated by q0
// (cos(q0 + a) = cos q0 cos a - sin q0 sin a, ...); the radius term is scaled by 5 (:43, :56)
void ArmtdPlanner::poly_zono(int t) {
    const double thr = prm.simplify_threshold;
    const Robot& r = robot;
    for (int i = 0; i < NF; i++) {
        const double* tb = &tab[(size_t)i * 6 * T];
        const double c_cos = tb[0 * T + t], g_cos = tb[1 * T + t], r_cos = tb[2 * T + t];
        const double c_sin = tb[3 * T + t], g_sin = tb[4 * T + t], r_sin = tb[5 * T + t];
        const double cq = std::cos(q0[i]), sq = std::sin(q0[i]);

        const double cos_c = cq * c_cos - sq * c_sin;
        double cos_coeff[2];
        cos_coeff[0] = cq * g_cos - sq * g_sin;
        cos_coeff[1] = std::fabs(cq) * r_cos + std::fabs(sq) * r_sin;
        cos_coeff[1] *= 5.0;
        uint64_t cos_deg[2][NF * 6] = {{0}};
        cos_deg[0][i] = 1;            // k
        cos_deg[1][i + NF * 4] = 1;   // cosqe

        const double sin_c = cq * c_sin + sq * c_cos;
        double sin_coeff[2];
        sin_coeff[0] = cq * g_sin + sq * g_cos;
        sin_coeff[1] = std::fabs(cq) * r_sin + std::fabs(sq) * r_cos;
        sin_coeff[1] *= 5.0;
        uint64_t sin_deg[2][NF * 6] = {{0}};
        sin_deg[0][i] = 1;            // k
        sin_deg[1][i + NF * 5] = 1;   // sinqe

        traj->cos_q_des[i * T + t] = PZ(cos_c, cos_coeff, cos_deg, 2, thr);
        traj->sin_q_des[i * T + t] = PZ(sin_c, sin_coeff, sin_deg, 2, thr);
        PZ Ri = PZ::rpy(r.rots[i * 3], r.rots[i * 3 + 1], r.rots[i * 3 + 2]);
        if (r.axes[i] != 0) {
            PZ rz = PZ::rot(cos_c, cos_coeff, cos_deg, 2, sin_c, sin_coeff, sin_deg, 2, r.axes[i], thr);
            Ri = mul(Ri, rz, thr);
        }
        traj->R[i * T + t] = Ri;
        traj->R_t[i * T + t] = Ri.transpose();
    }
    for (int i = NF; i < NJ; i++) {  // fixed joints at the end of the chain (:75-78)
        traj->R[i * T + t] = PZ::rpy(r.rots[i * 3], r.rots[i * 3 + 1], r.rots[i * 3 + 2]);
        traj->R_t[i * T + t] = traj->R[i * T + t].transpose();
    }
}

// ACMP/armtd_main.cu:113-164: JRS, FK + reduce_link_PZ, hyperplanes (no RNEA)
void ArmtdPlanner::reach() {
    traj = new Bezier(robot, prm, q0, qd0, qdd0);  // holds the R / R_t arrays (its curve is unused)
#pragma omp parallel for num_threads(num_threads) schedule(dynamic, 1)
    for (int t = 0; t < T; t++) poly_zono(t);
    kd = new KinDyn(traj);
    link_gens.assign((size_t)T * NJ * 18, 0.0);
#pragma omp parallel for num_threads(num_threads) schedule(dynamic)
    for (int t = 0; t < T; t++) {
        kd->fk(t);
        for (int i = 0; i < NJ; i++) kd->links[i * T + t].reduce_link_PZ(&link_gens[((size_t)t * NJ + i) * 18]);
    }
    torque_radius.assign((size_t)T * NF, 0.0);
    buffer_obstacles();
}

// ACMP/NLPclass.cu:75-140
void ArmtdPlanner::bounds(double* g_l, double* g_u) const {
    int off = 0;
    for (int i = 0; i < NJ * T * O; i++) { g_l[i] = -1e19; g_u[i] = 0; }
    off += NJ * T * O;
    for (int rep = 0; rep < 2; rep++) {
        for (int i = 0; i < NF; i++) { g_l[off + i] = robot.state_lb[i] + robot.qe; g_u[off + i] = robot.state_ub[i] - robot.qe; }
        off += NF;
    }
    for (int rep = 0; rep < 2; rep++) {
        for (int i = 0; i < NF; i++) { g_l[off + i] = -robot.speed_limits[i] + robot.qde; g_u[off + i] = robot.speed_limits[i] - robot.qde; }
        off += NF;
    }
}

static double wrap_pi(double a) {  // ACMP/NLPclass.cu:6-15
    double w = a;
    while (w < -M_PI) w += 2 * M_PI;
    while (w > M_PI) w -= 2 * M_PI;
    return w;
}

// ACMP/NLPclass.cu:186-216: q_plan = q0 + qd0 * 0.5 + k_range * x * 0.125; the four continuous
// joints (0, 2, 4, 6 on the Kinova: the robot's wrap mask) wrapped and summed first
double ArmtdPlanner::eval_f(const double* x) const {
    double qp[NF];
    for (int i = 0; i < NF; i++) qp[i] = q0[i] + qd0[i] * 0.5 + kr[i] * x[i] * 0.125;
    double f = 0.0;
    bool first = true;
    for (int pass = 1; pass >= 0; pass--)
        for (int i = 0; i < NF; i++) {
            if (robot.wrap_mask[i] != pass) continue;
            const double d = pass ? wrap_pi(q_des[i] - qp[i]) : (q_des[i] - qp[i]);
            const double term = std::pow(d, 2);
            f = first ? term : f + term;
            first = false;
        }
    return f * prm.cost_scale;
}

// ACMP/NLPclass.cu:221-246
void ArmtdPlanner::eval_grad_f(const double* x, double* grad) const {
    for (int i = 0; i < NF; i++) {
        const double qp = q0[i] + qd0[i] * 0.5 + kr[i] * x[i] * 0.125;
        const double dk = kr[i] * 0.125;
        grad[i] = robot.wrap_mask[i] ? (2 * wrap_pi(qp - q_des[i]) * dk) : (2 * (qp - q_des[i]) * dk);
        grad[i] *= prm.cost_scale;
    }
}

// ACMP/Trajectory.cu:83-383 (value and, when grad is not null, the reference's gradient rows)
void ArmtdPlanner::extremum(const double* k, double* ext, double* grad) const {
    const double t_move = 0.5, t_total = 1.0, t_to_stop = t_total - t_move;
    if (grad) std::memset(grad, 0, sizeof(double) * 4 * NF * NF);
    for (int i = 0; i < NF; i++) {
        const double k_actual = kr[i] * k[i];
        const double q_peak = q0[i] + qd0[i] * t_move + k_actual * t_move * t_move * 0.5;
        const double q_dot_peak = qd0[i] + k_actual * t_move;
        const double q_ddot_to_stop = -q_dot_peak / t_to_stop;
        const double q_stop = q_peak + q_dot_peak * t_to_stop + 0.5 * q_ddot_to_stop * t_to_stop * t_to_stop;
        const double t_mm = -qd0[i] / k_actual;
        double q_max_tp, q_min_tp, qd_max_tp, qd_min_tp, g_q_max_tp, g_q_min_tp, g_qd_max_tp, g_qd_min_tp;
        double q_max_ts, q_min_ts, qd_max_ts, qd_min_ts, g_q_max_ts, g_q_min_ts, g_qd_max_ts, g_qd_min_ts;
        double qe_o[2], gqe_o[2];
        if (q_peak >= q0[i]) {
            qe_o[0] = q0[i]; qe_o[1] = q_peak; gqe_o[0] = 0; gqe_o[1] = 0.5 * t_move * t_move;
        } else {
            qe_o[0] = q_peak; qe_o[1] = q0[i]; gqe_o[0] = 0.5 * t_move * t_move; gqe_o[1] = 0;
        }
        if (t_mm > 0 && t_mm < t_move) {
            if (k_actual >= 0) {
                q_min_tp = q0[i] + qd0[i] * t_mm + 0.5 * k_actual * t_mm * t_mm;
                q_max_tp = qe_o[1];
                g_q_min_tp = (0.5 * qd0[i] * qd0[i]) / (k_actual * k_actual);
                g_q_max_tp = gqe_o[1];
            } else {
                q_min_tp = qe_o[0];
                q_max_tp = q0[i] + qd0[i] * t_mm + 0.5 * k_actual * t_mm * t_mm;
                g_q_min_tp = gqe_o[0];
                g_q_max_tp = (0.5 * qd0[i] * qd0[i]) / (k_actual * k_actual);
            }
        } else {
            q_min_tp = qe_o[0]; q_max_tp = qe_o[1];
            g_q_min_tp = gqe_o[0]; g_q_max_tp = gqe_o[1];
        }
        if (q_dot_peak >= qd0[i]) {
            qd_min_tp = qd0[i]; qd_max_tp = q_dot_peak; g_qd_min_tp = 0; g_qd_max_tp = t_move;
        } else {
            qd_min_tp = q_dot_peak; qd_max_tp = qd0[i]; g_qd_min_tp = t_move; g_qd_max_tp = 0;
        }
        if (q_stop >= q_peak) {
            q_min_ts = q_peak; q_max_ts = q_stop;
            g_q_min_ts = 0.5 * t_move * t_move; g_q_max_ts = 0.5 * t_move * t_move + 0.5 * t_move * t_to_stop;
        } else {
            q_min_ts = q_stop; q_max_ts = q_peak;
            g_q_min_ts = 0.5 * t_move * t_move + 0.5 * t_move * t_to_stop; g_q_max_ts = 0.5 * t_move * t_move;
        }
        if (q_dot_peak >= 0) {
            qd_min_ts = 0; qd_max_ts = q_dot_peak; g_qd_min_ts = 0; g_qd_max_ts = t_move;
        } else {
            qd_min_ts = q_dot_peak; qd_max_ts = 0; g_qd_min_ts = t_move; g_qd_max_ts = 0;
        }
        const bool a = q_min_tp <= q_min_ts, b = q_max_tp >= q_max_ts;
        const bool c = qd_min_tp <= qd_min_ts, d = qd_max_tp >= qd_max_ts;
        ext[i] = a ? q_min_tp : q_min_ts;
        ext[i + NF] = b ? q_max_tp : q_max_ts;
        ext[i + 2 * NF] = c ? qd_min_tp : qd_min_ts;
        ext[i + 3 * NF] = d ? qd_max_tp : qd_max_ts;
        if (grad) {
            grad[i * NF + i] = a ? g_q_min_tp : g_q_min_ts;
            grad[(i + NF) * NF + i] = b ? g_q_max_tp : g_q_max_ts;
            grad[(i + 2 * NF) * NF + i] = c ? g_qd_min_tp : g_qd_min_ts;
            grad[(i + 3 * NF) * NF + i] = d ? g_qd_max_tp : g_qd_max_ts;
        }
    }
}

// ACMP/NLPclass.cu:252-330: link slices, collision rows from offset 0, extrema after them
void ArmtdPlanner::eval_g_jac(const double* x, double* g, double* jac, double* link_center_out) const {
    std::vector<double> lc((size_t)T * NJ * 3), dlc(jac ? (size_t)T * NJ * NF * 3 : 0);
#pragma omp parallel for num_threads(num_threads) schedule(dynamic)
    for (int t = 0; t < T; t++)
        for (int l = 0; l < NJ; l++)
            link_slice(t, l, x, &lc[((size_t)t * NJ + l) * 3], jac ? &dlc[((size_t)t * NJ + l) * NF * 3] : nullptr);
#pragma omp parallel for num_threads(num_threads) schedule(static) collapse(2)
    for (int l = 0; l < NJ; l++)
        for (int t = 0; t < T; t++)
            for (int o = 0; o < O; o++) {
                const size_t row = ((size_t)l * T + t) * O + o;
                collision_row(t, l, o, &lc[((size_t)t * NJ + l) * 3], jac ? &dlc[((size_t)t * NJ + l) * NF * 3] : nullptr,
                              &g[row], jac ? &jac[row * NF] : nullptr);
            }
    const size_t off = (size_t)T * NJ * O;
    extremum(x, &g[off], jac ? &jac[off * NF] : nullptr);
    if (link_center_out) std::memcpy(link_center_out, lc.data(), lc.size() * sizeof(double));
}

// ACMP/NLPclass.cu:358-452
bool ArmtdPlanner::feasible(const double* g) const {
    int off = 0;
    for (int i = 0; i < NF - 1; i++)  // links 0 .. NUM_FACTORS-2 (:375)
        for (int j = 0; j < T; j++)
            for (int h = 0; h < O; h++)
                if (g[(i * T + j) * O + h + off] > prm.collision_violation) return false;
    off += NJ * T * O;
    for (int rep = 0; rep < 2; rep++) {
        for (int i = off; i < off + NF; i++)
            if (g[i] < robot.state_lb[i - off] + robot.qe || g[i] > robot.state_ub[i - off] - robot.qe) return false;
        off += NF;
    }
    for (int rep = 0; rep < 2; rep++) {
        for (int i = off; i < off + NF; i++)
            if (g[i] < -robot.speed_limits[i - off] + robot.qde || g[i] > robot.speed_limits[i - off] - robot.qde) return false;
        off += NF;
    }
    return true;
}

}  // namespace oracle
