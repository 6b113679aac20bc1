// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
#include "planner.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle {

Planner::Planner(const Robot& r, const Params& p, const double* q0_, const double* qd0_, const double* qdd0_,
                 const double* q_des_, int num_obstacles, const double* obs)
    : robot(r), prm(p), T(p.T), NJ(r.num_joints), O(num_obstacles) {
    if (O < 0 || O > MAX_OBS) throw std::runtime_error("Number of obstacles out of range");
    for (int i = 0; i < NF; i++) { q0[i] = q0_[i]; qd0[i] = qd0_[i]; qdd0[i] = qdd0_[i]; q_des[i] = q_des_[i]; }
    obstacles.assign(obs, obs + O * (OBS_GEN + 1) * 3);
}

Planner::~Planner() {
    delete kd;
    delete traj;
}

void Planner::reach() {
    traj = new Bezier(robot, prm, q0, qd0, qdd0);
    // armour_main.cu:97-104
#pragma omp parallel for num_threads(num_threads) schedule(dynamic, 1)
    for (int t = 0; t < T; t++) traj->makePolyZono(t);

    // armour_main.cu:113-143
    kd = new KinDyn(traj);
    link_gens.assign((size_t)T * NJ * 18, 0.0);
#pragma omp parallel for num_threads(num_threads) schedule(dynamic)
    for (int t = 0; t < T; t++) {
        kd->fk(t);
        for (int i = 0; i < NJ; i++) kd->links[i * T + t].reduce_link_PZ(&link_gens[((size_t)t * NJ + i) * 18]);
        kd->rnea_nominal(t);
        kd->rnea_interval(t);
        for (int i = 0; i < NF; i++)
            kd->u_nom_int[i * T + t] = sub(kd->u_nom_int[i * T + t], kd->u_nom[i * T + t], prm.simplify_threshold);
        for (int i = 0; i < NF; i++) kd->u_nom[i * T + t].reduce();
    }

    // armour_main.cu:173-211
    torque_radius.assign((size_t)T * NF, 0.0);
    const double ub_const = robot.alpha * (robot.M_max - robot.M_min) * robot.eps;
    for (int t = 0; t < T; t++) {
        Interval rho(0.0);
        for (int i = 0; i < NF; i++) {
            double lo, hi;
            kd->u_nom_int[i * T + t].toInterval(&lo, &hi);
            const Interval tmp(lo, hi);
            rho += tmp * tmp;
            torque_radius[t * NF + i] = ub_const + 0.5 * std::max(std::fabs(tmp.lower()), std::fabs(tmp.upper()));
        }
        rho = sqrt(rho);
        for (int i = 0; i < NF; i++) torque_radius[t * NF + i] += 0.5 * rho.upper();
        for (int i = 0; i < NF; i++) torque_radius[t * NF + i] += kd->u_nom[i * T + t].indep[0];
        for (int i = 0; i < NF; i++) torque_radius[t * NF + i] += robot.friction[i];
    }

    buffer_obstacles();
}

// CollisionChecking.cu:26-39 pair tables; :136-228 buffer + polytope_PH as CPU loops. Depends on
// the link generators of reach() and the obstacles only, so set_obstacles() can rerun it alone.
void Planner::buffer_obstacles() {
    int combA[COMB], combB[COMB];
    {
        int a = 0, b = 1;
        for (int i = 0; i < COMB; i++) {
            combA[i] = a; combB[i] = b;
            if (b < BUF_GEN - 1) b++;
            else { a++; b = a + 1; }
        }
    }
    const size_t nh = (size_t)T * NJ * O * COMB;
    hA.assign(nh * 3, 0.0);
    hd.assign(nh, 0.0);
    hdelta.assign(nh, 0.0);
#pragma omp parallel for num_threads(num_threads) schedule(static)
    for (int t = 0; t < T; t++) {
        for (int l = 0; l < NJ; l++) {
            const double* lg = &link_gens[((size_t)t * NJ + l) * 18];
            for (int o = 0; o < O; o++) {
                const double* ob = &obstacles[(size_t)o * 12];
                double G[BUF_GEN][3];
                for (int i = 0; i < OBS_GEN; i++)
                    for (int r = 0; r < 3; r++) G[i][r] = ob[(i + 1) * 3 + r];
                for (int i = 0; i < 6; i++)
                    for (int r = 0; r < 3; r++) G[OBS_GEN + i][r] = lg[r + 3 * i];
                const double* c = ob;
                for (int p = 0; p < COMB; p++) {
                    const int a = combA[p], b = combB[p];
                    double gc[3];
                    gc[0] = G[a][1] * G[b][2] - G[a][2] * G[b][1];
                    gc[1] = G[a][2] * G[b][0] - G[a][0] * G[b][2];
                    gc[2] = G[a][0] * G[b][1] - G[a][1] * G[b][0];
                    const double nrm = std::sqrt(gc[0] * gc[0] + gc[1] * gc[1] + gc[2] * gc[2]);
                    double C[3] = {0, 0, 0};
                    if (nrm > 0) { C[0] = gc[0] / nrm; C[1] = gc[1] / nrm; C[2] = gc[2] / nrm; }
                    const size_t idx = (((size_t)t * NJ + l) * O + o) * COMB + p;
                    hA[idx * 3 + 0] = C[0]; hA[idx * 3 + 1] = C[1]; hA[idx * 3 + 2] = C[2];
                    hd[idx] = C[0] * c[0] + C[1] * c[1] + C[2] * c[2];
                    double del = 0.0;
                    for (int j = 0; j < BUF_GEN; j++) del += std::fabs(C[0] * G[j][0] + C[1] * G[j][1] + C[2] * G[j][2]);
                    hdelta[idx] = del;
                }
            }
        }
    }
}

void Planner::set_obstacles(int num_obstacles, const double* obs) {
    if (num_obstacles < 0 || num_obstacles > MAX_OBS) throw std::runtime_error("Number of obstacles out of range");
    O = num_obstacles;
    obstacles.assign(obs, obs + O * (OBS_GEN + 1) * 3);
    if (!link_gens.empty()) buffer_obstacles();
}

// NLPclass.cu:87-165
void Planner::bounds(double* g_l, double* g_u) const {
    int off = 0;
    for (int t = 0; t < T; t++)
        for (int j = 0; j < NF; j++) {
            g_l[t * NF + j] = -robot.torque_limits[j] + torque_radius[t * NF + j];
            g_u[t * NF + j] = robot.torque_limits[j] - torque_radius[t * NF + j];
        }
    off += NF * T;
    for (int i = off; i < off + T * NJ * O; i++) { g_l[i] = -1e19; g_u[i] = 0; }
    off += T * NJ * O;
    for (int rep = 0; rep < 2; rep++) {
        for (int i = 0; i < NF; i++) { g_l[off + i] = robot.state_lb[i] + robot.qe; g_u[off + i] = robot.state_ub[i] - robot.qe; }
        off += NF;
    }
    for (int rep = 0; rep < 2; rep++) {
        for (int i = 0; i < NF; i++) { g_l[off + i] = -robot.speed_limits[i] + robot.qde; g_u[off + i] = robot.speed_limits[i] - robot.qde; }
        off += NF;
    }
}

static double wrap_to_pi(double a) {  // NLPclass.cu:6-15
    double w = a;
    while (w < -M_PI) w += 2 * M_PI;
    while (w > M_PI) w -= 2 * M_PI;
    return w;
}

// NLPclass.cu:207-236 ; wrapped joints are summed first (the reference's order for Kinova)
double Planner::eval_f(const double* x) const {
    double qp[NF];
    for (int i = 0; i < NF; i++)
        qp[i] = q_des_func(traj->q0[i], traj->Tqd0[i], traj->TTqdd0[i], prm.k_range[i] * x[i], prm.t_plan);
    double f = 0.0;
    bool first = true;
    for (int pass = 1; pass >= 0; pass--)
        for (int i = 0; i < NF; i++) {
            if (robot.wrap_mask[i] != pass) continue;
            const double d = pass ? wrap_to_pi(q_des[i] - qp[i]) : (q_des[i] - qp[i]);
            const double term = std::pow(d, 2);
            f = first ? term : f + term;
            first = false;
        }
    return f * prm.cost_scale;
}

// NLPclass.cu:241-267
void Planner::eval_grad_f(const double* x, double* grad) const {
    const double tp = prm.t_plan;
    for (int i = 0; i < NF; i++) {
        const double qp = q_des_func(traj->q0[i], traj->Tqd0[i], traj->TTqdd0[i], prm.k_range[i] * x[i], tp);
        const double dk = tp * tp * tp * (6 * tp * tp - 15 * tp + 10) * prm.k_range[i];
        grad[i] = robot.wrap_mask[i] ? (2 * wrap_to_pi(qp - q_des[i]) * dk) : (2 * (qp - q_des[i]) * dk);
        grad[i] *= prm.cost_scale;
    }
}

// PZsparse.cu:404-435 + getCenter of the resulting Interval (NLPclass.cu:313), and :477-516
void Planner::link_slice(int t, int l, const double* x, double* c3, double* grad21) const {
    const PZ& pz = kd->links[l * T + t];
    double rc[3], rr[3];
    pz.slice(x, rc, rr);
    for (int e = 0; e < 3; e++) c3[e] = getCenter(Interval(rc[e] - rr[e], rc[e] + rr[e]));
    if (grad21) pz.slice_grad(x, grad21);
}

void Planner::torque_slice(int t, int j, const double* x, double* val, double* grad7) const {
    const PZ& pz = kd->u_nom[j * T + t];
    double rc, rr;
    pz.slice(x, &rc, &rr);
    *val = getCenter(Interval(rc - rr, rc + rr));
    if (grad7) pz.slice_grad(x, grad7);
}

// CollisionChecking.cu:230-299 for one (t, link, obstacle) block, as a CPU loop
void Planner::collision_row(int t, int l, int o, const double* c, const double* dc, double* g, double* grad7) const {
    double pos[COMB], neg[COMB];
    const size_t base = (((size_t)t * NJ + l) * O + o) * COMB;
    for (int p = 0; p < COMB; p++) {
        const double* A = &hA[(base + p) * 3];
        const double d = hd[base + p], del = hdelta[base + p];
        const double nrm = std::sqrt(A[0] * A[0] + A[1] * A[1] + A[2] * A[2]);
        if (nrm > 0) {
            const double Ac = A[0] * c[0] + A[1] * c[1] + A[2] * c[2];
            pos[p] = Ac - (d + del);
            neg[p] = -Ac - (-d + del);
        } else {
            pos[p] = -100000000;
            neg[p] = -100000000;
        }
    }
    double mx = -100000000;
    int id = 0;
    bool isneg = false;
    for (int i = 0; i < COMB; i++) {
        if (pos[i] > mx) { mx = pos[i]; id = i; isneg = false; }
        if (neg[i] > mx) { mx = neg[i]; id = i; isneg = true; }
    }
    *g = -mx;
    if (grad7) {
        const double* A = &hA[(base + id) * 3];
        for (int k = 0; k < NF; k++) {
            const double* v = &dc[k * 3];
            const double dot = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
            grad7[k] = isneg ? dot : -dot;
        }
    }
}

// NLPclass.cu:272-396
void Planner::eval_g_jac(const double* x, double* g, double* jac, double* link_center_out) const {
    std::vector<double> lc((size_t)T * NJ * 3), dlc(jac ? (size_t)T * NJ * NF * 3 : 0);
#pragma omp parallel for num_threads(num_threads) schedule(dynamic)
    for (int t = 0; t < T; t++) {
        for (int k = 0; k < NF; k++)
            torque_slice(t, k, x, &g[t * NF + k], jac ? &jac[(size_t)(t * NF + k) * NF] : nullptr);
        for (int l = 0; l < NJ; l++)
            link_slice(t, l, x, &lc[((size_t)t * NJ + l) * 3], jac ? &dlc[((size_t)t * NJ + l) * NF * 3] : nullptr);
    }
    const size_t off = (size_t)NF * T;
#pragma omp parallel for num_threads(num_threads) schedule(static) collapse(2)
    for (int l = 0; l < NJ; l++)
        for (int t = 0; t < T; t++)
            for (int o = 0; o < O; o++) {
                const size_t row = off + ((size_t)l * T + t) * O + o;
                collision_row(t, l, o, &lc[((size_t)t * NJ + l) * 3], jac ? &dlc[((size_t)t * NJ + l) * NF * 3] : nullptr,
                              &g[row], jac ? &jac[row * NF] : nullptr);
            }
    const size_t off2 = off + (size_t)T * NJ * O;
    traj->returnJointPositionExtremum(&g[off2], x);
    traj->returnJointVelocityExtremum(&g[off2 + 2 * NF], x);
    if (jac) {
        traj->returnJointPositionExtremumGradient(&jac[off2 * NF], x);
        traj->returnJointVelocityExtremumGradient(&jac[(off2 + 2 * NF) * NF], x);
    }
    if (link_center_out) std::memcpy(link_center_out, lc.data(), lc.size() * sizeof(double));
}

// NLPclass.cu:449-538
bool Planner::feasible(const double* g) const {
    int off = 0;
    for (int t = 0; t < T; t++)
        for (int j = 0; j < NF; j++) {
            const double v = g[t * NF + j];
            const double tr = torque_radius[t * NF + j], tl = robot.torque_limits[j];
            if (v < -tl + tr - prm.torque_violation || v > tl - tr + prm.torque_violation) return false;
        }
    off += NF * T;
    for (int i = 0; i < NJ; i++)
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
