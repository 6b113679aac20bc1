// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// C entry points of the CPU oracle, loaded by tests/ and bench.py's cpu_baseline leg via ctypes.
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>
#include "ipm.h"
#include "armtd.h"
#include "planner.h"

using namespace oracle;

namespace {
struct PlannerNlp : IpmProblem {
    Planner* P;
    explicit PlannerNlp(Planner* p) : P(p) {}
    int n() const override { return NF; }
    int m() const override { return P->m(); }
    void bounds(double* xl, double* xu, double* gl, double* gu) const override {
        for (int i = 0; i < NF; i++) { xl[i] = -1.0; xu[i] = 1.0; }  // NLPclass.cu:105-113
        P->bounds(gl, gu);
    }
    void eval(const double* x, double* f, double* grad, double* g, double* jac) override {
        *f = P->eval_f(x);
        P->eval_grad_f(x, grad);
        P->eval_g_jac(x, g, jac);
        if (noise > 0) {
            // sensitivity study only: g and J scaled by 1 + noise u, u uniform in [-1, 1), a fixed
            // xorshift sequence per solve (tools/mu_study.py --noise)
            const int m = P->m();
            for (long i = 0; i < (long)m * (NF + 1); i++) {
                rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
                const double u = (double)(rng >> 11) * 0x1p-52 - 1.0;
                if (i < m) g[i] *= 1.0 + noise * u;
                else if (jac) jac[i - m] *= 1.0 + noise * u;
            }
        }
    }
    double noise = 0;
    unsigned long long rng = 0x9E3779B97F4A7C15ull;
};

Robot robot_by_id(int id) {
    (void)id;
    return kinova_without_gripper();
}

// robot tables in the layout of include/armour_hip.h armour_robot (the tests hand the same bytes to
// the product and to this checker)
constexpr int RD_J = 9;
struct RobotDesc {
    int num_joints;
    int axes[RD_J];
    int wrap[NF];
    double trans[(RD_J + 1) * 3];
    double rots[RD_J * 3];
    double mass[RD_J];
    double com[RD_J * 3];
    double inertia[RD_J * 9];
    double mass_uncertainty, inertia_uncertainty;
    double friction[RD_J], damping[RD_J], armature[RD_J];
    double state_lb[NF], state_ub[NF];
    double speed_limits[NF], torque_limits[NF];
    double gravity;
    double link_center[RD_J * 3], link_generators[RD_J * 3];
    double alpha, V_m, M_max, M_min, K;
};

Robot robot_from_desc(const RobotDesc& t) {
    Robot r{};
    r.num_joints = t.num_joints;
    for (int i = 0; i < RD_J; i++) {
        r.axes[i] = t.axes[i];
        r.mass[i] = t.mass[i];
        r.friction[i] = t.friction[i];
        r.damping[i] = t.damping[i];
        r.armature[i] = t.armature[i];
        for (int e = 0; e < 3; e++) {
            r.rots[3 * i + e] = t.rots[3 * i + e];
            r.com[3 * i + e] = t.com[3 * i + e];
            r.link_c[i][e] = t.link_center[3 * i + e];
            r.link_g[i][e] = t.link_generators[3 * i + e];
        }
        for (int e = 0; e < 9; e++) r.inertia[9 * i + e] = t.inertia[9 * i + e];
    }
    for (int e = 0; e < (RD_J + 1) * 3; e++) r.trans[e] = t.trans[e];
    r.mass_uncertainty = t.mass_uncertainty;
    r.inertia_uncertainty = t.inertia_uncertainty;
    for (int i = 0; i < NF; i++) {
        r.state_lb[i] = t.state_lb[i];
        r.state_ub[i] = t.state_ub[i];
        r.speed_limits[i] = t.speed_limits[i];
        r.torque_limits[i] = t.torque_limits[i];
        r.wrap_mask[i] = t.wrap[i] ? 1 : 0;
    }
    r.gravity = t.gravity;
    r.alpha = t.alpha;
    r.V_m = t.V_m;
    r.M_max = t.M_max;
    r.M_min = t.M_min;
    r.K = t.K;
    r.eps = std::sqrt(2 * r.V_m / r.M_min);  // KinovaWithoutGripperInfo.h:102-112
    r.qe = r.eps / r.K;
    r.qde = 2 * r.eps;
    r.qdae = r.eps;
    r.qddae = 2 * r.K * r.eps;
    return r;
}
}  // namespace

extern "C" {

void* oracle_create(int robot_id, int T, int O, const double* q0, const double* qd0, const double* qdd0,
                    const double* q_des, const double* obstacles, int threads) {
    try {
        Robot r = robot_by_id(robot_id);
        Params p = default_params(T);
        Planner* P = new Planner(r, p, q0, qd0, qdd0, q_des, O, obstacles);
        P->num_threads = threads > 0 ? threads : 1;
        return P;
    } catch (...) {
        return nullptr;
    }
}

// the same with robot tables (RobotDesc = armour_robot layout)
void* oracle_create_robot(const void* robot, int T, int O, const double* q0, const double* qd0, const double* qdd0,
                          const double* q_des, const double* obstacles, int threads) {
    try {
        Robot r = robot_from_desc(*static_cast<const RobotDesc*>(robot));
        Params p = default_params(T);
        Planner* P = new Planner(r, p, q0, qd0, qdd0, q_des, O, obstacles);
        P->num_threads = threads > 0 ? threads : 1;
        return P;
    } catch (...) {
        return nullptr;
    }
}

// the ARMTD comparison planner (armtd.h): tables [joint][6][T] = c_cos, g_cos, r_cos, c_sin,
// g_sin, r_sin (ACMP/armtd_main.cu:70-90), k_range [7]; robot: null (Kinova) or a RobotDesc
void* oracle_create_armtd(const void* robot, int T, int O, const double* q0, const double* qd0, const double* q_des,
                          const double* tables, const double* k_range, const double* obstacles, int threads) {
    try {
        Robot r = robot ? robot_from_desc(*static_cast<const RobotDesc*>(robot)) : robot_by_id(0);
        Params p = default_params(T);
        Planner* P = new ArmtdPlanner(r, p, q0, qd0, q_des, tables, k_range, O, obstacles);
        P->num_threads = threads > 0 ? threads : 1;
        return P;
    } catch (...) {
        return nullptr;
    }
}

void oracle_free(void* h) { delete static_cast<Planner*>(h); }

// runs the reach-set half of a plan (armour_main.cu:97-222); returns elapsed ms or -1
double oracle_reach(void* h) {
    Planner* P = static_cast<Planner*>(h);
    auto t0 = std::chrono::high_resolution_clock::now();
    try {
        P->reach();
    } catch (...) {
        return -1.0;
    }
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

// test tooling: replace the obstacles after oracle_reach (hyperplanes only; 0 / -1)
int oracle_set_obstacles(void* h, int O, const double* obstacles) {
    try {
        static_cast<Planner*>(h)->set_obstacles(O, obstacles);
    } catch (...) {
        return -1;
    }
    return 0;
}

int oracle_num_constraints(void* h) { return static_cast<Planner*>(h)->m(); }

void oracle_bounds(void* h, double* gl, double* gu) { static_cast<Planner*>(h)->bounds(gl, gu); }

// eval_g (+ eval_jac_g when jac != null) at x; link_center (T*NJ*3) optional
void oracle_eval(void* h, const double* x, double* g, double* jac, double* link_center) {
    static_cast<Planner*>(h)->eval_g_jac(x, g, jac, link_center);
}

double oracle_cost(void* h, const double* x, double* grad) {
    Planner* P = static_cast<Planner*>(h);
    if (grad) P->eval_grad_f(x, grad);
    return P->eval_f(x);
}

int oracle_feasible(void* h, const double* g) { return static_cast<Planner*>(h)->feasible(g) ? 1 : 0; }

// what: 0 link_gens (T*NJ*18), 1 torque_radius (T*7), 2 hyperplane A (T*NJ*O*36*3), 3 d, 4 delta
int oracle_get(void* h, int what, double* out) {
    Planner* P = static_cast<Planner*>(h);
    const std::vector<double>* v = nullptr;
    switch (what) {
        case 0: v = &P->link_gens; break;
        case 1: v = &P->torque_radius; break;
        case 2: v = &P->hA; break;
        case 3: v = &P->hd; break;
        case 4: v = &P->hdelta; break;
        default: return -1;
    }
    std::memcpy(out, v->data(), v->size() * sizeof(double));
    return (int)v->size();
}

// monomial table of a reach-set PZ. kind: 0 link (index l*T+t, 3x1 after reduce_link_PZ),
// 1 u_nom (j*T+t, after reduce), 2 u_nom_int - u_nom (disturbance), 3 JRS R (i*T+t, 3x3),
// 4 qd_des, 5 qda_des, 6 qdda_des, 7 cos_q_des, 8 sin_q_des.
// Writes center[9], indep[9], and up to cap monomials (hash, coeff[9]); returns count or -1.
int oracle_pz(void* h, int kind, int idx, double* center, double* indep, unsigned long long* hashes, double* coeffs, int cap, int* rows, int* cols) {
    Planner* P = static_cast<Planner*>(h);
    const PZ* pz = nullptr;
    switch (kind) {
        case 0: pz = &P->kd->links[idx]; break;
        case 1: pz = &P->kd->u_nom[idx]; break;
        case 2: pz = &P->kd->u_nom_int[idx]; break;
        case 3: pz = &P->traj->R[idx]; break;
        case 4: pz = &P->traj->qd_des[idx]; break;
        case 5: pz = &P->traj->qda_des[idx]; break;
        case 6: pz = &P->traj->qdda_des[idx]; break;
        case 7: pz = &P->traj->cos_q_des[idx]; break;
        case 8: pz = &P->traj->sin_q_des[idx]; break;
        default: return -1;
    }
    const int n = pz->R * pz->C;
    *rows = pz->R;
    *cols = pz->C;
    for (int e = 0; e < 9; e++) { center[e] = e < n ? pz->center[e] : 0.0; indep[e] = e < n ? pz->indep[e] : 0.0; }
    const int cnt = (int)pz->poly.size();
    for (int i = 0; i < cnt && i < cap; i++) {
        hashes[i] = pz->poly[i].h;
        for (int e = 0; e < 9; e++) coeffs[i * 9 + e] = e < n ? pz->poly[i].c[e] : 0.0;
    }
    return cnt;
}

// full plan: reach + NLP + finalize. stats[0]=reach ms, [1]=nlp ms, [2]=iterations, [3]=evals,
// [4]=solver status, [5]=objective/cost_scale, [6]=kkt error, [7]=iteration count at the last
// restart after a restoration phase (-1: none). Returns 1 feasible, 0 infeasible, -1 error.
int oracle_plan_mu(void* h, double* k_opt, double* g_out, double* stats, int max_iter, int mu_strategy);
int oracle_plan(void* h, double* k_opt, double* g_out, double* stats, int max_iter) {
    return oracle_plan_mu(h, k_opt, g_out, stats, max_iter, 1);
}

// the same with the barrier strategy chosen (1 adaptive, the default: IPOPT_MU_STRATEGY "adaptive",
// KPR/Parameters.h:57; 0 monotone: DESIGN.md §5)
int oracle_plan_ex(void* h, double* k_opt, double* g_out, double* stats, int max_iter, int mu_strategy, int flags,
                   double noise);
int oracle_plan_mu(void* h, double* k_opt, double* g_out, double* stats, int max_iter, int mu_strategy) {
    return oracle_plan_ex(h, k_opt, g_out, stats, max_iter, mu_strategy, 0, 0.0);
}
// flags: bits 0-1 IpmOptions::mu_study, bit 2 no restoration phase; noise: relative perturbation of
// every g / J value the solver sees (sensitivity studies only)
int oracle_plan_ex(void* h, double* k_opt, double* g_out, double* stats, int max_iter, int mu_strategy, int flags,
                   double noise) {
    Planner* P = static_cast<Planner*>(h);
    auto t0 = std::chrono::high_resolution_clock::now();
    try {
        if (!P->kd) P->reach();
    } catch (...) {
        return -1;
    }
    auto t1 = std::chrono::high_resolution_clock::now();
    PlannerNlp nlp(P);
    nlp.noise = noise;
    IpmOptions opt;
    opt.tol = P->tol;
    if (max_iter > 0) opt.max_iter = max_iter;
    opt.mu_strategy = mu_strategy;
    opt.mu_study = flags & 3;
    opt.qf_grid = (flags >> 8) & 255;  // studies: bits 8-15
    opt.lbfgs_hist = (flags >> 16) & 255;  // studies: bits 16-23 (0: the product's damped BFGS)
    if (flags & 4) opt.resto_max = 0;  // no restoration phase (studies)
    double x[NF] = {0, 0, 0, 0, 0, 0, 0};  // NLPclass.cu:193-199
    std::vector<double> g(P->m());
    IpmResult r = ipm_solve(nlp, opt, x, g.data());
    auto t2 = std::chrono::high_resolution_clock::now();
    const bool feas = P->feasible(g.data());
    for (int i = 0; i < NF; i++) k_opt[i] = x[i];
    if (g_out) std::memcpy(g_out, g.data(), g.size() * sizeof(double));
    if (stats) {
        stats[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats[1] = std::chrono::duration<double, std::milli>(t2 - t1).count();
        stats[2] = r.iterations;
        stats[3] = r.evaluations;
        stats[4] = r.status;
        stats[5] = r.obj / P->prm.cost_scale;
        stats[6] = r.kkt_error;
        stats[7] = r.restart_iter;
    }
    return feas ? 1 : 0;
}

}  // extern "C"
