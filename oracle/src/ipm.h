// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
//
// CPU statement of the build's NLP solver ("armour-IPM"). The reference drives the NLP with
// Ipopt + HSL MA97 + L-BFGS (KPR/armour_main.cu:238-290), none of which exist in this image
// (SURVEY §8c). The product ships its own interior-point solver that runs on the GPU; this file
// is the CPU statement of exactly the same algorithm, used to check the GPU solver
// (DESIGN.md §NLP). Algorithm (per iteration):
//   rows r = 0..m-1 (constraints, bounds [L_r, U_r], |bound| >= 1e19 means infinite) plus the
//   n box bounds; each finite side k has slack s_k > 0 and multiplier z_k > 0;
//   1. residuals r_d = grad f - sum_k z_k a_k, r_p = c_k(x) - s_k, errors E_0 / E_mu (Ipopt-scaled)
//   2. barrier update: adaptive (the default, mu_strategy 1; Ipopt's mu_strategy "adaptive",
//      KPR/Parameters.h:57): LOQO oracle mu = 0.1 min(0.05 (1 - xi) / xi, 2)^3 avg(s z) in free
//      mode, floor tol/10, mu on the 2^(j/8) grid, with the kkt-error globalisation falling back
//      to the monotone rule; or monotone (option 0):
//      mu <- max(tol/10, min(kappa_mu*mu, mu^theta)) while E_mu <= kappa_eps*mu
//   3. Newton step on the reduced 7x7 system (H + sum_k sigma_k a_k a_k^T) dx = -grad f + sum_k a_k (mu/s_k - sigma_k r_p,k)
//   4. ds, dz, fraction-to-boundary step sizes
//   5. Ipopt's filter line search on theta = ||c(x) - s||_1 and the barrier objective
//      phi = f - mu sum ln s, at most max_ls backtracking trials; when it fails, a restoration
//      phase (Gauss-Newton on the violation with a box barrier, at most resto_max phases) that
//      restarts the interior point from a feasible point or ends in local infeasibility (status 4)
//   6. multiplier update with Ipopt's kappa_sigma safeguard; damped BFGS update of H
#pragma once

namespace oracle {

struct IpmOptions {
    double tol = 1e-4;          // IPOPT_OPTIMIZATION_TOLERANCE (Parameters.h:50)
    int max_iter = 100;
    double mu0 = 0.1;
    double kappa_eps = 10.0;
    double kappa_mu = 0.2;
    double theta_mu = 1.5;
    double tau_min = 0.99;
    double bound_push = 1e-2;
    double eta = 1e-4;
    int max_ls = 10;
    double kappa_sigma = 1e10;
    double s_max = 100.0;
    double inf_bound = 1e19;
    // barrier strategy: 1 adaptive (the default: the reference's IPOPT_MU_STRATEGY "adaptive",
    // KPR/Parameters.h:57, restated with Ipopt's mu_oracle loqo and adaptive_mu_globalization
    // kkt-error — not Ipopt's default quality-function / obj-constr-filter pair — with mu on a
    // 2^(1/8) grid and the floor tol / 10; ipm.cpp); 0 monotone (Fiacco-McCormick);
    // 2 (pricing study only, not on the device): Ipopt's default adaptive pair, mu_oracle
    // quality-function and adaptive_mu_globalization obj-constr-filter, with Ipopt's mu_min 1e-11
    int mu_strategy = 1;
    int qf_grid = 0;  // mu_strategy 2 / 3 studies: > 0 replaces the golden section by a fixed grid of this many sigmas
    // studies of the adaptive rule only (tools/mu_sensitivity.py): bit 0 drops the 2^(1/8) grid
    // (ipm.cpp mu_grid), bit 1 the tol / 10 floor (Ipopt's mu_min 1e-11 instead)
    int mu_study = 0;
    // Hessian approximation (pricing study only, not on the device): 0 the product's damped BFGS
    // matrix; h > 0 Ipopt's limited-memory BFGS (hessian_approximation limited-memory,
    // KPR/armour_main.cu:259), restated from its documented options: history h (Ipopt's
    // limited_memory_max_history default 6), update type bfgs, initialisation scalar1
    // (sigma = s'y / s's, clamped to [1e-8, 1e8]), a pair skipped when s'y <= sqrt(eps) |s| |y|
    // and the history reset after more than limited_memory_max_skipping = 2 skips in a row
    int lbfgs_hist = 0;
    // restoration phase (ipm.cpp restoration): phases per solve (0: none; a failed line search
    // then takes the last trial, and three in a row end the solve), violation target inside the
    // bounds, box barrier weight, stall ratio
    int resto_max = 3;
    double resto_delta = 1e-6;
    double resto_mu = 1e-8;
    double resto_stall = 1e-4;
};

struct IpmResult {
    int status;        // 0 converged, 1 max_iter, 2 line-search failure, 4 local infeasibility
                       // (the restoration phase stalled or failed; 3 is the ABI's "not planned")
    int iterations;
    int evaluations;
    double obj;
    double kkt_error;
    int restart_iter;  // iteration count at the last restoration phase that ended in a restart (-1: none)
};

// evaluation callback: f, grad f (n), g (m), dense row-major Jacobian (m x n)
struct IpmProblem {
    virtual ~IpmProblem() {}
    virtual int n() const = 0;
    virtual int m() const = 0;
    virtual void bounds(double* xl, double* xu, double* gl, double* gu) const = 0;
    virtual void eval(const double* x, double* f, double* grad, double* g, double* jac) = 0;
};

// x: in = start point, out = final iterate; g_out (m) = constraints at the final iterate
IpmResult ipm_solve(IpmProblem& prob, const IpmOptions& opt, double* x, double* g_out);

}  // namespace oracle
