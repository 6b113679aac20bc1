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
//   2. barrier update: monotone (default, mu_strategy 0):
//      mu <- max(tol/10, min(kappa_mu*mu, mu^theta)) while E_mu <= kappa_eps*mu; or adaptive
//      (option 1; Ipopt's mu_strategy "adaptive", KPR/Parameters.h:57): LOQO oracle
//      mu = 0.1 min(0.05 (1 - xi) / xi, 2)^3 avg(s z) in free mode, with the kkt-error
//      globalisation falling back to the monotone rule
//   3. Newton step on the reduced 7x7 system (H + sum_k sigma_k a_k a_k^T) dx = -grad f + sum_k a_k (mu/s_k - sigma_k r_p,k)
//   4. ds, dz, fraction-to-boundary step sizes
//   5. Ipopt's filter line search (no restoration phase) on theta = ||c(x) - s||_1 and the
//      barrier objective phi = f - mu sum ln s, at most max_ls backtracking trials
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
    // barrier strategy: 0 monotone (the build's solver, GPU and CPU); 1 adaptive (Ipopt's
    // mu_strategy "adaptive", KPR/Parameters.h:57, with the LOQO mu oracle and the kkt-error
    // globalisation, restated in ipm.cpp; an option, see DESIGN.md §5 for why it is not the default)
    int mu_strategy = 0;
};

struct IpmResult {
    int status;        // 0 converged, 1 max_iter, 2 line-search failure
    int iterations;
    int evaluations;
    double obj;
    double kkt_error;
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
