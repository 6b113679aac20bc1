// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// CPU statement of armour-IPM (see ipm.h). The GPU solver (armour-dev_amd/csrc/nlp_kernels.hip)
// implements the same passes; reductions there run in a different order, so iterates agree to
// rounding, not bit for bit.
#include "ipm.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include <cstdio>
#include <cstdlib>

namespace oracle {

static const int NMAX = 8;

// The barrier parameter on a fixed logarithmic grid, 2^(j/8) x 2^e: the nearest grid point in
// log2 (ties up), with the grid values and the midpoints between them as exact constants so that
// the device solver (nlp_kernels.hip mu_grid) forms the same bits. The adaptive rule's mu is a
// smooth function of the complementarity products; on the grid a rounding-level difference in
// those sums leaves mu unchanged (unless it straddles a midpoint), where the LOQO sigma
// (a cube of xi) would carry it into the next iterate amplified.
static double mu_grid(double x) {
    static const double G[9] = {0x1.0000000000000p+0, 0x1.172b83c7d517bp+0, 0x1.306fe0a31b715p+0,
                                0x1.4bfdad5362a27p+0, 0x1.6a09e667f3bcdp+0, 0x1.8ace5422aa0dbp+0,
                                0x1.ae89f995ad3adp+0, 0x1.d5818dcfba487p+0, 0x1.0000000000000p+1};
    static const double B[8] = {0x1.0b5586cf9890fp+0, 0x1.2387a6e756238p+0, 0x1.3dea64c123422p+0,
                                0x1.5ab07dd485429p+0, 0x1.7a11473eb0187p+0, 0x1.9c49182a3f090p+0,
                                0x1.c199bdd85529cp+0, 0x1.ea4afa2a490dap+0};
    if (!(x > 0) || !std::isfinite(x)) return x;
    int e;
    const double y = 2.0 * std::frexp(x, &e);  // x = y 2^(e-1), y in [1, 2)
    int j = 0;
    for (int q = 0; q < 8; q++) j += y >= B[q];
    return std::ldexp(G[j], e - 1);
}

// Cholesky of a dense n x n SPD matrix (row-major) with diagonal shift; returns false if not PD
static bool chol_solve(const double* M, int n, double shift, const double* b, double* x) {
    double L[NMAX * NMAX];
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = M[i * n + j] + (i == j ? shift : 0.0);
            for (int k = 0; k < j; k++) s -= L[i * n + k] * L[j * n + k];
            if (i == j) {
                if (!(s > 0)) return false;
                L[i * n + i] = std::sqrt(s);
            } else {
                L[i * n + j] = s / L[j * n + j];
            }
        }
    double y[NMAX];
    for (int i = 0; i < n; i++) {
        double s = b[i];
        for (int k = 0; k < i; k++) s -= L[i * n + k] * y[k];
        y[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = y[i];
        for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
        x[i] = s / L[i * n + i];
    }
    return true;
}

IpmResult ipm_solve(IpmProblem& prob, const IpmOptions& opt, double* x, double* g_out) {
    const int n = prob.n(), m = prob.m();
    const int R = m + n;  // constraint rows + box rows
    std::vector<double> L(R), U(R);
    {
        std::vector<double> xl(n), xu(n), gl(m), gu(m);
        prob.bounds(xl.data(), xu.data(), gl.data(), gu.data());
        for (int r = 0; r < m; r++) { L[r] = gl[r]; U[r] = gu[r]; }
        for (int j = 0; j < n; j++) { L[m + j] = xl[j]; U[m + j] = xu[j]; }
        // Ipopt-style push of the start point into the box interior
        for (int j = 0; j < n; j++) {
            const double p = std::min(opt.bound_push * std::max(1.0, std::fabs(xl[j])), opt.bound_push * (xu[j] - xl[j]));
            x[j] = std::min(std::max(x[j], xl[j] + p), xu[j] - p);
        }
    }
    std::vector<char> hlo(R), hhi(R);
    for (int r = 0; r < R; r++) { hlo[r] = L[r] > -opt.inf_bound; hhi[r] = U[r] < opt.inf_bound; }

    // evaluation buffers (current and trial)
    std::vector<double> g(m), J((size_t)m * n), gt(m), Jt((size_t)m * n);
    double f, ft, grad[NMAX], gradt[NMAX];
    prob.eval(x, &f, grad, g.data(), J.data());
    int nevals = 1;

    auto val = [&](const std::vector<double>& gv, const double* xv, int r) { return r < m ? gv[r] : xv[r - m]; };
    auto grow = [&](const std::vector<double>& Jv, int r, double* a) {
        if (r < m) for (int j = 0; j < n; j++) a[j] = Jv[(size_t)r * n + j];
        else for (int j = 0; j < n; j++) a[j] = (j == r - m) ? 1.0 : 0.0;
    };

    std::vector<double> slo(R, 0), shi(R, 0), zlo(R, 0), zhi(R, 0);
    std::vector<double> dslo(R, 0), dshi(R, 0), dzlo(R, 0), dzhi(R, 0), rplo(R, 0), rphi(R, 0);
    double mu = opt.mu0;
    // slacks pushed into the interior and multipliers mu / s at the current point (the start, and
    // the restart after a successful restoration phase)
    auto init_slacks = [&]() {
        for (int r = 0; r < R; r++) {
            const double v = val(g, x, r);
            double p = 0;
            if (hlo[r] && hhi[r]) p = std::min(opt.bound_push * std::max(1.0, std::fabs(L[r])), opt.bound_push * (U[r] - L[r]));
            slo[r] = 0; zlo[r] = 0; shi[r] = 0; zhi[r] = 0;
            if (hlo[r]) {
                const double pl = hhi[r] ? p : opt.bound_push * std::max(1.0, std::fabs(L[r]));
                slo[r] = std::max(v - L[r], pl);
                zlo[r] = mu / slo[r];
            }
            if (hhi[r]) {
                const double pu = hlo[r] ? p : opt.bound_push * std::max(1.0, std::fabs(U[r]));
                shi[r] = std::max(U[r] - v, pu);
                zhi[r] = mu / shi[r];
            }
        }
    };
    init_slacks();

    double H[NMAX * NMAX] = {0};
    for (int j = 0; j < n; j++) H[j * n + j] = 1.0;
    bool first_update = true;
    // limited-memory BFGS (opt.lbfgs_hist > 0, study only): the stored (s, y) pairs, oldest first;
    // H is rebuilt after every update as sigma I followed by the BFGS updates of the stored pairs in
    // order, the dense form of the compact representation
    std::vector<std::vector<double>> lb_s, lb_y;
    int lb_skips = 0;
    auto lbfgs_rebuild = [&](double sigma) {
        for (int i = 0; i < n * n; i++) H[i] = 0;
        for (int j = 0; j < n; j++) H[j * n + j] = sigma;
        for (size_t q = 0; q < lb_s.size(); q++) {
            const double* sv = lb_s[q].data();
            const double* y = lb_y[q].data();
            double Hs[NMAX], sHs = 0, sy = 0;
            for (int i = 0; i < n; i++) {
                Hs[i] = 0;
                for (int j = 0; j < n; j++) Hs[i] += H[i * n + j] * sv[j];
                sHs += sv[i] * Hs[i];
                sy += sv[i] * y[i];
            }
            for (int i = 0; i < n; i++)
                for (int j = 0; j < n; j++) H[i * n + j] += -Hs[i] * Hs[j] / sHs + y[i] * y[j] / sy;
        }
    };
    std::vector<double> filt_theta, filt_phi;
    double theta_max = -1, theta_min = -1;
    int nfail = 0;
    // adaptive barrier (mu_strategy 1): free mode takes mu from the LOQO oracle every iteration;
    // the kkt-error globalisation switches to monotone (fixed) mode when the KKT error has not
    // fallen below 0.9999 x the largest of the last 4 reference values, and back to free mode once
    // it has (Ipopt: adaptive_mu_globalization kkt-error, kkterror_red_iters 4, red_fact 0.9999,
    // adaptive_mu_monotone_init_factor 0.8, mu_oracle loqo)
    bool free_mode = opt.mu_strategy >= 1;
    std::vector<double> kkt_ref;
    // mu_strategy 2 (study only): Ipopt's default adaptive pair, mu_oracle quality-function with
    // adaptive_mu_globalization obj-constr-filter (qf_mu below); the filter of (f, theta) of the
    // free-mode iterates, and Ipopt's mu bounds (mu_min 1e-11, mu_max = min(1e5, 1e3 avg(s z) at the start))
    std::vector<double> gf_f, gf_t;
    double mu_max_qf = -1;
    // the adaptive rule's floor: tol / 10, the monotone rule's floor (Ipopt's mu_min default is
    // 1e-11; below ~tol / 10 the reduced system's Sigma = z / s ~ z^2 / mu of the active rows makes
    // the 1e-4-tolerance solution reproducible to ~1e-5 only: DESIGN.md §5, tools/mu_sensitivity.py)
    // mu_strategy 3 (study only): the quality-function pair with the product's floor tol / 10 and grid
    const bool qf = opt.mu_strategy == 2 || opt.mu_strategy == 3;
    const double mu_min = (opt.mu_study & 2) || opt.mu_strategy == 2 ? 1e-11 : opt.tol / 10;
    auto qf_grid = [&](double v) { return opt.mu_strategy == 3 ? mu_grid(v) : v; };
    IpmResult res{1, 0, 0, 0.0, 0.0, -1};
    double a[NMAX], at[NMAX];
    int it;
    int nresto = 0;
    // Restoration phase (the device statement is nlp_kernels.hip resto_*). From the
    // current x (g, J at x), Gauss-Newton steps on
    //   Phi(x) = 1/2 sum_r e_r(x)^2 + mu_R sum_j (-ln(1 - x_j) - ln(1 + x_j)),
    //   e_r = max(0, (L_r + delta) - g_r, g_r - (U_r - delta)) over the constraint rows' finite sides
    // (targets delta inside the bounds, so a point that reaches them is strictly feasible; the box
    // |x| < 1 by the barrier and the fraction to the boundary), Levenberg-Marquardt damping
    // lambda = 1e-2 min(1, |e|_2) (1 + max_j M_jj), an Armijo backtracking search over max_ls
    // halvings. Each iteration in order: (1) every original row within its bounds -> 0 (restart the
    // interior point); (2) the iteration cap -> 1; (3) Phi decreased by at most resto_stall x Phi
    // in two consecutive iterations -> 4 (local infeasibility); (4) the step, or 4 when the
    // factorisation or the line search fails. Accepted steps count as iterations.
    auto restoration = [&](int& iter, int& ne) -> int {
        double phi_prev = -1;
        int stall = 0;
        for (;;) {
            double Mr[NMAX * NMAX] = {0}, br[NMAX] = {0}, V = 0, e0max = 0;
            for (int r = 0; r < m; r++) {
                const double v = g[r];
                double e = 0, sg = 0, e0 = 0;
                if (hlo[r]) {
                    e0 = std::max(e0, L[r] - v);
                    const double el = (L[r] + opt.resto_delta) - v;
                    if (el > 0) { e = el; sg = -1.0; }
                }
                if (hhi[r]) {
                    e0 = std::max(e0, v - U[r]);
                    const double eh = v - (U[r] - opt.resto_delta);
                    if (e == 0 && eh > 0) { e = eh; sg = 1.0; }
                }
                e0max = std::max(e0max, e0);
                if (e > 0) {
                    grow(J, r, a);
                    V += e * e;
                    const double es = e * sg;
                    for (int i = 0; i < n; i++) {
                        br[i] += es * a[i];
                        for (int j = 0; j < n; j++) Mr[i * n + j] += a[i] * a[j];
                    }
                }
            }
            if (e0max <= 0) return 0;
            if (iter >= opt.max_iter) return 1;
            auto barrier = [&](const double* xv) {
                double b = 0;
                for (int j = 0; j < n; j++) b += -std::log(1.0 - xv[j]) - std::log(1.0 + xv[j]);
                return opt.resto_mu * b;
            };
            const double phi = 0.5 * V + barrier(x);
            if (phi_prev >= 0) {
                stall = (phi_prev - phi <= opt.resto_stall * phi_prev) ? stall + 1 : 0;
                if (stall >= 2) return 4;
            }
            phi_prev = phi;
            double dmax = 0;
            for (int j = 0; j < n; j++) dmax = std::max(dmax, Mr[j * n + j]);
            const double lam = 1e-2 * std::min(1.0, std::sqrt(V)) * (1.0 + dmax);
            double A[NMAX * NMAX], rhs[NMAX], gp[NMAX], dxr[NMAX];
            for (int i = 0; i < n * n; i++) A[i] = Mr[i];
            for (int j = 0; j < n; j++) {
                const double u = 1.0 - x[j], l = 1.0 + x[j];
                gp[j] = br[j] + opt.resto_mu * (1.0 / u - 1.0 / l);
                A[j * n + j] += opt.resto_mu * (1.0 / (u * u) + 1.0 / (l * l)) + lam;
                rhs[j] = -gp[j];
            }
            double shift = 0.0;
            bool ok = false;
            for (int tries = 0; tries < 40 && !ok; tries++) {
                ok = chol_solve(A, n, shift, rhs, dxr);
                shift = (shift == 0.0) ? 1e-8 : shift * 10;
            }
            if (!ok) return 4;
            double amax = 1.0, dphi = 0;
            for (int j = 0; j < n; j++) {
                if (dxr[j] > 0) amax = std::min(amax, opt.tau_min * (1.0 - x[j]) / dxr[j]);
                if (dxr[j] < 0) amax = std::min(amax, opt.tau_min * (-1.0 - x[j]) / dxr[j]);
                dphi += gp[j] * dxr[j];
            }
            double al = amax, xr[NMAX];
            bool acc = false;
            for (int ls = 0; ls < opt.max_ls && !acc; ls++) {
                for (int j = 0; j < n; j++) xr[j] = x[j] + al * dxr[j];
                prob.eval(xr, &ft, gradt, gt.data(), Jt.data());
                ne++;
                double Vt = 0;
                for (int r = 0; r < m; r++) {
                    const double v = gt[r];
                    double e = 0;
                    if (hlo[r]) { const double el = (L[r] + opt.resto_delta) - v; if (el > 0) e = el; }
                    if (hhi[r]) { const double eh = v - (U[r] - opt.resto_delta); if (e == 0 && eh > 0) e = eh; }
                    Vt += e * e;
                }
                const double phit = 0.5 * Vt + barrier(xr);
                if (phit <= phi + opt.eta * al * dphi) acc = true;
                else al *= 0.5;
            }
            if (!acc) return 4;
            for (int j = 0; j < n; j++) { x[j] = xr[j]; grad[j] = gradt[j]; }
            f = ft;
            g.swap(gt);
            J.swap(Jt);
            iter++;
        }
    };
    // the quality-function oracle's sigma at the current iterate (mu_strategy 2 only): reads the
    // dual residual rd_q and the slack residuals rplo / rphi of step 1
    double rd_q[NMAX];
    auto qf_sigma = [&](double avg) -> double {
        double M[NMAX * NMAX], b0[NMAX], b1[NMAX], dx0[NMAX], dx1[NMAX];
        for (int i = 0; i < n * n; i++) M[i] = H[i];
        for (int j = 0; j < n; j++) { b0[j] = -grad[j]; b1[j] = 0; }
        for (int r = 0; r < R; r++) {
            grow(J, r, a);
            double sig = 0, c0 = 0, c1 = 0;
            if (hlo[r]) { const double sr = zlo[r] / slo[r]; sig += sr; c0 -= sr * rplo[r]; c1 += 1.0 / slo[r]; }
            if (hhi[r]) { const double sr = zhi[r] / shi[r]; sig += sr; c0 += sr * rphi[r]; c1 -= 1.0 / shi[r]; }
            for (int i = 0; i < n; i++) {
                b0[i] += a[i] * c0;
                b1[i] += a[i] * c1;
                for (int j = 0; j < n; j++) M[i * n + j] += sig * a[i] * a[j];
            }
        }
        double shift = 0.0;
        bool ok = false;
        for (int tries = 0; tries < 40 && !ok; tries++) {
            ok = chol_solve(M, n, shift, b0, dx0) && chol_solve(M, n, shift, b1, dx1);
            shift = (shift == 0.0) ? 1e-8 : shift * 10;
        }
        if (!ok) return 0.1;
        std::vector<double> adx0(R), adx1(R);
        for (int r = 0; r < R; r++) {
            grow(J, r, a);
            double u0 = 0, u1 = 0;
            for (int j = 0; j < n; j++) { u0 += a[j] * dx0[j]; u1 += a[j] * dx1[j]; }
            adx0[r] = u0;
            adx1[r] = u1;
        }
        double nd = 0, np = 0;
        for (int j = 0; j < n; j++) nd += rd_q[j] * rd_q[j];
        int ns = 0;
        for (int r = 0; r < R; r++) {
            if (hlo[r]) { np += rplo[r] * rplo[r]; ns++; }
            if (hhi[r]) { np += rphi[r] * rphi[r]; ns++; }
        }
        nd /= std::max(1, n);
        np /= std::max(1, ns);
        auto q = [&](double sg) {
            const double mu_s = sg * avg;
            const double tau = std::max(opt.tau_min, 1.0 - mu_s);
            double ap = 1.0, ad = 1.0;
            for (int r = 0; r < R; r++) {
                const double adx = adx0[r] + mu_s * adx1[r];
                if (hlo[r]) {
                    const double ds = adx + rplo[r], dz = mu_s / slo[r] - zlo[r] - zlo[r] / slo[r] * ds;
                    if (ds < 0) ap = std::min(ap, -tau * slo[r] / ds);
                    if (dz < 0) ad = std::min(ad, -tau * zlo[r] / dz);
                }
                if (hhi[r]) {
                    const double ds = -adx + rphi[r], dz = mu_s / shi[r] - zhi[r] - zhi[r] / shi[r] * ds;
                    if (ds < 0) ap = std::min(ap, -tau * shi[r] / ds);
                    if (dz < 0) ad = std::min(ad, -tau * zhi[r] / dz);
                }
            }
            double cc = 0;
            for (int r = 0; r < R; r++) {
                const double adx = adx0[r] + mu_s * adx1[r];
                if (hlo[r]) {
                    const double ds = adx + rplo[r], dz = mu_s / slo[r] - zlo[r] - zlo[r] / slo[r] * ds;
                    const double c = (slo[r] + ap * ds) * (zlo[r] + ad * dz);
                    cc += c * c;
                }
                if (hhi[r]) {
                    const double ds = -adx + rphi[r], dz = mu_s / shi[r] - zhi[r] - zhi[r] / shi[r] * ds;
                    const double c = (shi[r] + ap * ds) * (zhi[r] + ad * dz);
                    cc += c * c;
                }
            }
            return (1 - ad) * (1 - ad) * nd + (1 - ap) * (1 - ap) * np + cc / std::max(1, ns);
        };
        const double smin = std::max(1e-6, mu_min / avg), smax = std::min(100.0, mu_max_qf / avg);
        if (opt.qf_grid > 0) {
            // the device's form (study): q on a fixed log grid of sigma over [1e-6, 100], argmin
            // (first of equals), clipped to [smin, smax]
            double best = 1.0, fb = 1e300;
            for (int k = 0; k < opt.qf_grid; k++) {
                const double sg = std::pow(10.0, -6.0 + 8.0 * k / (opt.qf_grid - 1));
                const double fq = q(sg);
                if (fq < fb) { fb = fq; best = sg; }
            }
            return std::min(std::max(best, smin), std::max(smax, smin));
        }
        const double q1 = q(1.0);
        const bool up = q(1.0 - 1e-4) > q1;  // q decreases towards sigma > 1
        const double gr = 0.5 * (std::sqrt(5.0) - 1.0);
        // golden section on [lo, hi] (log scale below 1), at most 8 steps
        double lo = up ? 1.0 : std::log(std::min(smin, 1.0)), hi = up ? std::max(smax, 1.0) : 0.0;
        auto sig_of = [&](double t) { return up ? t : std::exp(t); };
        double m1 = hi - gr * (hi - lo), m2 = lo + gr * (hi - lo);
        double f1 = q(sig_of(m1)), f2 = q(sig_of(m2));
        for (int k = 0; k < 8; k++) {
            if (sig_of(hi) - sig_of(lo) < 1e-2 * sig_of(hi)) break;
            if (f1 <= f2) { hi = m2; m2 = m1; f2 = f1; m1 = hi - gr * (hi - lo); f1 = q(sig_of(m1)); }
            else { lo = m1; m1 = m2; f1 = f2; m2 = lo + gr * (hi - lo); f2 = q(sig_of(m2)); }
        }
        double best = f1 <= f2 ? sig_of(m1) : sig_of(m2), fb = std::min(f1, f2);
        if (q1 < fb) best = 1.0;
        return std::min(std::max(best, smin), std::max(smax, smin));
    };
    for (it = 0; it < opt.max_iter; it++) {
        // 1. residuals and errors
        double rd[NMAX];
        for (int j = 0; j < n; j++) rd[j] = grad[j];
        double inf_p = 0, compl0 = 0, sumz = 0;
        int nside = 0;
        for (int r = 0; r < R; r++) {
            const double v = val(g, x, r);
            grow(J, r, a);
            double w = 0;
            if (hlo[r]) {
                rplo[r] = (v - L[r]) - slo[r];
                w += zlo[r];
                inf_p = std::max(inf_p, std::fabs(rplo[r]));
                compl0 = std::max(compl0, slo[r] * zlo[r]);
                sumz += zlo[r];
                nside++;
            }
            if (hhi[r]) {
                rphi[r] = (U[r] - v) - shi[r];
                w -= zhi[r];
                inf_p = std::max(inf_p, std::fabs(rphi[r]));
                compl0 = std::max(compl0, shi[r] * zhi[r]);
                sumz += zhi[r];
                nside++;
            }
            for (int j = 0; j < n; j++) rd[j] -= w * a[j];
        }
        double inf_d = 0;
        for (int j = 0; j < n; j++) inf_d = std::max(inf_d, std::fabs(rd[j]));
        for (int j = 0; j < n; j++) rd_q[j] = rd[j];
        const double sd = std::max(opt.s_max, sumz / std::max(1, nside)) / opt.s_max;
        const double E0 = std::max(std::max(inf_d / sd, inf_p), compl0 / sd);
        res.kkt_error = E0;
        if (E0 <= opt.tol) { res.status = 0; break; }
        // 2. barrier update. Emu is the barrier problem's error at the iteration's starting mu.
        double Emu;
        {
            double cm = 0;
            for (int r = 0; r < R; r++) {
                if (hlo[r]) cm = std::max(cm, std::fabs(slo[r] * zlo[r] - mu));
                if (hhi[r]) cm = std::max(cm, std::fabs(shi[r] * zhi[r] - mu));
            }
            Emu = std::max(std::max(inf_d / sd, inf_p), cm / sd);
        }
        if (qf) {
            // Ipopt's default adaptive pair (IpAdaptiveMuUpdate.cpp, IpQualityFunctionMuOracle.cpp
            // with their default options), restated for the pricing study of DESIGN.md §5:
            //   globalisation obj-constr-filter: in free mode the iterate must be acceptable to a
            //   filter of the earlier free-mode iterates' (f, theta) with margin 1e-5 min(1, theta)
            //   (filter_margin_fact, filter_max_margin); else fixed (monotone) mode from
            //   0.8 avg(s z) (adaptive_mu_monotone_init_factor), back to free mode once acceptable;
            //   oracle quality-function: mu = sigma avg(s z), sigma minimising the quality function
            //   q = (1 - a_D)^2 |r_d|^2 / n_d + (1 - a_P)^2 |r_p|^2 / n_p + |(s + a_P ds)(z + a_D dz)|^2 / n_c
            //   (quality_function_norm_type 2-norm-squared, no centrality or balancing term) of the
            //   step dx(mu) = dx_aff + mu dx_1 with fraction-to-boundary step sizes a_P, a_D,
            //   by golden section (at most 8 steps, sigma tolerance 1e-2) on [sigma_min = 1e-6, 1] in
            //   log scale or [1, sigma_max = 100], whichever side q decreases into from sigma = 1.
            double sum = 0, theta = 0;
            for (int r = 0; r < R; r++) {
                if (hlo[r]) { sum += slo[r] * zlo[r]; theta += std::fabs(rplo[r]); }
                if (hhi[r]) { sum += shi[r] * zhi[r]; theta += std::fabs(rphi[r]); }
            }
            const double avg = sum / std::max(1, nside);
            if (mu_max_qf < 0) mu_max_qf = std::min(1e5, 1e3 * avg);
            const double margin = 1e-5 * std::min(1.0, theta);
            bool acceptable = true;
            for (size_t q = 0; q < gf_f.size(); q++)
                if (!(f + margin < gf_f[q] || theta + margin < gf_t[q])) acceptable = false;
            const double mu_old = mu;
            if (free_mode && !acceptable) {
                free_mode = false;
                mu = std::max(mu_min, qf_grid(0.8 * avg));
            } else if (!free_mode && acceptable) {
                free_mode = true;
            }
            if (free_mode) {
                gf_f.push_back(f);
                gf_t.push_back(theta);
                mu = std::max(mu_min, std::min(qf_grid(qf_sigma(avg) * avg), mu_max_qf));
            } else if (Emu <= opt.kappa_eps * mu && mu > mu_min) {
                mu = std::max(mu_min, std::min(opt.kappa_mu * mu, std::pow(mu, opt.theta_mu)));
            }
            if (mu != mu_old) {
                filt_theta.clear();
                filt_phi.clear();
            }
        } else if (opt.mu_strategy == 1) {
            // adaptive (Ipopt's mu_strategy "adaptive", KPR/Parameters.h:57): free mode takes mu
            // from the LOQO oracle, sigma = 0.1 min(0.05 (1 - xi) / xi, 2)^3 with xi = min(s z) /
            // avg(s z); the kkt-error globalisation switches to fixed (monotone) mode, from
            // 0.8 x avg(s z), when E0 has not fallen below 0.9999 x the largest of the last four
            // free-mode values, and back to free mode once E0 is below 0.9999 x its value at the switch
            double sum = 0, mn = 1e300;
            for (int r = 0; r < R; r++) {
                if (hlo[r]) { const double c = slo[r] * zlo[r]; sum += c; mn = std::min(mn, c); }
                if (hhi[r]) { const double c = shi[r] * zhi[r]; sum += c; mn = std::min(mn, c); }
            }
            const double avg = sum / std::max(1, nside);
            bool progress = kkt_ref.size() < 4;
            if (!progress) {
                double mx = 0;
                for (double v : kkt_ref) mx = std::max(mx, v);
                progress = E0 <= 0.9999 * mx;
            }
            const double mu_old = mu;
            if (free_mode && !progress) {
                free_mode = false;
                mu = std::max(mu_min, (opt.mu_study & 1) ? 0.8 * avg : mu_grid(0.8 * avg));
                kkt_ref.assign(1, E0);
            } else if (!free_mode && progress && !kkt_ref.empty() && E0 <= 0.9999 * kkt_ref.back()) {
                free_mode = true;
                kkt_ref.clear();
            }
            if (free_mode) {
                kkt_ref.push_back(E0);
                if (kkt_ref.size() > 4) kkt_ref.erase(kkt_ref.begin());
                const double xi = mn / avg;
                const double sg = 0.1 * std::pow(std::min(0.05 * (1 - xi) / xi, 2.0), 3);
                mu = std::max(mu_min, std::min((opt.mu_study & 1) ? sg * avg : mu_grid(sg * avg), 1e5));
            } else if (Emu <= opt.kappa_eps * mu && mu > opt.tol / 10) {
                mu = std::max(opt.tol / 10, std::min(opt.kappa_mu * mu, std::pow(mu, opt.theta_mu)));
            }
            if (mu != mu_old) {
                filt_theta.clear();
                filt_phi.clear();
            }
        } else if (Emu <= opt.kappa_eps * mu && mu > opt.tol / 10) {
            // monotone: at most one decrease per iteration
            mu = std::max(opt.tol / 10, std::min(opt.kappa_mu * mu, std::pow(mu, opt.theta_mu)));
            filt_theta.clear();
            filt_phi.clear();
        }
        // 3. reduced Newton system
        double M[NMAX * NMAX], rhs[NMAX];
        for (int i = 0; i < n * n; i++) M[i] = H[i];
        for (int j = 0; j < n; j++) rhs[j] = -grad[j];
        for (int r = 0; r < R; r++) {
            grow(J, r, a);
            double sig = 0, c = 0;
            if (hlo[r]) { const double s = zlo[r] / slo[r]; sig += s; c += mu / slo[r] - s * rplo[r]; }
            if (hhi[r]) { const double s = zhi[r] / shi[r]; sig += s; c -= mu / shi[r] - s * rphi[r]; }
            for (int i = 0; i < n; i++) {
                rhs[i] += a[i] * c;
                for (int j = 0; j < n; j++) M[i * n + j] += sig * a[i] * a[j];
            }
        }
        double dx[NMAX];
        {
            // inertia correction: shift the diagonal until the factorisation succeeds (bounded)
            double shift = 0.0;
            bool ok = false;
            for (int tries = 0; tries < 40 && !ok; tries++) {
                ok = chol_solve(M, n, shift, rhs, dx);
                shift = (shift == 0.0) ? 1e-8 : shift * 10;
            }
            if (!ok) { res.status = 2; break; }
        }
        // 4. step components and fraction to boundary
        const double tau = std::max(opt.tau_min, 1.0 - mu);
        double ap = 1.0, ad = 1.0, rp1 = 0, bdir = 0, logs = 0;
        for (int r = 0; r < R; r++) {
            grow(J, r, a);
            double adx = 0;
            for (int j = 0; j < n; j++) adx += a[j] * dx[j];
            if (hlo[r]) {
                const double s = zlo[r] / slo[r];
                dslo[r] = adx + rplo[r];
                dzlo[r] = mu / slo[r] - zlo[r] - s * dslo[r];
                if (dslo[r] < 0) ap = std::min(ap, -tau * slo[r] / dslo[r]);
                if (dzlo[r] < 0) ad = std::min(ad, -tau * zlo[r] / dzlo[r]);
                rp1 += std::fabs(rplo[r]); bdir += dslo[r] / slo[r]; logs += std::log(slo[r]);
            }
            if (hhi[r]) {
                const double s = zhi[r] / shi[r];
                dshi[r] = -adx + rphi[r];
                dzhi[r] = mu / shi[r] - zhi[r] - s * dshi[r];
                if (dshi[r] < 0) ap = std::min(ap, -tau * shi[r] / dshi[r]);
                if (dzhi[r] < 0) ad = std::min(ad, -tau * zhi[r] / dzhi[r]);
                rp1 += std::fabs(rphi[r]); bdir += dshi[r] / shi[r]; logs += std::log(shi[r]);
            }
        }
        // 5. filter line search (Ipopt's, without restoration): theta = ||c(x) - s||_1,
        //    barrier objective phi = f - mu sum ln s
        double gdx = 0;
        for (int i = 0; i < n; i++) gdx += grad[i] * dx[i];
        const double theta0 = rp1;
        if (theta_min < 0) theta_min = 1e-4 * std::max(1.0, theta0);
        const double phi0 = f - mu * logs;
        const double Dphi = gdx - mu * bdir;
        if (theta_max < 0) theta_max = 1e4 * std::max(1.0, theta0);
        // BFGS needs sum_r w_r a_r(x) with the updated multipliers z + ad*dz
        double wa_old[NMAX] = {0};
        for (int r = 0; r < R; r++) {
            double w = 0;
            if (hlo[r]) w += zlo[r] + ad * dzlo[r];
            if (hhi[r]) w -= zhi[r] + ad * dzhi[r];
            grow(J, r, a);
            for (int j = 0; j < n; j++) wa_old[j] += w * a[j];
        }
        double alpha = ap, xt[NMAX];
        bool accepted = false, ftype = false;
        for (int ls = 0; ls < opt.max_ls; ls++) {
            for (int j = 0; j < n; j++) xt[j] = x[j] + alpha * dx[j];
            prob.eval(xt, &ft, gradt, gt.data(), Jt.data());
            nevals++;
            double logt = 0, rpt = 0;
            for (int r = 0; r < R; r++) {
                const double v = val(gt, xt, r);
                if (hlo[r]) { const double st = slo[r] + alpha * dslo[r]; logt += std::log(st); rpt += std::fabs((v - L[r]) - st); }
                if (hhi[r]) { const double st = shi[r] + alpha * dshi[r]; logt += std::log(st); rpt += std::fabs((U[r] - v) - st); }
            }
            const double phit = ft - mu * logt, thetat = rpt;
            bool ok = thetat <= theta_max;
            for (size_t q = 0; ok && q < filt_theta.size(); q++)
                if (!(thetat < filt_theta[q] || phit < filt_phi[q])) ok = false;
            if (ok) {
                const bool switching = Dphi < 0 && alpha * std::pow(-Dphi, 2.3) > std::pow(theta0, 1.1);
                if (switching && theta0 <= theta_min) {
                    ok = phit <= phi0 + opt.eta * alpha * Dphi;
                    ftype = ok;
                } else {
                    ok = thetat <= (1 - 1e-5) * theta0 || phit <= phi0 - 1e-8 * theta0;
                    if (!ok && switching) { ok = phit <= phi0 + opt.eta * alpha * Dphi; ftype = ok; }
                }
            }
            if (ok) { accepted = true; break; }
            if (ls + 1 < opt.max_ls) alpha *= 0.5;
        }
        if (!accepted && nresto < opt.resto_max) {
            // 5b. restoration phase (the role of Ipopt's, which it enters when the line search finds
            //     no acceptable trial): minimise the constraint violation from x, then restart
            nresto++;
            it++;  // the failed iteration counts
            const int rs = restoration(it, nevals);
            if (rs == 1) { res.status = 1; break; }
            if (rs == 4) { res.status = 4; break; }
            // every row within its bounds: the interior point restarts at x (slacks and multipliers
            // as at the start, at the current mu; a fresh filter and BFGS matrix)
            res.restart_iter = it;
            init_slacks();
            for (int i = 0; i < n * n; i++) H[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
            first_update = true;
            lb_s.clear();
            lb_y.clear();
            lb_skips = 0;
            filt_theta.clear();
            filt_phi.clear();
            theta_max = -1;
            theta_min = -1;
            nfail = 0;
            free_mode = opt.mu_strategy >= 1;
            kkt_ref.clear();
            gf_f.clear();
            gf_t.clear();
            it--;  // (the loop's increment; restoration counted its own iterations)
            continue;
        }
        if (accepted && !ftype) { filt_theta.push_back((1 - 1e-5) * theta0); filt_phi.push_back(phi0 - 1e-8 * theta0); }
        // a trial forced after max_ls halvings counts as a failed line search; three in a row end
        // the solve (the role of Ipopt's failed restoration phase, which this solver does not have)
        nfail = accepted ? 0 : nfail + 1;
        // 6. accept the trial point; multipliers with kappa_sigma safeguard
        double wa_new[NMAX] = {0};
        for (int r = 0; r < R; r++) {
            double w = 0;
            if (hlo[r]) {
                const double zn = zlo[r] + ad * dzlo[r];
                w += zn;
                slo[r] = slo[r] + alpha * dslo[r];
                zlo[r] = std::min(std::max(zn, mu / (opt.kappa_sigma * slo[r])), opt.kappa_sigma * mu / slo[r]);
            }
            if (hhi[r]) {
                const double zn = zhi[r] + ad * dzhi[r];
                w -= zn;
                shi[r] = shi[r] + alpha * dshi[r];
                zhi[r] = std::min(std::max(zn, mu / (opt.kappa_sigma * shi[r])), opt.kappa_sigma * mu / shi[r]);
            }
            grow(Jt, r, at);
            for (int j = 0; j < n; j++) wa_new[j] += w * at[j];
        }
        if (opt.lbfgs_hist > 0) {
            // Ipopt's limited-memory BFGS of the Lagrangian Hessian (study only)
            std::vector<double> sv(n), y(n);
            double ss = 0, yy = 0, sy = 0;
            for (int j = 0; j < n; j++) {
                sv[j] = xt[j] - x[j];
                y[j] = (gradt[j] - grad[j]) - (wa_new[j] - wa_old[j]);
                ss += sv[j] * sv[j];
                yy += y[j] * y[j];
                sy += sv[j] * y[j];
            }
            if (sy <= std::sqrt(2.220446049250313e-16) * std::sqrt(ss) * std::sqrt(yy) || ss <= 0) {
                if (++lb_skips > 2) {
                    lb_s.clear();
                    lb_y.clear();
                    lb_skips = 0;
                    lbfgs_rebuild(1.0);
                }
            } else {
                lb_skips = 0;
                if ((int)lb_s.size() == opt.lbfgs_hist) {
                    lb_s.erase(lb_s.begin());
                    lb_y.erase(lb_y.begin());
                }
                lb_s.push_back(sv);
                lb_y.push_back(y);
                lbfgs_rebuild(std::min(std::max(sy / ss, 1e-8), 1e8));
            }
        } else {
        // damped BFGS on the Lagrangian Hessian
            double sv[NMAX], y[NMAX], Hs[NMAX];
            double ss = 0;
            for (int j = 0; j < n; j++) {
                sv[j] = xt[j] - x[j];
                y[j] = (gradt[j] - grad[j]) - (wa_new[j] - wa_old[j]);
                ss += sv[j] * sv[j];
            }
            double sy = 0;
            for (int j = 0; j < n; j++) sy += sv[j] * y[j];
            if (first_update && sy > 0 && ss > 1e-20) {
                double yy = 0;
                for (int j = 0; j < n; j++) yy += y[j] * y[j];
                const double sc = yy / sy;
                for (int i = 0; i < n * n; i++) H[i] = 0;
                for (int j = 0; j < n; j++) H[j * n + j] = sc;
                first_update = false;
            }
            double sHs = 0;
            for (int i = 0; i < n; i++) {
                Hs[i] = 0;
                for (int j = 0; j < n; j++) Hs[i] += H[i * n + j] * sv[j];
                sHs += sv[i] * Hs[i];
            }
            if (ss > 1e-20 && sHs > 1e-20) {
                const double theta = (sy >= 0.2 * sHs) ? 1.0 : 0.8 * sHs / (sHs - sy);
                double rv[NMAX], sr = 0;
                for (int j = 0; j < n; j++) { rv[j] = theta * y[j] + (1 - theta) * Hs[j]; sr += sv[j] * rv[j]; }
                if (sr > 1e-20)
                    for (int i = 0; i < n; i++)
                        for (int j = 0; j < n; j++) H[i * n + j] += -Hs[i] * Hs[j] / sHs + rv[i] * rv[j] / sr;
            }
        }
        for (int j = 0; j < n; j++) { x[j] = xt[j]; grad[j] = gradt[j]; }
        f = ft;
        g.swap(gt);
        J.swap(Jt);
        if (nfail >= 3) { res.status = 2; it++; break; }
    }
    res.iterations = it;
    res.evaluations = nevals;
    res.obj = f;
    std::memcpy(g_out, g.data(), sizeof(double) * m);
    return res;
}

}  // namespace oracle
