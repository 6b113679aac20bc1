// armour-mi355x — one reach-set job = one (world, time interval): JRS -> PZ forward kinematics ->
// reduce_link_PZ -> PZ RNEA (nominal and interval fused) -> disturbance -> reduce -> torque radius.
// Follows, op for op, KPR/Trajectory.cu:63-254, KPR/Dynamics.cu:69-181 and
// KPR/armour_main.cu:118-211; runs as one 256-thread workgroup on gfx950 (reach_kernel in
// reach_kernel.hip) or sequentially in the CPU emulation used by tests.
#pragma once
#include "interval.h"
#include "pz_engine.h"

namespace armour {

constexpr int CAP_LM = 64;    // k-only monomials kept per link PZ after reduce_link_PZ
constexpr int CAP_UM = 256;   // k-only monomials kept per torque PZ after reduce

// Outputs of all jobs (global memory); index j = world * T + t
struct ReachOut {
    int T, NJ;
    uint16_t* link_hash;   // [j][NJ][CAP_LM]   (k-only hash < 2^14)
    double* link_coef;     // [j][NJ][CAP_LM][3]
    int* link_cnt;         // [j][NJ]
    double* link_center;   // [j][NJ][3]
    double* link_rad;      // [j][NJ][3]
    double* link_gens;     // [j][NJ][18]  3x6 column-major (KPR/armour_main.cu:114,125)
    uint16_t* tq_hash;     // [j][NF][CAP_UM]
    double* tq_coef;       // [j][NF][CAP_UM]
    int* tq_cnt;           // [j][NF]
    double* tq_center;     // [j][NF]
    double* tq_rad;        // [j][NF]
    double* torque_radius; // [j][NF]   (KPR/armour_main.cu:173-211)
    int* err;              // [world]
};

// per-joint JRS scalars of one interval (KPR/Trajectory.cu:71-245)
struct JrsJoint {
    double cos_c, cos_k, cos_e;
    double sin_c, sin_k, sin_e;
    double qd_c, qd_k, qd_e, qda_e;
    double qdd_c, qdd_k, qdd_e;
};

// ---- Bernstein trajectory, written in Bernstein form (same as oracle/src/traj.cpp) ----
AD double bz_q(double q0, double Tqd0, double TTqdd0, double k, double t) {
    const double b0 = q0, b1 = q0 + Tqd0 / 5, b2 = q0 + (2 * Tqd0) / 5 + TTqdd0 / 20, b3 = q0 + k;
    const double u = 1.0 - t, u2 = u * u, t2 = t * t;
    const double B0 = u2 * u2 * u, B1 = 5 * t * u2 * u2, B2 = 10 * t2 * u2 * u;
    const double B345 = t2 * t * (10 * u2 + 5 * t * u + t2);
    return B0 * b0 + B1 * b1 + B2 * b2 + B345 * b3;
}
AD double bz_qd(double q0, double Tqd0, double TTqdd0, double k, double t) {
    const double b0 = q0, b1 = q0 + Tqd0 / 5, b2 = q0 + (2 * Tqd0) / 5 + TTqdd0 / 20, b3 = q0 + k;
    const double u = 1.0 - t, u2 = u * u;
    return 5 * (u2 * u2 * (b1 - b0) + 4 * t * u2 * u * (b2 - b1) + 6 * t * t * u2 * (b3 - b2));
}
AD double bz_qdd(double q0, double Tqd0, double TTqdd0, double k, double t) {
    const double b0 = q0, b1 = q0 + Tqd0 / 5, b2 = q0 + (2 * Tqd0) / 5 + TTqdd0 / 20, b3 = q0 + k;
    const double u = 1.0 - t;
    return 20 * (u * u * u * (b2 - 2 * b1 + b0) + 3 * t * u * u * (b3 - 2 * b2 + b1) + 3 * t * t * u * (b2 - b3));
}
AD void q_roots(double Tqd0, double TTqdd0, double k, double* r2, double* r3) {
    const double disc = sqrt(64 * Tqd0 * Tqd0 + 14 * Tqd0 * TTqdd0 - 120 * k * Tqd0 + TTqdd0 * TTqdd0);
    const double den = 5 * (6 * Tqd0 - 12 * k + TTqdd0);
    *r2 = (2 * Tqd0 + TTqdd0 + disc) / den;
    *r3 = (2 * Tqd0 + TTqdd0 - disc) / den;
}
AD void qd_roots(double Tqd0, double TTqdd0, double k, double* r2, double* r3) {
    const double disc = sqrt(6 * (150 * k * k - 180 * k * Tqd0 - 20 * k * TTqdd0 + 54 * Tqd0 * Tqd0 + 14 * Tqd0 * TTqdd0 + TTqdd0 * TTqdd0));
    const double den = 10 * (6 * Tqd0 - 12 * k + TTqdd0);
    *r2 = (18 * Tqd0 - 30 * k + 4 * TTqdd0 + disc) / den;
    *r3 = (18 * Tqd0 - 30 * k + 4 * TTqdd0 - disc) / den;
}
AD void qdd_roots_k0(double Tqd0, double TTqdd0, double* r1, double* r2) {
    const double disc = sqrt(2 * (152 * Tqd0 * Tqd0 + 42 * Tqd0 * TTqdd0 + 3 * TTqdd0 * TTqdd0));
    const double den = 10 * (6 * Tqd0 + TTqdd0);
    *r1 = (32 * Tqd0 + 6 * TTqdd0 + disc) / den;
    *r2 = (32 * Tqd0 + 6 * TTqdd0 - disc) / den;
}
AD void bound_k_indep(double vlb, double vub, double s_lb, double s_ub, double e1, double v1, double e2, double v2, double* lo, double* hi) {
    if (vlb > vub) { const double t = vlb; vlb = vub; vub = t; }
    if (s_lb < e1 && e1 < s_ub) { vlb = fmin(vlb, v1); vub = fmax(vub, v1); }
    if (s_lb < e2 && e2 < s_ub) { vlb = fmin(vlb, v2); vub = fmax(vub, v2); }
    *lo = vlb;
    *hi = vub;
}

// KPR/Trajectory.cu:63-245 for joint i over [s_ind/T, (s_ind+1)/T]
ADN JrsJoint jrs_joint(const RobotParams& rp, int T, int s_ind, int i, double q0, double qd0, double qdd0) {
    const double D = rp.duration;
    const double Tqd0 = qd0 * D, TTqdd0 = qdd0 * D * D;
    const double ds = 1.0 / T;
    const double s_lb = s_ind * ds, s_ub = (s_ind + 1) * ds;
    const double kr = rp.k_range[i];
    JrsJoint J;
    // k-independent extrema (Trajectory.cu:36-58)
    double qe1, qe2, qde1, qde2, qdde1, qdde2;
    q_roots(Tqd0, TTqdd0, 0.0, &qe1, &qe2);
    qd_roots(Tqd0, TTqdd0, 0.0, &qde1, &qde2);
    qdd_roots_k0(Tqd0, TTqdd0, &qdde1, &qdde2);
    const double qv1 = bz_q(q0, Tqd0, TTqdd0, 0.0, qe1), qv2 = bz_q(q0, Tqd0, TTqdd0, 0.0, qe2);
    const double qdv1 = bz_qd(q0, Tqd0, TTqdd0, 0.0, qde1) / D, qdv2 = bz_qd(q0, Tqd0, TTqdd0, 0.0, qde2) / D;
    const double qddv1 = bz_qdd(q0, Tqd0, TTqdd0, 0.0, qdde1) / (D * D), qddv2 = bz_qdd(q0, Tqd0, TTqdd0, 0.0, qdde2) / (D * D);

    // Part 1: q_des
    double kc_lb = s_lb * s_lb * s_lb * (6 * s_lb * s_lb - 15 * s_lb + 10);
    double kc_ub = s_ub * s_ub * s_ub * (6 * s_ub * s_ub - 15 * s_ub + 10);
    double kdc = (kc_ub + kc_lb) * 0.5;
    double kdr = (kc_ub - kc_lb) * 0.5 * kr;
    double ki_lb, ki_ub;
    bound_k_indep(bz_q(q0, Tqd0, TTqdd0, 0.0, s_lb), bz_q(q0, Tqd0, TTqdd0, 0.0, s_ub), s_lb, s_ub, qe1, qv1, qe2, qv2, &ki_lb, &ki_ub);
    double kir = (ki_ub - ki_lb) * 0.5;
    const double qc = (ki_lb + ki_ub) * 0.5;
    const Ival qri = iv(-kdr - kir - rp.qe, kdr + kir + rp.qe);
    const Ival kI = iv(-kr, kr);
    const Ival arg = iadd(iadd(qc, imul(kdc, kI)), qri);
    const Ival sq = isqr(iadd(qri, imul(kdc, kI)));
    // Part 1.a cos (Trajectory.cu:103-117)
    {
        double cc = cos(qc);
        Ival r = isub(imul(sin(qc), ineg(qri)), imul(imul(0.5, icos(arg)), sq));
        cc += icenter(r);
        r = isub(r, icenter(r));
        J.cos_c = cc;
        J.cos_k = -kdc * kr * sin(qc);
        J.cos_e = iradius(r);
    }
    // Part 1.b sin (Trajectory.cu:120-134)
    {
        double sc = sin(qc);
        Ival r = isub(imul(cos(qc), qri), imul(imul(0.5, isin(arg)), sq));
        sc += icenter(r);
        r = isub(r, icenter(r));
        J.sin_c = sc;
        J.sin_k = kdc * kr * cos(qc);
        J.sin_e = iradius(r);
    }
    // Part 2: qd_des (Trajectory.cu:151-192)
    kc_lb = (30 * s_lb * s_lb * (s_lb - 1) * (s_lb - 1)) / D;
    kc_ub = (30 * s_ub * s_ub * (s_ub - 1) * (s_ub - 1)) / D;
    if (kc_ub < kc_lb) { const double t = kc_lb; kc_lb = kc_ub; kc_ub = t; }
    kdc = (kc_ub + kc_lb) * 0.5 * kr;
    kdr = (kc_ub - kc_lb) * 0.5 * kr;
    bound_k_indep(bz_qd(q0, Tqd0, TTqdd0, 0.0, s_lb) / D, bz_qd(q0, Tqd0, TTqdd0, 0.0, s_ub) / D, s_lb, s_ub, qde1, qdv1, qde2, qdv2, &ki_lb, &ki_ub);
    kir = (ki_ub - ki_lb) * 0.5;
    J.qd_c = (ki_lb + ki_ub) * 0.5;
    J.qd_k = kdc;
    J.qd_e = kdr + kir + rp.qde;
    J.qda_e = kdr + kir + rp.qdae;
    // Part 3: qdd_des (Trajectory.cu:195-244)
    const double MAXIMA = 0.5 - sqrt(3.0) / 6, MINIMA = 0.5 + sqrt(3.0) / 6;
    const double tl = (60 * s_lb * (2 * s_lb * s_lb - 3 * s_lb + 1)) / D / D;
    const double tu = (60 * s_ub * (2 * s_ub * s_ub - 3 * s_ub + 1)) / D / D;
    if (s_ub <= MAXIMA) { kc_lb = tl; kc_ub = tu; }
    else if (s_lb <= MAXIMA) { kc_lb = fmin(tl, tu); kc_ub = (60 * MAXIMA * (2 * MAXIMA * MAXIMA - 3 * MAXIMA + 1)) / D / D; }
    else if (s_ub <= MINIMA) { kc_lb = tu; kc_ub = tl; }
    else if (s_lb <= MINIMA) { kc_lb = (60 * MINIMA * (2 * MINIMA * MINIMA - 3 * MINIMA + 1)) / D / D; kc_ub = fmax(tl, tu); }
    else { kc_lb = tl; kc_ub = tu; }
    kdc = (kc_ub + kc_lb) * 0.5 * kr;
    kdr = (kc_ub - kc_lb) * 0.5 * kr;
    bound_k_indep(bz_qdd(q0, Tqd0, TTqdd0, 0.0, s_lb) / (D * D), bz_qdd(q0, Tqd0, TTqdd0, 0.0, s_ub) / (D * D), s_lb, s_ub, qdde1, qddv1, qdde2, qddv2, &ki_lb, &ki_ub);
    kir = (ki_ub - ki_lb) * 0.5;
    J.qdd_c = (ki_lb + ki_ub) * 0.5;
    J.qdd_k = kdc;
    J.qdd_e = kdr + kir + rp.qddae;
    return J;
}

// PZ from raw candidate monomials with the reference constructor's simplify (PZsparse.cu:120-205)
// — tiny lists, done by thread 0
ADN void h_make_raw(Ctx& x, int o, int R, int C, const double* center, int nc, const uint64_t* hs, const double (*cf)[9]) {
    if (x.g.tid == 0) {
        const int n = R * C;
        int ord[4];
        for (int i = 0; i < nc; i++) ord[i] = i;
        for (int i = 1; i < nc; i++)  // insertion sort by hash (stable, as std::sort for n <= 16)
            for (int j = i; j > 0 && hs[ord[j]] < hs[ord[j - 1]]; j--) { const int t = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = t; }
        double keep_c[4][9];
        uint64_t keep_h[4];
        int K = 0;
        double red[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        int i = 0;
        while (i < nc) {
            double acc[9];
            for (int e = 0; e < n; e++) acc[e] = cf[ord[i]][e];
            int j = i + 1;
            for (; j < nc && hs[ord[j]] == hs[ord[i]]; j++)
                for (int e = 0; e < n; e++) acc[e] = acc[e] + cf[ord[j]][e];
            if (frob_norm(acc, n) <= x.thr) {
                for (int e = 0; e < n; e++) red[e] = red[e] + fabs(acc[e]);
            } else {
                for (int e = 0; e < n; e++) keep_c[K][e] = acc[e];
                keep_h[K] = hs[ord[i]];
                K++;
            }
            i = j;
        }
        PZH& h = x.H[o];
        h.R = R; h.C = C; h.comp = -1; h.scaled = 0; h.neg = 0; h.scale = 1.0; h.stride = n;
        for (int e = 0; e < 9; e++) { h.center[e] = e < n ? center[e] : 0.0; h.ind[0][e] = 0.0; h.ind[1][e] = 0.0; }
        if (frob_norm(red, n) != 0)
            for (int e = 0; e < n; e++) { h.ind[0][e] += red[e]; h.ind[1][e] += red[e]; }
        if (x.A->hused + K > x.A->hcap || x.A->cused + (long)K * n > x.A->ccap) {
            *x.err |= ERR_ARENA;
            h.cnt = 0; h.hoff = 0; h.coff = 0;
        } else {
            h.cnt = K; h.hoff = x.A->hused; h.coff = x.A->cused;
            for (int k = 0; k < K; k++) {
                x.A->h[h.hoff + k] = keep_h[k];
                for (int e = 0; e < n; e++) x.A->c[h.coff + (long)k * n + e] = keep_c[k][e];
            }
            x.A->hused += K;
            x.A->cused += (long)K * n;
        }
    }
    x.g.sync();
}

// constant PZ (no monomials): PZsparse(const MatrixXd&, double uncertainty) (PZsparse.cu:75-98)
AD void h_const(Ctx& x, int o, int R, int C, const double* center, double unc_int) {
    if (x.g.tid == 0) {
        PZH& h = x.H[o];
        const int n = R * C;
        h.R = R; h.C = C; h.cnt = 0; h.hoff = 0; h.coff = 0; h.stride = n; h.comp = -1; h.scaled = 0; h.neg = 0; h.scale = 1.0;
        for (int e = 0; e < 9; e++) {
            h.center[e] = e < n ? center[e] : 0.0;
            h.ind[0][e] = 0.0;
            h.ind[1][e] = e < n ? unc_int * fabs(center[e]) : 0.0;
        }
    }
    x.g.sync();
}

// materialised transpose of a full handle (PZsparse.cu:1050-1066)
ADN void op_transpose(Ctx& x, int o, int a) {
    if (x.g.tid == 0) {
        x.H[x.opa] = x.H[a];
        const PZH& A = x.H[x.opa];
        PZH& h = x.H[o];
        hdr_init(h, A.C, A.R);
        for (int i = 0; i < A.R; i++)
            for (int j = 0; j < A.C; j++) {
                h.center[j + i * A.C] = A.center[i + j * A.R];
                h.ind[0][j + i * A.C] = A.ind[0][i + j * A.R];
                h.ind[1][j + i * A.C] = A.ind[1][i + j * A.R];
            }
    }
    x.g.sync();
    const PZH& A = x.H[x.opa];
    const int n = nel(A);
    alloc_out(x, o, A.cnt, n);
    const PZH& O = x.H[o];
    if (O.cnt == A.cnt)
        for (int k = x.g.tid; k < A.cnt; k += x.g.n) {
            double m[9];
            read_mono(x, A, k, m);
            x.A->h[O.hoff + k] = mono_hash(x, A, k);
            for (int i = 0; i < A.R; i++)
                for (int j = 0; j < A.C; j++) x.A->c[O.coff + (long)k * n + j + i * A.C] = m[i + j * A.R];
        }
    x.g.sync();
}

// handle slots
namespace hs {
constexpr int R0 = 0;                       // R[0..MAX_J]       (MAX_J + 1)
constexpr int RT0 = R0 + MAX_J + 1;         // R_t[0..MAX_J-1]
constexpr int QD0 = RT0 + MAX_J;            // qd_des[0..NF-1]
constexpr int QDA0 = QD0 + NF;              // qda_des
constexpr int QDD0 = QDA0 + NF;             // qdda_des
constexpr int F0 = QDD0 + NF;               // F[0..MAX_J-1]
constexpr int N0 = F0 + MAX_J;              // N[0..MAX_J-1]
constexpr int W = N0 + MAX_J, WDOT = W + 1, WAUX = W + 2, LIN = W + 3, FF = W + 4, NN = W + 5;
constexpr int T1 = W + 6, T2 = T1 + 1, T3 = T1 + 2, T4 = T1 + 3, T5 = T1 + 4, T6 = T1 + 5, T7 = T1 + 6;
constexpr int CA = T1 + 8;                  // cross scratch A (11 slots)
constexpr int CB = CA + 11;                 // cross scratch B (11 slots)
constexpr int OPA = CB + 11, OPB = OPA + 1, OPC = OPA + 2;  // operand staging
constexpr int COUNT = OPA + 3;
}  // namespace hs

// outputs of one link / torque PZ
ADN void emit_link(Ctx& x, const ReachOut& out, long j, int l) {
    // reduce_link_PZ (PZsparse.cu:370-402) in monomial order, then emit the k-only part
    const int L = l;
    if (x.g.tid == 0) {
        PZH& h = x.H[hs::T7];
        const long base = (j * out.NJ + L);
        double* gens = out.link_gens + base * 18;
        for (int e = 0; e < 18; e++) gens[e] = 0.0;
        int jg = 0, kk = 0;
        double ind[3] = {h.ind[0][0], h.ind[0][1], h.ind[0][2]};
        for (int k = 0; k < h.cnt; k++) {
            const uint64_t hh = x.A->h[h.hoff + k];
            const double* c = x.A->c + h.coff + (long)k * 3;
            if (hh < HASH_K_ONLY) {
                if (kk < CAP_LM) {
                    out.link_hash[base * CAP_LM + kk] = (uint16_t)hh;
                    for (int e = 0; e < 3; e++) out.link_coef[(base * CAP_LM + kk) * 3 + e] = c[e];
                } else {
                    *x.err |= ERR_OUTCAP;
                }
                kk++;
            } else if (hh < HASH_K_LINKS_ONLY && (hh & K_MASK) == 0) {
                if (jg < 3) { for (int e = 0; e < 3; e++) gens[e + 3 * jg] = c[e]; }
                else *x.err |= ERR_LINKGEN;
                jg++;
            } else {
                for (int e = 0; e < 3; e++) ind[e] += fabs(c[e]);
            }
        }
        gens[0 + 3 * 3] = ind[0];
        gens[1 + 3 * 4] = ind[1];
        gens[2 + 3 * 5] = ind[2];
        out.link_cnt[base] = kk < CAP_LM ? kk : CAP_LM;
        for (int e = 0; e < 3; e++) { out.link_center[base * 3 + e] = h.center[e]; out.link_rad[base * 3 + e] = ind[e]; }
    }
    x.g.sync();
}

ADN void emit_torque(Ctx& x, const ReachOut& out, long j, int i, double* rdist, double* ured) {
    if (x.g.tid == 0) {
        PZH& h = x.H[hs::T7];
        const long base = j * NF + i;
        // disturbance u_int - u_nom: centres and monomials cancel exactly, the independent parts
        // add (armour_main.cu:135-137, PZsparse.cu:813-834)
        rdist[i] = h.ind[1][0] + h.ind[0][0];
        // reduce (PZsparse.cu:352-368)
        double ind = h.ind[0][0];
        int kk = 0;
        for (int k = 0; k < h.cnt; k++) {
            const uint64_t hh = x.A->h[h.hoff + k];
            double c = x.A->c[h.coff + (long)k * h.stride + (h.comp >= 0 ? h.comp : 0)];
            if (h.scaled) c = h.scale * c;
            if (h.neg) c = -c;
            if (hh < HASH_K_ONLY) {
                if (kk < CAP_UM) {
                    out.tq_hash[base * CAP_UM + kk] = (uint16_t)hh;
                    out.tq_coef[base * CAP_UM + kk] = c;
                } else {
                    *x.err |= ERR_OUTCAP;
                }
                kk++;
            } else {
                ind += fabs(c);
            }
        }
        out.tq_cnt[base] = kk < CAP_UM ? kk : CAP_UM;
        out.tq_center[base] = h.center[0];
        out.tq_rad[base] = ind;
        ured[i] = ind;
    }
    x.g.sync();
}

// The whole job. q0/qd0/qdd0: this world's initial state.
AD void reach_job(Ctx& x, const RobotParams& rp, int T, int t, const double* q0, const double* qd0, const double* qdd0,
                  const ReachOut& out, long j, JrsJoint* jrs, double* scratch) {
    const int NJ = rp.num_joints;
    // ---- JRS (Trajectory.cu:63-254): scalars in parallel, PZs by thread 0 ----
    for (int i = x.g.tid; i < NF; i += x.g.n) jrs[i] = jrs_joint(rp, T, t, i, q0[i], qd0[i], qdd0[i]);
    x.g.sync();
    for (int i = 0; i < NF; i++) {
        const JrsJoint& J = jrs[i];
        uint64_t hh[4];
        double cf[4][9];
        // qd / qda / qdda 1-D PZs: k_i and qde_i / qdae_i / qddae_i monomials
        for (int v = 0; v < 3; v++) {
            const double c0 = v == 2 ? J.qdd_c : J.qd_c;
            hh[0] = slot_hash(SLOT_K + i);
            cf[0][0] = v == 2 ? J.qdd_k : J.qd_k;
            hh[1] = slot_hash((v == 0 ? SLOT_QDE : v == 1 ? SLOT_QDAE : SLOT_QDDAE) + i);
            cf[1][0] = v == 0 ? J.qd_e : v == 1 ? J.qda_e : J.qdd_e;
            h_make_raw(x, (v == 0 ? hs::QD0 : v == 1 ? hs::QDA0 : hs::QDD0) + i, 1, 1, &c0, 2, hh, cf);
        }
        if (rp.axes[i] != 0) {
            // rotation PZ about the joint axis (PZsparse.cu:179-205 + makeRotationMatrix :211-250)
            const int ax = rp.axes[i];
            double cen[9];
            for (int e = 0; e < 9; e++) cen[e] = (e % 4 == 0) ? 1.0 : 0.0;
            auto put = [&](double* Rm, double c, double s) {
                const double ns = -1.0 * s;
                if (ax == 1) { Rm[1 + 3] = c; Rm[1 + 6] = ns; Rm[2 + 3] = s; Rm[2 + 6] = c; }
                else if (ax == 2) { Rm[0] = c; Rm[0 + 6] = s; Rm[2] = ns; Rm[2 + 6] = c; }
                else { Rm[0] = c; Rm[0 + 3] = ns; Rm[1] = s; Rm[1 + 3] = c; }
            };
            put(cen, J.cos_c, J.sin_c);
            for (int m = 0; m < 4; m++) for (int e = 0; e < 9; e++) cf[m][e] = 0.0;
            put(cf[0], J.cos_k, 0.0); hh[0] = slot_hash(SLOT_K + i);
            put(cf[1], J.cos_e, 0.0); hh[1] = slot_hash(SLOT_COS + i);
            put(cf[2], 0.0, J.sin_k); hh[2] = slot_hash(SLOT_K + i);
            put(cf[3], 0.0, J.sin_e); hh[3] = slot_hash(SLOT_SIN + i);
            h_make_raw(x, hs::T1, 3, 3, cen, 4, hh, cf);
            h_const(x, hs::T2, 3, 3, rp.rpy[i], 0.0);
            op_mul(x, hs::R0 + i, hs::T2, hs::T1);
        } else {
            h_const(x, hs::R0 + i, 3, 3, rp.rpy[i], 0.0);
        }
        op_transpose(x, hs::RT0 + i, hs::R0 + i);
    }
    for (int i = NF; i < NJ; i++) {
        h_const(x, hs::R0 + i, 3, 3, rp.rpy[i], 0.0);
        op_transpose(x, hs::RT0 + i, hs::R0 + i);
    }
    h_const(x, hs::R0 + NJ, 3, 3, rp.rpy[MAX_J], 0.0);  // PZsparse(0, 0, 0)

    // ---- forward kinematics (Dynamics.cu:69-81) + reduce_link_PZ (armour_main.cu:124-126) ----
    {
        const int FKR = hs::W, FKT = hs::WDOT, P = hs::T1, TMP = hs::T2, BOX = hs::T3;
        h_const(x, FKR, 3, 3, rp.rpy[MAX_J], 0.0);
        h_zero(x, FKT, 3, 1);
        for (int i = 0; i < NJ; i++) {
            h_const(x, P, 3, 1, &rp.trans[3 * i], 0.0);
            op_mul(x, TMP, FKR, P);
            op_add(x, FKT, FKT, TMP, +1);
            op_mul(x, FKR, FKR, hs::R0 + i);
            // link box: generators on the qde_0 / qdae_0 / qddae_0 slots (Dynamics.cu:98-116)
            uint64_t hh[4];
            double cf[4][9];
            for (int m = 0; m < 3; m++) {
                for (int e = 0; e < 9; e++) cf[m][e] = 0.0;
                cf[m][m] = rp.link_g[i][m];
                hh[m] = slot_hash(NF * (m + 1));
            }
            h_make_raw(x, BOX, 3, 1, rp.link_c[i], 3, hh, cf);
            op_mul(x, TMP, FKR, BOX);
            op_add(x, hs::T7, TMP, FKT, +1);
            emit_link(x, out, j, i);
        }
    }

    // ---- RNEA, nominal and interval fused (Dynamics.cu:83-181) ----
    h_zero(x, hs::W, 3, 1);
    h_zero(x, hs::WDOT, 3, 1);
    h_zero(x, hs::WAUX, 3, 1);
    h_zero(x, hs::LIN, 3, 1);
    if (x.g.tid == 0) x.H[hs::LIN].center[2] = rp.gravity;
    x.g.sync();
    for (int i = 0; i < NJ; i++) {
        const int RT = hs::RT0 + i;
        const double* p = &rp.trans[3 * i];
        const double* c = &rp.com[3 * i];
        // line 16
        op_cross_pm(x, hs::T1, hs::WDOT, p, hs::CA);
        op_add(x, hs::T2, hs::LIN, hs::T1, +1);
        op_cross_pm(x, hs::T3, hs::WAUX, p, hs::CB);
        op_cross_pp(x, hs::T4, hs::W, hs::T3, hs::CA);
        op_add(x, hs::T5, hs::T2, hs::T4, +1);
        op_mul(x, hs::LIN, RT, hs::T5);
        // line 13
        op_mul(x, hs::W, RT, hs::W);
        if (rp.axes[i] != 0) {
            const int ax = (rp.axes[i] < 0 ? -rp.axes[i] : rp.axes[i]) - 1;
            op_add_one_dim(x, hs::W, hs::W, hs::QD0 + i, ax, 0);
            op_mul(x, hs::WAUX, RT, hs::WAUX);
            op_mul(x, hs::WDOT, RT, hs::WDOT);
            h_zero(x, hs::T1, 3, 1);
            op_add_one_dim(x, hs::T1, hs::T1, hs::QD0 + i, ax, 0);
            op_cross_pp(x, hs::T2, hs::WAUX, hs::T1, hs::CA);
            op_add(x, hs::WDOT, hs::WDOT, hs::T2, +1);
            op_add_one_dim(x, hs::WDOT, hs::WDOT, hs::QDD0 + i, ax, 0);
            op_add_one_dim(x, hs::WAUX, hs::WAUX, hs::QDA0 + i, ax, 0);
        } else {
            op_mul(x, hs::WAUX, RT, hs::WAUX);
            op_mul(x, hs::WDOT, RT, hs::WDOT);
        }
        // line 23 & 27
        op_cross_pm(x, hs::T1, hs::WDOT, c, hs::CA);
        op_add(x, hs::T2, hs::LIN, hs::T1, +1);
        op_cross_pm(x, hs::T3, hs::WAUX, c, hs::CB);
        op_cross_pp(x, hs::T4, hs::W, hs::T3, hs::CA);
        op_add(x, hs::T5, hs::T2, hs::T4, +1);
        {
            double m = rp.mass[i];
            h_const(x, hs::T6, 1, 1, &m, rp.mass_uncertainty);
        }
        op_mul(x, hs::F0 + i, hs::T6, hs::T5);
        // line 29
        h_const(x, hs::T6, 3, 3, &rp.inertia[i * 9], rp.inertia_uncertainty);
        op_mul(x, hs::T1, hs::T6, hs::WDOT);
        op_mul(x, hs::T2, hs::T6, hs::W);
        op_cross_pp(x, hs::T3, hs::WAUX, hs::T2, hs::CA);
        op_add(x, hs::N0 + i, hs::T1, hs::T3, +1);
    }
    h_zero(x, hs::FF, 3, 1);
    h_zero(x, hs::NN, 3, 1);
    double* rdist = scratch;
    double* ured = scratch + NF;
    for (int i = NJ - 1; i >= 0; i--) {
        const int R1 = hs::R0 + i + 1;
        // line 29: n = N + R*n + cross(com, F) + cross(p_{i+1}, R*f); R*f evaluated once
        op_mul(x, hs::T1, R1, hs::NN);
        op_add(x, hs::T2, hs::N0 + i, hs::T1, +1);
        op_cross_mp(x, hs::T3, &rp.com[3 * i], hs::F0 + i, hs::CA);
        op_add(x, hs::T4, hs::T2, hs::T3, +1);
        op_mul(x, hs::T5, R1, hs::FF);
        op_cross_mp(x, hs::T6, &rp.trans[3 * (i + 1)], hs::T5, hs::CA);
        op_add(x, hs::NN, hs::T4, hs::T6, +1);
        // line 28
        op_add(x, hs::FF, hs::T5, hs::F0 + i, +1);
        if (rp.axes[i] != 0 && i < NF) {
            const int ax = (rp.axes[i] < 0 ? -rp.axes[i] : rp.axes[i]) - 1;
            h_elem(x, hs::T1, hs::NN, ax, 0);
            h_scale(x, hs::T2, rp.armature[i], hs::QDD0 + i);
            op_add(x, hs::T3, hs::T1, hs::T2, +1);
            h_scale(x, hs::T2, rp.damping[i], hs::QD0 + i);
            op_add(x, hs::T7, hs::T3, hs::T2, +1);
            emit_torque(x, out, j, i, rdist, ured);
        }
    }

    // ---- torque radius (armour_main.cu:173-211) ----
    if (x.g.tid == 0) {
        const double ubc = rp.alpha * (rp.M_max - rp.M_min) * rp.eps;
        double tr[NF];
        Ival rho = Ival{0.0, 0.0};
        for (int i = 0; i < NF; i++) {
            const Ival tmp = iv(0.0 - rdist[i], 0.0 + rdist[i]);
            rho = iadd(rho, imul(tmp, tmp));
            tr[i] = ubc + 0.5 * fmax(fabs(tmp.lo), fabs(tmp.hi));
        }
        rho = isqrt(rho);
        for (int i = 0; i < NF; i++) tr[i] += 0.5 * rho.hi;
        for (int i = 0; i < NF; i++) tr[i] += ured[i];
        for (int i = 0; i < NF; i++) tr[i] += rp.friction[i];
        for (int i = 0; i < NF; i++) out.torque_radius[j * NF + i] = tr[i];
    }
    x.g.sync();
}

}  // namespace armour
