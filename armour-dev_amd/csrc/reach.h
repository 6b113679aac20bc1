// armour-mi355x — one reach-set job = one (world, time interval): JRS -> PZ forward kinematics ->
// reduce_link_PZ -> PZ RNEA (nominal and interval fused) -> disturbance -> reduce -> torque radius.
// Follows, op for op, KPR/Trajectory.cu:63-254, KPR/Dynamics.cu:69-181 and
// KPR/armour_main.cu:118-211; runs as one 256-thread workgroup on gfx950 (reach_kernel in
// reach_kernel.hip) or sequentially in the CPU emulation used by tests.
#pragma once
#include <initializer_list>
#include <vector>
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
__host__ __device__ __attribute__((noinline)) JrsJoint jrs_joint(const RobotParams& rp, int T, int s_ind, int i, double q0, double qd0, double qdd0) {
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

// ---------------------------------------------------------------------------------------------
// The reach program. The op sequence of one job depends only on the robot (joint axes, NJ), so
// the host builds it once (ProgramBuilder) as a tape of Ops with SSA-style handle slots (an
// output never aliases an operand, so operands are read in place — no staging copies), and the
// kernel interprets it: one switch whose bodies are force-inlined, one barrier per op.

enum : int {
    OP_JRS, OP_MAKE1D, OP_MAKEROT, OP_MAKEBOX, OP_CONST, OP_ZERO, OP_VIEW, OP_TRANSPOSE,
    OP_MUL, OP_ADD, OP_STACK3, OP_ADD1D, OP_EMIT_LINK, OP_EMIT_TORQUE, OP_TORQUE_RADIUS,
    OP_CROSS_C,   // fused cross with a constant vector: o, a = PZ, b = vector table (0 trans, 1 com), c = row, i = 0: a x v, 1: v x a
    OP_CROSS_PP,  // fused PZ x PZ cross: o, a, b
    OP_NCODES
};
constexpr int VEC_TRANS = 0, VEC_COM = 1;
enum : int { CONST_RPY = 0, CONST_TRANS = 1, CONST_MASS = 2, CONST_INERTIA = 3 };

struct Op {
    int code;
    int o, a, b, c;
    int i;
    int sync;   // barrier after this op
    int par;    // > 1: first of a lane-parallel group of par independent thread-0 ops of one code
    double s;
};


// thread-0 bodies are inlined too: an out-of-line variant (stack arrays passed through a lambda
// into a nested out-of-line call) was miscompiled for gfx950 — tools/dump_ops.py localised it to
// MAKEROT writing the wrong centre element
#define T0FN __host__ __device__ inline __attribute__((always_inline))

// ---- thread-0 bodies ----------------------------------------------------------------------

// PZ from raw candidate monomials with the reference constructor's simplify (PZsparse.cu:120-205)
T0FN void t0_make_raw(Ctx& x, int o, int R, int C, const double* center, int nc, const uint64_t* hs, const double (*cf)[9]) {
    // the reference's stable sort + merge + prune of <= 4 monomials, written with static indices
    // only (a run-time index into these small arrays would put them in scratch memory): members
    // of an equal-hash group are summed in index order (the stable order), pruned amounts and
    // |kept| sums are added in hash order, kept rows land at their hash rank
    constexpr int M = 4;
    const int n = R * C;
    uint64_t h[M];
    UNR for (int m = 0; m < M; m++) h[m] = m < nc ? hs[m] : ~(uint64_t)0;
    bool head[M], keep[M];
    double acc[M][9];
    UNR for (int m = 0; m < M; m++) {
        head[m] = m < nc;
        UNR for (int m2 = 0; m2 < m; m2++) if (h[m2] == h[m]) head[m] = false;
        UNR for (int e = 0; e < 9; e++) acc[m][e] = (m < nc && e < n) ? cf[m][e] : 0.0;
        UNR for (int m2 = m + 1; m2 < M; m2++)
            if (m2 < nc && h[m2] == h[m]) UNR for (int e = 0; e < 9; e++) if (e < n) acc[m][e] = acc[m][e] + cf[m2][e];
        keep[m] = head[m] && !(frob_norm(acc[m], n) <= x.thr);
    }
    int rk[M], pos[M], K = 0;
    UNR for (int m = 0; m < M; m++) {
        rk[m] = 0;
        pos[m] = 0;
        UNR for (int m2 = 0; m2 < M; m2++) {
            if (head[m2] && h[m2] < h[m]) rk[m]++;
            if (keep[m2] && h[m2] < h[m]) pos[m]++;
        }
        K += keep[m] ? 1 : 0;
    }
    double red[9], ab[9];
    UNR for (int e = 0; e < 9; e++) { red[e] = 0.0; ab[e] = 0.0; }
    UNR for (int r = 0; r < M; r++)
        UNR for (int m = 0; m < M; m++) {
            if (head[m] && !keep[m] && rk[m] == r) UNR for (int e = 0; e < 9; e++) red[e] = red[e] + fabs(acc[m][e]);
            if (keep[m] && pos[m] == r) UNR for (int e = 0; e < 9; e++) ab[e] = ab[e] + fabs(acc[m][e]);
        }
    PZH& hd = x.H[o];
    hdr_init(x, hd, R, C);
    for (int e = 0; e < n; e++) cen(x, hd)[e] = center[e];
    if (frob_norm(red, n) != 0)
        for (int e = 0; e < n; e++) { ind(x, hd, 0)[e] += red[e]; ind(x, hd, 1)[e] += red[e]; }
    UNR for (int e = 0; e < 9; e++) if (e < n) abs_(x, hd)[e] += ab[e];
    arena_alloc_t0(x, hd, K, n);
    if (hd.cnt == K)
        UNR for (int m = 0; m < M; m++)
            if (keep[m]) {
                x.ah[hd.hoff + pos[m]] = h[m];
                UNR for (int e = 0; e < 9; e++) if (e < n) x.ac[hd.coff + (long)pos[m] * n + e] = acc[m][e];
            }
}

// constant PZ (no monomials): PZsparse(const MatrixXd&, double uncertainty) (PZsparse.cu:75-98);
// the uncertainty enters only the interval part (ind[1]) of the fused nominal/interval pair
T0FN void t0_const(Ctx& x, int o, int R, int C, const double* center, double unc_int) {
    PZH& h = x.H[o];
    hdr_init(x, h, R, C);
    const int n = R * C;
    for (int e = 0; e < n; e++) {
        cen(x, h)[e] = center[e];
        ind(x, h, 1)[e] = unc_int * fabs(center[e]);
    }
}

// element (e >= 0) and/or scale view of a full handle: operator()(r,c) (PZsparse.cu:678-697)
// and PZ * double (PZsparse.cu:996-1030) — lazy, no simplify
T0FN void t0_view(Ctx& x, int o, int a, int e, int scaled, double s) {
    const PZH& P = x.H[a];
    PZH& h = x.H[o];
    const int n = e >= 0 ? 1 : nel(P);
    h.R = e >= 0 ? 1 : P.R;
    h.C = e >= 0 ? 1 : P.C;
    h.cnt = P.cnt; h.stride = P.stride; h.hoff = P.hoff; h.coff = P.coff;
    h.comp = e >= 0 ? e : P.comp;
    h.scaled = scaled;
    h.scale = scaled ? s : 1.0;
    if (P.comp >= 0 || P.scaled) err_or(x, ERR_HANDLES);  // views of views never occur in this program
    for (int q = 0; q < n; q++) {
        const int src = e >= 0 ? e : q;
        double c = cen(x, P)[src], i0 = ind(x, P, 0)[src], i1 = ind(x, P, 1)[src], ab = abs_(x, P)[src];
        if (scaled) { c = c * s; i0 = i0 * fabs(s); i1 = i1 * fabs(s); ab = ab * fabs(s); }
        cen(x, h)[q] = c; ind(x, h, 0)[q] = i0; ind(x, h, 1)[q] = i1; abs_(x, h)[q] = ab;
    }
}

// materialised transpose of a full handle (PZsparse.cu:1050-1066); operands are rotations with
// a handful of monomials, so thread 0 copies them
T0FN void t0_transpose(Ctx& x, int o, int a) {
    const PZH& A = x.H[a];
    PZH& h = x.H[o];
    hdr_init(x, h, A.C, A.R);
    for (int i = 0; i < A.R; i++)
        for (int j = 0; j < A.C; j++) {
            cen(x, h)[j + i * A.C] = cen(x, A)[i + j * A.R];
            ind(x, h, 0)[j + i * A.C] = ind(x, A, 0)[i + j * A.R];
            ind(x, h, 1)[j + i * A.C] = ind(x, A, 1)[i + j * A.R];
            abs_(x, h)[j + i * A.C] = abs_(x, A)[i + j * A.R];
        }
    const int n = nel(A);
    arena_alloc_t0(x, h, A.cnt, n);
    if (h.cnt == A.cnt)
        for (int k = 0; k < A.cnt; k++) {
            double m[9];
            read_mono(x, A, k, m);
            x.ah[h.hoff + k] = mono_hash(x, A, k);
            for (int i = 0; i < A.R; i++)
                for (int jj = 0; jj < A.C; jj++) x.ac[h.coff + (long)k * n + jj + i * A.C] = m[i + jj * A.R];
        }
    bytes_add(x, 2.0 * A.cnt * (8.0 + 8.0 * n));
}

T0FN void t0_make_1d(Ctx& x, int o, const JrsJoint& J, int i, int v) {
    // qd / qda / qdda 1-D PZs: k_i and qde_i / qdae_i / qddae_i monomials (Trajectory.cu:151-244)
    const double c0 = v == 2 ? J.qdd_c : J.qd_c;
    uint64_t hh[2];
    double cf[2][9];
    hh[0] = slot_hash(SLOT_K + i);
    cf[0][0] = v == 2 ? J.qdd_k : J.qd_k;
    hh[1] = slot_hash((v == 0 ? SLOT_QDE : v == 1 ? SLOT_QDAE : SLOT_QDDAE) + i);
    cf[1][0] = v == 0 ? J.qd_e : v == 1 ? J.qda_e : J.qdd_e;
    t0_make_raw(x, o, 1, 1, &c0, 2, hh, cf);
}

T0FN void t0_make_rot(Ctx& x, int o, const RobotParams& rp, const JrsJoint& J, int i) {
    // rotation PZ about the joint axis (PZsparse.cu:179-205 + makeRotationMatrix :211-250)
    const int ax = rp.axes[i];
    double cen[9], cf[4][9];
    uint64_t hh[4];
    for (int e = 0; e < 9; e++) cen[e] = (e % 4 == 0) ? 1.0 : 0.0;
    for (int m = 0; m < 4; m++) for (int e = 0; e < 9; e++) cf[m][e] = 0.0;
    auto put = [&](double* Rm, double c, double s) {
        const double ns = -1.0 * s;
        if (ax == 1) { Rm[1 + 3] = c; Rm[1 + 6] = ns; Rm[2 + 3] = s; Rm[2 + 6] = c; }
        else if (ax == 2) { Rm[0] = c; Rm[0 + 6] = s; Rm[2] = ns; Rm[2 + 6] = c; }
        else { Rm[0] = c; Rm[0 + 3] = ns; Rm[1] = s; Rm[1 + 3] = c; }
    };
    put(cen, J.cos_c, J.sin_c);
    put(cf[0], J.cos_k, 0.0); hh[0] = slot_hash(SLOT_K + i);
    put(cf[1], J.cos_e, 0.0); hh[1] = slot_hash(SLOT_COS + i);
    put(cf[2], 0.0, J.sin_k); hh[2] = slot_hash(SLOT_K + i);
    put(cf[3], 0.0, J.sin_e); hh[3] = slot_hash(SLOT_SIN + i);
    t0_make_raw(x, o, 3, 3, cen, 4, hh, cf);
}

T0FN void t0_make_box(Ctx& x, int o, const RobotParams& rp, int i) {
    // link box: generators on the qde_0 / qdae_0 / qddae_0 slots (Dynamics.cu:98-116)
    uint64_t hh[3];
    double cf[3][9];
    for (int m = 0; m < 3; m++) {
        for (int e = 0; e < 9; e++) cf[m][e] = 0.0;
        cf[m][m] = rp.link_g[i][m];
        hh[m] = slot_hash(NF * (m + 1));
    }
    t0_make_raw(x, o, 3, 1, rp.link_c[i], 3, hh, cf);
}

// reduce_link_PZ (PZsparse.cu:370-402) in monomial order, then emit the k-only part
T0FN void t0_emit_link(Ctx& x, const ReachOut& out, long j, int a, int l) {
    const PZH& h = x.H[a];
    const long base = j * out.NJ + l;
    double* gens = out.link_gens + base * 18;
    double gl[18];
    for (int e = 0; e < 18; e++) gl[e] = 0.0;
    int jg = 0, kk = 0;
    double rad[3] = {ind(x, h, 0)[0], ind(x, h, 0)[1], ind(x, h, 0)[2]};
    for (int k = 0; k < h.cnt; k++) {
        const uint64_t hh = x.ah[h.hoff + k];
        const double* c = x.ac + h.coff + (long)k * 3;
        if (hh < HASH_K_ONLY) {
            if (kk < CAP_LM) {
                out.link_hash[base * CAP_LM + kk] = (uint16_t)hh;
                for (int e = 0; e < 3; e++) out.link_coef[(base * CAP_LM + kk) * 3 + e] = c[e];
            } else {
                err_or(x, ERR_OUTCAP);
            }
            kk++;
        } else if (hh < HASH_K_LINKS_ONLY && (hh & K_MASK) == 0) {
            if (jg < 3) { for (int e = 0; e < 3; e++) gl[e + 3 * jg] = c[e]; }
            else err_or(x, ERR_LINKGEN);
            jg++;
        } else {
            for (int e = 0; e < 3; e++) rad[e] += fabs(c[e]);
        }
    }
    gl[0 + 3 * 3] = rad[0];
    gl[1 + 3 * 4] = rad[1];
    gl[2 + 3 * 5] = rad[2];
    for (int e = 0; e < 18; e++) gens[e] = gl[e];
    out.link_cnt[base] = kk < CAP_LM ? kk : CAP_LM;
    for (int e = 0; e < 3; e++) { out.link_center[base * 3 + e] = cen(x, h)[e]; out.link_rad[base * 3 + e] = rad[e]; }
}

T0FN void t0_emit_torque(Ctx& x, const ReachOut& out, long j, int a, int i, double* rdist, double* ured) {
    const PZH& h = x.H[a];
    const long base = j * NF + i;
    // disturbance u_int - u_nom: centres and monomials cancel exactly, the independent parts add
    // (armour_main.cu:135-137, PZsparse.cu:813-834)
    rdist[i] = ind(x, h, 1)[0] + ind(x, h, 0)[0];
    // reduce (PZsparse.cu:352-368)
    double rad = ind(x, h, 0)[0];
    int kk = 0;
    for (int k = 0; k < h.cnt; k++) {
        const uint64_t hh = x.ah[h.hoff + k];
        double c = x.ac[h.coff + (long)k * h.stride + (h.comp >= 0 ? h.comp : 0)];
        if (h.scaled) c = h.scale * c;
        if (hh < HASH_K_ONLY) {
            if (kk < CAP_UM) {
                out.tq_hash[base * CAP_UM + kk] = (uint16_t)hh;
                out.tq_coef[base * CAP_UM + kk] = c;
            } else {
                err_or(x, ERR_OUTCAP);
            }
            kk++;
        } else {
            rad += fabs(c);
        }
    }
    out.tq_cnt[base] = kk < CAP_UM ? kk : CAP_UM;
    out.tq_center[base] = cen(x, h)[0];
    out.tq_rad[base] = rad;
    ured[i] = rad;
}

// torque radius (armour_main.cu:173-211)
T0FN void t0_torque_radius(const RobotParams& rp, const ReachOut& out, long j, const double* rdist, const double* ured) {
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

// ---- operator dispatch ----------------------------------------------------------------------
// number of candidate terms of a simplifying op (uniform: every thread reads the same headers)
AI int op_terms(const Ctx& x, const Op& op) {
    const PZH& A = x.H[op.a];
    const PZH& B = x.H[op.b];
    if (op.code == OP_CROSS_C) return A.cnt;
    if (op.code == OP_MUL || op.code == OP_CROSS_PP) return A.cnt + B.cnt + A.cnt * B.cnt;
    if (op.code == OP_STACK3) return A.cnt + B.cnt + x.H[op.c].cnt;
    return A.cnt + B.cnt;
}

// term list of a simplifying op (all threads, uniform)
AI void op_terms_of(const Ctx& x, const Op& op, Terms& T) {
    switch (op.code) {
        case OP_MUL: terms_mul(x, op.a, op.b, T); break;
        case OP_ADD: terms_add(x, op.a, op.b, op.i, T); break;
        case OP_STACK3: terms_stack3(x, op.a, op.b, op.c, T); break;
        default: terms_add_one_dim(x, op.a, op.b, op.i, T); break;
    }
}
// output header, element-parallel: called by lanes e = 0..8 of wave 0
AI void op_header_par(Ctx& x, const Op& op, int e) {
    switch (op.code) {
        case OP_MUL: header_mul_par(x, op.o, op.a, op.b, e); break;
        case OP_ADD: header_add_par(x, op.o, op.a, op.b, op.i, e); break;
        case OP_STACK3: header_stack3_par(x, op.o, op.a, op.b, op.c, e); break;
        default: header_add_one_dim_par(x, op.o, op.a, op.b, op.i, e); break;
    }
}
// output header (thread 0)
AI void op_header(Ctx& x, const Op& op, const Terms& T) {
    switch (op.code) {
        case OP_MUL: header_mul(x, op.o, op.a, op.b, T); break;
        case OP_ADD: header_add(x, op.o, op.a, op.b, op.i); break;
        case OP_STACK3: header_stack3(x, op.o, op.a, op.b, op.c); break;
        default: header_add_one_dim(x, op.o, op.a, op.b, op.i); break;
    }
}

// One job (world w, interval t): the interpreter. jrs / scratch live in LDS.
// dump (diagnostics, may be null): per op, the output handle's [cnt, R*C, centre[0..2], ind0[0],
// ind1[0], absum[0]] after the op
constexpr int DUMP_W = 8;
#if !defined(__HIP_DEVICE_COMPILE__)
// host emulation statistics (tests/emu): per op [code, class, term kind, |S0|, |S1|, N, runs, output count]
inline int* g_op_stats = nullptr;
// host emulation: per op, the output handle's monomial hashes (structure studies)
inline void (*g_hash_sink)(int pc, const uint64_t* h, int n) = nullptr;
#endif
AI void run_program(Ctx& x, const RobotParams& rp, const Op* prog, int nops, int T, int t, const double* q0,
                    const double* qd0, const double* qdd0, const ReachOut& out, long j, JrsJoint* jrs,
                    double* scratch, unsigned long long* prof, double* dump = nullptr, const JrsJoint* jrs_in = nullptr) {
    const int tid = x.g.tid;
    double* rdist = scratch;
    double* ured = scratch + NF;
#if defined(__HIP_DEVICE_COMPILE__)
    const bool stamp = (prof || x.phase) && tid == 0;
    long long c_end = stamp ? clock64() : 0;
#endif
    // every handle empty at the job's start: a slot named before its first definition (an operand
    // field an op does not use) must not carry what the previous job or kernel left in LDS
    for (int k = x.g.tid; k < MAX_SLOTS; k += x.g.n) {
        x.H[k].cnt = 0;
        x.H[k].hoff = 0;
        x.H[k].coff = 0;
    }
    x.g.sync();
    for (int pc = 0; pc < nops; pc++) {
        const Op op = prog[pc];
        const int par = op.par > 1 ? op.par : 1;  // ops pc .. pc + par - 1 run as one group
#if defined(__HIP_DEVICE_COMPILE__)
        long long c0 = 0;
        if (stamp) {
            c0 = clock64();
            if (x.phase) x.phase[13] += (unsigned long long)(c0 - c_end);  // between ops
        }
#endif
        switch (op.code) {
            case OP_JRS:
                // on the device the JRS scalars come from jrs_kernel (their interval arithmetic
                // would otherwise set this kernel's register budget); the emulation computes them
#if defined(__HIP_DEVICE_COMPILE__)
                for (int i = tid; i < NF; i += x.g.n) jrs[i] = jrs_in[i];
#else
                for (int i = tid; i < NF; i += x.g.n) jrs[i] = jrs_in ? jrs_in[i] : jrs_joint(rp, T, t, i, q0[i], qd0[i], qdd0[i]);
#endif
                break;
            case OP_MAKE1D:
            case OP_MAKEROT:
            case OP_MAKEBOX:
            case OP_CONST:
            case OP_ZERO:
            case OP_VIEW:
            case OP_TRANSPOSE:
            case OP_EMIT_LINK:
            case OP_EMIT_TORQUE:
                // thread-0 ops; a group of par independent ones runs one per lane of wave 0
                for (int mi = tid; mi < par; mi += x.g.n) {
                    const Op m = mi == 0 ? op : prog[pc + mi];
                    switch (m.code) {
                        case OP_MAKE1D: t0_make_1d(x, m.o, jrs[m.i], m.i, m.b); break;
                        case OP_MAKEROT: t0_make_rot(x, m.o, rp, jrs[m.i], m.i); break;
                        case OP_MAKEBOX: t0_make_box(x, m.o, rp, m.i); break;
                        case OP_CONST:
                            if (m.a == CONST_RPY) t0_const(x, m.o, 3, 3, rp.rpy[m.i], 0.0);
                            else if (m.a == CONST_TRANS) t0_const(x, m.o, 3, 1, &rp.trans[3 * m.i], 0.0);
                            else if (m.a == CONST_MASS) t0_const(x, m.o, 1, 1, &rp.mass[m.i], rp.mass_uncertainty);
                            else t0_const(x, m.o, 3, 3, &rp.inertia[9 * m.i], rp.inertia_uncertainty);
                            break;
                        case OP_ZERO:
                            hdr_init(x, x.H[m.o], m.b, m.c);
                            if (m.i) cen(x, x.H[m.o])[2] = rp.gravity;
                            break;
                        case OP_VIEW: t0_view(x, m.o, m.a, m.i, m.b, m.s); break;
                        case OP_TRANSPOSE: t0_transpose(x, m.o, m.a); break;
                        case OP_EMIT_LINK: t0_emit_link(x, out, j, m.a, m.i); break;
                        default: t0_emit_torque(x, out, j, m.a, m.i, rdist, ured); break;
                    }
                }
                break;
            case OP_TORQUE_RADIUS: if (tid == 0) t0_torque_radius(rp, out, j, rdist, ured); break;
            case OP_CROSS_C: {
                const double* v = op.b == VEC_TRANS ? &rp.trans[3 * op.c] : &rp.com[3 * op.c];
                const CrossC C = cross_const_table(op.i, v);
                if (tid == 0) hdr_init(x, x.H[op.o], 3, 1);
                cross_const(x, op.o, op.a, C);
                break;
            }
            default: {
                // MUL / ADD / STACK3 / ADD1D / CROSS_PP: term list, header, simplify. The ordering of
                // large term lists is shared; the group passes are instantiated per output class.
                Terms Tm;
                int cls;  // 0: 1x1, 1: 3x1, 2: 3x3 plain simplify, 3: fused PZ x PZ cross
                if (op.code == OP_CROSS_PP) {
                    terms_cross_pp(x, op.a, op.b, Tm);
                    cls = 3;
                } else {
                    op_terms_of(x, op, Tm);
                    cls = Tm.nout == 1 ? 0 : (Tm.nout == 3 ? 1 : 2);
                }
                const int N = op_terms(x, op);
#if !defined(__HIP_DEVICE_COMPILE__)
                if (g_op_stats) {
                    int* st = g_op_stats + 8 * pc;
                    st[0] = op.code; st[1] = cls; st[2] = Tm.kind; st[3] = Tm.S[0].cnt;
                    st[4] = Tm.ns > 1 ? Tm.S[1].cnt : 0; st[5] = N; st[6] = Tm.runs();
                }
#endif
#if defined(__HIP_DEVICE_COMPILE__)
                long long ph0 = (x.phase && tid == 0) ? clock64() : 0;
#endif
#if defined(__HIP_DEVICE_COMPILE__)
                if (tid < 9) {
                    if (cls == 3) { if (tid == 0) hdr_init(x, x.H[op.o], 3, 1); }
                    else op_header_par(x, op, tid);
                }
#else
                if (cls == 3) hdr_init(x, x.H[op.o], 3, 1);
                else for (int e = 0; e < 9; e++) op_header_par(x, op, e);
#endif
#if defined(__HIP_DEVICE_COMPILE__)
                if (x.phase && tid == 0) x.phase[14] += (unsigned long long)(clock64() - ph0);
#endif
                PolBlock<1> p1{x.thr};
                PolBlock<3> p3{x.thr};
                PolBlock<9> p9{x.thr};
                PolCrossPP pp;
                pp.thr = x.thr;
                pp.ac = cen(x, x.H[op.a]);
                pp.bc = cen(x, x.H[op.b]);
                pp.a = op.a;
                pp.b = op.b;
#if defined(__HIP_DEVICE_COMPILE__)
                if (N <= 64 && !(x.mode & 1)) {
                    if (tid < 64) {
                        if (cls == 0) simplify_small(x, op.o, Tm, p1, N);
                        else if (cls == 1) simplify_small(x, op.o, Tm, p3, N);
                        else if (cls == 2) simplify_small(x, op.o, Tm, p9, N);
                        else simplify_small(x, op.o, Tm, pp, N);
                    }
                    break;
                }
                long long pt = (x.phase && tid == 0) ? clock64() : 0;
#endif
                stage_sources(x, Tm);
                x.g.sync();
#if defined(__HIP_DEVICE_COMPILE__)
                if (x.phase && tid == 0) { const long long c_ = clock64(); x.phase[6] += (unsigned long long)(c_ - pt); pt = c_; }
#endif
                KeyBufs K;
                if (!order_keys(x, Tm, N, K)) {
                    if (tid == 0) { *x.err |= ERR_SORTCAP; x.H[op.o].cnt = 0; }
                    break;
                }
#if defined(__HIP_DEVICE_COMPILE__)
                if (x.phase && tid == 0) x.phase[1] += (unsigned long long)(clock64() - pt);
#endif
                if (cls == 0) simplify_groups<decltype(p1)>(x, op.o, Tm, p1, N, K);
                else if (cls == 1) simplify_groups<decltype(p3)>(x, op.o, Tm, p3, N, K);
                else if (cls == 2) simplify_groups<decltype(p9)>(x, op.o, Tm, p9, N, K);
                else simplify_groups<decltype(pp)>(x, op.o, Tm, pp, N, K);
                break;
            }
        }
        if (op.sync) x.g.sync();
#if !defined(__HIP_DEVICE_COMPILE__)
        if (g_op_stats && op.o >= 0) g_op_stats[8 * pc + 7] = x.H[op.o].cnt;
        if (g_hash_sink)
            for (int mi = 0; mi < par; mi++) {
                const int mo = prog[pc + mi].o;
                if (mo >= 0) g_hash_sink(pc + mi, x.ah + x.H[mo].hoff, x.H[mo].cnt);
            }
#endif
        if (dump) {
            x.g.sync();
            if (tid == 0)
                for (int mi = 0; mi < par; mi++) {
                    const int mo = prog[pc + mi].o;
                    if (mo < 0) continue;
                    const PZH& h = x.H[mo];
                    double* d = dump + (long)(pc + mi) * DUMP_W;
                    d[0] = h.cnt; d[1] = h.R * h.C; d[2] = cen(x, h)[0]; d[3] = cen(x, h)[1]; d[4] = cen(x, h)[2];
                    d[5] = ind(x, h, 0)[0]; d[6] = ind(x, h, 1)[0]; d[7] = abs_(x, h)[0];
                }
            x.g.sync();
        }
#if defined(__HIP_DEVICE_COMPILE__)
        if (stamp) {
            c_end = clock64();
            if (prof) {
                atomicAdd(&prof[2 * pc], (unsigned long long)(c_end - c0));
                if ((op.code >= OP_MUL && op.code <= OP_ADD1D) || op.code >= OP_CROSS_C)
                    atomicAdd(&prof[2 * pc + 1], (unsigned long long)op_terms(x, op));
                c_end = clock64();
            }
        }
#endif
        pc += par - 1;
    }
}

// ---- host: program builder --------------------------------------------------------------------
struct ProgramBuilder {
    std::vector<Op> ops;
    // handle slots, SSA style: every op writes a fresh (or freed) slot, so no op's output aliases
    // an operand. Each slot has a fixed payload class n = R*C (1, 3 or 9), so the LDS payload pool
    // holds 4n doubles per slot instead of the 3x3 worst case.
    std::vector<int> cls;
    std::vector<int> free_by[10];
    int nslots = 0;

    int alloc(int n) {
        if (!free_by[n].empty()) { const int s = free_by[n].back(); free_by[n].pop_back(); return s; }
        cls.push_back(n);
        return nslots++;
    }
    void rel(int s) { free_by[cls[s]].push_back(s); }
    // payload offsets (doubles) of every slot in the pool, and the pool size
    std::vector<int> slot_offsets(int* total) const {
        std::vector<int> off(nslots);
        int acc = 0;
        for (int k = 0; k < nslots; k++) { off[k] = acc; acc += 4 * cls[k]; }
        *total = acc;
        return off;
    }
    int out_class(int code, int a, int b, int c, int i) const {
        switch (code) {
            case OP_MUL: {
                const int ca = cls[a], cb = cls[b];
                return ca == 1 ? cb : (cb == 1 ? ca : (cb == 9 ? 9 : 3));
            }
            case OP_ADD: case OP_ADD1D: case OP_TRANSPOSE: return cls[a];
            case OP_VIEW: return i >= 0 ? 1 : cls[a];
            case OP_CONST: return (a == CONST_RPY || a == CONST_INERTIA) ? 9 : (a == CONST_TRANS ? 3 : 1);
            case OP_ZERO: return b * c;
            case OP_MAKE1D: return 1;
            case OP_MAKEROT: return 9;
            default: return 3;  // MAKEBOX, STACK3, CROSS_C, CROSS_PP
        }
    }
    void rel(std::initializer_list<int> l) { for (int s : l) rel(s); }
    void emit(int code, int o = -1, int a = 0, int b = 0, int c = 0, int i = 0, double s = 0.0) {
        Op op;
        op.code = code; op.o = o; op.a = a; op.b = b; op.c = c; op.i = i; op.s = s; op.sync = 1; op.par = 0;
        ops.push_back(op);
    }
    int out(int code, int a = 0, int b = 0, int c = 0, int i = 0, double s = 0.0) {
        const int o = alloc(out_class(code, a, b, c, i));
        emit(code, o, a, b, c, i, s);
        return o;
    }
    int mul(int a, int b) { return out(OP_MUL, a, b); }
    int add(int a, int b) { return out(OP_ADD, a, b, 0, +1); }
    int sub(int a, int b) { return out(OP_ADD, a, b, 0, -1); }
    int stack3(int a, int b, int c) { return out(OP_STACK3, a, b, c); }
    int add1d(int self, int a, int e) { return out(OP_ADD1D, self, a, 0, e); }
    int elem(int a, int e) { return out(OP_VIEW, a, 0, 0, e); }
    int scaled_elem(int a, int e, double s) { return out(OP_VIEW, a, 1, 0, e, s); }
    int scaled(int a, double s) { return out(OP_VIEW, a, 1, 0, -1, s); }
    int cnst(int kind, int i) { return out(OP_CONST, kind, 0, 0, i); }
    int zero(int R, int C, int gravity = 0) { return out(OP_ZERO, 0, R, C, gravity); }

    // cross products (PZsparse.cu:1118-1167). fused = true: one op each (OP_CROSS_C / OP_CROSS_PP,
    // every intermediate simplify replicated inside); false: composed from element views, products,
    // differences and a stack, op by op as the reference composes them (kept for A/B checks)
    bool fused = true;
    const RobotParams* rp = nullptr;
    const double* vec(int src, int row) const { return src == VEC_TRANS ? &rp->trans[3 * row] : &rp->com[3 * row]; }
    int cross_pm(int a, int src, int row) {  // PZ x const
        if (fused) return out(OP_CROSS_C, a, src, row, 0);
        const double* b = vec(src, row);
        const int s0 = scaled_elem(a, 1, b[2]), s1 = scaled_elem(a, 2, b[1]);
        const int r0 = sub(s0, s1);
        rel({s0, s1});
        const int s2 = scaled_elem(a, 2, b[0]), s3 = scaled_elem(a, 0, b[2]);
        const int r1 = sub(s2, s3);
        rel({s2, s3});
        const int s4 = scaled_elem(a, 0, b[1]), s5 = scaled_elem(a, 1, b[0]);
        const int r2 = sub(s4, s5);
        rel({s4, s5});
        const int o = stack3(r0, r1, r2);
        rel({r0, r1, r2});
        return o;
    }
    int cross_mp(int src, int row, int b) {  // const x PZ
        if (fused) return out(OP_CROSS_C, b, src, row, 1);
        const double* a = vec(src, row);
        const int s0 = scaled_elem(b, 2, a[1]), s1 = scaled_elem(b, 1, a[2]);
        const int r0 = sub(s0, s1);
        rel({s0, s1});
        const int s2 = scaled_elem(b, 0, a[2]), s3 = scaled_elem(b, 2, a[0]);
        const int r1 = sub(s2, s3);
        rel({s2, s3});
        const int s4 = scaled_elem(b, 1, a[0]), s5 = scaled_elem(b, 0, a[1]);
        const int r2 = sub(s4, s5);
        rel({s4, s5});
        const int o = stack3(r0, r1, r2);
        rel({r0, r1, r2});
        return o;
    }
    int cross_pp(int a, int b) {  // PZ x PZ
        if (fused) return out(OP_CROSS_PP, a, b);
        const int a0 = elem(a, 0), a1 = elem(a, 1), a2 = elem(a, 2);
        const int b0 = elem(b, 0), b1 = elem(b, 1), b2 = elem(b, 2);
        int p = mul(a1, b2), q = mul(a2, b1);
        const int r0 = sub(p, q);
        rel({p, q});
        p = mul(a2, b0); q = mul(a0, b2);
        const int r1 = sub(p, q);
        rel({p, q});
        p = mul(a0, b1); q = mul(a1, b0);
        const int r2 = sub(p, q);
        rel({p, q, a0, a1, a2, b0, b1, b2});
        const int o = stack3(r0, r1, r2);
        rel({r0, r1, r2});
        return o;
    }

    // the whole job, op for op KPR/Trajectory.cu:63-254, Dynamics.cu:69-181, armour_main.cu:118-211
    // fk_only: the ARMTD comparison planner's program (ACMP/armtd_main.cu:141-156): joint
    // rotations, forward kinematics and reduce_link_PZ; no velocity PZs, no RNEA, no torque
    void build(const RobotParams& rp, bool fk_only = false) {
        this->rp = &rp;
        const int NJ = rp.num_joints;
        int R[MAX_J + 1], RT[MAX_J], QD[NF], QDA[NF], QDD[NF];
        emit(OP_JRS);
        // ops of one kind that do not depend on each other are emitted back to back, so that
        // group() can run them lane-parallel
        for (int i = 0; i < NF && !fk_only; i++) {
            QD[i] = out(OP_MAKE1D, 0, 0, 0, i);
            QDA[i] = out(OP_MAKE1D, 0, 1, 0, i);
            QDD[i] = out(OP_MAKE1D, 0, 2, 0, i);
        }
        for (int i = 0; i < NF; i++) {
            if (rp.axes[i] != 0) {
                const int rot = out(OP_MAKEROT, 0, 0, 0, i);
                const int c = cnst(CONST_RPY, i);
                R[i] = mul(c, rot);
                rel({rot, c});
            } else {
                R[i] = cnst(CONST_RPY, i);
            }
        }
        for (int i = NF; i < NJ; i++) R[i] = cnst(CONST_RPY, i);
        if (!fk_only) {
            for (int i = 0; i < NJ; i++) RT[i] = out(OP_TRANSPOSE, R[i]);
            R[NJ] = cnst(CONST_RPY, MAX_J);  // PZsparse(0, 0, 0)
        }

        // forward kinematics (Dynamics.cu:69-81) + reduce_link_PZ (armour_main.cu:124-126)
        {
            int FKR = cnst(CONST_RPY, MAX_J), FKT = zero(3, 1), links[MAX_J];
            for (int i = 0; i < NJ; i++) {
                const int P = cnst(CONST_TRANS, i);
                const int tmp = mul(FKR, P);
                const int fkt = add(FKT, tmp);
                rel({P, tmp, FKT});
                FKT = fkt;
                const int fkr = mul(FKR, R[i]);
                rel(FKR);
                FKR = fkr;
                const int box = out(OP_MAKEBOX, 0, 0, 0, i);
                const int tmp2 = mul(FKR, box);
                links[i] = add(tmp2, FKT);
                rel({box, tmp2});
            }
            rel({FKR, FKT});
            for (int i = 0; i < NJ; i++) emit(OP_EMIT_LINK, -1, links[i], 0, 0, i);
            for (int i = 0; i < NJ; i++) rel(links[i]);
        }
        if (fk_only) {
            finish();
            return;
        }

        // RNEA, nominal and interval fused (Dynamics.cu:83-181)
        int W = zero(3, 1), WDOT = zero(3, 1), WAUX = zero(3, 1), LIN = zero(3, 1, 1);
        int F[MAX_J], N[MAX_J];
        for (int i = 0; i < NJ; i++) {
            // line 16
            {
                const int t1 = cross_pm(WDOT, VEC_TRANS, i);
                const int t2 = add(LIN, t1);
                const int t3 = cross_pm(WAUX, VEC_TRANS, i);
                const int t4 = cross_pp(W, t3);
                const int t5 = add(t2, t4);
                const int lin = mul(RT[i], t5);
                rel({t1, t2, t3, t4, t5, LIN});
                LIN = lin;
            }
            // line 13
            {
                int w = mul(RT[i], W);
                rel(W);
                W = w;
            }
            if (rp.axes[i] != 0) {
                const int ax = (rp.axes[i] < 0 ? -rp.axes[i] : rp.axes[i]) - 1;
                int w = add1d(W, QD[i], ax);
                rel(W);
                W = w;
                const int waux = mul(RT[i], WAUX);
                rel(WAUX);
                WAUX = waux;
                const int wdot = mul(RT[i], WDOT);
                rel(WDOT);
                WDOT = wdot;
                const int z = zero(3, 1);
                const int t1 = add1d(z, QD[i], ax);
                const int t2 = cross_pp(WAUX, t1);
                const int wd2 = add(WDOT, t2);
                rel({z, t1, t2, WDOT});
                WDOT = add1d(wd2, QDD[i], ax);
                rel(wd2);
                const int wa2 = add1d(WAUX, QDA[i], ax);
                rel(WAUX);
                WAUX = wa2;
            } else {
                const int waux = mul(RT[i], WAUX);
                rel(WAUX);
                WAUX = waux;
                const int wdot = mul(RT[i], WDOT);
                rel(WDOT);
                WDOT = wdot;
            }
            // line 23 & 27
            {
                const int t1 = cross_pm(WDOT, VEC_COM, i);
                const int t2 = add(LIN, t1);
                const int t3 = cross_pm(WAUX, VEC_COM, i);
                const int t4 = cross_pp(W, t3);
                const int t5 = add(t2, t4);
                const int m = cnst(CONST_MASS, i);
                F[i] = mul(m, t5);
                rel({t1, t2, t3, t4, t5, m});
            }
            // line 29
            {
                const int I = cnst(CONST_INERTIA, i);
                const int t1 = mul(I, WDOT);
                const int t2 = mul(I, W);
                const int t3 = cross_pp(WAUX, t2);
                N[i] = add(t1, t3);
                rel({I, t1, t2, t3});
            }
        }
        rel({W, WDOT, WAUX, LIN});
        int FF = zero(3, 1), NN = zero(3, 1), us[MAX_J];
        for (int i = 0; i < MAX_J; i++) us[i] = -1;
        for (int i = NJ - 1; i >= 0; i--) {
            // line 29: n = N + R*n + cross(com, F) + cross(p_{i+1}, R*f); R*f evaluated once
            const int t1 = mul(R[i + 1], NN);
            const int t2 = add(N[i], t1);
            const int t3 = cross_mp(VEC_COM, i, F[i]);
            const int t4 = add(t2, t3);
            const int t5 = mul(R[i + 1], FF);
            const int t6 = cross_mp(VEC_TRANS, i + 1, t5);
            const int nn = add(t4, t6);
            rel({t1, t2, t3, t4, t6, NN});
            NN = nn;
            // line 28
            const int ff = add(t5, F[i]);
            rel({t5, FF});
            FF = ff;
            if (rp.axes[i] != 0 && i < NF) {
                const int ax = (rp.axes[i] < 0 ? -rp.axes[i] : rp.axes[i]) - 1;
                const int e = elem(NN, ax);
                const int s1 = scaled(QDD[i], rp.armature[i]);
                const int u1 = add(e, s1);
                const int s2 = scaled(QD[i], rp.damping[i]);
                us[i] = add(u1, s2);
                rel({e, s1, u1, s2});
            }
        }
        for (int i = NJ - 1; i >= 0; i--)
            if (us[i] >= 0) emit(OP_EMIT_TORQUE, -1, us[i], 0, 0, i);
        for (int i = NJ - 1; i >= 0; i--)
            if (us[i] >= 0) rel(us[i]);
        emit(OP_TORQUE_RADIUS);
        finish();
    }
    void finish() {
        // thread-0 ops chained back to back need no barrier between them
        auto t0_only = [](int c) {
            return c == OP_MAKE1D || c == OP_MAKEROT || c == OP_MAKEBOX || c == OP_CONST || c == OP_ZERO ||
                   c == OP_VIEW || c == OP_TRANSPOSE || c == OP_EMIT_LINK || c == OP_EMIT_TORQUE;
        };
        for (size_t k = 0; k + 1 < ops.size(); k++)
            if (t0_only(ops[k].code) && t0_only(ops[k + 1].code)) ops[k].sync = 0;
        group(t0_only);
    }
    // consecutive thread-0 ops of one code none of which reads another's output become one
    // lane-parallel group (at most a wave); a barrier follows every group
    template <class F>
    void group(F t0_only) {
        auto reads = [](const Op& op, int slot) {
            return (op.code == OP_VIEW || op.code == OP_TRANSPOSE || op.code == OP_EMIT_LINK || op.code == OP_EMIT_TORQUE) &&
                   op.a == slot;
        };
        for (size_t k = 0; k < ops.size();) {
            size_t e = k + 1;
            if (t0_only(ops[k].code)) {
                while (e < ops.size() && e - k < 64 && ops[e].code == ops[k].code) {
                    bool dep = false;
                    for (size_t q = k; q < e; q++) dep = dep || (ops[q].o >= 0 && reads(ops[e], ops[q].o));
                    if (dep) break;
                    e++;
                }
            }
            if (e - k > 1) {
                ops[k].par = (int)(e - k);
                ops[k].sync = 1;
                if (k > 0) ops[k - 1].sync = 1;  // members on other lanes read what thread 0 wrote
            }
            k = e;
        }
    }
};

}  // namespace armour
