// armour-mi355x — NLP kernels for a batch of W worlds:
//   bounds_kernel       constraint bounds (KPR/NLPclass.cu:87-165)
//   eval_kernel         g(x) and its dense Jacobian (KPR/NLPclass.cu:207-396): PZ slicing
//                       (PZsparse.cu:404-555), collision rows (CollisionChecking.cu:230-299) with
//                       the buffered-obstacle hyperplanes (:136-228) computed in place and a
//                       per-(link, obstacle) scan in the reference's plane order, torque and
//                       extremum rows
//   ipm_*               armour-IPM (oracle/src/ipm.cpp), one row-parallel pass per phase with
//                       deterministic block partials and one wave per world for the 7x7 algebra
//   feasible_kernel     finalize_solution's re-check (KPR/NLPclass.cu:449-538)
#include "nlp.h"

namespace armour {

// ------------------------------------------------------------------------------------------
// helpers
// wave_sum (wave.h): DPP / permlane butterfly
__device__ inline double wave_max(double v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = fmax(v, xor_f64(v, m));
    return v;
}
__device__ inline double wave_min(double v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = fmin(v, xor_f64(v, m));
    return v;
}
// N values at once, the arithmetic of N block_reduce calls (wave reduction, then the waves in
// order) with one barrier: the N wave reductions are independent and interleave. kinds[i]: 0 sum,
// 1 max, 2 min. out[i] written by thread i; lds holds (blockDim / 64) * N doubles.
template <int N>
__device__ inline void block_reduce_n(double (&v)[N], const int (&kinds)[N], double* lds, double* out) {
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    // groups of 8 interleave; a scheduling barrier between groups bounds the live registers
#pragma unroll
    for (int g = 0; g < N; g += 8) {
#pragma unroll
        for (int i = g; i < (g + 8 < N ? g + 8 : N); i++)
            v[i] = kinds[i] == 0 ? wave_sum(v[i]) : kinds[i] == 1 ? wave_max(v[i]) : wave_min(v[i]);
        if ((threadIdx.x & 63) == 0) {
#pragma unroll
            for (int i = g; i < (g + 8 < N ? g + 8 : N); i++) lds[wave * N + i] = v[i];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    const int i = threadIdx.x;
    if (i < N) {
        int kind = 0;
#pragma unroll
        for (int q = 0; q < N; q++) if (q == i) kind = kinds[q];
        double s = lds[i];
        for (int k = 1; k < nw; k++) {
            const double t = lds[k * N + i];
            s = kind == 0 ? s + t : kind == 1 ? fmax(s, t) : fmin(s, t);
        }
        out[i] = s;
    }
}

// row bounds: a collision row's are the constants bounds_kernel stores (-1e19, 0), not re-read
__device__ inline void row_bounds(const NlpDev& d, long i, int r, double& L, double& U) {
    const bool col = r >= d.nt && r < d.nt + d.T * d.NJ * d.O;
    L = col ? -1e19 : d.L[i];
    U = col ? 0.0 : d.U[i];
}
// The row passes read a row's state in one batch before its arithmetic: the slack and multiplier
// slots of both sides exist for every row (zero where a side is absent) and are read
// unconditionally, and a collision row's bounds load comes from one cached word of its world
// (wb = w * R) instead of the row's own slot. A row then waits for memory once; loads behind each
// side's branch and re-reads after each store had waited a round trip apiece (~6 per row).
// A collision row has no lower side (L = -1e19): its lower-side slots are read from those of the
// world's first collision row (lo; unused, and never written by a row pass), one cached word, so
// the batch costs no bytes for them.
struct RowBounds {
    double Lm, Um;
    bool col;
    long lo;  // index of the row's lower-side slots
    __device__ RowBounds(const NlpDev& d, long i, long wb, int r) {
        col = r >= d.nt && r < d.nt + d.T * d.NJ * d.O;
        const long ib = col ? wb : i;
        Lm = d.L[ib];
        Um = d.U[ib];
        lo = col ? wb + d.nt : i;
    }
    __device__ double L() const { return col ? -1e19 : Lm; }
    __device__ double U() const { return col ? 0.0 : Um; }
};
__device__ inline bool has_lo(const NlpDev& d, double L) { return L > -d.opt.inf_bound; }
__device__ inline bool has_hi(const NlpDev& d, double U) { return U < d.opt.inf_bound; }

// value and gradient of row r of world w from eval slot `slot` at point x; a collision row's
// gradient is n . dc/dx from the compact form (bitwise the value eval_kernel forms densely)
__device__ inline double row_va(const NlpDev& d, int slot, int w, int r, const double* x, double* a) {
    const int nc = d.T * d.NJ * d.O;
    // the value's load ahead of the branches (a box row's, from row 0, goes unused), so that it
    // travels with the row's other loads instead of after them
    const long gi = gidx(d, slot, w, r < d.m ? r : 0);
    const double v = d.g[gi];
    if (r >= d.nt && r < d.nt + nc) {
        const int q = r - d.nt, lt = q / d.O, l = lt / d.T, t = lt % d.T;
        const double* n = d.jn + slot * d.njn + ((long)w * nc + q) * 3;
        const double* D = d.jd + slot * d.njd + (((long)w * d.T + t) * d.NJ + l) * NF * 3;
        const double n0 = n[0], n1 = n[1], n2 = n[2];
#pragma unroll
        for (int j = 0; j < NF; j++) a[j] = n0 * D[3 * j] + n1 * D[3 * j + 1] + n2 * D[3 * j + 2];
        return v;
    }
    if (r < d.m) {
        const double* J = d.J + gi * NF;
#pragma unroll
        for (int j = 0; j < NF; j++) a[j] = J[j];
        return v;
    }
#pragma unroll
    for (int j = 0; j < NF; j++) a[j] = (j == r - d.m) ? 1.0 : 0.0;
    return x[r - d.m];
}

// normalised cross product of a generator pair, zero for a parallel pair (CollisionChecking.cu:136-228)
template <typename R>
__device__ inline __attribute__((always_inline)) void plane_normal(const R* ga, const R* gb, R& C0,
                                                                   R& C1, R& C2) {
    const R gc0 = ga[1] * gb[2] - ga[2] * gb[1];
    const R gc1 = ga[2] * gb[0] - ga[0] * gb[2];
    const R gc2 = ga[0] * gb[1] - ga[1] * gb[0];
    const R nrm = sqrt(gc0 * gc0 + gc1 * gc1 + gc2 * gc2);
    C0 = 0; C1 = 0; C2 = 0;
    if (nrm > 0) { C0 = gc0 / nrm; C1 = gc1 / nrm; C2 = gc2 / nrm; }
}

// Link generators 3..5 are reduce_link_PZ's radii: r_e on axis e with exact zeros elsewhere
// (lane_engine.h emit_link). A product with one of those zeros is ±0 and adding ±0 leaves a sum
// unchanged, so the terms below drop them: equal to the general arithmetic up to the sign of a
// zero. E >= 0 marks a normal whose component E is zero (a plane spanned with radius E).
template <int E, typename R>
__device__ inline __attribute__((always_inline)) R dot_z(const R* C, const R* g) {
    if constexpr (E == 0) return C[1] * g[1] + C[2] * g[2];
    else if constexpr (E == 1) return C[0] * g[0] + C[2] * g[2];
    else if constexpr (E == 2) return C[0] * g[0] + C[1] * g[1];
    else return C[0] * g[0] + C[1] * g[1] + C[2] * g[2];
}

// plane of obstacle generator ga and link generator gb (CollisionChecking.cu:136-228): the
// normalised cross product (zero for a parallel pair), d = A . c_obs and delta = sum_k |A . g_k| over
// the 9 buffered generators in order (the obstacle's 3, the link's 3 box generators and 3 radii).
// E < 0 for a box generator gb, E = e for radius e; the radius terms are A_f r_f (none for f = E,
// where A_E = 0)
template <int E, typename R>
__device__ inline __attribute__((always_inline)) void mixed_plane(const R* ga, const R* gb, const R (*G)[3],
                                                                  const R* oc, R* C, R& dd, R& del) {
    R gc[3];
    R nrm;
    if constexpr (E < 0) {
        gc[0] = ga[1] * gb[2] - ga[2] * gb[1];
        gc[1] = ga[2] * gb[0] - ga[0] * gb[2];
        gc[2] = ga[0] * gb[1] - ga[1] * gb[0];
        nrm = sqrt(gc[0] * gc[0] + gc[1] * gc[1] + gc[2] * gc[2]);
    } else {
        const R r = gb[E];
        if constexpr (E == 0) { gc[0] = 0.0; gc[1] = ga[2] * r; gc[2] = -(ga[1] * r); }
        else if constexpr (E == 1) { gc[0] = -(ga[2] * r); gc[1] = 0.0; gc[2] = ga[0] * r; }
        else { gc[0] = ga[1] * r; gc[1] = -(ga[0] * r); gc[2] = 0.0; }
        constexpr int P = E == 0 ? 1 : 0, Q = E == 2 ? 1 : 2;
        nrm = sqrt(gc[P] * gc[P] + gc[Q] * gc[Q]);
    }
    C[0] = 0; C[1] = 0; C[2] = 0;
    if (nrm > 0) {
#pragma unroll
        for (int e = 0; e < 3; e++)
            if (e != E) C[e] = gc[e] / nrm;
    }
    dd = dot_z<E>(C, oc);
    del = 0.0;
#pragma unroll
    for (int k = 0; k < BUF_GEN - 3; k++) del += fabs(dot_z<E>(C, G[k]));
#pragma unroll
    for (int f = 0; f < 3; f++)
        if (f != E) del += fabs(C[f] * G[BUF_GEN - 3 + f][f]);
}

// mixed plane of obstacle generator ga and link generator j (0..2 box, 3..5 the radii): the
// mixed_plane<E> specialisation for j (folds to one call once j is a constant)
template <typename R>
__device__ inline __attribute__((always_inline)) void mixed_plane_j(int j, const R* ga, const R (*G)[3], const R* oc,
                                                                    R* C, R& dd, R& del) {
    // every case indexes G with a constant: a run-time row index would place a private G in scratch
    switch (j) {
        case 0: mixed_plane<-1>(ga, G[OBS_GEN + 0], G, oc, C, dd, del); break;
        case 1: mixed_plane<-1>(ga, G[OBS_GEN + 1], G, oc, C, dd, del); break;
        case 2: mixed_plane<-1>(ga, G[OBS_GEN + 2], G, oc, C, dd, del); break;
        case 3: mixed_plane<0>(ga, G[OBS_GEN + 3], G, oc, C, dd, del); break;
        case 4: mixed_plane<1>(ga, G[OBS_GEN + 4], G, oc, C, dd, del); break;
        default: mixed_plane<2>(ga, G[OBS_GEN + 5], G, oc, C, dd, del); break;
    }
}

// table entry of link-link plane p (generators i < j of the link's 6): the normal, A . c (c: the
// sliced centre in the evaluation, the centre of its range in the cache build) and |A . g_k| of the
// link's 6 generators (the link's part of delta, kept per summand for the reference's order)
template <typename R>
__device__ inline __attribute__((always_inline)) void ll_table(const R* lg, int p, const R* c, R* P) {
    int i = 0, rem = p;
    while (rem >= 5 - i) { rem -= 5 - i; i++; }
    const int j = i + 1 + rem;
    R A0, A1, A2;
    plane_normal(lg + 3 * i, lg + 3 * j, A0, A1, A2);
    P[0] = A0; P[1] = A1; P[2] = A2;
    P[3] = A0 * c[0] + A1 * c[1] + A2 * c[2];
#pragma unroll
    for (int k = 0; k < 6; k++) P[4 + k] = fabs(A0 * lg[3 * k] + A1 * lg[3 * k + 1] + A2 * lg[3 * k + 2]);
}
// table entry of obstacle-obstacle plane p: the normal, d = A . c_obs and the obstacle's part of delta
template <typename R>
__device__ inline __attribute__((always_inline)) void oo_table(const R* ob, int p, R* P) {
    const int i = p == 2 ? 1 : 0, j = p == 0 ? 1 : 2;
    R A0, A1, A2;
    plane_normal(ob + 3 * (i + 1), ob + 3 * (j + 1), A0, A1, A2);
    P[0] = A0; P[1] = A1; P[2] = A2;
    P[3] = A0 * ob[0] + A1 * ob[1] + A2 * ob[2];
    R del = 0.0;
#pragma unroll
    for (int k = 0; k < OBS_GEN; k++) del += fabs(A0 * ob[3 * (k + 1)] + A1 * ob[3 * (k + 1) + 1] + A2 * ob[3 * (k + 1) + 2]);
    P[4] = del;
}
// d and delta of a link-link plane for one obstacle (generators G[0..2], centre oc), delta summed
// in the reference's order: the obstacle's generators first, then the link's
template <typename R>
__device__ inline __attribute__((always_inline)) void ll_complete(const R* P, const R (*G)[3], const R* oc, R& dd, R& del) {
    const R A0 = P[0], A1 = P[1], A2 = P[2];
    dd = A0 * oc[0] + A1 * oc[1] + A2 * oc[2];
    del = 0.0;
#pragma unroll
    for (int k = 0; k < OBS_GEN; k++) del += fabs(A0 * G[k][0] + A1 * G[k][1] + A2 * G[k][2]);
#pragma unroll
    for (int k = 0; k < 6; k++) del += P[4 + k];
}
// d and delta of an obstacle-obstacle plane for one link (generators L[0..2], radii L[3..5] on
// axes 0..2: their products with the other components are exact zeros and dropped)
template <typename R>
__device__ inline __attribute__((always_inline)) void oo_complete(const R* P, const R (*L)[3], R& dd, R& del) {
    const R A0 = P[0], A1 = P[1], A2 = P[2];
    dd = P[3];
    del = P[4];
#pragma unroll
    for (int k = 0; k < 3; k++) del += fabs(A0 * L[k][0] + A1 * L[k][1] + A2 * L[k][2]);
    del += fabs(A0 * L[3][0]);
    del += fabs(A1 * L[4][1]);
    del += fabs(A2 * L[5][2]);
}

// one monomial's contribution to a slice (k = 0) or to its derivative in x_{k-1}: the products
// of PZsparse.cu:404-435 / 477-516 in factor order, v * 1.0 standing in for a skipped factor
// ptab[j][g] = x_j^g (g = 0: 1.0, the skipped factor exactly), ptab[j][4 + g] = g x_j^(g-1): one
// LDS read per factor instead of a select chain (eval_kernel is VALU-issue bound). The reference
// skips a term whose derivative variable has degree 0; here its factor ptab[k-1][4] = 0 makes the
// term ±0 (coefficients and x are finite), and adding ±0 is the skip up to the sign of a zero.
template <typename R>
__device__ inline __attribute__((always_inline)) R slice_term(R co, int h, int k, const R (*ptab)[8]) {
    R v = co;
#pragma unroll
    for (int j = 0; j < NF; j++) {
        const int g = (h >> (2 * j)) & 3;
        v = v * ptab[j][g + (j == k - 1 ? 4 : 0)];
    }
    return v;
}

// ------------------------------------------------------------------------------------------
// constraint bounds (NLPclass.cu:87-165) of row r of world w; rows m..m+NF-1 are the box bounds on
// x. Formed by ipm_rows_init on the solver stream (no kernel of its own on the reach stream).
__device__ inline void bounds_of(const NlpDev& d, int w, int r, double& L, double& U) {
    const RobotParams& rp = *d.rp;
    {
        const int nt = d.nt, nc = d.T * d.NJ * d.O;
        if (r < nt) {
            const int t = r / NF, j = r % NF;
            const double tr = d.ro.torque_radius[((long)w * d.T + t) * NF + j];
            L = -rp.torque_limits[j] + tr;
            U = rp.torque_limits[j] - tr;
        } else if (r < nt + nc) {
            L = -1e19; U = 0;
        } else if (r < nt + nc + 2 * NF) {
            const int j = (r - nt - nc) % NF;
            L = rp.state_lb[j] + rp.qe;
            U = rp.state_ub[j] - rp.qe;
        } else if (r < d.m) {
            const int j = (r - nt - nc - 2 * NF) % NF;
            L = -rp.speed_limits[j] + rp.qde;
            U = rp.speed_limits[j] - rp.qde;
        } else {
            L = -1.0; U = 1.0;  // NLPclass.cu:105-113
        }
    }
}

// ------------------------------------------------------------------------------------------
// trajectory extrema (Trajectory.cu:256-540; restated as in oracle/src/traj.cpp)
__device__ void extremum(int kind, double q0, double Tqd0, double TTqdd0, double ka, double* mn, double* mx, int* mnid, int* mxid, double* e2o, double* e3o) {
    double e2, e3;
    if (kind == 0) q_roots(Tqd0, TTqdd0, ka, &e2, &e3);
    else qd_roots(Tqd0, TTqdd0, ka, &e2, &e3);
    auto f = [&](double t) { return kind == 0 ? bz_q(q0, Tqd0, TTqdd0, ka, t) : bz_qd(q0, Tqd0, TTqdd0, ka, t); };
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
    *e2o = e2;
    *e3o = e3;
}
// EVAL_PROF=1 (diagnostic builds only: make lane_variant LW=4 LX=_evprof EXTRA=-DEVAL_PROF=1): thread 0
// of blocks (t = 0 | 50, list entry 0) prints its phase boundaries (wall clock, 10 ns ticks)
#ifndef EVAL_PROF
#define EVAL_PROF 0
#endif
#define EVP_DECL unsigned long long evp_[10]; int evn_ = 0;
#define EVP_MARK if (EVAL_PROF && threadIdx.x == 0 && evn_ < 10) evp_[evn_++] = wall_clock64();
#define EVP_PRINT(tag)                                                                                   \
    if (EVAL_PROF && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 50) && blockIdx.y == 0) {      \
        EVP_MARK                                                                                           \
        printf("%s t=%d grid=%d n=%d: %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", tag, (int)blockIdx.x,    \
               (int)gridDim.y, evn_, evn_ > 1 ? evp_[1] - evp_[0] : 0ull, evn_ > 2 ? evp_[2] - evp_[1] : 0ull,      \
               evn_ > 3 ? evp_[3] - evp_[2] : 0ull, evn_ > 4 ? evp_[4] - evp_[3] : 0ull,                         \
               evn_ > 5 ? evp_[5] - evp_[4] : 0ull, evn_ > 6 ? evp_[6] - evp_[5] : 0ull,                         \
               evn_ > 7 ? evp_[7] - evp_[6] : 0ull, evn_ > 8 ? evp_[8] - evp_[7] : 0ull,                         \
               evn_ > 9 ? evp_[9] - evp_[8] : 0ull);                                                             \
    }
__device__ double extremum_grad(int kind, int id, double e2, double e3) {
    // envelope theorem: d/dk of the value at an interior critical point (oracle/src/traj.cpp)
    if (id == 1) return 0.0;
    if (id == 4) return 1.0;  // the reference returns 1 at t = 1 for both position and velocity
    const double r = id == 2 ? e2 : e3;
    return kind == 0 ? r * r * r * (6 * r * r - 15 * r + 10) : 30 * r * r * (r - 1) * (r - 1);
}
__device__ double wrap_to_pi(double a) {
    double w = a;
    while (w < -M_PI) w += 2 * M_PI;
    while (w > M_PI) w -= 2 * M_PI;
    return w;
}

// ARMTD comparison planner: constant-acceleration extrema (ACMP/Trajectory.cu:83-383, the
// gradient with respect to k_actual = k_range * x as the reference) and cost (ACMP/NLPclass.cu:
// 186-246), one thread; restated as in oracle/src/armtd.cpp
__device__ __noinline__ void armtd_extrema_cost(const NlpDev& d, int w, const double* x, double* Gb, double* Jb,
                                                double* fb, double* gradb) {
    const RobotParams& rp = *d.rp;
    const long off = (long)d.T * d.NJ * d.O;
    const double* q0 = d.q0 + w * NF;
    const double* qd0 = d.qd0 + w * NF;
    const double* kr = d.krange + w * NF;
    const double t_move = 0.5, t_total = 1.0, t_to_stop = t_total - t_move;
    for (int i = 0; i < NF; i++) {
        const double k_actual = kr[i] * x[i];
        const double q_peak = q0[i] + qd0[i] * t_move + k_actual * t_move * t_move * 0.5;
        const double q_dot_peak = qd0[i] + k_actual * t_move;
        const double q_ddot_to_stop = -q_dot_peak / t_to_stop;
        const double q_stop = q_peak + q_dot_peak * t_to_stop + 0.5 * q_ddot_to_stop * t_to_stop * t_to_stop;
        const double t_mm = -qd0[i] / k_actual;
        double q_max_tp, q_min_tp, qd_max_tp, qd_min_tp, g_q_max_tp, g_q_min_tp, g_qd_max_tp, g_qd_min_tp;
        double q_max_ts, q_min_ts, qd_max_ts, qd_min_ts, g_q_max_ts, g_q_min_ts, g_qd_max_ts, g_qd_min_ts;
        double qe0, qe1, gqe0, gqe1;
        if (q_peak >= q0[i]) { qe0 = q0[i]; qe1 = q_peak; gqe0 = 0; gqe1 = 0.5 * t_move * t_move; }
        else { qe0 = q_peak; qe1 = q0[i]; gqe0 = 0.5 * t_move * t_move; gqe1 = 0; }
        if (t_mm > 0 && t_mm < t_move) {
            if (k_actual >= 0) {
                q_min_tp = q0[i] + qd0[i] * t_mm + 0.5 * k_actual * t_mm * t_mm;
                q_max_tp = qe1;
                g_q_min_tp = (0.5 * qd0[i] * qd0[i]) / (k_actual * k_actual);
                g_q_max_tp = gqe1;
            } else {
                q_min_tp = qe0;
                q_max_tp = q0[i] + qd0[i] * t_mm + 0.5 * k_actual * t_mm * t_mm;
                g_q_min_tp = gqe0;
                g_q_max_tp = (0.5 * qd0[i] * qd0[i]) / (k_actual * k_actual);
            }
        } else {
            q_min_tp = qe0; q_max_tp = qe1; g_q_min_tp = gqe0; g_q_max_tp = gqe1;
        }
        if (q_dot_peak >= qd0[i]) { qd_min_tp = qd0[i]; qd_max_tp = q_dot_peak; g_qd_min_tp = 0; g_qd_max_tp = t_move; }
        else { qd_min_tp = q_dot_peak; qd_max_tp = qd0[i]; g_qd_min_tp = t_move; g_qd_max_tp = 0; }
        if (q_stop >= q_peak) {
            q_min_ts = q_peak; q_max_ts = q_stop;
            g_q_min_ts = 0.5 * t_move * t_move; g_q_max_ts = 0.5 * t_move * t_move + 0.5 * t_move * t_to_stop;
        } else {
            q_min_ts = q_stop; q_max_ts = q_peak;
            g_q_min_ts = 0.5 * t_move * t_move + 0.5 * t_move * t_to_stop; g_q_max_ts = 0.5 * t_move * t_move;
        }
        if (q_dot_peak >= 0) { qd_min_ts = 0; qd_max_ts = q_dot_peak; g_qd_min_ts = 0; g_qd_max_ts = t_move; }
        else { qd_min_ts = q_dot_peak; qd_max_ts = 0; g_qd_min_ts = t_move; g_qd_max_ts = 0; }
        const bool a = q_min_tp <= q_min_ts, b = q_max_tp >= q_max_ts;
        const bool c = qd_min_tp <= qd_min_ts, e = qd_max_tp >= qd_max_ts;
        const double val[4] = {a ? q_min_tp : q_min_ts, b ? q_max_tp : q_max_ts, c ? qd_min_tp : qd_min_ts,
                               e ? qd_max_tp : qd_max_ts};
        const double grd[4] = {a ? g_q_min_tp : g_q_min_ts, b ? g_q_max_tp : g_q_max_ts, c ? g_qd_min_tp : g_qd_min_ts,
                               e ? g_qd_max_tp : g_qd_max_ts};
        for (int q = 0; q < 4; q++) {
            const long row = off + q * NF + i;
            Gb[row] = val[q];
            for (int k = 0; k < NF; k++) Jb[row * NF + k] = k == i ? grd[q] : 0.0;
        }
    }
    // cost: q_plan = q0 + qd0 * 0.5 + k_range * x * 0.125, wrapped joints summed first
    double qp[NF];
    for (int i = 0; i < NF; i++) qp[i] = q0[i] + qd0[i] * 0.5 + kr[i] * x[i] * 0.125;
    double fv = 0.0;
    bool first = true;
    for (int pass = 1; pass >= 0; pass--)
        for (int i = 0; i < NF; i++) {
            if (rp.wrap_mask[i] != pass) continue;
            const double dd = pass ? wrap_to_pi(d.qdes[w * NF + i] - qp[i]) : (d.qdes[w * NF + i] - qp[i]);
            const double term = dd * dd;
            fv = first ? term : fv + term;
            first = false;
        }
    *fb = fv * rp.cost_scale;
    for (int i = 0; i < NF; i++) {
        const double dk = kr[i] * 0.125;
        const double gv = rp.wrap_mask[i] ? (2 * wrap_to_pi(qp[i] - d.qdes[w * NF + i]) * dk) : (2 * (qp[i] - d.qdes[w * NF + i]) * dk);
        gradb[i] = gv * rp.cost_scale;
    }
}

// ------------------------------------------------------------------------------------------
// Certified plane cache, grid (T, W), once per reach. The collision value of
// a (link, obstacle) pair is max over the 36 planes of the buffered obstacle of
// max(A . c - (d + delta), -A . c - (-d + delta)) (CollisionChecking.cu:230-299), where A, d and
// delta depend on the reach sets and the obstacle only and c = c(x) is the sliced link centre.
// Over the box |x_i| <= PC_XBOX, c(x) lies in centre +- rad (rad = sum of |coefficient| of the
// link's k-monomials, times PC_RADF), which bounds each candidate between lo and hi. With M the
// largest lo, a plane whose hi < M - PC_MARGIN is below the maximum for every x in the box, by far
// more than the rounding of the evaluation: the scan over the remaining planes, in the reference's
// order with the same arithmetic, returns the same value, the same winning plane and the same
// first-maximum tie-break. Those planes are stored (A, d + delta, -d + delta) for eval_kernel.
__device__ inline __attribute__((always_inline)) void pc_bounds(const double* A, double P, double N, const double* cen,
                                                                const double* rad, double& lo, double& hi) {
    const double Ac = A[0] * cen[0] + A[1] * cen[1] + A[2] * cen[2];
    const double S = fabs(A[0]) * rad[0] + fabs(A[1]) * rad[1] + fabs(A[2]) * rad[2];
    lo = fmax(Ac - S - P, -Ac - S - N);
    hi = fmax(Ac + S - P, -Ac + S - N);
}
__device__ inline bool nonzero3(const double* A) { return A[0] != 0 || A[1] != 0 || A[2] != 0; }
// order-preserving 64-bit keys of (non-NaN) doubles, for LDS atomicMax
__device__ inline unsigned long long okey(double x) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ inline double dkey(unsigned long long k) {
    return __builtin_bit_cast(double, (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k);
}

__global__ __launch_bounds__(EVAL_THREADS) void plane_cache_kernel(NlpDev d) {
    const int t = blockIdx.x, w = blockIdx.y, tid = threadIdx.x;
    const long jt = (long)w * d.T + t;
    const int NJ = d.NJ, O = d.O, NP = NJ * O;
    __shared__ double cen[MAX_J][3], rad[MAX_J][3];
    __shared__ double lgen[MAX_J][18];
    __shared__ double obs[MAX_OBS][12];
    __shared__ double llp[MAX_J][LL_PLANES][10];
    __shared__ double oop[MAX_OBS][OO_PLANES][5];
    __shared__ double mixlo[MAX_J * MAX_OBS * OBS_GEN];
    __shared__ unsigned char mixbits[MAX_J * MAX_OBS * OBS_GEN];
    __shared__ double pairM[MAX_J * MAX_OBS];
    __shared__ unsigned cntp[MAX_J * MAX_OBS];
    __shared__ unsigned long long pbits[MAX_J * MAX_OBS];  // surviving planes of a pair, bit = scan position
    __shared__ unsigned total_s;
    for (int i = tid; i < NJ * 18; i += blockDim.x) lgen[i / 18][i % 18] = d.ro.link_gens[jt * NJ * 18 + i];
    for (int i = tid; i < O * 12; i += blockDim.x) obs[i / 12][i % 12] = d.obs[(long)w * O * 12 + i];
    if (tid < NJ * 3) {
        const int l = tid / 3, e = tid % 3;
        const long b = jt * NJ + l;
        const int cnt = d.ro.link_cnt[b];
        double r = 0.0;
        for (int q = 0; q < cnt; q++) r += fabs(d.ro.link_coef[(b * CAP_LM + q) * 3 + e]);
        cen[l][e] = d.ro.link_center[b * 3 + e];
        rad[l][e] = r * PC_RADF;
    }
    __syncthreads();
    for (int u = tid; u < NJ * LL_PLANES + O * OO_PLANES; u += blockDim.x) {
        if (u < NJ * LL_PLANES) ll_table(lgen[u / LL_PLANES], u % LL_PLANES, cen[u / LL_PLANES], llp[u / LL_PLANES][u % LL_PLANES]);
        else oo_table(obs[(u - NJ * LL_PLANES) / OO_PLANES], (u - NJ * LL_PLANES) % OO_PLANES,
                      oop[(u - NJ * LL_PLANES) / OO_PLANES][(u - NJ * LL_PLANES) % OO_PLANES]);
    }
    const int nmix = NP * OBS_GEN;
    // the 9 buffered generators of pair (l, o) (obstacle's 3, the link's 6) and the obstacle centre
    auto load_gens = [&](int l, int o, double (*G)[3], double* oc) {
#pragma unroll
        for (int r = 0; r < 3; r++) oc[r] = obs[o][r];
#pragma unroll
        for (int q = 0; q < OBS_GEN; q++)
#pragma unroll
            for (int r = 0; r < 3; r++) G[q][r] = obs[o][(q + 1) * 3 + r];
#pragma unroll
        for (int q = 0; q < 6; q++)
#pragma unroll
            for (int r = 0; r < 3; r++) G[OBS_GEN + q][r] = lgen[l][r + 3 * q];
    };
    // pass 1 over the mixed planes: the largest lower bound of each (link, obstacle, i) item
    __syncthreads();
    for (int u = tid; u < nmix; u += blockDim.x) {
        const int l = u / (O * OBS_GEN), o = (u / OBS_GEN) % O, i = u % OBS_GEN;
        double G[BUF_GEN][3], oc[3];
        load_gens(l, o, G, oc);
        double M = -1e300;
        const double* const ga = obs[o] + 3 * (i + 1);  // G[i], read from LDS (a run-time row of G would be scratch)
#pragma unroll
        for (int j = 0; j < 6; j++) {
            double A[3], dd, del, lo, hi;
            mixed_plane_j(j, ga, G, oc, A, dd, del);
            pc_bounds(A, dd + del, -dd + del, cen[l], rad[l], lo, hi);
            if (nonzero3(A)) M = fmax(M, lo);
        }
        mixlo[u] = M;
    }
    __syncthreads();
    // pass 1 over the pairs: M, the largest lower bound over all 36 planes
    for (int pr = tid; pr < NP; pr += blockDim.x) {
        const int l = pr / O, o = pr % O;
        double G[BUF_GEN][3], oc[3];
        load_gens(l, o, G, oc);
        double M = fmax(fmax(mixlo[pr * 3], mixlo[pr * 3 + 1]), mixlo[pr * 3 + 2]);
#pragma unroll
        for (int p = 0; p < OO_PLANES; p++) {
            double dd, del, lo, hi;
            oo_complete(oop[o][p], G + OBS_GEN, dd, del);
            pc_bounds(oop[o][p], dd + del, -dd + del, cen[l], rad[l], lo, hi);
            if (nonzero3(oop[o][p])) M = fmax(M, lo);
        }
        for (int p = 0; p < LL_PLANES; p++) {
            double dd, del, lo, hi;
            ll_complete(llp[l][p], G, oc, dd, del);
            pc_bounds(llp[l][p], dd + del, -dd + del, cen[l], rad[l], lo, hi);
            if (nonzero3(llp[l][p])) M = fmax(M, lo);
        }
        pairM[pr] = M;
    }
    __syncthreads();
    // pass 2 over the mixed planes: which can reach M
    for (int u = tid; u < nmix; u += blockDim.x) {
        const int l = u / (O * OBS_GEN), o = (u / OBS_GEN) % O, i = u % OBS_GEN;
        double G[BUF_GEN][3], oc[3];
        load_gens(l, o, G, oc);
        const double M = pairM[u / OBS_GEN] - PC_MARGIN;
        unsigned bits = 0;
        const double* const ga = obs[o] + 3 * (i + 1);
#pragma unroll
        for (int j = 0; j < 6; j++) {
            double A[3], dd, del, lo, hi;
            mixed_plane_j(j, ga, G, oc, A, dd, del);
            pc_bounds(A, dd + del, -dd + del, cen[l], rad[l], lo, hi);
            if (nonzero3(A) && hi >= M) bits |= 1u << j;
        }
        mixbits[u] = (unsigned char)bits;
    }
    __syncthreads();
    // pass 2 over the pairs: the surviving planes in the reference's order (a < b over the 9
    // buffered generators, CollisionChecking.cu:26-39); count, then offsets, then the records
    auto survives = [&](int pr, int l, int o, int a, int b, const double (*G)[3], const double* oc) -> bool {
        if (a < OBS_GEN && b >= OBS_GEN) return (mixbits[pr * OBS_GEN + a] >> (b - OBS_GEN)) & 1;
        const double* P = b < OBS_GEN ? oop[o][a + b - 1] : llp[l][(a - OBS_GEN) * (11 - (a - OBS_GEN)) / 2 + b - a - 1];
        double dd, del, lo, hi;
        if (b < OBS_GEN) oo_complete(P, G + OBS_GEN, dd, del);
        else ll_complete(P, G, oc, dd, del);
        pc_bounds(P, dd + del, -dd + del, cen[l], rad[l], lo, hi);
        return nonzero3(P) && hi >= pairM[pr] - PC_MARGIN;
    };
    for (int pr = tid; pr < NP; pr += blockDim.x) {
        const int l = pr / O, o = pr % O;
        double G[BUF_GEN][3], oc[3];
        load_gens(l, o, G, oc);
        unsigned n = 0;
        unsigned long long bits = 0;
        int pos = 0;
        for (int a = 0; a < BUF_GEN; a++)
            for (int b = a + 1; b < BUF_GEN; b++, pos++)
                if (survives(pr, l, o, a, b, G, oc)) {
                    n++;
                    bits |= 1ull << pos;
                }
        cntp[pr] = n;
        pbits[pr] = bits;
    }
    __syncthreads();
    if (tid < 64) {  // exclusive prefix over the pairs, one wave: lane k sums a contiguous chunk
        const int per = (NP + 63) / 64, b0 = tid * per;
        unsigned s = 0;
        for (int q = b0; q < b0 + per && q < NP; q++) s += cntp[q];
        unsigned incl = s;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned v = __shfl_up(incl, off);
            if (tid >= off) incl += v;
        }
        unsigned run = incl - s;
        for (int q = b0; q < b0 + per && q < NP; q++) {
            const unsigned c = cntp[q];
            cntp[q] = run;
            run += c;
            d.pcoff[jt * NP + q] = (run - c) << 8 | c;
        }
        if (tid == 63) total_s = incl;
    }
    __syncthreads();
    // the block's records from the pool: one atomic per block; a build that runs out of pool is
    // repeated by the host on a larger one (ensure_plane_cache)
    __shared__ unsigned long long base_s;
    if (tid == 0) {
        const unsigned long long b0 = atomicAdd(d.pcnext, total_s);
        const bool fits = b0 + total_s <= (unsigned long long)d.pc_pool;
        d.pcok[jt] = fits ? 1 : 0;
        d.pcbase[jt] = fits ? b0 : 0;
        base_s = fits ? b0 : ~0ull;
    }
    __syncthreads();
    if (base_s == ~0ull) return;
    double* const rec = d.pc + 5 * base_s;
    uint16_t* const pcp = d.pcp + base_s;
    const int cap = (int)total_s;  // the block's [5][n] record arrays
    for (int pr = tid; pr < NP; pr += blockDim.x) {
        const int l = pr / O, o = pr % O;
        double G[BUF_GEN][3], oc[3];
        load_gens(l, o, G, oc);
        unsigned q = cntp[pr];
        const unsigned long long bits = pbits[pr];
        int pos = 0;
        for (int a = 0; a < BUF_GEN; a++)
            for (int b = a + 1; b < BUF_GEN; b++) {
                if (!((bits >> pos++) & 1ull)) continue;
                double A[3], dd, del;
                if (a < OBS_GEN && b >= OBS_GEN) {
                    mixed_plane_j(b - OBS_GEN, obs[o] + 3 * (a + 1), G, oc, A, dd, del);
                } else {
                    const double* P = b < OBS_GEN ? oop[o][a + b - 1] : llp[l][(a - OBS_GEN) * (11 - (a - OBS_GEN)) / 2 + b - a - 1];
                    A[0] = P[0]; A[1] = P[1]; A[2] = P[2];
                    if (b < OBS_GEN) oo_complete(P, G + OBS_GEN, dd, del);
                    else ll_complete(P, G, oc, dd, del);
                }
                rec[q] = A[0];
                rec[cap + q] = A[1];
                rec[2 * cap + q] = A[2];
                rec[3 * cap + q] = dd + del;
                rec[4 * cap + q] = -dd + del;
                pcp[q] = (uint16_t)pr;
                q++;
            }
    }
}

// ------------------------------------------------------------------------------------------
// g(x) and dense Jacobian, grid (T, W). mode 0: ws.x into slot 0 (start point,
// armour_eval_constraints); mode 1: the line-search trial ws.xt into the non-current slot (worlds
// still searching only). The sliced link centres go to the slot's own region (feasible_kernel
// copies the current slot's, the final iterate's, out).
// ARMTD selects the comparison planner's extrema and cost at compile time: a call into them from
// the ARMOUR instantiation would cost it registers and a stack frame (occupancy 4 -> 3 waves/SIMD)
// CACHED (fp64 only): the collision rows from the certified plane cache, for points in its box
// (every solver point; armour_eval_constraints checks x on the host); otherwise the full scan.
// LM, UM, UB: LDS capacities — monomials per link / torque PZ and the staging buffer (doubles).
// eval_kernel_t reserves the reach's caps (CAP_LM, CAP_UM); eval_kernel_small the small ones, for
// batches whose largest PZs and pair tables fit (planner.hip checks): 16 KB of LDS, held to eight
// waves per SIMD (64 VGPRs, 26 spilled) — eight resident blocks per CU instead of four. Measured per
// 327-world solve: 16.4 ms (four blocks), 16.1 (five), 14.9 (six), 14.1 (seven), 13.6 (eight); the
// latency of the staged phases hides behind more blocks, the spills cost less.
constexpr int UB_FULL = MAX_J * CAP_LM * 3 + NF * CAP_UM;
constexpr int LM_S = 16, UM_S = 64;
constexpr int UB_S = 1544;   // >= MAX_J * LM_S * 3 + NF * UM_S, and the pair tables of 280 pairs (5.5 NP + 1)
static_assert(UB_S >= MAX_J * LM_S * 3 + NF * UM_S, "small staging buffer");
__host__ __device__ constexpr int eval_pair_doubles(int np) { return np + (np + 1) / 2 + 4 * np; }
template <typename R, bool ARMTD, bool CACHED, int LM, int UM, int UB>
__device__ __attribute__((always_inline)) void eval_body(const NlpDev& d, int mode) {
    static_assert(!CACHED || std::is_same<R, double>::value, "the plane cache is fp64");
    // mode 5: the trial point the speculative round chose (ipm_world_Cs: spec_k >= 0), in full,
    // into the world's trial slot (list entries, blockIdx.y -> wl)
    if ((mode == 1 || mode == 5) && d.lcount && blockIdx.y >= *d.lcount) return;
    const int t = blockIdx.x, w = world_of(d, blockIdx.y);
    WorldState& S = d.ws[w];
    // (restoration launches, d.resto: the worlds in the restoration phase, WS_RESTO)
    if (mode == 1 && !((d.resto ? S.status == WS_RESTO : S.status == 0) && S.searching)) return;
    if (mode == 5 && !(d.resto ? (S.status == WS_RESTO && S.rpend) : (S.status == 0 && S.spec_k >= 0))) return;
    EVP_DECL EVP_MARK
    const int slot = mode == 0 ? 0 : 1 - S.cur;
    double* const Gb = d.g + gidx(d, slot, w, 0);
    double* const Jb = d.J + gidx(d, slot, w, 0) * NF;
    double* const Lcb = d.link_c + slot * d.lcs + (long)w * d.T * d.NJ * 3;
    double* const fb = d.f + slot * d.W + w;
    double* const gradb = d.grad + ((long)slot * d.W + w) * NF;
    // compact collision Jacobian (NlpDev::jn / jd); mode 0 also writes those rows densely into Jb
    const long ncol = (long)d.T * d.NJ * d.O;
    double* const Jnb = d.jn + slot * d.njn + (long)w * ncol * 3;
    double* const Jdb = d.jd + slot * d.njd + (long)w * d.T * d.NJ * NF * 3;
    const RobotParams& rp = *d.rp;
    const int tid = threadIdx.x;
    const long jt = (long)w * d.T + t;
    const int NJ = d.NJ, O = d.O;
    // everything this (world, t) reads is staged into LDS with coalesced loads first
    __shared__ double x[NF];   // the point itself stays fp64 (cost and extremum rows)
    __shared__ R lc[MAX_J][3];
    __shared__ R dlc[MAX_J][NF][3];
    __shared__ R lgen[MAX_J][18];
    __shared__ R obs[MAX_OBS][12];
    __shared__ uint16_t lh[MAX_J][LM];
    __shared__ uint16_t th[NF][UM];
    // monomial coefficients while slicing; afterwards the same LDS holds the obstacle-independent
    // link-link planes and the link-independent obstacle-obstacle planes (full scan), or the pair
    // tables of the cached scan
    __shared__ double ubuf[UB];
    static_assert(MAX_J * LM * 3 + NF * UM <= UB, "monomial staging");
    auto lco = reinterpret_cast<R (*)[LM][3]>(ubuf);
    auto tco = reinterpret_cast<R (*)[UM]>(ubuf + MAX_J * LM * 3);
    constexpr int NMIX = MAX_J * MAX_OBS * OBS_GEN;
    static_assert(CACHED || MAX_J * LL_PLANES * 10 + MAX_OBS * OO_PLANES * 5 + NMIX + (NMIX + 7) / 8 <= UB, "plane tables");
    auto llp = reinterpret_cast<R (*)[LL_PLANES][10]>(ubuf);
    auto oop = reinterpret_cast<R (*)[OO_PLANES][5]>(ubuf + MAX_J * LL_PLANES * 10);
    R* mixv = reinterpret_cast<R*>(ubuf + MAX_J * LL_PLANES * 10 + MAX_OBS * OO_PLANES * 5);   // per (link, obstacle, i)
    int8_t* mixc = reinterpret_cast<int8_t*>(mixv + NMIX);
    __shared__ int lcnt[MAX_J], tcnt[NF];
    __shared__ R ptab[NF][8];
    if (tid < NF) {
        const double xd = mode == 0 ? S.x[tid] : S.xt[tid];
        x[tid] = xd;
        const R xj = (R)xd;
        ptab[tid][0] = (R)1.0; ptab[tid][1] = xj; ptab[tid][2] = xj * xj; ptab[tid][3] = xj * xj * xj;
        ptab[tid][4] = (R)0.0; ptab[tid][5] = (R)1.0 * (R)1.0; ptab[tid][6] = (R)2.0 * xj; ptab[tid][7] = (R)3.0 * (xj * xj);
    }
    if (tid < NJ) lcnt[tid] = d.ro.link_cnt[jt * NJ + tid];
    if (tid >= 32 && tid < 32 + NF) tcnt[tid - 32] = d.nt ? d.ro.tq_cnt[jt * NF + tid - 32] : 0;  // ARMTD: no torque PZs
    if constexpr (!CACHED) {
        for (int i = tid; i < NJ * 18; i += blockDim.x) lgen[i / 18][i % 18] = d.ro.link_gens[jt * NJ * 18 + i];
        for (int i = tid; i < O * 12; i += blockDim.x) obs[i / 12][i % 12] = d.obs[(long)w * O * 12 + i];
    }
    __syncthreads();
    EVP_MARK
    if (!(d.diag & 1)) {
        // only the valid monomials, enumerated compactly (one load round per thread): u < L are
        // link monomials, the rest torque monomials; prefix offsets from the per-PZ counts
        int lpre[MAX_J + 1], tpre[NF + 1];
        lpre[0] = 0;
#pragma unroll
        for (int l = 0; l < MAX_J; l++) lpre[l + 1] = lpre[l] + (l < NJ ? lcnt[l] : 0);
        tpre[0] = 0;
#pragma unroll
        for (int j = 0; j < NF; j++) tpre[j + 1] = tpre[j] + tcnt[j];
        const int L = lpre[MAX_J], M = tpre[NF];
        for (int u = tid; u < L + M; u += blockDim.x) {
            if (u < L) {
                int l = 0, q0 = 0;
#pragma unroll
                for (int k = 1; k < MAX_J; k++) if (u >= lpre[k]) { l = k; q0 = lpre[k]; }
                const int q = u - q0;
                const long b = (jt * NJ + l) * CAP_LM + q;
                lh[l][q] = d.ro.link_hash[b];
                lco[l][q][0] = d.ro.link_coef[b * 3];
                lco[l][q][1] = d.ro.link_coef[b * 3 + 1];
                lco[l][q][2] = d.ro.link_coef[b * 3 + 2];
            } else {
                const int v = u - L;
                int j = 0, q0 = 0;
#pragma unroll
                for (int k = 1; k < NF; k++) if (v >= tpre[k]) { j = k; q0 = tpre[k]; }
                const int q = v - q0;
                const long b = (jt * NF + j) * CAP_UM + q;
                th[j][q] = d.ro.tq_hash[b];
                tco[j][q] = d.ro.tq_coef[b];
            }
        }
    }
    __syncthreads();
    EVP_MARK
    // slices (PZsparse.cu:404-435 value, :477-516 gradient): one thread per output — k = 0 the
    // value, k = 1..7 the derivative in x_{k-1} — summing its terms in monomial order. Powers come
    // from a per-variable table (ptab, filled with the staging), x_j^g as the reference forms it.
    // The NF * 8 torque outputs (the longest sums) fill wave 0 alone, the link outputs start at
    // thread 64: no wave runs both loops.
    const int nlk = NJ * 3 * 8;
    for (int u = tid; u < ((d.diag & 1) ? 0 : 64 + nlk); u += blockDim.x) {
      if (u >= 64) {
        const int ul = u - 64;
        const int l = ul / 24, e = (ul / 8) % 3, k = ul % 8;
        const long base = jt * NJ + l;
        R c = k == 0 ? d.ro.link_center[base * 3 + e] : 0.0;
        const int cnt = lcnt[l];
        // four independent products in flight, summed in monomial order
        int q = 0;
        for (; q + 4 <= cnt; q += 4) {
            const R v0 = slice_term(lco[l][q][e], lh[l][q], k, ptab);
            const R v1 = slice_term(lco[l][q + 1][e], lh[l][q + 1], k, ptab);
            const R v2 = slice_term(lco[l][q + 2][e], lh[l][q + 2], k, ptab);
            const R v3 = slice_term(lco[l][q + 3][e], lh[l][q + 3], k, ptab);
            c = c + v0; c = c + v1; c = c + v2; c = c + v3;
        }
        for (; q < cnt; q++) c = c + slice_term(lco[l][q][e], lh[l][q], k, ptab);
        if (k == 0) {
            const R r = d.ro.link_rad[base * 3 + e];
            const R cc = ((c - r) + (c + r)) * 0.5;  // getCenter(Interval(c - r, c + r))
            lc[l][e] = cc;
            Lcb[((long)t * NJ + l) * 3 + e] = cc;
        } else {
            dlc[l][k - 1][e] = c;
            Jdb[(((long)t * NJ + l) * NF + k - 1) * 3 + e] = c;
        }
      } else {
        // torque rows (NLPclass.cu:304-309, 376-380)
        if (u >= NF * 8 || d.nt == 0) continue;
        const int j = u / 8, k = u % 8;
        const long base = jt * NF + j;
        R c = k == 0 ? d.ro.tq_center[base] : 0.0;
        const int cnt = tcnt[j];
        int q = 0;
        for (; q + 4 <= cnt; q += 4) {
            const R v0 = slice_term(tco[j][q], th[j][q], k, ptab);
            const R v1 = slice_term(tco[j][q + 1], th[j][q + 1], k, ptab);
            const R v2 = slice_term(tco[j][q + 2], th[j][q + 2], k, ptab);
            const R v3 = slice_term(tco[j][q + 3], th[j][q + 3], k, ptab);
            c = c + v0; c = c + v1; c = c + v2; c = c + v3;
        }
        for (; q < cnt; q++) c = c + slice_term(tco[j][q], th[j][q], k, ptab);
        const long gi = (long)t * NF + j;
        if (k == 0) {
            const R r = d.ro.tq_rad[base];
            Gb[gi] = ((c - r) + (c + r)) * 0.5;
        } else {
            Jb[gi * NF + k - 1] = c;
        }
      }
    }
    if constexpr (ARMTD) {
        if (tid == blockDim.x - 1 && t == 0) armtd_extrema_cost(d, w, x, Gb, Jb, fb, gradb);
    } else if (t == 0 && tid >= (int)blockDim.x - 2 * NF - 1) {
        // extremum rows (NLPclass.cu:319-320, 390-391), one thread per (kind, joint), and the cost
        // (NLPclass.cu:207-267) on one more thread
        const double* q0 = d.q0 + w * NF;
        const double* qd0 = d.qd0 + w * NF;
        const double* qdd0 = d.qdd0 + w * NF;
        const double D = rp.duration;
        const int v = tid - ((int)blockDim.x - 2 * NF - 1);
        if (v < 2 * NF) {
            const long off2 = (long)NF * d.T + (long)d.T * d.NJ * d.O;
            const int kind = v / NF, i = v % NF;
            const double Tq = qd0[i] * D, TTq = qdd0[i] * D * D;
            const double ka = rp.k_range[i] * x[i];
            double mn, mx, e2, e3;
            int mnid, mxid;
            extremum(kind, q0[i], Tq, TTq, ka, &mn, &mx, &mnid, &mxid, &e2, &e3);
            const double scale = kind == 0 ? 1.0 : D;
            const long gmin = off2 + kind * 2 * NF + i, gmax = gmin + NF;
            Gb[gmin] = mn / scale;
            Gb[gmax] = mx / scale;
            const double gmn = extremum_grad(kind, mnid, e2, e3) * rp.k_range[i] / scale;
            const double gmx = extremum_grad(kind, mxid, e2, e3) * rp.k_range[i] / scale;
#pragma unroll
            for (int k = 0; k < NF; k++) {
                Jb[gmin * NF + k] = (k == i) ? gmn : 0.0;
                Jb[gmax * NF + k] = (k == i) ? gmx : 0.0;
            }
        } else {
            // cost: wrapped joints summed first (NLPclass.cu:225-233)
            const double tp = rp.t_plan;
            double qp[NF];
            for (int i = 0; i < NF; i++) qp[i] = bz_q(q0[i], qd0[i] * D, qdd0[i] * D * D, rp.k_range[i] * x[i], tp);
            double fv = 0.0;
            bool first = true;
            for (int pass = 1; pass >= 0; pass--)
                for (int i = 0; i < NF; i++) {
                    if (rp.wrap_mask[i] != pass) continue;
                    const double dd = pass ? wrap_to_pi(d.qdes[w * NF + i] - qp[i]) : (d.qdes[w * NF + i] - qp[i]);
                    const double term = dd * dd;
                    fv = first ? term : fv + term;
                    first = false;
                }
            *fb = fv * rp.cost_scale;
            for (int i = 0; i < NF; i++) {
                const double dk = tp * tp * tp * (6 * tp * tp - 15 * tp + 10) * rp.k_range[i];
                double gv = rp.wrap_mask[i] ? (2 * wrap_to_pi(qp[i] - d.qdes[w * NF + i]) * dk) : (2 * (qp[i] - d.qdes[w * NF + i]) * dk);
                gradb[i] = gv * rp.cost_scale;
            }
        }
    }
    __syncthreads();
    EVP_MARK
    // collision rows (CollisionChecking.cu:230-299). Of the 36 planes of a buffered obstacle, the
    // 15 spanned by two link generators do not depend on the obstacle and the 3 spanned by two
    // obstacle generators do not depend on the link: those are formed once per block, with the
    // parts of d and delta they determine alone (delta's summands kept separate where the
    // reference's left-to-right sum needs them in order), then the per-(link, obstacle) scan only
    // completes them.
    const long nt = d.nt;
    bool coll = !(d.diag & 2);
    if constexpr (CACHED) {
        // the certified plane cache (plane_cache_kernel): the scan over the kept planes, same order,
        // same arithmetic. A point outside the cache's box cannot come from the solver (its box
        // slacks keep |x_i| <= 1 up to rounding); should one arrive, its rows are NaN (the line
        // search rejects the trial) and the miss is counted (armour_get_plane_cache_stats).
        bool inbox = true;
#pragma unroll
        for (int j = 0; j < NF; j++) inbox = inbox && fabs(x[j]) <= PC_XBOX;
        if (coll && !inbox) {
            for (int pr = tid; pr < NJ * O; pr += blockDim.x)
                Gb[nt + ((long)(pr / O) * d.T + t) * O + pr % O] = __builtin_nan("");
            if (tid == 0) atomicAdd(d.cnt + 7, 1u);
        } else if (coll) {
            // Record-parallel scan. Every thread takes records q = tid, tid + 256, ... of the block's
            // kept planes straight from global memory and forms both candidates, A . c - P before
            // -A . c - N (position 2 q + neg in the serial scan order). Pass 1: the pair's maximum by
            // an LDS atomicMax on an order-preserving key; pass 2: the first position holding that
            // maximum (atomicMin); pass 3: that record publishes its plane. A candidate wins only
            // above the serial scan's start value (-1e8, strict >), NaN never: the serial scan's
            // strict-> first maximum, value, plane and sign exactly. The pair tables live in the
            // slicing buffer (free now).
            const int NP = NJ * O;
            const unsigned last = d.pcoff[jt * NP + NP - 1];
            const int total = (int)(last >> 8) + (int)(last & 255);
            const unsigned long long pb = d.pcbase[jt];
            const double* const rec = d.pc + 5 * pb;
            const uint16_t* const pcp = d.pcp + pb;
            const int cap = total;  // the block's [5][n] record arrays
            // eval_pair_doubles(NP) <= UB: always for UB_FULL, checked by the host for UB_S
            unsigned long long* const pkey = reinterpret_cast<unsigned long long*>(ubuf);  // [NP]
            unsigned* const pidx = reinterpret_cast<unsigned*>(ubuf + NP);                   // [NP]
            double* const pB = ubuf + NP + (NP + 1) / 2;                                     // [NP][4]: A, value
            static_assert(eval_pair_doubles(MAX_J * MAX_OBS) <= UB_FULL, "pair tables");
            const double start = -100000000.0;
            for (int pr = tid; pr < NP; pr += blockDim.x) {
                pkey[pr] = okey(start);
                pidx[pr] = 0xFFFFFFFFu;
            }
            __syncthreads();
            EVP_MARK
            auto cand = [&](int q, double& v, int& sub, int& pr, double* a) {
                a[0] = rec[q];
                a[1] = rec[cap + q];
                a[2] = rec[2 * cap + q];
                const double P = rec[3 * cap + q], N = rec[4 * cap + q];
                pr = pcp[q];
                const int l = pr / O;
                const double Ac = a[0] * lc[l][0] + a[1] * lc[l][1] + a[2] * lc[l][2];
                const double pos = Ac - P, neg = -Ac - N;
                sub = (neg > pos || pos != pos) ? 1 : 0;  // the serial scan takes neg only when it beats pos
                v = sub ? neg : pos;
            };
            constexpr int RPT = 3;
            if (total <= RPT * EVAL_THREADS) {
                double v[RPT], a[RPT][3];
                int sub[RPT], pq[RPT];
#pragma unroll
                for (int s = 0; s < RPT; s++) {
                    const int q = tid + s * EVAL_THREADS;
                    v[s] = start;
                    sub[s] = 0;
                    pq[s] = 0;
                    if (q < total) {
                        cand(q, v[s], sub[s], pq[s], a[s]);
                        if (v[s] > start) atomicMax(&pkey[pq[s]], okey(v[s]));
                    }
                }
                __syncthreads();
                EVP_MARK
#pragma unroll
                for (int s = 0; s < RPT; s++) {
                    const int q = tid + s * EVAL_THREADS;
                    if (q < total && v[s] > start && v[s] == dkey(pkey[pq[s]])) atomicMin(&pidx[pq[s]], (unsigned)(2 * q + sub[s]));
                }
                __syncthreads();
                EVP_MARK
#pragma unroll
                for (int s = 0; s < RPT; s++) {
                    const int q = tid + s * EVAL_THREADS;
                    if (q < total && pidx[pq[s]] == (unsigned)(2 * q + sub[s])) {
                        double* const b = pB + pq[s] * 4;
                        b[0] = a[s][0]; b[1] = a[s][1]; b[2] = a[s][2]; b[3] = v[s];
                    }
                }
            } else {
                for (int q = tid; q < total; q += blockDim.x) {
                    double v, a[3];
                    int sub, pr;
                    cand(q, v, sub, pr, a);
                    if (v > start) atomicMax(&pkey[pr], okey(v));
                }
                __syncthreads();
                EVP_MARK
                for (int q = tid; q < total; q += blockDim.x) {
                    double v, a[3];
                    int sub, pr;
                    cand(q, v, sub, pr, a);
                    if (v > start && v == dkey(pkey[pr])) atomicMin(&pidx[pr], (unsigned)(2 * q + sub));
                }
                __syncthreads();
                EVP_MARK
                for (int q = tid; q < total; q += blockDim.x) {
                    double v, a[3];
                    int sub, pr;
                    cand(q, v, sub, pr, a);
                    if (pidx[pr] == (unsigned)(2 * q + sub)) {
                        double* const b = pB + pr * 4;
                        b[0] = a[0]; b[1] = a[1]; b[2] = a[2]; b[3] = v;
                    }
                }
            }
            __syncthreads();
            EVP_MARK
            for (int pr = tid; pr < NP; pr += blockDim.x) {
                const int l = pr / O, o = pr % O;
                const unsigned wi = pidx[pr];
                const bool won = wi != 0xFFFFFFFFu, isneg = won && (wi & 1u);
                const double* const b = pB + pr * 4;
                const double best = won ? b[3] : start;
                const double B0 = won ? b[0] : 0.0, B1 = won ? b[1] : 0.0, B2 = won ? b[2] : 0.0;
                const long row = nt + ((long)l * d.T + t) * O + o;
                Gb[row] = -best;
                // J = isneg ? B . dc : -(B . dc) = n . dc with n = isneg ? B : -B (negation is exact)
                double* const jn = Jnb + (row - nt) * 3;
                jn[0] = isneg ? B0 : -B0;
                jn[1] = isneg ? B1 : -B1;
                jn[2] = isneg ? B2 : -B2;
                if (mode == 0) {
#pragma unroll
                    for (int kk = 0; kk < NF; kk++) {
                        const double dot = B0 * dlc[l][kk][0] + B1 * dlc[l][kk][1] + B2 * dlc[l][kk][2];
                        Jb[row * NF + kk] = isneg ? dot : -dot;
                    }
                }
            }
            coll = false;
        }
    }
    if constexpr (!CACHED) {
    for (int u = tid; u < (coll ? NJ * LL_PLANES + O * OO_PLANES : 0); u += blockDim.x) {
        if (u < NJ * LL_PLANES) {
            const int l = u / LL_PLANES, p = u % LL_PLANES;
            ll_table(lgen[l], p, lc[l], llp[l][p]);
        } else {
            const int v = u - NJ * LL_PLANES, o = v / OO_PLANES, p = v % OO_PLANES;
            oo_table(obs[o], p, oop[o][p]);
        }
    }
    // the 18 mixed planes (one obstacle generator i, one link generator j) depend on both: one item
    // per (link, obstacle, i) scans its 6 planes j = 0..5 in order and keeps the first maximum
    // (value, and j * 2 + neg; -1: none) — 3 items per pair fill the waves that one thread per
    // pair leaves idle
    const int nmix = coll ? NJ * O * OBS_GEN : 0;
    for (int u = tid; u < nmix; u += blockDim.x) {
        const int l = u / (O * OBS_GEN), o = (u / OBS_GEN) % O, i = u % OBS_GEN;
        const R c0 = lc[l][0], c1 = lc[l][1], c2 = lc[l][2];
        R G[BUF_GEN][3], oc[3];
#pragma unroll
        for (int r = 0; r < 3; r++) oc[r] = obs[o][r];
#pragma unroll
        for (int q = 0; q < OBS_GEN; q++)
#pragma unroll
            for (int r = 0; r < 3; r++) G[q][r] = obs[o][(q + 1) * 3 + r];
#pragma unroll
        for (int q = 0; q < 6; q++)
#pragma unroll
            for (int r = 0; r < 3; r++) G[OBS_GEN + q][r] = lgen[l][r + 3 * q];
        R ga[3];
#pragma unroll
        for (int r = 0; r < 3; r++) ga[r] = obs[o][(i + 1) * 3 + r];
        const R cc[3] = {c0, c1, c2};
        R best = -100000000.0;
        int code = -1;
        auto scan = [&](auto e_tag, int j) {
            constexpr int E = decltype(e_tag)::value;
            R A[3], dd, del;
            mixed_plane<E>(ga, G[OBS_GEN + j], G, oc, A, dd, del);
            const R Ac = dot_z<E>(A, cc);
            if (A[0] != 0 || A[1] != 0 || A[2] != 0) {
                const R pos = Ac - (dd + del);
                const R neg = -Ac - (-dd + del);
                if (pos > best) { best = pos; code = 2 * j; }
                if (neg > best) { best = neg; code = 2 * j + 1; }
            }
        };
        using gen = std::integral_constant<int, -1>;
        scan(gen{}, 0);
        scan(gen{}, 1);
        scan(gen{}, 2);
        scan(std::integral_constant<int, 0>{}, 3);
        scan(std::integral_constant<int, 1>{}, 4);
        scan(std::integral_constant<int, 2>{}, 5);
        mixv[u] = best;
        mixc[u] = (int8_t)code;
    }
    __syncthreads();
    EVP_MARK
    // one thread per (link, obstacle) completes the 36-plane scan in the reference's order (pairs
    // (a, b), a < b, lexicographic: CollisionChecking.cu:26-39; pos_p before neg_p, strict >), so the
    // first maximum wins as in the reference's serial loop; a mixed run (a < 3 <= b) enters as its
    // item's first maximum, and a winning mixed plane's normal is formed again at the end
    for (int pr = tid; pr < (coll ? NJ * O : 0); pr += blockDim.x) {
        const int l = pr / O, o = pr % O;
        R best = -100000000.0;
        R B0 = 0, B1 = 0, B2 = 0;
        bool isneg = false;
        int mwin = -1;  // winning mixed plane: i * 6 + j
        const R c0 = lc[l][0], c1 = lc[l][1], c2 = lc[l][2];
        // the 9 buffered generators in registers: obstacle's 3, then the link's 6
        R G[BUF_GEN][3], oc[3];
#pragma unroll
        for (int r = 0; r < 3; r++) oc[r] = obs[o][r];
#pragma unroll
        for (int i = 0; i < OBS_GEN; i++)
#pragma unroll
            for (int r = 0; r < 3; r++) G[i][r] = obs[o][(i + 1) * 3 + r];
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int r = 0; r < 3; r++) G[OBS_GEN + i][r] = lgen[l][r + 3 * i];
#pragma unroll
        for (int a = 0; a < BUF_GEN; a++)
#pragma unroll
            for (int b = a + 1; b < BUF_GEN; b++) {
                if (a < OBS_GEN && b >= OBS_GEN) {
                    if (b == OBS_GEN) {
                        const int u = pr * OBS_GEN + a;
                        const R v = mixv[u];
                        const int cd = mixc[u];
                        if (v > best) { best = v; mwin = a * 6 + (cd >> 1); isneg = cd & 1; }
                    }
                    continue;
                }
                R A0, A1, A2, dd, del, Ac;
                if (b < OBS_GEN) {
                    const R* P = oop[o][a + b - 1];
                    A0 = P[0]; A1 = P[1]; A2 = P[2];
                    oo_complete(P, G + OBS_GEN, dd, del);
                    Ac = A0 * c0 + A1 * c1 + A2 * c2;
                } else {
                    const int i = a - OBS_GEN, j = b - OBS_GEN;
                    const R* P = llp[l][i * (11 - i) / 2 + j - i - 1];
                    A0 = P[0]; A1 = P[1]; A2 = P[2]; Ac = P[3];
                    ll_complete(P, G, oc, dd, del);
                }
                // the reference skips a zero normal (norm > 0); for a normalised or zeroed A
                // that is exactly "some component non-zero"
                if (A0 != 0 || A1 != 0 || A2 != 0) {
                    const R pos = Ac - (dd + del);
                    const R neg = -Ac - (-dd + del);
                    if (pos > best) { best = pos; B0 = A0; B1 = A1; B2 = A2; isneg = false; mwin = -1; }
                    if (neg > best) { best = neg; B0 = A0; B1 = A1; B2 = A2; isneg = true; mwin = -1; }
                }
            }
        if (mwin >= 0) plane_normal(obs[o] + 3 * (mwin / 6 + 1), lgen[l] + 3 * (mwin % 6), B0, B1, B2);
        const long row = nt + ((long)l * d.T + t) * O + o;
        Gb[row] = -best;
        double* const jn = Jnb + (row - nt) * 3;
        jn[0] = isneg ? B0 : -B0;
        jn[1] = isneg ? B1 : -B1;
        jn[2] = isneg ? B2 : -B2;
        if (mode == 0) {
#pragma unroll
            for (int k = 0; k < NF; k++) {
                const R dot = B0 * dlc[l][k][0] + B1 * dlc[l][k][1] + B2 * dlc[l][k][2];
                Jb[row * NF + k] = isneg ? dot : -dot;
            }
        }
    }
    }
    EVP_PRINT("EV")
}

// the product evaluation is fp64; eval_kernel_t<float> serves only the fp32 tolerance study
// (ARMOUR_EVAL_F32, tools/fp32_study.py): reach sets stay fp64, the slicing and collision
// arithmetic runs in float
template <typename R, bool ARMTD, bool CACHED>
__global__ __launch_bounds__(EVAL_THREADS) void eval_kernel_t(NlpDev d, int mode) {
    eval_body<R, ARMTD, CACHED, CAP_LM, CAP_UM, UB_FULL>(d, mode);
}
__global__ __launch_bounds__(EVAL_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void eval_kernel_small(NlpDev d, int mode) {
    eval_body<double, false, true, LM_S, UM_S, UB_S>(d, mode);
}
template __global__ void eval_kernel_t<double, false, false>(NlpDev, int);
template __global__ void eval_kernel_t<float, false, false>(NlpDev, int);
template __global__ void eval_kernel_t<double, true, false>(NlpDev, int);
template __global__ void eval_kernel_t<float, true, false>(NlpDev, int);
template __global__ void eval_kernel_t<double, false, true>(NlpDev, int);
template __global__ void eval_kernel_t<double, true, true>(NlpDev, int);

// ------------------------------------------------------------------------------------------
// Speculative line-search round, values only. Block (t, list entry i) evaluates the K = max_ls - 1
// remaining trial points of world wl[i] (alpha halved k times from the round's alpha: the points
// ipm_world_C's sequential rounds would visit) — the constraint values and the cost, all the
// acceptance test reads (ipm_rows_Cs / ipm_world_Cs); the Jacobian is formed only for the trial
// chosen, by a full evaluation (eval_kernel_t mode 5). The monomials are staged and each
// certified-plane record is loaded once for all K points; every value is formed with
// eval_kernel_t's arithmetic.
// LM, UM, UB as eval_body; the staging buffer then holds the (trial, pair) keys, K * NP <= UB
constexpr int UB_TS = EV_MAXK * 280;   // small variant: 9 trials of up to 280 pairs (7 links x 40 obstacles)
static_assert(UB_TS >= MAX_J * LM_S * 3 + NF * UM_S, "small trials staging buffer");
__device__ inline double pass_b_alpha(const NlpDev& d, int w);
template <int LM, int UM, int UB, int KM = EV_MAXK>
__device__ __attribute__((always_inline)) void eval_trials_body(const NlpDev& d) {
    if (d.lcount && blockIdx.y >= *d.lcount) return;
    const int t = blockIdx.x, i = blockIdx.y, w = d.wl[i];
    const WorldState& S = d.ws[w];
    // (restoration launches, d.resto: the trials of the phase's Armijo search)
    if (!(d.resto ? (S.status == WS_RESTO && S.searching) : (S.status == 0 && (d.b_in_cs || S.searching)))) return;
    EVP_DECL EVP_MARK
    const RobotParams& rp = *d.rp;
    const int tid = threadIdx.x, K = d.K;
    const long jt = (long)w * d.T + t;
    const int NJ = d.NJ, O = d.O, NP = NJ * O;
    const long nt = d.nt;
    __shared__ double xk[KM][NF];
    __shared__ double ptab[KM][NF][4];  // x_j^g of trial k (the value slices' factors)
    __shared__ double lck[KM][MAX_J][3];
    __shared__ uint16_t lh[MAX_J][LM];
    __shared__ uint16_t th[NF][UM];
    __shared__ double ubuf[UB];
    static_assert(MAX_J * LM * 3 + NF * UM <= UB, "monomial staging");
    __shared__ int lcnt[MAX_J], tcnt[NF];
    auto lco = reinterpret_cast<double (*)[LM][3]>(ubuf);
    auto tco = reinterpret_cast<double (*)[UM]>(ubuf + MAX_J * LM * 3);
    if (tid < K * NF) {
        const int kk = tid / NF, j = tid % NF;
        double a = d.b_in_cs ? pass_b_alpha(d, w) : S.alpha;
        for (int q = 0; q < kk; q++) a *= 0.5;
        const double xj = S.x[j] + a * S.dx[j];
        xk[kk][j] = xj;
        ptab[kk][j][0] = 1.0; ptab[kk][j][1] = xj; ptab[kk][j][2] = xj * xj; ptab[kk][j][3] = xj * xj * xj;
    }
    if (tid >= 64 && tid < 64 + NJ) lcnt[tid - 64] = d.ro.link_cnt[jt * NJ + tid - 64];
    if (tid >= 96 && tid < 96 + NF) tcnt[tid - 96] = d.nt ? d.ro.tq_cnt[jt * NF + tid - 96] : 0;
    __syncthreads();
    EVP_MARK
    {
        int lpre[MAX_J + 1], tpre[NF + 1];
        lpre[0] = 0;
#pragma unroll
        for (int l = 0; l < MAX_J; l++) lpre[l + 1] = lpre[l] + (l < NJ ? lcnt[l] : 0);
        tpre[0] = 0;
#pragma unroll
        for (int j = 0; j < NF; j++) tpre[j + 1] = tpre[j] + tcnt[j];
        const int L = lpre[MAX_J], M = tpre[NF];
        for (int u = tid; u < L + M; u += blockDim.x) {
            if (u < L) {
                int l = 0, q0 = 0;
#pragma unroll
                for (int k = 1; k < MAX_J; k++) if (u >= lpre[k]) { l = k; q0 = lpre[k]; }
                const int q = u - q0;
                const long b = (jt * NJ + l) * CAP_LM + q;
                lh[l][q] = d.ro.link_hash[b];
                lco[l][q][0] = d.ro.link_coef[b * 3];
                lco[l][q][1] = d.ro.link_coef[b * 3 + 1];
                lco[l][q][2] = d.ro.link_coef[b * 3 + 2];
            } else {
                const int v = u - L;
                int j = 0, q0 = 0;
#pragma unroll
                for (int k = 1; k < NF; k++) if (v >= tpre[k]) { j = k; q0 = tpre[k]; }
                const int q = v - q0;
                const long b = (jt * NF + j) * CAP_UM + q;
                th[j][q] = d.ro.tq_hash[b];
                tco[j][q] = d.ro.tq_coef[b];
            }
        }
    }
    __syncthreads();
    EVP_MARK
    // value slices of every trial: link centres (k, l, e) and torque rows (k, j), monomial order
    auto vterm = [&](double co, int h, int kk) {
        double v = co;
#pragma unroll
        for (int j = 0; j < NF; j++) v = v * ptab[kk][j][(h >> (2 * j)) & 3];
        return v;
    };
    const int nlv = K * NJ * 3, ntv = d.nt ? K * NF : 0;
    for (int u = tid; u < nlv + ntv; u += blockDim.x) {
        if (u < nlv) {
            const int kk = u / (NJ * 3), l = (u / 3) % NJ, e = u % 3;
            const long base = jt * NJ + l;
            double c = d.ro.link_center[base * 3 + e];
            const int cnt = lcnt[l];
            int q = 0;
            for (; q + 4 <= cnt; q += 4) {
                const double v0 = vterm(lco[l][q][e], lh[l][q], kk), v1 = vterm(lco[l][q + 1][e], lh[l][q + 1], kk);
                const double v2 = vterm(lco[l][q + 2][e], lh[l][q + 2], kk), v3 = vterm(lco[l][q + 3][e], lh[l][q + 3], kk);
                c = c + v0; c = c + v1; c = c + v2; c = c + v3;
            }
            for (; q < cnt; q++) c = c + vterm(lco[l][q][e], lh[l][q], kk);
            const double r = d.ro.link_rad[base * 3 + e];
            lck[kk][l][e] = ((c - r) + (c + r)) * 0.5;  // getCenter(Interval(c - r, c + r))
        } else {
            const int v = u - nlv, kk = v / NF, j = v % NF;
            const long base = jt * NF + j;
            double c = d.ro.tq_center[base];
            const int cnt = tcnt[j];
            int q = 0;
            for (; q + 4 <= cnt; q += 4) {
                const double v0 = vterm(tco[j][q], th[j][q], kk), v1 = vterm(tco[j][q + 1], th[j][q + 1], kk);
                const double v2 = vterm(tco[j][q + 2], th[j][q + 2], kk), v3 = vterm(tco[j][q + 3], th[j][q + 3], kk);
                c = c + v0; c = c + v1; c = c + v2; c = c + v3;
            }
            for (; q < cnt; q++) c = c + vterm(tco[j][q], th[j][q], kk);
            const double r = d.ro.tq_rad[base];
            d.gs[((long)i * K + kk) * d.m + (long)t * NF + j] = ((c - r) + (c + r)) * 0.5;
        }
    }
    // extremum rows (NLPclass.cu:319-320, 390-391) and cost (NLPclass.cu:207-267) of every trial:
    // task v = (kind, joint) for v < 2 NF, the cost for v = 2 NF, on blocks t = v (mod T), one lane
    // per trial in the last wave. Each extremum is a chain of dependent fp64 divisions and roots
    // (~0.8 us); spread over blocks, no block's critical path holds more than one (all on block 0
    // they were 14 in a row, about half the launch in the solver's tail).
    for (int v = t; v <= 2 * NF && tid >= (int)blockDim.x - K; v += d.T) {
        const int kk = tid - ((int)blockDim.x - K);
        const double* x = xk[kk];
        double* const Gb = d.gs + ((long)i * K + kk) * d.m;
        const double* q0 = d.q0 + w * NF;
        const double* qd0 = d.qd0 + w * NF;
        const double* qdd0 = d.qdd0 + w * NF;
        const double D = rp.duration;
        if (v < 2 * NF) {
            const long off2 = (long)NF * d.T + (long)d.T * d.NJ * d.O;
            const int kind = v / NF, j = v % NF;
            double mn, mx, e2, e3;
            int mnid, mxid;
            extremum(kind, q0[j], qd0[j] * D, qdd0[j] * D * D, rp.k_range[j] * x[j], &mn, &mx, &mnid, &mxid, &e2, &e3);
            const double scale = kind == 0 ? 1.0 : D;
            const long rmin = off2 + kind * 2 * NF + j;
            Gb[rmin] = mn / scale;
            Gb[rmin + NF] = mx / scale;
            continue;
        }
        const double tp = rp.t_plan;
        double qp[NF];
        for (int j = 0; j < NF; j++) qp[j] = bz_q(q0[j], qd0[j] * D, qdd0[j] * D * D, rp.k_range[j] * x[j], tp);
        double fv = 0.0;
        bool first = true;
        for (int pass = 1; pass >= 0; pass--)
            for (int j = 0; j < NF; j++) {
                if (rp.wrap_mask[j] != pass) continue;
                const double dd = pass ? wrap_to_pi(d.qdes[w * NF + j] - qp[j]) : (d.qdes[w * NF + j] - qp[j]);
                const double term = dd * dd;
                fv = first ? term : fv + term;
                first = false;
            }
        d.fs[(long)i * K + kk] = fv * rp.cost_scale;
    }
    __syncthreads();
    EVP_MARK
    // collision rows of every trial from the plane cache, record-parallel as eval_kernel_t's scan:
    // every thread takes records straight from global memory and forms each trial's two candidates;
    // the (trial, pair) maximum by an LDS atomicMax on an order-preserving key (the value is all a
    // trial needs; a +-0 tie cannot change the line search's terms). Tables in the slicing buffer.
    // (Measured slower: one thread per pair scanning its records, 2x in the solver's tail: a pair's
    // records are a dependent chain of loads on one lane; and each thread reducing four consecutive
    // records before its atomics, strided loads.)
    const unsigned last = NP > 0 ? d.pcoff[jt * NP + NP - 1] : 0u;
    const int total = (int)(last >> 8) + (int)(last & 255);
    const unsigned long long pb = d.pcbase[jt];
    const double* const rec = d.pc + 5 * pb;
    const uint16_t* const pcp = d.pcp + pb;
    const int cap = total;  // the block's [5][n] record arrays
    unsigned long long* const pkey = reinterpret_cast<unsigned long long*>(ubuf);  // [K][NP]
    static_assert(EV_MAXK * MAX_J * MAX_OBS <= UB_FULL, "trial pair table");  // K * NP <= UB_TS: host check
    const double start = -100000000.0;
    for (int u = tid; u < K * NP; u += blockDim.x) pkey[u] = okey(start);
    __syncthreads();
    EVP_MARK
    for (int q = tid; q < total; q += blockDim.x) {
        const double a0 = rec[q], a1 = rec[cap + q], a2 = rec[2 * cap + q];
        const double P = rec[3 * cap + q], N = rec[4 * cap + q];
        const int pr = pcp[q], l = pr / O;
        for (int kk = 0; kk < K; kk++) {
            const double Ac = a0 * lck[kk][l][0] + a1 * lck[kk][l][1] + a2 * lck[kk][l][2];
            const double pos = Ac - P, neg = -Ac - N;
            const double v = (neg > pos || pos != pos) ? neg : pos;
            if (v > start) atomicMax(&pkey[kk * NP + pr], okey(v));
        }
    }
    __syncthreads();
    EVP_MARK
    for (int u = tid; u < K * NP; u += blockDim.x) {
        const int kk = u / NP, pr = u - kk * NP;
        const int l = pr / O, o = pr % O;
        d.gs[((long)i * K + kk) * d.m + nt + ((long)l * d.T + t) * O + o] = -dkey(pkey[u]);
    }
    EVP_PRINT("TR")
}
__global__ __launch_bounds__(EVAL_THREADS) void eval_trials_kernel(NlpDev d) { eval_trials_body<CAP_LM, CAP_UM, UB_FULL>(d); }
// the sync-free tail's single line-search round: all max_ls trials (K = EV_MAXK + 1) of the few
// running worlds, round 0's trial included (ipm_world_Cs_all); K * NJ * O <= UB_FULL (host check)
__global__ __launch_bounds__(EVAL_THREADS) void eval_trials_all(NlpDev d) { eval_trials_body<CAP_LM, CAP_UM, UB_FULL, EV_MAXK + 1>(d); }
// five waves per SIMD (91 VGPRs): six measured slower (5.5 -> 5.7 ms per solve)
__global__ __launch_bounds__(EVAL_THREADS) __attribute__((amdgpu_waves_per_eu(5, 5))) void eval_trials_small(NlpDev d) {
    eval_trials_body<LM_S, UM_S, UB_TS>(d);
}

// ------------------------------------------------------------------------------------------
// armour-IPM
__global__ __launch_bounds__(64) void ipm_world_init(NlpDev d) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= d.W) return;
    WorldState& S = d.ws[w];
    for (int j = 0; j < NF; j++) {
        const double xl = -1.0, xu = 1.0;
        const double p = fmin(d.opt.bound_push * fmax(1.0, fabs(xl)), d.opt.bound_push * (xu - xl));
        S.x[j] = fmin(fmax(0.0, xl + p), xu - p);  // start point x = 0 (NLPclass.cu:193-199)
        S.xt[j] = S.x[j];
        S.dx[j] = 0.0;
    }
    for (int i = 0; i < NF * NF; i++) S.H[i] = (i % (NF + 1) == 0) ? 1.0 : 0.0;
    S.mu = d.opt.mu0;
    S.theta_max = -1;
    S.theta_min = -1;
    S.nfilt = 0;
    S.cur = 0;
    S.status = d.ro.err[w] ? 4 : 0;  // 4: reach set over capacity (planner.hip run_reach), not planned
    d.wl_run[w] = w;                 // the first iteration covers every world
    if (w == 0) { d.cnt[0] = 0; d.cnt[1] = 0; d.cnt[2] = 0; }
    S.searching = 0;
    S.first_update = 1;
    S.nfail = 0;
    S.iter = 0;
    S.nevals = 1;
    S.kkt = 0;
    S.free_mode = d.opt.mu_strategy == 1 ? 1 : 0;
    S.nref = 0;
    S.nresto = 0;
    S.rstall = 0;
    S.rpend = 0;
    S.rphi = -1;
}

__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_init(NlpDev d) {
    const int w = world_of(d, blockIdx.y);  // every world, or the list restarted by a restoration phase
    const WorldState& S = d.ws[w];
    const long r0 = (long)blockIdx.x * d.chunk;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        double a[NF];
        const double v = row_va(d, S.cur, w, (int)r, S.x, a);
        const long i = (long)w * d.R + r;
        double L, U;
        bounds_of(d, w, (int)r, L, U);
        d.L[i] = L;
        d.U[i] = U;
        const bool hl = has_lo(d, L), hh = has_hi(d, U);
        double p = 0;
        if (hl && hh) p = fmin(d.opt.bound_push * fmax(1.0, fabs(L)), d.opt.bound_push * (U - L));
        d.slo[i] = 0; d.zlo[i] = 0; d.shi[i] = 0; d.zhi[i] = 0;
        if (hl) {
            const double pl = hh ? p : d.opt.bound_push * fmax(1.0, fabs(L));
            d.slo[i] = fmax(v - L, pl);
            d.zlo[i] = S.mu / d.slo[i];
        }
        if (hh) {
            const double pu = hl ? p : d.opt.bound_push * fmax(1.0, fabs(U));
            d.shi[i] = fmax(U - v, pu);
            d.zhi[i] = S.mu / d.shi[i];
        }
    }
}

// pass A: residuals, errors, reduced Newton system sums
// pass A's row accumulation (residuals, Newton system) at the current point: value v, gradient a
struct AAcc {
    double rdp[NF], M[28], u1[NF], u2[NF];
    double inf_p, compl0, cm, sumz;
    double sumc, minc;  // sum and minimum of s z over the finite sides (the adaptive barrier's oracle)
    __device__ void zero() {
#pragma unroll
        for (int j = 0; j < NF; j++) { rdp[j] = 0; u1[j] = 0; u2[j] = 0; }
#pragma unroll
        for (int k = 0; k < 28; k++) M[k] = 0;
        inf_p = 0; compl0 = 0; cm = 0; sumz = 0;
        sumc = 0; minc = 1e300;
    }
};
// pass A's row accumulation with the row's slacks and multipliers given (registers)
template <int ML = 0>
__device__ inline __attribute__((always_inline)) void row_A_sz(const NlpDev& d, long i, double v, const double* a, double L,
                                                               double U, double mu, double slo, double zlo, double shi,
                                                               double zhi, AAcc& c, double* ml = nullptr) {
    double wr = 0, sig = 0, c1 = 0, c2 = 0;
    if (has_lo(d, L)) {
        const double s = slo, z = zlo;
        const double rp = (v - L) - s;  // (not stored: pass B forms it again from v and s)
        wr += z;
        c.inf_p = fmax(c.inf_p, fabs(rp));
        c.compl0 = fmax(c.compl0, s * z);
        c.cm = fmax(c.cm, fabs(s * z - mu));
        c.sumz += z;
        c.sumc += s * z;
        c.minc = fmin(c.minc, s * z);
        const double sg = z / s;
        sig += sg;
        c1 += 1.0 / s;
        c2 += sg * rp;
    }
    if (has_hi(d, U)) {
        const double s = shi, z = zhi;
        const double rp = (U - v) - s;
        wr -= z;
        c.inf_p = fmax(c.inf_p, fabs(rp));
        c.compl0 = fmax(c.compl0, s * z);
        c.cm = fmax(c.cm, fabs(s * z - mu));
        c.sumz += z;
        c.sumc += s * z;
        c.minc = fmin(c.minc, s * z);
        const double sg = z / s;
        sig += sg;
        c1 -= 1.0 / s;
        c2 -= sg * rp;
    }
    int k = 0;
#pragma unroll
    for (int p = 0; p < NF; p++) {
        c.rdp[p] += wr * a[p];
        c.u1[p] += a[p] * c1;
        c.u2[p] += a[p] * c2;
#pragma unroll
        for (int q = p; q < NF; q++, k++) {
            if (k < ML) ml[k * ROW_THREADS] += sig * a[p] * a[q];
            else c.M[k] += sig * a[p] * a[q];
        }
    }
}
__device__ inline __attribute__((always_inline)) void row_A(const NlpDev& d, long i, double v, const double* a, double L,
                                                            double U, double mu, AAcc& c) {
    row_A_sz(d, i, v, a, L, U, mu, d.slo[i], d.zlo[i], d.shi[i], d.zhi[i], c);
}
constexpr int NA = 55;  // pass A's partial sums per row block (<= KA)
static_assert(NA <= KA, "pass A partials fit the partial slots");
template <int ML = 0>
__device__ inline void reduce_A(const NlpDev& d, int w, AAcc& c, double* lds, const double* ml = nullptr) {
    double* out = d.partial + ((long)w * d.nblk + blockIdx.x) * KA;
    double v[NA];
    int kinds[NA];
#pragma unroll
    for (int j = 0; j < NF; j++) { v[j] = c.rdp[j]; v[39 + j] = c.u1[j]; v[46 + j] = c.u2[j]; }
    v[7] = c.inf_p; v[8] = c.compl0; v[9] = c.cm; v[10] = c.sumz;
#pragma unroll
    for (int k = 0; k < 28; k++) v[11 + k] = k < ML ? ml[k * ROW_THREADS] : c.M[k];
    v[53] = c.sumc; v[54] = c.minc;
#pragma unroll
    for (int k = 0; k < NA; k++) kinds[k] = (k >= 7 && k <= 9) ? 1 : k == 54 ? 2 : 0;
    block_reduce_n(v, kinds, lds, out);
}
// pass B's multiplier step of one side, dz = mu / s - z - (z / s) ds, exactly as ipm_rows_B forms
// it: pass D forms it again from the same s, z, ds and mu (pass A's barrier update comes after D)
// instead of storing and re-reading it
__device__ inline double dual_step(double mu, double s, double z, double ds) {
    const double sg = z / s;
    return mu / s - z - sg * ds;
}
// pass D's row update (accept the trial: slacks, multipliers) and the BFGS ingredient sum w a
__device__ inline __attribute__((always_inline)) void row_D(const NlpDev& d, long i, const double* a, double L, double U,
                                                            double mu, double ad, double alpha, double* wn) {
    const double ks = d.opt.kappa_sigma;
    double wv = 0;
    if (has_lo(d, L)) {
        const double zn = d.zlo[i] + ad * dual_step(mu, d.slo[i], d.zlo[i], d.dslo[i]);
        wv += zn;
        const double s = d.slo[i] + alpha * d.dslo[i];
        d.slo[i] = s;
        d.zlo[i] = fmin(fmax(zn, mu / (ks * s)), ks * mu / s);
    }
    if (has_hi(d, U)) {
        const double zn = d.zhi[i] + ad * dual_step(mu, d.shi[i], d.zhi[i], d.dshi[i]);
        wv -= zn;
        const double s = d.shi[i] + alpha * d.dshi[i];
        d.shi[i] = s;
        d.zhi[i] = fmin(fmax(zn, mu / (ks * s)), ks * mu / s);
    }
#pragma unroll
    for (int j = 0; j < NF; j++) wn[j] += wv * a[j];
}

__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_A(NlpDev d) {
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (S.status != 0) return;
    __shared__ double lds[(ROW_THREADS / 64) * NA];
    AAcc c;
    c.zero();
    const double mu = S.mu;
    const long r0 = (long)blockIdx.x * d.chunk;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        double a[NF];
        const double v = row_va(d, S.cur, w, (int)r, S.x, a);
        const long i = (long)w * d.R + r;
        double L, U;
        row_bounds(d, i, (int)r, L, U);
        row_A(d, i, v, a, L, U, mu, c);
    }
    reduce_A(d, w, c, lds);
}

// passes D (of the previous iteration) and A (of this one) in one sweep over the rows: the trial
// point D accepts is the point A works at, so each row's value and gradient are read once; the
// arithmetic of ipm_rows_D then ipm_rows_A. D's sums go to partial2, A's to partial.
// ML > 0 (ipm_rows_DA_lds, the wide launches): the first ML of pass A's 28 Newton-matrix
// accumulators live in LDS, one slot per thread, with the same additions in the same order, so the
// kernel holds 166 VGPRs instead of 216 and runs three waves per SIMD instead of two: a 1308-world
// launch 744 -> 651 us, but a small grid's latency 17.2 -> 19.9 us (the slots' LDS round trips), so
// grids below four blocks per CU keep the register form (planner.hip ipm_loop)
constexpr int DA_ML = 20;
template <int ML>
__device__ __attribute__((always_inline)) void rows_DA_body(const NlpDev& d) {
    if (d.lcount && blockIdx.y >= *d.lcount) return;
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (S.status != 0) return;
    __shared__ double lds[(ROW_THREADS / 64) * NA];
    double* ml = nullptr;
    if constexpr (ML > 0) {
        __shared__ double mls[ML * ROW_THREADS];
        ml = mls + threadIdx.x;
#pragma unroll
        for (int k = 0; k < ML; k++) ml[k * ROW_THREADS] = 0.0;
    }
    const double mu = S.mu, ad = S.ad, alpha = S.alpha;
    double wn[NF];
#pragma unroll
    for (int j = 0; j < NF; j++) wn[j] = 0;
    AAcc c;
    c.zero();
    const double ks = d.opt.kappa_sigma;
    const long r0 = (long)blockIdx.x * d.chunk, wb = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        // the row's loads in one batch, then row_D's and row_A's arithmetic on registers (A reads
        // the slacks and multipliers D has just formed)
        const long i = wb + r;
        const RowBounds B(d, i, wb, (int)r);
        const double slo = d.slo[B.lo], zlo = d.zlo[B.lo], dslo = d.dslo[B.lo];
        const double shi = d.shi[i], zhi = d.zhi[i], dshi = d.dshi[i];
        double a[NF];
        const double v = row_va(d, 1 - S.cur, w, (int)r, S.xt, a);
        const double L = B.L(), U = B.U();
        double wv = 0, sl = slo, zl = zlo, sh = shi, zh = zhi;
        if (has_lo(d, L)) {
            const double zn = zlo + ad * dual_step(mu, slo, zlo, dslo);
            wv += zn;
            sl = slo + alpha * dslo;
            zl = fmin(fmax(zn, mu / (ks * sl)), ks * mu / sl);
            d.slo[i] = sl;
            d.zlo[i] = zl;
        }
        if (has_hi(d, U)) {
            const double zn = zhi + ad * dual_step(mu, shi, zhi, dshi);
            wv -= zn;
            sh = shi + alpha * dshi;
            zh = fmin(fmax(zn, mu / (ks * sh)), ks * mu / sh);
            d.shi[i] = sh;
            d.zhi[i] = zh;
        }
#pragma unroll
        for (int j = 0; j < NF; j++) wn[j] += wv * a[j];
        row_A_sz<ML>(d, i, v, a, L, U, mu, sl, zl, sh, zh, c, ml);
        if constexpr (ML > 0) __asm__ volatile("" ::: "memory");  // the slots stay in LDS across rows
    }
    const int kinds[NF] = {};
    block_reduce_n(wn, kinds, lds, d.partial2 + ((long)w * d.nblk + blockIdx.x) * KA2);
    __syncthreads();
    reduce_A<ML>(d, w, c, lds, ml);
}
__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_DA(NlpDev d) { rows_DA_body<0>(d); }
__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_DA_lds(NlpDev d) { rows_DA_body<DA_ML>(d); }

__device__ bool chol_solve7(const double* M, double shift, const double* b, double* x) {
    double L[NF * NF];
    for (int i = 0; i < NF; i++)
        for (int j = 0; j <= i; j++) {
            double s = M[i * NF + j] + (i == j ? shift : 0.0);
            for (int k = 0; k < j; k++) s -= L[i * NF + k] * L[j * NF + k];
            if (i == j) {
                if (!(s > 0)) return false;
                L[i * NF + i] = sqrt(s);
            } else {
                L[i * NF + j] = s / L[j * NF + j];
            }
        }
    double y[NF];
    for (int i = 0; i < NF; i++) {
        double s = b[i];
        for (int k = 0; k < i; k++) s -= L[i * NF + k] * y[k];
        y[i] = s / L[i * NF + i];
    }
    for (int i = NF - 1; i >= 0; i--) {
        double s = y[i];
        for (int k = i + 1; k < NF; k++) s -= L[k * NF + i] * x[k];
        x[i] = s / L[i * NF + i];
    }
    return true;
}

// world w's row-block partials [0, N) combined over the blocks in block order, one lane per value
// (the arithmetic of a serial loop over the blocks), returned wave-uniform. op: 0 sum, 1 max, 2 min
// onto init. The per-world kernels run one wave per world: the nblk dependent load rounds of a
// single thread become one round per lane.
template <int N>
__device__ inline void world_partials_at(const double* base, int nblk, int stride, const double (&init)[N],
                                         const int (&op)[N], double (&P)[N]);
template <int N>
__device__ inline void world_partials(const NlpDev& d, int w, const double (&init)[N], const int (&op)[N], double (&P)[N]) {
    world_partials_at(d.partial + (long)w * d.nblk * KA, d.nblk, KA, init, op, P);
}
template <int N>
__device__ inline void world_partials_at(const double* base, int nblk, int stride, const double (&init)[N],
                                         const int (&op)[N], double (&P)[N]) {
    const int lane = threadIdx.x & 63;
    double s = 0;
    int o = 0;
#pragma unroll
    for (int q = 0; q < N; q++)
        if (q == lane) { s = init[q]; o = op[q]; }
    if (lane < N) {
        // sixteen block partials in flight per step (clamped loads), combined in block order
        const double* in = base + lane;
        for (int b0 = 0; b0 < nblk; b0 += 16) {
            double x[16];
#pragma unroll
            for (int u = 0; u < 16; u++) x[u] = in[(long)min(b0 + u, nblk - 1) * stride];
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (b0 + u < nblk) s = o == 0 ? s + x[u] : o == 1 ? fmax(s, x[u]) : fmin(s, x[u]);
        }
    }
    const uint64_t u = __builtin_bit_cast(uint64_t, s);
#pragma unroll
    for (int q = 0; q < N; q++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, q);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), q);
        P[q] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    }
}

__device__ inline void world_A_body(const NlpDev& d, WorldState& S, int w, int nside);
// The adaptive barrier parameter on a fixed logarithmic grid 2^(j/8) x 2^e (oracle/src/ipm.cpp
// mu_grid, the same constants and comparisons): a rounding-level difference in the complementarity
// sums leaves mu's bits unchanged unless it straddles a midpoint
__device__ inline double mu_grid(double x) {
    constexpr double G[9] = {0x1.0000000000000p+0, 0x1.172b83c7d517bp+0, 0x1.306fe0a31b715p+0,
                             0x1.4bfdad5362a27p+0, 0x1.6a09e667f3bcdp+0, 0x1.8ace5422aa0dbp+0,
                             0x1.ae89f995ad3adp+0, 0x1.d5818dcfba487p+0, 0x1.0000000000000p+1};
    constexpr double B[8] = {0x1.0b5586cf9890fp+0, 0x1.2387a6e756238p+0, 0x1.3dea64c123422p+0,
                             0x1.5ab07dd485429p+0, 0x1.7a11473eb0187p+0, 0x1.9c49182a3f090p+0,
                             0x1.c199bdd85529cp+0, 0x1.ea4afa2a490dap+0};
    if (!(x > 0) || !isfinite(x)) return x;
    int e;
    const double y = 2.0 * frexp(x, &e);
    int j = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) j += y >= B[q];
    double gj = G[0];
#pragma unroll
    for (int q = 1; q < 9; q++) gj = j == q ? G[q] : gj;
    return ldexp(gj, e - 1);
}
// A world kernel (one wave) works on its world's state staged in LDS: one coalesced round trip in
// and one out, where lane 0's steps would otherwise wait on a dependent global load per field. The
// way out is taken only for a world the kernel works on (interior point: status 0 at entry;
// restoration: WS_RESTO): an iteration's list may still name a world whose line search failed after
// the list was formed, and that world's restoration phase can run concurrently on the planner's
// second stream (planner.hip ipm_loop), so a copy of its state taken here must not be written back.
__device__ inline void ws_copy(WorldState& dst, const WorldState& src) {
    static_assert(sizeof(WorldState) % 8 == 0, "WorldState in 8-byte words");
    const uint64_t* s = reinterpret_cast<const uint64_t*>(&src);
    uint64_t* t = reinterpret_cast<uint64_t*>(&dst);
    for (int k = threadIdx.x; k < (int)(sizeof(WorldState) / 8); k += blockDim.x) t[k] = s[k];
}
__global__ __launch_bounds__(64) void ipm_world_A(NlpDev d, int nside) {
    const int w = world_of(d, blockIdx.x);
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == 0;
    world_A_body(d, S, w, nside);
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
}
// pass A's world step: convergence test, barrier update, Newton step; every lane of the wave calls it
__device__ inline void world_A_body(const NlpDev& d, WorldState& S, int w, int nside) {
    if (S.status != 0) return;
    if (S.iter >= d.opt.max_iter) {  // oracle: loop ends without a final check
        if (threadIdx.x == 0) S.status = 2;
        return;
    }
    double P[NA], init[NA];
    int op[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) { init[k] = k == 54 ? 1e300 : 0; op[k] = (k >= 7 && k <= 9) ? 1 : k == 54 ? 2 : 0; }
    world_partials(d, w, init, op, P);
    if (threadIdx.x != 0) return;
    const double* grad = d.grad + ((long)S.cur * d.W + w) * NF;
    double rd[NF], inf_d = 0;
    for (int j = 0; j < NF; j++) { rd[j] = grad[j] - P[j]; inf_d = fmax(inf_d, fabs(rd[j])); }
    const double sd = fmax(d.opt.s_max, P[10] / (double)(nside > 0 ? nside : 1)) / d.opt.s_max;
    const double E0 = fmax(fmax(inf_d / sd, P[7]), P[8] / sd);
    S.kkt = E0;
    if (E0 <= d.opt.tol) { S.status = 1; return; }
    const double Emu = fmax(fmax(inf_d / sd, P[7]), P[9] / sd);
    if (d.opt.mu_strategy == 1) {
        // adaptive barrier (oracle/src/ipm.cpp, same order of decisions): free mode takes mu from
        // the LOQO oracle; the kkt-error globalisation switches to fixed (monotone) mode when E0 has
        // not fallen below 0.9999 x the largest of the last four, back once below the switch value.
        // mu on the 2^(1/8) grid, floor tol / 10
        const double mu_min = d.opt.tol / 10;
        const double avg = P[53] / (double)(nside > 0 ? nside : 1), mn = P[54];
        bool progress = S.nref < 4;
        if (!progress) {
            double mx = 0;
            for (int q = 0; q < 4; q++) mx = fmax(mx, S.kkt_ref[q]);
            progress = E0 <= 0.9999 * mx;
        }
        const double mu_old = S.mu;
        if (S.free_mode && !progress) {
            S.free_mode = 0;
            S.mu = fmax(mu_min, mu_grid(0.8 * avg));
            S.kkt_ref[0] = E0;
            S.nref = 1;
        } else if (!S.free_mode && progress && S.nref >= 1 && E0 <= 0.9999 * S.kkt_ref[S.nref - 1]) {
            S.free_mode = 1;
            S.nref = 0;
        }
        if (S.free_mode) {
            if (S.nref == 4) {
                for (int q = 0; q < 3; q++) S.kkt_ref[q] = S.kkt_ref[q + 1];
                S.kkt_ref[3] = E0;
            } else {
                S.kkt_ref[S.nref++] = E0;
            }
            const double xi = mn / avg;
            const double sg = 0.1 * pow(fmin(0.05 * (1 - xi) / xi, 2.0), 3);
            S.mu = fmax(mu_min, fmin(mu_grid(sg * avg), 1e5));
        } else if (Emu <= d.opt.kappa_eps * S.mu && S.mu > d.opt.tol / 10) {
            S.mu = fmax(d.opt.tol / 10, fmin(d.opt.kappa_mu * S.mu, pow(S.mu, d.opt.theta_mu)));
        }
        if (S.mu != mu_old) S.nfilt = 0;
    } else if (Emu <= d.opt.kappa_eps * S.mu && S.mu > d.opt.tol / 10) {
        S.mu = fmax(d.opt.tol / 10, fmin(d.opt.kappa_mu * S.mu, pow(S.mu, d.opt.theta_mu)));
        S.nfilt = 0;
    }
    double M[NF * NF], rhs[NF];
    int k = 0;
    for (int p = 0; p < NF; p++)
        for (int q = p; q < NF; q++) {
            M[p * NF + q] = S.H[p * NF + q] + P[11 + k];
            M[q * NF + p] = S.H[q * NF + p] + P[11 + k];
            k++;
        }
    for (int j = 0; j < NF; j++) rhs[j] = -grad[j] + S.mu * P[39 + j] - P[46 + j];
    // inertia correction: shift the diagonal until the factorisation succeeds (bounded)
    double shift = 0.0;
    bool ok = false;
    for (int tries = 0; tries < 40 && !ok; tries++) {
        ok = chol_solve7(M, shift, rhs, S.dx);
        shift = (shift == 0.0) ? 1e-8 : shift * 10;
    }
    if (!ok) {
        for (int j = 0; j < NF; j++) S.dx[j] = 0.0;
        S.status = 3;
    }
}

// pass B: step components, fraction to boundary, line-search ingredients. Held to four waves per
// SIMD (128 VGPRs, 2 spilled): 3.66 ms per 327-world solve against 3.95 at three. ipm_rows_DA held
// to three spills 32 registers and slows from 6.5 to 7.9 ms, so it stays at two.
__global__ __launch_bounds__(ROW_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4))) void ipm_rows_B(NlpDev d) {
    if (d.lcount && blockIdx.y >= *d.lcount) return;
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (S.status != 0) return;
    __shared__ double lds[(ROW_THREADS / 64) * NA];
    const double mu = S.mu;
    const double tau = fmax(d.opt.tau_min, 1.0 - mu);
    double ap = 1.0, ad = 1.0, rp1 = 0, bdir = 0, logs = 0, wa[NF], wb[NF];
#pragma unroll
    for (int j = 0; j < NF; j++) { wa[j] = 0; wb[j] = 0; }
    double dx[NF];
#pragma unroll
    for (int j = 0; j < NF; j++) dx[j] = S.dx[j];
    const long r0 = (long)blockIdx.x * d.chunk, w0 = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        const long i = w0 + r;  // the row's loads in one batch (RowBounds)
        const RowBounds B(d, i, w0, (int)r);
        const double slo = d.slo[B.lo], zlo = d.zlo[B.lo];
        const double shi = d.shi[i], zhi = d.zhi[i];
        double a[NF];
        const double v = row_va(d, S.cur, w, (int)r, S.x, a);
        double adx = 0;
#pragma unroll
        for (int j = 0; j < NF; j++) adx += a[j] * dx[j];
        const double L = B.L(), U = B.U();
        // pass A's primal residuals, formed as row_A_sz forms them (same point, slot and slacks)
        // instead of stored there and re-read
        const double rplo = (v - L) - slo, rphi = (U - v) - shi;
        double za = 0, zb = 0;
        if (has_lo(d, L)) {
            const double s = slo, z = zlo, sg = z / s;
            const double ds = adx + rplo;
            const double dz = mu / s - z - sg * ds;  // = dual_step(mu, s, z, ds), formed again by pass D
            d.dslo[i] = ds;
            if (ds < 0) ap = fmin(ap, -tau * s / ds);
            if (dz < 0) ad = fmin(ad, -tau * z / dz);
            rp1 += fabs(rplo); bdir += ds / s; logs += log(s);
            za += z; zb += dz;
        }
        if (has_hi(d, U)) {
            const double s = shi, z = zhi, sg = z / s;
            const double ds = -adx + rphi;
            const double dz = mu / s - z - sg * ds;
            d.dshi[i] = ds;
            if (ds < 0) ap = fmin(ap, -tau * s / ds);
            if (dz < 0) ad = fmin(ad, -tau * z / dz);
            rp1 += fabs(rphi); bdir += ds / s; logs += log(s);
            za -= z; zb -= dz;
        }
#pragma unroll
        for (int j = 0; j < NF; j++) { wa[j] += za * a[j]; wb[j] += zb * a[j]; }
    }
    double* out = d.partial + ((long)w * d.nblk + blockIdx.x) * KA;
    double v[19];
    int kinds[19];
    v[0] = ap; v[1] = ad; v[2] = rp1; v[3] = bdir; v[4] = logs;
#pragma unroll
    for (int j = 0; j < NF; j++) { v[5 + j] = wa[j]; v[12 + j] = wb[j]; }
#pragma unroll
    for (int k = 0; k < 19; k++) kinds[k] = k < 2 ? 2 : 0;
    block_reduce_n(v, kinds, lds, out);
}

// pass B's world step: step sizes, line-search ingredients, the first trial point (every lane of
// the wave calls it; ipm_world_B, or ipm_world_Cs_all in the sync-free tail)
__device__ inline void world_B_body(const NlpDev& d, WorldState& S, int w) {
    if (S.status != 0) return;
    double P[19], init[19];
    int op[19];
#pragma unroll
    for (int k = 0; k < 19; k++) { init[k] = k < 2 ? 1.0 : 0.0; op[k] = k < 2 ? 2 : 0; }
    world_partials(d, w, init, op, P);
    if (threadIdx.x != 0) return;
    const double* grad = d.grad + ((long)S.cur * d.W + w) * NF;
    const double f = d.f[S.cur * d.W + w];
    double gdx = 0;
    for (int j = 0; j < NF; j++) gdx += grad[j] * S.dx[j];
    S.ap = P[0];
    S.ad = P[1];
    S.theta0 = P[2];
    if (S.theta_min < 0) S.theta_min = 1e-4 * fmax(1.0, S.theta0);
    if (S.theta_max < 0) S.theta_max = 1e4 * fmax(1.0, S.theta0);
    S.phi0 = f - S.mu * P[4];
    S.Dphi = gdx - S.mu * P[3];
    S.sw_dphi = S.Dphi < 0 ? pow(-S.Dphi, 2.3) : 0.0;
    S.sw_theta = pow(S.theta0, 1.1);
    for (int j = 0; j < NF; j++) { S.wa_old_a[j] = P[5 + j]; S.wa_old_b[j] = P[12 + j]; }
    S.alpha = S.ap;
    for (int j = 0; j < NF; j++) S.xt[j] = S.x[j] + S.alpha * S.dx[j];
    S.searching = 1;
    S.ls = 0;
    S.ftype = 0;
    S.accepted_ok = 0;
}
__global__ __launch_bounds__(64) void ipm_world_B(NlpDev d) {
    if (d.lcount && blockIdx.x >= *d.lcount) return;
    const int w = world_of(d, blockIdx.x);
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == 0;
    world_B_body(d, S, w);
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
}
// the first trial's step alpha = S.ap as world_B_body forms it: pass B's block partials of the
// primal fraction to the boundary, min onto 1 in block order (world_partials' arithmetic), for the
// tail's trial passes that run before the world step (NlpDev::b_in_cs)
__device__ inline double pass_b_alpha(const NlpDev& d, int w) {
    const double* in = d.partial + (long)w * d.nblk * KA;
    double a = 1.0;
    for (int b0 = 0; b0 < d.nblk; b0 += 16) {
        double x[16];
#pragma unroll
        for (int u = 0; u < 16; u++) x[u] = in[(long)min(b0 + u, d.nblk - 1) * KA];
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (b0 + u < d.nblk) a = fmin(a, x[u]);
    }
    return a;
}

// pass C: barrier objective and constraint violation at the trial point
__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_C(NlpDev d) {
    if (d.lcount && blockIdx.y >= *d.lcount) return;
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (!(S.status == 0 && S.searching)) return;
    __shared__ double lds[(ROW_THREADS / 64) * NA];
    double logt = 0, rpt = 0;
    const double alpha = S.alpha;
    const long r0 = (long)blockIdx.x * d.chunk, wb = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        const long i = wb + r;  // the row's loads in one batch (RowBounds)
        const RowBounds B(d, i, wb, (int)r);
        const double slo = d.slo[B.lo], dslo = d.dslo[B.lo], shi = d.shi[i], dshi = d.dshi[i];
        double a[NF];
        const double v = row_va(d, 1 - S.cur, w, (int)r, S.xt, a);
        const double L = B.L(), U = B.U();
        if (has_lo(d, L)) { const double st = slo + alpha * dslo; logt += log(st); rpt += fabs((v - L) - st); }
        if (has_hi(d, U)) { const double st = shi + alpha * dshi; logt += log(st); rpt += fabs((U - v) - st); }
    }
    double* out = d.partial + ((long)w * d.nblk + blockIdx.x) * KA;
    double v[2] = {logt, rpt};
    const int kinds[2] = {0, 0};
    block_reduce_n(v, kinds, lds, out);
}

__device__ inline void accept_trial(const NlpDev& d, WorldState& S, double logt, double rpt, double ft, bool filt, int w);
// the filter test of a trial (theta_t, phi_t) on a whole wave, one filter entry per lane
// (MAX_FILTER <= 64): acceptable to the filter iff no entry dominates it
__device__ inline bool filter_pass(const WorldState& S, double thetat, double phit) {
    const int q = threadIdx.x & 63;
    const bool fail = q < S.nfilt && !(thetat < S.filt_theta[q] || phit < S.filt_phi[q]);
    return __ballot(fail) == 0;
}
__device__ inline void world_C_body(const NlpDev& d, WorldState& S, int w) {
    if (!(S.status == 0 && S.searching)) return;
    double P[2];
    const double init[2] = {0.0, 0.0};
    const int op[2] = {0, 0};
    world_partials(d, w, init, op, P);
    const double ft = d.f[(1 - S.cur) * d.W + w];
    const bool filt = filter_pass(S, P[1], ft - S.mu * P[0]);
    if (threadIdx.x != 0) return;
    accept_trial(d, S, P[0], P[1], ft, filt, w);
}

// the filter acceptance test of one trial point (barrier terms logt, violation rpt, objective ft);
// on failure the next trial (alpha halved) or, after max_ls trials, the forced last one
__device__ inline void accept_trial(const NlpDev& d, WorldState& S, double logt, double rpt, double ft, bool filt, int w) {
    S.nevals++;
    const double phit = ft - S.mu * logt, thetat = rpt;
    bool ok = thetat <= S.theta_max && filt;  // filt: filter_pass of (thetat, phit)
    bool ftype = false;
    if (ok) {
        const bool switching = S.Dphi < 0 && S.alpha * S.sw_dphi > S.sw_theta;
        if (switching && S.theta0 <= S.theta_min) {
            ok = phit <= S.phi0 + d.opt.eta * S.alpha * S.Dphi;
            ftype = ok;
        } else {
            ok = thetat <= (1 - 1e-5) * S.theta0 || phit <= S.phi0 - 1e-8 * S.theta0;
            if (!ok && switching) { ok = phit <= S.phi0 + d.opt.eta * S.alpha * S.Dphi; ftype = ok; }
        }
    }
    if (ok) {
        S.searching = 0;
        S.accepted_ok = 1;
        if (!ftype && S.nfilt < MAX_FILTER) {
            S.filt_theta[S.nfilt] = (1 - 1e-5) * S.theta0;
            S.filt_phi[S.nfilt] = S.phi0 - 1e-8 * S.theta0;
            S.nfilt++;
        }
        return;
    }
    S.ls++;
    if (S.ls >= d.opt.max_ls) {  // keep the last trial (oracle: accepted = false)
        S.searching = 0;
        S.accepted_ok = 0;
        if (S.nresto < d.opt.resto_max) {
            // the restoration phase instead of the forced step (oracle/src/ipm.cpp 5b; run after the
            // interior-point loop by planner.hip run_resto): the failed iteration counts
            S.status = WS_RESTO;
            S.nresto++;
            S.iter++;
            S.rphi = -1;
            S.rstall = 0;
            S.rpend = 0;
            if (d.rl_app) d.rl_app[atomicAdd(&d.cnt[12], 1u)] = w;  // the loop's phase list
        }
        return;
    }
    S.alpha *= 0.5;
    for (int j = 0; j < NF; j++) S.xt[j] = S.x[j] + S.alpha * S.dx[j];
}

// one line-search round's acceptance test per world, then the compaction bookkeeping: the worlds
// still running (round 0) and still searching are appended to the next lists (their order only
// decides which block serves which world), and the last block to finish publishes both counts to
// the mapped host flags and resets the counters for the next launch.
__global__ __launch_bounds__(64) void ipm_world_C(NlpDev d) {
    const bool valid = !d.lcount || blockIdx.x < *d.lcount;
    const int w = valid ? world_of(d, blockIdx.x) : 0;
    __shared__ WorldState S;
    if (valid) {
        ws_copy(S, d.ws[w]);
        __syncthreads();
        const bool act = S.status == 0;
        world_C_body(d, S, w);
        __syncthreads();
        if (act) ws_copy(d.ws[w], S);
    }
    if (threadIdx.x != 0) return;
    if (valid && S.status == 0) {
        if (d.ls0) d.wl_run[atomicAdd(&d.cnt[0], 1u)] = w;
        if (S.searching) d.wl_search[atomicAdd(&d.cnt[1], 1u)] = w;
    }
    __threadfence();
    if (atomicAdd(&d.cnt[2], 1u) == gridDim.x - 1) {
        __threadfence();
        const unsigned nrun = atomicAdd(&d.cnt[0], 0u), nsearch = atomicAdd(&d.cnt[1], 0u);
        if (d.ls0) d.flags[0] = (int)nrun;
        if (d.ls0 && d.lrun_out) *d.lrun_out = nrun;
        if (d.ls0 && d.nrun_flag) *d.nrun_flag = (int)nrun;
        if (d.ls0 && d.bt_flag) *d.bt_flag = (int)nsearch;
        d.flags[1] = (int)nsearch;
        if (d.lcount_out) *d.lcount_out = nsearch;
        if (d.pend_flag) *d.pend_flag = (int)atomicAdd(&d.cnt[12], 0u);
        d.cnt[0] = 0;
        d.cnt[1] = 0;
        d.cnt[2] = 0;
    }
}

// Speculative line-search round (the tail: few worlds still searching after round 0). Pass C of
// every remaining trial k = 0 .. K-1 (alpha halved k times) of list entry i, blockIdx.y = i * K + k,
// from the trial's own slot; the arithmetic of ipm_rows_C at that trial.
__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_Cs(NlpDev d) {
    const int i = blockIdx.y / d.K, k = blockIdx.y % d.K;
    if (d.lcount && (unsigned)i >= *d.lcount) return;
    const int w = d.wl[i];
    const WorldState& S = d.ws[w];
    if (!(S.status == 0 && (d.b_in_cs || S.searching))) return;
    __shared__ double lds[(ROW_THREADS / 64) * NA];
    double alpha = d.b_in_cs ? pass_b_alpha(d, w) : S.alpha;
    for (int q = 0; q < k; q++) alpha *= 0.5;
    const double* G = d.gs + (long)blockIdx.y * d.m;
    double logt = 0, rpt = 0;
    const long r0 = (long)blockIdx.x * d.chunk, wb = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        const long ii = wb + r;  // the row's loads in one batch (RowBounds)
        const RowBounds B(d, ii, wb, (int)r);
        const double slo = d.slo[B.lo], dslo = d.dslo[B.lo], shi = d.shi[ii], dshi = d.dshi[ii];
        const double v = r < d.m ? G[r] : S.x[r - d.m] + alpha * S.dx[r - d.m];  // box row: the trial's x
        const double L = B.L(), U = B.U();
        if (has_lo(d, L)) { const double st = slo + alpha * dslo; logt += log(st); rpt += fabs((v - L) - st); }
        if (has_hi(d, U)) { const double st = shi + alpha * dshi; logt += log(st); rpt += fabs((U - v) - st); }
    }
    double* out = d.partial_s + ((long)blockIdx.y * d.nblk + blockIdx.x) * KA;
    double v[2] = {logt, rpt};
    const int kinds[2] = {0, 0};
    block_reduce_n(v, kinds, lds, out);
}

// the trials of a speculative round tested in order, exactly as the sequential rounds would
// (ipm_world_C): the first acceptable one ends the search, or the last (forced) one
// list entry blockIdx.x (one wave): every trial's two partial sums at once (lane 2 k + q, block
// partials summed in order as world_partials_at), then the acceptance tests in trial order on lane 0
__device__ inline void world_Cs_body(const NlpDev& d, WorldState& S, int i);
__global__ __launch_bounds__(64) void ipm_world_Cs(NlpDev d) {
    if (d.lcount && blockIdx.x >= *d.lcount) return;
    const int w = d.wl[blockIdx.x];
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == 0;
    world_Cs_body(d, S, blockIdx.x);
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
}
// The tail's whole line search in one round (planner.hip run_solver, sync-free tail): every trial
// k = 0 .. max_ls - 1 of every running world was evaluated values-only (eval_trials_kernel with
// K = max_ls) and summed (ipm_rows_Cs), so this is round 0 and every later round of
// ipm_world_C's sequential search at once: the acceptance tests in trial order (world_Cs_body),
// then round 0's bookkeeping — the worlds still running appended to the next iteration's list, the
// last block publishing the count as ipm_world_C does for ls0. The chosen trial is then evaluated in
// full (eval_kernel_t mode 5).
__global__ __launch_bounds__(64) void ipm_world_Cs_all(NlpDev d) {
    const bool valid = !d.lcount || blockIdx.x < *d.lcount;
    const int w = valid ? d.wl[blockIdx.x] : 0;
    __shared__ WorldState S;
    if (valid) {
        ws_copy(S, d.ws[w]);
        __syncthreads();
        const bool act = S.status == 0;
        if (d.b_in_cs) world_B_body(d, S, w);
        __syncthreads();  // lane 0's WorldState stores before every lane's reads (filter_pass)
        world_Cs_body(d, S, blockIdx.x);
        __syncthreads();
        if (act) ws_copy(d.ws[w], S);
    }
    if (threadIdx.x != 0) return;
    if (valid && S.status == 0) {
        d.wl_run[atomicAdd(&d.cnt[0], 1u)] = w;
        if (S.spec_k > 0) atomicAdd(&d.cnt[1], 1u);  // searched past round 0
    }
    __threadfence();
    if (atomicAdd(&d.cnt[2], 1u) == gridDim.x - 1) {
        __threadfence();
        const unsigned nrun = atomicAdd(&d.cnt[0], 0u), nbt = atomicAdd(&d.cnt[1], 0u);
        d.flags[0] = (int)nrun;
        d.flags[1] = 0;
        if (d.lrun_out) *d.lrun_out = nrun;
        if (d.nrun_flag) *d.nrun_flag = (int)nrun;
        if (d.bt_flag) *d.bt_flag = (int)nbt;
        if (d.pend_flag) *d.pend_flag = (int)atomicAdd(&d.cnt[12], 0u);
        d.cnt[0] = 0;
        d.cnt[1] = 0;
        d.cnt[2] = 0;
    }
}
__device__ inline void world_Cs_body(const NlpDev& d, WorldState& S, int i) {
    const int lane = threadIdx.x & 63;
    double s = 0.0;
    if (lane < 2 * d.K) {
        const double* in = d.partial_s + ((long)i * d.K + (lane >> 1)) * d.nblk * KA + (lane & 1);
        const int nb = d.nblk;
        for (int b0 = 0; b0 < nb; b0 += 16) {
            double x[16];
#pragma unroll
            for (int u = 0; u < 16; u++) x[u] = in[(long)min(b0 + u, nb - 1) * KA];
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (b0 + u < nb) s = s + x[u];
        }
    }
    const uint64_t u = __builtin_bit_cast(uint64_t, s);
    // the trials' objective values, one per lane in a single load round (a load per trial inside
    // the loop below waited a memory latency per trial)
    const uint64_t uf = __builtin_bit_cast(uint64_t, lane < d.K ? d.fs[(long)i * d.K + lane] : 0.0);
    int chosen = -1;
    const double mu = S.mu;
    for (int k = 0; k < d.K; k++) {
        const uint32_t lo0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 2 * k);
        const uint32_t hi0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 2 * k);
        const uint32_t lo1 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 2 * k + 1);
        const uint32_t hi1 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 2 * k + 1);
        const uint32_t lof = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)uf, k);
        const uint32_t hif = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uf >> 32), k);
        const double logt = __builtin_bit_cast(double, ((uint64_t)hi0 << 32) | lo0);
        const double rpt = __builtin_bit_cast(double, ((uint64_t)hi1 << 32) | lo1);
        const double ft = __builtin_bit_cast(double, ((uint64_t)hif << 32) | lof);
        // (the filter does not change while a search goes on: an acceptance ends it)
        const bool filt = filter_pass(S, rpt, ft - mu * logt);
        if (threadIdx.x == 0 && chosen == k - 1 && S.status == 0 && S.searching) {
            accept_trial(d, S, logt, rpt, ft, filt, d.wl[i]);
            chosen = k;
        }
    }
    if (threadIdx.x == 0) S.spec_k = chosen;
}

// pass D: accept the trial point — slacks, multipliers, BFGS ingredients
__global__ __launch_bounds__(ROW_THREADS) void ipm_rows_D(NlpDev d) {
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (S.status != 0) return;
    __shared__ double lds[(ROW_THREADS / 64) * NA];
    const double mu = S.mu, ad = S.ad, alpha = S.alpha;
    double wn[NF];
#pragma unroll
    for (int j = 0; j < NF; j++) wn[j] = 0;
    const long r0 = (long)blockIdx.x * d.chunk;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.R; r += blockDim.x) {
        double a[NF];
        row_va(d, 1 - S.cur, w, (int)r, S.xt, a);
        const long i = (long)w * d.R + r;
        double L, U;
        row_bounds(d, i, (int)r, L, U);
        row_D(d, i, a, L, U, mu, ad, alpha, wn);
    }
    double* out = d.partial2 + ((long)w * d.nblk + blockIdx.x) * KA2;
    const int kinds[NF] = {};
    block_reduce_n(wn, kinds, lds, out);
}

// pass D's world step: BFGS update, accept the trial point; every lane of the wave calls it. The
// vectors and scalars are formed by every lane alike (the same arithmetic in the same order, so the
// same values on every lane, at the cost of one lane), and lane l < 49 updates H's element l: the
// update's 98 divisions run side by side instead of one after another on lane 0. Within the one
// wave, every lane's reads of H precede the first write in program order.
__device__ inline void world_D_body(const NlpDev& d, WorldState& S, int w) {
    if (S.status != 0) return;
    double wn[NF];
    const double init[NF] = {};
    const int op[NF] = {};
    world_partials_at(d.partial2 + (long)w * d.nblk * KA2, d.nblk, KA2, init, op, wn);
    const int lane = threadIdx.x;
    const double* grad = d.grad + ((long)S.cur * d.W + w) * NF;
    const double* gradt = d.grad + ((long)(1 - S.cur) * d.W + w) * NF;
    double sv[NF], y[NF], Hs[NF], ss = 0, sy = 0;
    for (int j = 0; j < NF; j++) {
        sv[j] = S.xt[j] - S.x[j];
        const double wo = S.wa_old_a[j] + S.ad * S.wa_old_b[j];
        y[j] = (gradt[j] - grad[j]) - (wn[j] - wo);
        ss += sv[j] * sv[j];
    }
    for (int j = 0; j < NF; j++) sy += sv[j] * y[j];
    double Hm[NF * NF];
#pragma unroll
    for (int e = 0; e < NF * NF; e++) Hm[e] = S.H[e];
    const bool first = S.first_update && sy > 0 && ss > 1e-20;
    if (first) {
        double yy = 0;
        for (int j = 0; j < NF; j++) yy += y[j] * y[j];
        const double sc = yy / sy;
#pragma unroll
        for (int e = 0; e < NF * NF; e++) Hm[e] = (e % (NF + 1) == 0) ? sc : 0.0;
    }
    double sHs = 0;
#pragma unroll
    for (int i = 0; i < NF; i++) {
        Hs[i] = 0;
#pragma unroll
        for (int j = 0; j < NF; j++) Hs[i] += Hm[i * NF + j] * sv[j];
        sHs += sv[i] * Hs[i];
    }
    // this lane's element (row li, column lj) and its current value
    const int le = lane < NF * NF ? lane : 0, li = le / NF, lj = le % NF;
    double h = 0, Hsi = 0, Hsj = 0;
#pragma unroll
    for (int e = 0; e < NF * NF; e++) h = e == le ? Hm[e] : h;
#pragma unroll
    for (int q = 0; q < NF; q++) {
        Hsi = q == li ? Hs[q] : Hsi;
        Hsj = q == lj ? Hs[q] : Hsj;
    }
    if (ss > 1e-20 && sHs > 1e-20) {
        const double theta = (sy >= 0.2 * sHs) ? 1.0 : 0.8 * sHs / (sHs - sy);
        double rv[NF], sr = 0;
        for (int j = 0; j < NF; j++) { rv[j] = theta * y[j] + (1 - theta) * Hs[j]; sr += sv[j] * rv[j]; }
        if (sr > 1e-20) {
            double rvi = 0, rvj = 0;
#pragma unroll
            for (int q = 0; q < NF; q++) {
                rvi = q == li ? rv[q] : rvi;
                rvj = q == lj ? rv[q] : rvj;
            }
            h += -Hsi * Hsj / sHs + rvi * rvj / sr;
        }
    }
    if (lane < NF * NF) S.H[lane] = h;
    if (lane != 0) return;
    if (first) S.first_update = 0;
    for (int j = 0; j < NF; j++) S.x[j] = S.xt[j];
    S.cur = 1 - S.cur;
    S.nfail = S.accepted_ok ? 0 : S.nfail + 1;
    S.iter++;
    if (S.nfail >= 3) S.status = 3;
}
__global__ __launch_bounds__(64) void ipm_world_D(NlpDev d) {
    const int w = world_of(d, blockIdx.x);
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == 0;
    world_D_body(d, S, w);
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
}
// the fused passes' world step: D's (of the previous iteration), then A's, one wave
__global__ __launch_bounds__(64) void ipm_world_DA(NlpDev d, int nside) {
    if (d.lcount && blockIdx.x >= *d.lcount) return;
    const int w = world_of(d, blockIdx.x);
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == 0;
    world_D_body(d, S, w);
    __syncthreads();  // lane 0's WorldState stores before every lane's reads in world_A_body
    world_A_body(d, S, w, nside);
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
}

// ------------------------------------------------------------------------------------------
// Restoration phase (oracle/src/ipm.cpp restoration). A world whose line search
// finds no acceptable trial (accept_trial) leaves the interior-point loop with status WS_RESTO;
// planner.hip run_resto then takes all of them together, one iteration per round of launches:
//   resto_rows_G / resto_world_G  the Gauss-Newton system of Phi at the current point, the
//                                 decisions (every row within its bounds -> restart; the cap;
//                                 stall) and the step with its largest fraction to the box;
//   eval (mode 1) / resto_rows_V / resto_world_V  one Armijo trial per round, alpha halved, at
//                                 most max_ls rounds (the oracle's sequential search).
// The restarted worlds go back to the interior point (ipm_rows_init on their list, then the loop).
constexpr int NRG = 37;  // pass G's partial sums: M (28, upper triangle), b (7), sum e^2, max original violation

// the violation of one row against targets delta inside its bounds (e, and sg = -1 below the lower
// target / +1 above the upper one) and against the bounds themselves (e0): ipm.cpp's expressions
__device__ inline void resto_row(const NlpDev& d, double v, double L, double U, double& e, double& sg, double& e0) {
    const double delta = d.opt.resto_delta;
    e = 0; sg = 0; e0 = 0;
    if (has_lo(d, L)) {
        e0 = fmax(e0, L - v);
        const double el = (L + delta) - v;
        if (el > 0) { e = el; sg = -1.0; }
    }
    if (has_hi(d, U)) {
        e0 = fmax(e0, v - U);
        const double eh = v - (U - delta);
        if (e == 0 && eh > 0) { e = eh; sg = 1.0; }
    }
}
__device__ inline double resto_barrier(const NlpDev& d, const double* x) {
    double b = 0;
    for (int j = 0; j < NF; j++) b += -log(1.0 - x[j]) - log(1.0 + x[j]);
    return d.opt.resto_mu * b;
}

__global__ __launch_bounds__(ROW_THREADS) void resto_rows_G(NlpDev d) {
    if (d.lcount && blockIdx.y >= *d.lcount) return;
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (S.status != WS_RESTO) return;
    __shared__ double lds[(ROW_THREADS / 64) * NRG];
    const int slot = S.rpend ? 1 - S.cur : S.cur;  // a step chosen last iteration: its evaluation
    double M[28], b[NF], V = 0, e0m = 0;
#pragma unroll
    for (int k = 0; k < 28; k++) M[k] = 0;
#pragma unroll
    for (int j = 0; j < NF; j++) b[j] = 0;
    const long r0 = (long)blockIdx.x * d.chunk, wb = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.m; r += blockDim.x) {
        const long i = wb + r;
        const RowBounds B(d, i, wb, (int)r);
        double a[NF];
        const double v = row_va(d, slot, w, (int)r, S.x, a);
        double e, sg, e0;
        resto_row(d, v, B.L(), B.U(), e, sg, e0);
        e0m = fmax(e0m, e0);
        if (e > 0) {
            V += e * e;
            const double es = e * sg;
            int k = 0;
#pragma unroll
            for (int p = 0; p < NF; p++) {
                b[p] += es * a[p];
#pragma unroll
                for (int q = p; q < NF; q++) M[k++] += a[p] * a[q];
            }
        }
    }
    double v[NRG];
    int kinds[NRG];
#pragma unroll
    for (int k = 0; k < 28; k++) v[k] = M[k];
#pragma unroll
    for (int j = 0; j < NF; j++) v[28 + j] = b[j];
    v[35] = V;
    v[36] = e0m;
#pragma unroll
    for (int k = 0; k < NRG; k++) kinds[k] = k == 36 ? 1 : 0;
    block_reduce_n(v, kinds, lds, d.partial + ((long)w * d.nblk + blockIdx.x) * KA);
}

// a restoration phase that reached a point within every bound hands the world back to the
// interior point: a fresh filter and BFGS matrix at the current mu (slacks: ipm_rows_init)
__device__ inline void resto_restart(const NlpDev& d, WorldState& S) {
    S.status = WS_RESTART;  // running again once run_solver has set its slacks (ipm_collect)
    for (int i = 0; i < NF * NF; i++) S.H[i] = (i % (NF + 1) == 0) ? 1.0 : 0.0;
    S.first_update = 1;
    S.nfilt = 0;
    S.theta_max = -1;
    S.theta_min = -1;
    S.nfail = 0;
    S.free_mode = d.opt.mu_strategy == 1 ? 1 : 0;
    S.nref = 0;
    S.searching = 0;
    S.spec_k = -1;
}

// pass G's world step (lane 0 after the partials): ipm.cpp restoration's order of decisions
__device__ inline void resto_step(const NlpDev& d, WorldState& S, const double (&P)[NRG]) {
    if (P[36] <= 0) { resto_restart(d, S); return; }
    if (S.iter >= d.opt.max_iter) { S.status = 2; return; }
    const double V = P[35];
    const double phi = 0.5 * V + resto_barrier(d, S.x);
    if (S.rphi >= 0) {
        S.rstall = (S.rphi - phi <= d.opt.resto_stall * S.rphi) ? S.rstall + 1 : 0;
        if (S.rstall >= 2) { S.status = 5; return; }
    }
    S.rphi = phi;
    double A[NF * NF], rhs[NF], gp[NF], dx[NF];
    int k = 0;
    for (int p = 0; p < NF; p++)
        for (int q = p; q < NF; q++) {
            A[p * NF + q] = P[k];
            A[q * NF + p] = P[k];
            k++;
        }
    double dmax = 0;
    for (int j = 0; j < NF; j++) dmax = fmax(dmax, A[j * NF + j]);
    const double lam = 1e-2 * fmin(1.0, sqrt(V)) * (1.0 + dmax);
    const double mr = d.opt.resto_mu;
    for (int j = 0; j < NF; j++) {
        const double u = 1.0 - S.x[j], l = 1.0 + S.x[j];
        gp[j] = P[28 + j] + mr * (1.0 / u - 1.0 / l);
        A[j * NF + j] += mr * (1.0 / (u * u) + 1.0 / (l * l)) + lam;
        rhs[j] = -gp[j];
    }
    double shift = 0.0;
    bool ok = false;
    for (int tries = 0; tries < 40 && !ok; tries++) {
        ok = chol_solve7(A, shift, rhs, dx);
        shift = (shift == 0.0) ? 1e-8 : shift * 10;
    }
    if (!ok) { S.status = 5; return; }
    double amax = 1.0, dphi = 0;
    for (int j = 0; j < NF; j++) {
        if (dx[j] > 0) amax = fmin(amax, d.opt.tau_min * (1.0 - S.x[j]) / dx[j]);
        if (dx[j] < 0) amax = fmin(amax, d.opt.tau_min * (-1.0 - S.x[j]) / dx[j]);
        dphi += gp[j] * dx[j];
    }
    for (int j = 0; j < NF; j++) {
        S.dx[j] = dx[j];
        S.xt[j] = S.x[j] + amax * dx[j];
    }
    S.alpha = amax;
    S.phi0 = phi;
    S.Dphi = dphi;
    S.searching = 1;
    S.ls = 0;
}

// the last block of a restoration launch publishes a count (worlds still in the phase / still
// searching) into the mapped host flags and resets the ticket counters
__device__ inline void resto_count(const NlpDev& d, bool mine, int flag) {
    if (mine) atomicAdd(&d.cnt[0], 1u);
    __threadfence();
    if (atomicAdd(&d.cnt[2], 1u) == gridDim.x - 1) {
        __threadfence();
        d.flags[flag] = (int)atomicAdd(&d.cnt[0], 0u);
        d.cnt[0] = 0;
        d.cnt[2] = 0;
    }
}

__global__ __launch_bounds__(64) void resto_world_G(NlpDev d) {
    if (d.lcount && blockIdx.x >= *d.lcount) return;  // (one-round search: no count published)
    const int w = world_of(d, blockIdx.x);
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == WS_RESTO;
    if (act) {
        double P[NRG], init[NRG];
        int op[NRG];
#pragma unroll
        for (int k = 0; k < NRG; k++) { init[k] = 0; op[k] = k == 36 ? 1 : 0; }
        world_partials(d, w, init, op, P);
        if (threadIdx.x == 0) {
            if (S.rpend) {  // the step chosen last iteration, evaluated in the trial slot
                for (int j = 0; j < NF; j++) S.x[j] = S.xt[j];
                S.cur = 1 - S.cur;
                S.iter++;
                S.rpend = 0;
            }
            resto_step(d, S, P);
        }
    }
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
    if (threadIdx.x == 0 && d.rflag >= 0) resto_count(d, S.status == WS_RESTO, d.rflag);
}

// sum e^2 at the trial point (the trial slot's full evaluation, mode 1)
__global__ __launch_bounds__(ROW_THREADS) void resto_rows_V(NlpDev d) {
    const int w = world_of(d, blockIdx.y);
    const WorldState& S = d.ws[w];
    if (!(S.status == WS_RESTO && S.searching)) return;
    __shared__ double lds[(ROW_THREADS / 64) * NRG];
    const int slot = 1 - S.cur;
    double V = 0;
    const long r0 = (long)blockIdx.x * d.chunk, wb = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.m; r += blockDim.x) {
        const long i = wb + r;
        const RowBounds B(d, i, wb, (int)r);
        const double v = d.g[gidx(d, slot, w, r)];
        double e, sg, e0;
        resto_row(d, v, B.L(), B.U(), e, sg, e0);
        V += e * e;
    }
    double vv[1] = {V};
    const int kinds[1] = {0};
    block_reduce_n(vv, kinds, lds, d.partial + ((long)w * d.nblk + blockIdx.x) * KA);
}

// the Armijo test of the round's trial; a rejected trial halves alpha (max_ls trials, then the
// phase fails: local infeasibility at the current point)
__global__ __launch_bounds__(64) void resto_world_V(NlpDev d) {
    const int w = world_of(d, blockIdx.x);
    __shared__ WorldState S;
    ws_copy(S, d.ws[w]);
    __syncthreads();
    const bool act = S.status == WS_RESTO;
    if (act && S.searching) {
        double P[1];
        const double init[1] = {0.0};
        const int op[1] = {0};
        world_partials(d, w, init, op, P);
        if (threadIdx.x == 0) {
            S.nevals++;
            const double phit = 0.5 * P[0] + resto_barrier(d, S.xt);
            if (phit <= S.phi0 + d.opt.eta * S.alpha * S.Dphi) {
                S.searching = 0;
                S.rpend = 1;
            } else if (++S.ls >= d.opt.max_ls) {
                S.searching = 0;
                S.status = 5;
            } else {
                S.alpha *= 0.5;
                for (int j = 0; j < NF; j++) S.xt[j] = S.x[j] + S.alpha * S.dx[j];
            }
        }
    }
    __syncthreads();
    if (act) ws_copy(d.ws[w], S);
    if (threadIdx.x == 0) resto_count(d, S.status == WS_RESTO && S.searching, 1);
}

// The phase's Armijo search in one round (planner.hip run_resto, when the speculative machinery is
// there): the values of all max_ls trials (eval_trials_all, d.resto) summed per trial
// (resto_rows_Vs, list entry i and trial k at blockIdx.y = i K + k, the rows and partial sums of
// resto_rows_V), the tests in trial order (resto_world_Vs), then the chosen trial in full (eval
// mode 5, d.resto). The decisions and the chosen point are those of the sequential rounds.
__global__ __launch_bounds__(ROW_THREADS) void resto_rows_Vs(NlpDev d) {
    const int i = blockIdx.y / d.K;
    if (d.lcount && (unsigned)i >= *d.lcount) return;
    const int w = d.wl[i];
    const WorldState& S = d.ws[w];
    if (!(S.status == WS_RESTO && S.searching)) return;
    __shared__ double lds[(ROW_THREADS / 64) * NRG];
    const double* G = d.gs + (long)blockIdx.y * d.m;
    double V = 0;
    const long r0 = (long)blockIdx.x * d.chunk, wb = (long)w * d.R;
    for (long r = r0 + threadIdx.x; r < r0 + d.chunk && r < d.m; r += blockDim.x) {
        const long ii = wb + r;
        const RowBounds B(d, ii, wb, (int)r);
        double e, sg, e0;
        resto_row(d, G[r], B.L(), B.U(), e, sg, e0);
        V += e * e;
    }
    double vv[1] = {V};
    const int kinds[1] = {0};
    block_reduce_n(vv, kinds, lds, d.partial_s + ((long)blockIdx.y * d.nblk + blockIdx.x) * KA);
}
// ... and the list compaction of the one-round iterations: the worlds still in the phase go to the
// next iteration's list (wl_run), whose length the last block stores for the next launches (lrun_out,
// device) and for the host (nrun_flag, mapped; read one iteration late)
__global__ __launch_bounds__(64) void resto_world_Vs(NlpDev d) {
    const bool valid = !d.lcount || blockIdx.x < *d.lcount;
    const int i = blockIdx.x, w = valid ? d.wl[i] : 0;
    __shared__ WorldState S;
    bool act = false;
    if (valid) {
        ws_copy(S, d.ws[w]);
        __syncthreads();
        act = S.status == WS_RESTO;
    }
    if (act && S.searching) {
        // trial k's sum on lane k, its blocks combined in order (world_partials_at's arithmetic)
        const int lane = threadIdx.x & 63;
        double v = 0.0;
        if (lane < d.K) {
            const double* in = d.partial_s + ((long)i * d.K + lane) * d.nblk * KA;
            for (int b0 = 0; b0 < d.nblk; b0 += 16) {
                double xb[16];
#pragma unroll
                for (int u = 0; u < 16; u++) xb[u] = in[(long)min(b0 + u, d.nblk - 1) * KA];
#pragma unroll
                for (int u = 0; u < 16; u++)
                    if (b0 + u < d.nblk) v = v + xb[u];
            }
        }
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        for (int k = 0; k < d.K; k++) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
            const double Vk = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
            if (threadIdx.x == 0 && S.searching) {
                // resto_world_V's test of trial k (S.xt, S.alpha are trial k's)
                S.nevals++;
                const double phit = 0.5 * Vk + resto_barrier(d, S.xt);
                if (phit <= S.phi0 + d.opt.eta * S.alpha * S.Dphi) {
                    S.searching = 0;
                    S.rpend = 1;
                } else if (++S.ls >= d.opt.max_ls) {
                    S.searching = 0;
                    S.status = 5;
                } else {
                    S.alpha *= 0.5;
                    for (int j = 0; j < NF; j++) S.xt[j] = S.x[j] + S.alpha * S.dx[j];
                }
            }
        }
    }
    if (valid) {
        __syncthreads();
        if (act) ws_copy(d.ws[w], S);
    }
    if (threadIdx.x != 0) return;
    if (d.rl_app) {  // inside the interior-point loop: the phase list, published by resto_publish
        if (valid && S.status == WS_RESTO) d.rl_app[atomicAdd(&d.cnt[12], 1u)] = w;
        return;
    }
    if (valid && S.status == WS_RESTO) d.wl_run[atomicAdd(&d.cnt[0], 1u)] = w;
    __threadfence();
    if (atomicAdd(&d.cnt[2], 1u) == gridDim.x - 1) {
        __threadfence();
        const unsigned n = atomicAdd(&d.cnt[0], 0u);
        *d.lrun_out = n;
        *d.nrun_flag = (int)n;
        d.cnt[0] = 0;
        d.cnt[2] = 0;
    }
}

// the phase list of the next phase iteration: the worlds appended since the last publish (failed
// line searches, and the worlds the last phase iteration kept) moved from the append list `src` to
// `dst`, its length into cnt[14] (the phase launches' lcount) and, for the host, into the mapped
// flag `pflag` (null: none); the append list starts empty again
__global__ __launch_bounds__(256) void resto_publish(NlpDev d, const int* src, int* dst, int* pflag) {
    __shared__ unsigned n;
    if (threadIdx.x == 0) n = atomicAdd(&d.cnt[12], 0u);
    __syncthreads();
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        d.cnt[14] = n;
        d.cnt[12] = 0;
        if (pflag) *pflag = (int)n;
    }
}

// the worlds of list `in` (n entries; null: worlds 0..n-1) with status `st`, into `out`; the count
// into the mapped host flag `flag` (one block)
// (set >= 0: the collected worlds' new status)
__global__ __launch_bounds__(1024) void ipm_collect(NlpDev d, const int* in, int n, int st, int* out, int flag, int set) {
    __shared__ unsigned c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int w = in ? in[i] : i;
        if (d.ws[w].status == st) {
            out[atomicAdd(&c, 1u)] = w;
            if (set >= 0) d.ws[w].status = set;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) d.flags[flag] = (int)c;
}

// finalize_solution's feasibility re-check (NLPclass.cu:449-538): one block per world
__global__ void feasible_kernel(NlpDev d, int* feasible) {
    const int w = blockIdx.x;
    const WorldState& S = d.ws[w];
    const RobotParams& rp = *d.rp;
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const int nt = d.nt, nc = d.T * d.NJ * d.O;
    // ARMTD's re-check covers the collision rows of links 0 .. NF-2 only (ACMP/NLPclass.cu:375)
    const int nc_checked = d.armtd ? d.T * (NF - 1) * d.O : nc;
    for (int r = threadIdx.x; r < d.m; r += blockDim.x) {
        const double v = d.g[gidx(d, S.cur, w, r)];
        const long i = (long)w * d.R + r;
        bool b;
        if (r < nt) b = v < d.L[i] - rp.torque_violation || v > d.U[i] + rp.torque_violation;
        else if (r < nt + nc) b = r < nt + nc_checked && v > rp.collision_violation;
        else b = v < d.L[i] || v > d.U[i];
        if (b) atomicOr(&bad, 1);
    }
    const long n = (long)d.T * d.NJ * 3;
    const double* src = d.link_c + S.cur * d.lcs + w * n;
    double* dst = d.link_c + 2 * d.lcs + w * n;
    for (long i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    if (threadIdx.x == 0) feasible[w] = (bad || S.status == 4) ? 0 : 1;
}

}  // namespace armour
