// armour-mi355x — workgroup-cooperative sparse polynomial-zonotope (PZ) engine for gfx950.
//
// Semantics are those of the reference's PZsparse (KPR/PZsparse.cu:284-1167): monomials carry a
// 63-bit degree hash, products add hashes without carry, and every operator ends in simplify():
// merge equal hashes, prune merged coefficients whose Frobenius norm is <= SIMPLIFY_THRESHOLD
// into the interval part `independent`. The data layout is MI355X-first:
//   * a PZ is a handle (dims, centre, independent part) in LDS plus a structure-of-arrays run of
//     monomials (hash[], coefficient block[]) in a per-workgroup HBM arena (bump allocated);
//   * element extraction, scaling by a constant and negation are lazy views on a parent's
//     monomials (no copies) — the reader applies s*c exactly as the reference's materialised copy;
//   * simplify() is a bitonic sort of (hash, term-index) keys in LDS, a segmented group sum in
//     term order, a norm test, and a block-wide scan/compaction into the arena;
//   * every PZ carries TWO independent parts (nominal / interval inertial parameters). The
//     reference runs RNEA twice (armour_main.cu:129,132) with identical centres and monomials —
//     only `independent` differs — so one pass with dual independent parts replaces both.
// Operators stage their operand handles in dedicated LDS slots (opa/opb/opc) so that an output
// may alias an input; coefficient blocks are fixed 9-element register arrays with unrolled loops.
// The group abstraction (Grp) lets the same code run as a sequential host emulation in tests.
#pragma once
#include "common.h"

#define ADN __host__ __device__ __attribute__((noinline))
#define UNR _Pragma("unroll")

namespace armour {

struct Grp {
    int tid, n;
    AD void sync() const {
#if defined(__HIP_DEVICE_COMPILE__)
        __syncthreads();
#endif
    }
};

// PZ handle. Views: comp >= 0 selects one element of the parent's coefficient block (the
// reference's operator()(r,c), PZsparse.cu:678-697); scaled applies s * c on read (PZ * double,
// :996-1030); neg applies -c on read (the second operand of operator-, :813-834).
struct PZH {
    int R, C;
    int cnt;
    int stride;
    long hoff, coff;
    int comp;
    int scaled;
    int neg;
    int pad_;
    double scale;
    double center[9];
    double ind[2][9];
};

struct Arena {
    uint64_t* h;
    double* c;
    long hcap, ccap;
    long hused, cused;
};

struct Ctx {
    Grp g;
    PZH* H;            // handle table (LDS)
    int opa, opb, opc; // operand staging slots in H
    Arena* A;          // bump arena state (LDS), storage in HBM
    uint64_t* kh;      // sort keys: hash        (LDS, cap_lds entries)
    uint32_t* ki;      // sort keys: term index
    int* kp;           // keep flags / scan
    int cap_lds;
    uint64_t* gkh;     // global fallback for large sorts
    uint32_t* gki;
    int* gkp;
    int cap_glb;
    double* red;       // reduction scratch (LDS): [waves * 9] on device, [n * 9] in the emulation
    int* iscan;        // [2 * n] scan scratch (LDS)
    int* err;          // error word (LDS)
    double thr;
};

enum : int { ERR_ARENA = 1, ERR_SORTCAP = 2, ERR_LINKGEN = 4, ERR_OUTCAP = 8, ERR_HANDLES = 16 };

// ---------------------------------------------------------------------------------------------
// scalar helpers (fixed 9-element blocks, unrolled so blocks stay in registers)
template <int N>
AD double frob_norm_n(const double* x) {
    // Eigen 3.3 MatrixXd::norm(): packet-of-2 redux order (same as oracle/src/pz.cpp)
    if (N == 1) return sqrt(x[0] * x[0]);
    if (N == 3) return sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
    const double s0 = x[0] * x[0], s1 = x[1] * x[1], s2 = x[2] * x[2], s3 = x[3] * x[3], s4 = x[4] * x[4];
    const double s5 = x[5] * x[5], s6 = x[6] * x[6], s7 = x[7] * x[7], s8 = x[8] * x[8];
    return sqrt((((s0 + s4) + (s2 + s6)) + ((s1 + s5) + (s3 + s7))) + s8);
}
AD double frob_norm(const double* x, int n) {
    return n == 1 ? frob_norm_n<1>(x) : n == 3 ? frob_norm_n<3>(x) : frob_norm_n<9>(x);
}

// column-major coefficient-based product, inner index summed in order; dims in {1,3}
AD void matmul(const double* A, int ra, int ca, const double* B, int cb, double* out) {
    if (ra == 3 && ca == 3 && cb == 1) {
        double t[3];
        UNR for (int i = 0; i < 3; i++) t[i] = (A[i] * B[0] + A[i + 3] * B[1]) + A[i + 6] * B[2];
        UNR for (int i = 0; i < 3; i++) out[i] = t[i];
    } else if (ra == 3 && ca == 3 && cb == 3) {
        double t[9];
        UNR for (int j = 0; j < 3; j++)
            UNR for (int i = 0; i < 3; i++) t[i + 3 * j] = (A[i] * B[3 * j] + A[i + 3] * B[3 * j + 1]) + A[i + 6] * B[3 * j + 2];
        UNR for (int e = 0; e < 9; e++) out[e] = t[e];
    } else {
        double t[9];
        for (int j = 0; j < cb; j++)
            for (int i = 0; i < ra; i++) {
                double acc = A[i] * B[j * ca];
                for (int k = 1; k < ca; k++) acc = acc + A[i + k * ra] * B[k + j * ca];
                t[i + j * ra] = acc;
            }
        for (int e = 0; e < ra * cb; e++) out[e] = t[e];
    }
}

AD int nel(const PZH& h) { return h.R * h.C; }

// read monomial k of handle h into a 9-block (entries >= nel(h) are zero)
AD void read_mono(const Ctx& x, const PZH& h, int k, double* out) {
    const double* base = x.A->c + h.coff + (long)k * h.stride;
    const int n = nel(h);
    UNR for (int e = 0; e < 9; e++) {
        double v = 0.0;
        if (e < n) {
            v = base[h.comp >= 0 ? h.comp : e];
            if (h.scaled) v = h.scale * v;
            if (h.neg) v = -v;
        }
        out[e] = v;
    }
}
AD uint64_t mono_hash(const Ctx& x, const PZH& h, int k) { return x.A->h[h.hoff + k]; }

// ---------------------------------------------------------------------------------------------
// block primitives
AD void block_sum9(const Ctx& x, double* v) {
    // deterministic reduction of a 9-block over the group; result in v on every thread
    const Grp& g = x.g;
#if defined(__HIP_DEVICE_COMPILE__)
    // wave64 butterfly (every lane ends with the same sum), then the waves in order
    UNR for (int e = 0; e < 9; e++)
        UNR for (int m = 32; m > 0; m >>= 1) v[e] = v[e] + __shfl_xor(v[e], m, 64);
    const int wave = g.tid >> 6, nw = (g.n + 63) >> 6;
    if ((g.tid & 63) == 0)
        UNR for (int e = 0; e < 9; e++) x.red[wave * 9 + e] = v[e];
    g.sync();
    UNR for (int e = 0; e < 9; e++) {
        double s = x.red[e];
        for (int w = 1; w < nw; w++) s = s + x.red[w * 9 + e];
        v[e] = s;
    }
    g.sync();
#else
    for (int e = 0; e < 9; e++) x.red[g.tid * 9 + e] = v[e];
    g.sync();
    for (int s = g.n / 2; s > 0; s >>= 1) {
        if (g.tid < s)
            for (int e = 0; e < 9; e++) x.red[g.tid * 9 + e] = x.red[g.tid * 9 + e] + x.red[(g.tid + s) * 9 + e];
        g.sync();
    }
    for (int e = 0; e < 9; e++) v[e] = x.red[e];
    g.sync();
#endif
}

// exclusive scan of kp[0..N) in place; returns total
AD int block_scan(const Ctx& x, int* kp, int N) {
    const Grp& g = x.g;
    const int chunk = (N + g.n - 1) / g.n;
    const int lo = g.tid * chunk, hi = (lo + chunk < N) ? lo + chunk : N;
    int s = 0;
    for (int i = lo; i < hi; i++) s += kp[i];
    int* a = x.iscan;
    int* b = x.iscan + g.n;
    a[g.tid] = s;
    g.sync();
    for (int off = 1; off < g.n; off <<= 1) {
        b[g.tid] = a[g.tid] + (g.tid >= off ? a[g.tid - off] : 0);
        g.sync();
        int* t = a; a = b; b = t;
    }
    const int incl = a[g.tid];
    const int total = a[g.n - 1];
    int run = incl - s;
    for (int i = lo; i < hi; i++) { const int v = kp[i]; kp[i] = run; run += v; }
    g.sync();
    return total;
}

AD bool key_less(uint64_t h1, uint32_t i1, uint64_t h2, uint32_t i2) { return h1 < h2 || (h1 == h2 && i1 < i2); }

// bitonic sort of P (power of two) keys ascending by (hash, index)
ADN void bitonic(const Ctx& x, uint64_t* kh, uint32_t* ki, int P) {
    const Grp& g = x.g;
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int q = g.tid; q < P / 2; q += g.n) {
                const int i = 2 * j * (q / j) + (q % j);
                const int l = i + j;
                const bool asc = (i & k) == 0;
                const uint64_t hi_ = kh[i], hl = kh[l];
                const uint32_t ii = ki[i], il = ki[l];
                const bool gt = key_less(hl, il, hi_, ii);
                if (gt == asc) { kh[i] = hl; kh[l] = hi_; ki[i] = il; ki[l] = ii; }
            }
            g.sync();
        }
}

// ---------------------------------------------------------------------------------------------
// arena / handles. Convention: thread 0 stages operand handles into x.opa/opb/opc and writes the
// output header (dims, centre, independent parts) into the shared table; after a sync every
// thread reads handles from LDS; simplify_terms() then fills the output's monomials.

AD void alloc_out(Ctx& x, int o, int K, int stride) {
    if (x.g.tid == 0) {
        PZH& h = x.H[o];
        h.stride = stride;
        if (x.A->hused + K > x.A->hcap || x.A->cused + (long)K * stride > x.A->ccap) {
            *x.err |= ERR_ARENA;
            h.cnt = 0; h.hoff = 0; h.coff = 0;
        } else {
            h.hoff = x.A->hused;
            h.coff = x.A->cused;
            h.cnt = K;
            x.A->hused += K;
            x.A->cused += (long)K * stride;
        }
    }
    x.g.sync();
}

AD void hdr_init(PZH& h, int R, int C) {
    h.R = R; h.C = C; h.cnt = 0; h.stride = R * C; h.hoff = 0; h.coff = 0;
    h.comp = -1; h.scaled = 0; h.neg = 0; h.scale = 1.0;
    UNR for (int e = 0; e < 9; e++) { h.center[e] = 0.0; h.ind[0][e] = 0.0; h.ind[1][e] = 0.0; }
}

// generic simplify over a term list (hash(p), coef(p)) into shared handle o, whose header
// (dims, centre, independent parts: the operator's own formula) is already set; the pruned
// amount is added to both independent parts as in PZsparse.cu:347-349.
template <class Terms>
ADN void simplify_terms(Ctx& x, int o, const Terms& T, int N) {
    const Grp& g = x.g;
    const int n = x.H[o].R * x.H[o].C;
    uint64_t* kh = x.kh;
    uint32_t* ki = x.ki;
    int* kp = x.kp;
    int P = 1;
    while (P < N) P <<= 1;
    if (P > x.cap_lds) {
        kh = x.gkh; ki = x.gki; kp = x.gkp;
        if (P > x.cap_glb) {
            if (g.tid == 0) { *x.err |= ERR_SORTCAP; x.H[o].cnt = 0; }
            g.sync();
            return;
        }
    }
    for (int q = g.tid; q < P; q += g.n) {
        kh[q] = q < N ? T.hash(q) : ~(uint64_t)0;
        ki[q] = (uint32_t)q;
    }
    g.sync();
    if (N > 1) bitonic(x, kh, ki, P);
    double red[9], acc[9], tmp[9];
    UNR for (int e = 0; e < 9; e++) red[e] = 0.0;
    for (int q = g.tid; q < N; q += g.n) {
        const bool head = q == 0 || kh[q] != kh[q - 1];
        int keep = 0;
        if (head) {
            T.coef(ki[q], acc);
            for (int r = q + 1; r < N && kh[r] == kh[q]; r++) {
                T.coef(ki[r], tmp);
                UNR for (int e = 0; e < 9; e++) acc[e] = acc[e] + tmp[e];
            }
            if (frob_norm(acc, n) <= x.thr) {
                UNR for (int e = 0; e < 9; e++) red[e] = red[e] + fabs(acc[e]);
            } else {
                keep = 1;
            }
        }
        kp[q] = keep;
    }
    g.sync();
    const int K = block_scan(x, kp, N);
    alloc_out(x, o, K, n);
    const long hoff = x.H[o].hoff, coff = x.H[o].coff;
    if (x.H[o].cnt == K) {
        for (int q = g.tid; q < N; q += g.n) {
            const bool head = q == 0 || kh[q] != kh[q - 1];
            if (!head) continue;
            const bool keep = (q + 1 < N) ? (kp[q + 1] != kp[q]) : (kp[q] != K);
            if (!keep) continue;
            T.coef(ki[q], acc);
            for (int r = q + 1; r < N && kh[r] == kh[q]; r++) {
                T.coef(ki[r], tmp);
                UNR for (int e = 0; e < 9; e++) acc[e] = acc[e] + tmp[e];
            }
            const long pos = kp[q];
            x.A->h[hoff + pos] = kh[q];
            double* dst = x.A->c + coff + pos * n;
            UNR for (int e = 0; e < 9; e++) if (e < n) dst[e] = acc[e];
        }
    }
    block_sum9(x, red);
    if (g.tid == 0) {
        if (frob_norm(red, n) != 0)
            UNR for (int v = 0; v < 2; v++)
                UNR for (int e = 0; e < 9; e++) if (e < n) x.H[o].ind[v][e] = x.H[o].ind[v][e] + red[e];
    }
    g.sync();
}

// ---------------------------------------------------------------------------------------------
// term lists (operands live in LDS handle slots)

// operator* (PZsparse.cu:864-994): T1 a_i x B.c, T2 A.c x b_j, T3 a_i x b_j (hash a_i + b_j)
struct MulTerms {
    const Ctx* x;
    const PZH* A;
    const PZH* B;
    AD uint64_t hash(int p) const {
        const int na = A->cnt, nb = B->cnt;
        if (p < na) return mono_hash(*x, *A, p);
        if (p < na + nb) return mono_hash(*x, *B, p - na);
        const int q = p - na - nb;
        return mono_hash(*x, *A, q / nb) + mono_hash(*x, *B, q % nb);
    }
    AD void prod(const double* a, const double* b, double* out) const {
        const bool as = A->R == 1 && A->C == 1, bs = B->R == 1 && B->C == 1;
        if (as) { UNR for (int e = 0; e < 9; e++) out[e] = a[0] * b[e]; }
        else if (bs) { UNR for (int e = 0; e < 9; e++) out[e] = a[e] * b[0]; }
        else {
            matmul(a, A->R, A->C, b, B->C, out);
            UNR for (int e = 0; e < 9; e++) if (e >= A->R * B->C) out[e] = 0.0;
        }
    }
    AD void coef(int p, double* out) const {
        const int na = A->cnt, nb = B->cnt;
        double a[9], b[9];
        if (p < na) { read_mono(*x, *A, p, a); prod(a, B->center, out); return; }
        if (p < na + nb) { read_mono(*x, *B, p - na, b); prod(A->center, b, out); return; }
        const int q = p - na - nb;
        read_mono(*x, *A, q / nb, a);
        read_mono(*x, *B, q % nb, b);
        prod(a, b, out);
    }
};

// concatenation of up to 3 sources, each either a full block (place = -1) or a 1x1 source
// placed at component `place` of the output block (stack / addOneDimPZ)
struct CatTerms {
    const Ctx* x;
    const PZH* S[3];
    int place[3];
    AD void which(int p, int& s, int& k) const {
        s = 0;
        if (p >= S[0]->cnt) { p -= S[0]->cnt; s = 1; if (p >= S[1]->cnt) { p -= S[1]->cnt; s = 2; } }
        k = p;
    }
    AD uint64_t hash(int p) const { int s, k; which(p, s, k); return mono_hash(*x, *S[s], k); }
    AD void coef(int p, double* out) const {
        int s, k;
        which(p, s, k);
        read_mono(*x, *S[s], k, out);
        const int pl = place[s];
        if (pl >= 0) {
            const double v = out[0];
            UNR for (int e = 0; e < 9; e++) out[e] = (e == pl) ? v : 0.0;
        }
    }
};

// ---------------------------------------------------------------------------------------------
// handle constructors

AD void h_zero(Ctx& x, int o, int R, int C) {
    if (x.g.tid == 0) hdr_init(x.H[o], R, C);
    x.g.sync();
}

// element view (r, c) of handle a  (operator()(r,c), PZsparse.cu:678-697)
AD void h_elem(Ctx& x, int o, int a, int r, int c) {
    if (x.g.tid == 0) {
        const PZH s = x.H[a];
        PZH& h = x.H[o];
        h = s;
        const int e = r + c * s.R;
        h.R = 1; h.C = 1;
        h.comp = (s.comp >= 0) ? s.comp : e;
        h.center[0] = s.center[e];
        h.ind[0][0] = s.ind[0][e];
        h.ind[1][0] = s.ind[1][e];
    }
    x.g.sync();
}

// s * a  (PZsparse.cu:996-1030): lazy, no simplify
AD void h_scale(Ctx& x, int o, double s, int a) {
    if (x.g.tid == 0) {
        const PZH src = x.H[a];
        PZH& h = x.H[o];
        h = src;
        const int n = nel(h);
        for (int e = 0; e < n; e++) {
            h.center[e] = h.center[e] * s;
            h.ind[0][e] = h.ind[0][e] * fabs(s);
            h.ind[1][e] = h.ind[1][e] * fabs(s);
        }
        if (src.scaled || src.neg) *x.err |= ERR_HANDLES;  // views never stack scales in this program
        h.scaled = 1;
        h.scale = s;
    }
    x.g.sync();
}

// ---------------------------------------------------------------------------------------------
// operators

// a + b (sign = +1) or a - b (sign = -1)  (PZsparse.cu:743-764, 813-834)
ADN void op_add(Ctx& x, int o, int a, int b, int sign) {
    if (x.g.tid == 0) {
        x.H[x.opa] = x.H[a];
        x.H[x.opb] = x.H[b];
        const PZH& A = x.H[x.opa];
        PZH& B = x.H[x.opb];
        if (sign < 0) B.neg = !B.neg;
        PZH& h = x.H[o];
        hdr_init(h, A.R, A.C);
        const int n = nel(A);
        for (int e = 0; e < n; e++) {
            h.center[e] = sign > 0 ? A.center[e] + B.center[e] : A.center[e] - B.center[e];
            h.ind[0][e] = A.ind[0][e] + B.ind[0][e];
            h.ind[1][e] = A.ind[1][e] + B.ind[1][e];
        }
    }
    x.g.sync();
    CatTerms T;
    T.x = &x; T.S[0] = &x.H[x.opa]; T.S[1] = &x.H[x.opb]; T.S[2] = &x.H[x.opb];
    T.place[0] = -1; T.place[1] = -1; T.place[2] = -1;
    simplify_terms(x, o, T, x.H[x.opa].cnt + x.H[x.opb].cnt);
}

// a * b  (PZsparse.cu:864-994)
ADN void op_mul(Ctx& x, int o, int a, int b) {
    if (x.g.tid == 0) { x.H[x.opa] = x.H[a]; x.H[x.opb] = x.H[b]; }
    x.g.sync();
    const PZH& A = x.H[x.opa];
    const PZH& B = x.H[x.opb];
    // |A.c| + sum|a_i| and |B.c| + sum|b_j| for the independent part, reduced over the group
    double sa[9], sb[9], m[9];
    UNR for (int e = 0; e < 9; e++) { sa[e] = 0.0; sb[e] = 0.0; }
    for (int k = x.g.tid; k < A.cnt; k += x.g.n) { read_mono(x, A, k, m); UNR for (int e = 0; e < 9; e++) sa[e] = sa[e] + fabs(m[e]); }
    block_sum9(x, sa);
    for (int k = x.g.tid; k < B.cnt; k += x.g.n) { read_mono(x, B, k, m); UNR for (int e = 0; e < 9; e++) sb[e] = sb[e] + fabs(m[e]); }
    block_sum9(x, sb);
    MulTerms T;
    T.x = &x; T.A = &A; T.B = &B;
    if (x.g.tid == 0) {
        const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
        PZH& h = x.H[o];
        hdr_init(h, as ? B.R : A.R, as ? B.C : (bs ? A.C : B.C));
        const int na = nel(A), nb = nel(B), nr = nel(h);
        double cen[9];
        T.prod(A.center, B.center, cen);
        for (int e = 0; e < nr; e++) h.center[e] = cen[e];
        double r2[9], r3[9];
        for (int e = 0; e < 9; e++) { r2[e] = 0.0; r3[e] = 0.0; }
        for (int e = 0; e < na; e++) r2[e] = fabs(A.center[e]) + sa[e];
        for (int e = 0; e < nb; e++) r3[e] = fabs(B.center[e]) + sb[e];
        for (int v = 0; v < 2; v++) {
            double t2[9], t3[9], ii[9];
            if (as) { for (int e = 0; e < nb; e++) t2[e] = r2[0] * B.ind[v][e]; }
            else if (bs) { for (int e = 0; e < na; e++) t2[e] = r2[e] * B.ind[v][0]; }
            else matmul(r2, A.R, A.C, B.ind[v], B.C, t2);
            if (as) { for (int e = 0; e < nb; e++) t3[e] = A.ind[v][0] * r3[e]; }
            else if (bs) { for (int e = 0; e < na; e++) t3[e] = A.ind[v][e] * r3[0]; }
            else matmul(A.ind[v], A.R, A.C, r3, B.C, t3);
            if (as) { for (int e = 0; e < nr; e++) ii[e] = A.ind[v][0] * B.ind[v][e]; }
            else if (bs) { for (int e = 0; e < nr; e++) ii[e] = A.ind[v][e] * B.ind[v][0]; }
            else matmul(A.ind[v], A.R, A.C, B.ind[v], B.C, ii);
            for (int e = 0; e < nr; e++) h.ind[v][e] = ii[e] + (t2[e] + t3[e]);
        }
        if (as && !bs && B.R != 1 && A.cnt > 0 && B.cnt > 0) *x.err |= ERR_HANDLES;  // Eigen assert in the reference
    }
    x.g.sync();
    simplify_terms(x, o, T, A.cnt + B.cnt + A.cnt * B.cnt);
}

// stack three 1x1 PZs into a 3x1 (PZsparse.cu:1087-1116)
ADN void op_stack3(Ctx& x, int o, int a0, int a1, int a2) {
    if (x.g.tid == 0) {
        x.H[x.opa] = x.H[a0];
        x.H[x.opb] = x.H[a1];
        x.H[x.opc] = x.H[a2];
        PZH& h = x.H[o];
        hdr_init(h, 3, 1);
        const PZH* S[3] = {&x.H[x.opa], &x.H[x.opb], &x.H[x.opc]};
        for (int i = 0; i < 3; i++) { h.center[i] = S[i]->center[0]; h.ind[0][i] = S[i]->ind[0][0]; h.ind[1][i] = S[i]->ind[1][0]; }
    }
    x.g.sync();
    CatTerms T;
    T.x = &x; T.S[0] = &x.H[x.opa]; T.S[1] = &x.H[x.opb]; T.S[2] = &x.H[x.opc];
    T.place[0] = 0; T.place[1] = 1; T.place[2] = 2;
    simplify_terms(x, o, T, x.H[x.opa].cnt + x.H[x.opb].cnt + x.H[x.opc].cnt);
}

// self(r,c) += a (1x1)  (PZsparse.cu:1068-1085); result written to o
ADN void op_add_one_dim(Ctx& x, int o, int self, int a, int r, int c) {
    const int e = r + c * 3;
    if (x.g.tid == 0) {
        x.H[x.opa] = x.H[self];
        x.H[x.opb] = x.H[a];
        const PZH& A = x.H[x.opa];
        const PZH& B = x.H[x.opb];
        PZH& h = x.H[o];
        hdr_init(h, A.R, A.C);
        for (int q = 0; q < 9; q++) { h.center[q] = A.center[q]; h.ind[0][q] = A.ind[0][q]; h.ind[1][q] = A.ind[1][q]; }
        h.center[e] += B.center[0];
        h.ind[0][e] += B.ind[0][0];
        h.ind[1][e] += B.ind[1][0];
    }
    x.g.sync();
    CatTerms T;
    T.x = &x; T.S[0] = &x.H[x.opa]; T.S[1] = &x.H[x.opb]; T.S[2] = &x.H[x.opb];
    T.place[0] = -1; T.place[1] = e; T.place[2] = -1;
    simplify_terms(x, o, T, x.H[x.opa].cnt + x.H[x.opb].cnt);
}

// cross products (PZsparse.cu:1118-1167); handles t0 .. t0+10 are scratch slots
ADN void op_cross_mp(Ctx& x, int o, const double* a, int b, int t0) {
    const int e0 = t0, e1 = t0 + 1, e2 = t0 + 2, s0 = t0 + 3, s1 = t0 + 4, r0 = t0 + 5, r1 = t0 + 6, r2 = t0 + 7;
    const double a0 = a[0], a1 = a[1], a2 = a[2];
    h_elem(x, e0, b, 0, 0); h_elem(x, e1, b, 1, 0); h_elem(x, e2, b, 2, 0);
    h_scale(x, s0, a1, e2); h_scale(x, s1, a2, e1); op_add(x, r0, s0, s1, -1);
    h_scale(x, s0, a2, e0); h_scale(x, s1, a0, e2); op_add(x, r1, s0, s1, -1);
    h_scale(x, s0, a0, e1); h_scale(x, s1, a1, e0); op_add(x, r2, s0, s1, -1);
    op_stack3(x, o, r0, r1, r2);
}

ADN void op_cross_pm(Ctx& x, int o, int a, const double* b, int t0) {
    const int e0 = t0, e1 = t0 + 1, e2 = t0 + 2, s0 = t0 + 3, s1 = t0 + 4, r0 = t0 + 5, r1 = t0 + 6, r2 = t0 + 7;
    const double b0 = b[0], b1 = b[1], b2 = b[2];
    h_elem(x, e0, a, 0, 0); h_elem(x, e1, a, 1, 0); h_elem(x, e2, a, 2, 0);
    h_scale(x, s0, b2, e1); h_scale(x, s1, b1, e2); op_add(x, r0, s0, s1, -1);
    h_scale(x, s0, b0, e2); h_scale(x, s1, b2, e0); op_add(x, r1, s0, s1, -1);
    h_scale(x, s0, b1, e0); h_scale(x, s1, b0, e1); op_add(x, r2, s0, s1, -1);
    op_stack3(x, o, r0, r1, r2);
}

ADN void op_cross_pp(Ctx& x, int o, int a, int b, int t0) {
    const int a0 = t0, a1 = t0 + 1, a2 = t0 + 2, b0 = t0 + 3, b1 = t0 + 4, b2 = t0 + 5;
    const int p = t0 + 6, q = t0 + 7, r0 = t0 + 8, r1 = t0 + 9, r2 = t0 + 10;
    h_elem(x, a0, a, 0, 0); h_elem(x, a1, a, 1, 0); h_elem(x, a2, a, 2, 0);
    h_elem(x, b0, b, 0, 0); h_elem(x, b1, b, 1, 0); h_elem(x, b2, b, 2, 0);
    op_mul(x, p, a1, b2); op_mul(x, q, a2, b1); op_add(x, r0, p, q, -1);
    op_mul(x, p, a2, b0); op_mul(x, q, a0, b2); op_add(x, r1, p, q, -1);
    op_mul(x, p, a0, b1); op_mul(x, q, a1, b0); op_add(x, r2, p, q, -1);
    op_stack3(x, o, r0, r1, r2);
}

}  // namespace armour
