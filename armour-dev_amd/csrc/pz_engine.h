// armour-mi355x — workgroup-cooperative sparse polynomial-zonotope (PZ) engine for gfx950.
//
// Semantics are those of the reference's PZsparse (KPR/PZsparse.cu:284-1167): monomials carry a
// 63-bit degree hash, products add hashes without carry, and every operator ends in simplify():
// merge equal hashes, prune merged coefficients whose Frobenius norm is <= SIMPLIFY_THRESHOLD
// into the interval part `independent`. The data layout and algorithms are MI355X-first:
//   * a PZ is a handle (dims, centre, independent parts, sum|m_k|) in LDS plus a structure-of-
//     arrays run of monomials (hash[], coefficient block[]) in a per-workgroup HBM arena (bump
//     allocated). Every materialised run is sorted by hash with unique hashes (it is the output
//     of a simplify), which the operators below exploit;
//   * element extraction and scaling by a constant are lazy views on a parent's monomials (no
//     copies) — the reader applies s*c exactly as the reference's materialised copy would;
//   * simplify() orders (hash, term-index) keys and sums each equal-hash group in term order:
//       - N <= 64 terms: wave 0 alone. Each lane loads its term (hash + coefficients, one memory
//         round trip), a bitonic network over DPP / permlane moves (wave.h) sorts the keys in
//         registers, the coefficients follow by ds_bpermute, groups are summed by lane shifts and
//         compacted with ballot/popcount — no workgroup barrier;
//       - larger: the operands are first staged into LDS; the order is built by RANK MERGE: the
//         term list is a union of sorted runs (the sources of a sum or stack; T1, T2 and the rows
//         or columns of T3 for a product), and each key's rank is the sum of its lower bounds in
//         the runs — no sort. The group sums park their kept values in HBM for the compaction;
//   * every PZ carries TWO independent parts (nominal / interval inertial parameters). The
//     reference runs RNEA twice (armour_main.cu:129,132) with identical centres and monomials —
//     only `independent` differs — so one pass with dual independent parts replaces both;
//   * each handle carries sum_k |m_k| (elementwise), so a product's independent part needs no
//     pass over its operands' monomials.
// All device functions are force-inlined: the reach kernel is an interpreter whose op bodies
// are inlined once each into one switch (reach.h), so the program runs with no device calls.
// The group abstraction (Grp) lets the same code run as a sequential host emulation in tests.
#pragma once
#include "common.h"
#include "wave.h"

namespace armour {
constexpr int MAX_SLOTS = 96;  // handle slots of a reach program (ProgramBuilder)
}

#define AI __host__ __device__ inline __attribute__((always_inline))
#define UNR _Pragma("unroll")

namespace armour {

struct Grp {
    int tid, n;
    AI void sync() const {
#if defined(__HIP_DEVICE_COMPILE__)
        __syncthreads();
#endif
    }
};

// PZ handle. Views: comp >= 0 selects one element of the parent's coefficient block (the
// reference's operator()(r,c), PZsparse.cu:678-697); scaled applies s * c on read (PZ * double,
// :996-1030). The handle's small dense blocks live in an LDS pool at `off`, sized by the slot's
// static shape class n = R*C (1, 3 or 9): centre[n], independent parts ind0[n], ind1[n] and
// sum_k |m_k| elementwise (absum[n]) — see cen() / ind() / abs_().
struct PZH {
    int R, C;
    int cnt;
    int stride;
    long hoff, coff;
    int comp;
    int scaled;
    double scale;
    int off;
};

struct Arena {
    long hcap, ccap;
    long hused, cused;
    double bytes;  // algorithmic monomial bytes read + written by the operators of this job
};

struct Ctx {
    Grp g;
    PZH* H;            // handle table (LDS)
    double* pool;      // handle payload pool (LDS)
    Arena* A;          // bump arena state (LDS)
    // arena storage (HBM, per workgroup), held here (registers)
    uint64_t* ah;
    double* ac;
    uint64_t* kh;      // ordered keys: hash        (LDS, cap_lds entries)
    uint32_t* ki;      // ordered keys: term index
    int* kp;           // keep flags / scan
    int cap_lds;
    uint64_t* gkh;     // global fallback for large operators
    uint32_t* gki;
    int* gkp;
    int cap_glb;
    double* gout;      // group sums of the simplify in flight, by key position (HBM): cap_glb * 9
    double* stage;     // operand staging (LDS), stage_cap doubles
    int stage_cap;
    double* red;       // reduction scratch (LDS): [waves * 18] on device, [n * 18] in the emulation
    int* iscan;        // scan scratch (LDS): [waves] on device, [2 * n] in the emulation
    int* err;          // error word (LDS)
    double thr;
    unsigned long long* phase;  // optional large-operator phase cycle counters [8] (profiling)
    int mode;          // diagnostics: bit 0 = no wave-0 path
};

enum : int { ERR_ARENA = 1, ERR_SORTCAP = 2, ERR_LINKGEN = 4, ERR_OUTCAP = 8, ERR_HANDLES = 16 };

// ---------------------------------------------------------------------------------------------
// scalar helpers (fixed 9-element blocks, unrolled so blocks stay in registers)
AI double frob_norm(const double* x, int n) {
    // Eigen 3.3 MatrixXd::norm(): packet-of-2 redux order (same as oracle/src/pz.cpp)
    if (n == 1) return sqrt(x[0] * x[0]);
    if (n == 3) return sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
    const double s0 = x[0] * x[0], s1 = x[1] * x[1], s2 = x[2] * x[2], s3 = x[3] * x[3], s4 = x[4] * x[4];
    const double s5 = x[5] * x[5], s6 = x[6] * x[6], s7 = x[7] * x[7], s8 = x[8] * x[8];
    return sqrt((((s0 + s4) + (s2 + s6)) + ((s1 + s5) + (s3 + s7))) + s8);
}

// column-major coefficient-based product, inner index summed in order. The program only forms
// (3x3)(3x3) and (3x3)(3x1) block products (1x1 operands are handled as scalings); any other
// shape is flagged by the caller.
AI void matmul(const double* A, int ra, int ca, const double* B, int cb, double* out) {
    double t[9];
    UNR for (int e = 0; e < 9; e++) t[e] = 0.0;
    UNR for (int j = 0; j < 3; j++)
        UNR for (int i = 0; i < 3; i++)
            if (j < cb) t[i + 3 * j] = (A[i] * B[3 * j] + A[i + 3] * B[3 * j + 1]) + A[i + 6] * B[3 * j + 2];
    UNR for (int e = 0; e < 9; e++) out[e] = t[e];
}

AI int nel(const PZH& h) { return h.R * h.C; }
AI double* cen(const Ctx& x, const PZH& h) { return x.pool + h.off; }
AI double* ind(const Ctx& x, const PZH& h, int v) { return x.pool + h.off + (1 + v) * (h.R * h.C); }
AI double* abs_(const Ctx& x, const PZH& h) { return x.pool + h.off + 3 * (h.R * h.C); }

// read monomial k of handle h into a 9-block (entries >= nel(h) are zero)
AI void read_mono(const Ctx& x, const PZH& h, int k, double* out) {
    const double* base = x.ac + h.coff + (long)k * h.stride;
    const int n = nel(h);
    UNR for (int e = 0; e < 9; e++) {
        double v = 0.0;
        if (e < n) {
            v = base[h.comp >= 0 ? h.comp : e];
            if (h.scaled) v = h.scale * v;
        }
        out[e] = v;
    }
}
AI uint64_t mono_hash(const Ctx& x, const PZH& h, int k) { return x.ah[h.hoff + k]; }

// ---------------------------------------------------------------------------------------------
// wave / block primitives
#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline __attribute__((always_inline)) double wsum(double v) { return wave_sum(v); }
__device__ inline __attribute__((always_inline)) long bcast0(long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), 0);
    return (long)(((uint64_t)hi << 32) | lo);
}
#endif

// deterministic reduction of an n-block (n <= 18) over the group; result in v on every thread
AI void block_sum(const Ctx& x, double* v, int n) {
    const Grp& g = x.g;
#if defined(__HIP_DEVICE_COMPILE__)
    UNR for (int e = 0; e < 18; e++) if (e < n) v[e] = wsum(v[e]);
    const int wave = g.tid >> 6, nw = (g.n + 63) >> 6;
    if ((g.tid & 63) == 0)
        UNR for (int e = 0; e < 18; e++) if (e < n) x.red[wave * 18 + e] = v[e];
    g.sync();
    UNR for (int e = 0; e < 18; e++) {
        if (e < n) {
            double s = x.red[e];
            for (int w = 1; w < nw; w++) s = s + x.red[w * 18 + e];
            v[e] = s;
        }
    }
    g.sync();
#else
    for (int e = 0; e < n; e++) x.red[g.tid * 18 + e] = v[e];
    g.sync();
    for (int s = g.n / 2; s > 0; s >>= 1) {
        if (g.tid < s)
            for (int e = 0; e < n; e++) x.red[g.tid * 18 + e] = x.red[g.tid * 18 + e] + x.red[(g.tid + s) * 18 + e];
        g.sync();
    }
    for (int e = 0; e < n; e++) v[e] = x.red[e];
    g.sync();
#endif
}

// exclusive scan of kp[0..N) in place (contiguous chunk per thread); returns total
AI int block_scan(const Ctx& x, int* kp, int N) {
    const Grp& g = x.g;
    const int chunk = (N + g.n - 1) / g.n;
    const int lo = g.tid * chunk, hi = (lo + chunk < N) ? lo + chunk : N;
    int s = 0;
    for (int i = lo; i < hi; i++) s += kp[i];
#if defined(__HIP_DEVICE_COMPILE__)
    const int lane = g.tid & 63, wave = g.tid >> 6, nw = (g.n + 63) >> 6;
    const int inc = wave_incl_scan(s);
    if (lane == 63) x.iscan[wave] = inc;
    g.sync();
    int base = 0, total = 0;
    for (int w = 0; w < nw; w++) {
        const int t = x.iscan[w];
        if (w < wave) base += t;
        total += t;
    }
    int run = base + inc - s;
    for (int i = lo; i < hi; i++) { const int v = kp[i]; kp[i] = run; run += v; }
    g.sync();
    return total;
#else
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
#endif
}

AI bool key_less(uint64_t h1, uint32_t i1, uint64_t h2, uint32_t i2) { return h1 < h2 || (h1 == h2 && i1 < i2); }

// ---------------------------------------------------------------------------------------------
// operands as the term generator sees them: a run of `cnt` monomials with hashes h[k] and
// coefficient rows c[k * stride + (comp >= 0 ? comp : e)], e < n, times scale if scaled.
struct Src {
    const uint64_t* h;
    const double* c;
    int cnt, n, stride, comp, scaled;
    double scale;
    AI uint64_t hash(int k) const { return h[k]; }
    AI void read(int k, bool neg, double* out) const {
        const double* base = c + (long)k * stride;
        UNR for (int e = 0; e < 9; e++) {
            double v = 0.0;
            if (e < n) {
                v = base[comp >= 0 ? comp : e];
                if (scaled) v = scale * v;
                if (neg) v = -v;
            }
            out[e] = v;
        }
    }
};

AI Src src_of(const Ctx& x, const PZH& p) {
    Src s;
    s.h = x.ah + p.hoff;
    s.c = x.ac + p.coff;
    s.cnt = p.cnt;
    s.n = nel(p);
    s.stride = p.stride;
    s.comp = p.comp;
    s.scaled = p.scaled;
    s.scale = p.scale;
    return s;
}

// first k in [0, cnt) with h[k] >= key (runs are strictly increasing)
AI int lower_bound(const uint64_t* h, int cnt, uint64_t key) {
    int lo = 0, len = cnt;
    while (len > 0) {
        const int half = len >> 1;
        if (h[lo + half] < key) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    return lo;
}
// same over the T3 row i of a product: keys off + h[j]
AI int lower_bound_off(const uint64_t* h, int cnt, uint64_t off, uint64_t key) {
    int lo = 0, len = cnt;
    while (len > 0) {
        const int half = len >> 1;
        if (off + h[lo + half] < key) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    return lo;
}
// T3 column j of a product: keys ha[i] + hb_j over i
AI int lower_bound_col(const uint64_t* ha, int cnt, uint64_t hbj, uint64_t key) { return lower_bound_off(ha, cnt, hbj, key); }
// RK searches over one run at once: out[u] = first k in [0, cnt) with off[u] + h[k] >= key[u].
// Branch-free, with a halving sequence that depends on cnt only, so the RK searches' loads are in
// flight together (one search is a chain of dependent loads; a term's rank sums many of them).
constexpr int RK = 4;
AI void lower_bounds(const uint64_t* h, int cnt, const uint64_t* off, const uint64_t* key, int* out) {
    int base[RK];
    UNR for (int u = 0; u < RK; u++) base[u] = 0;
    if (cnt <= 0) {
        UNR for (int u = 0; u < RK; u++) out[u] = 0;
        return;
    }
    for (int n = cnt; n > 1;) {
        const int half = n >> 1;
        uint64_t v[RK];
        UNR for (int u = 0; u < RK; u++) v[u] = h[base[u] + half];
        UNR for (int u = 0; u < RK; u++) base[u] = off[u] + v[u] < key[u] ? base[u] + half : base[u];
        n -= half;
    }
    uint64_t v[RK];
    UNR for (int u = 0; u < RK; u++) v[u] = h[base[u]];
    UNR for (int u = 0; u < RK; u++) out[u] = base[u] + (off[u] + v[u] < key[u] ? 1 : 0);
}

// term lists of an operator: kind 0 = product (PZsparse.cu:864-994: T1 a_i x B.c, T2 A.c x b_j,
// T3 a_i x b_j with hash a_i + b_j), kind 1 = concatenation of up to 3 sources, each a full block
// (place = -1) or a 1x1 source placed at component `place` (operator+/-, stack, addOneDimPZ)
struct Terms {
    int kind, ns;
    Src S[3];
    int places;        // 4 bits per source: component + 1 (0: full block)
    int negs;          // bit per source: negate on read
    const double* Ac;  // product: operand centres (LDS handles)
    const double* Bc;
    int AR, AC, BC;
    int nout;          // elements of the output block
    uint32_t nbm;      // product: ceil(2^32 / |S1|), so T3 index q splits as q / nb = mulhi(q, nbm)
    // T3 index q -> (row i, column j) without an integer division: exact for q, nb < 2^16
    AI void split(int q, int& i, int& j) const {
        const int nb = S[1].cnt;
#if defined(__HIP_DEVICE_COMPILE__)
        i = nb == 1 ? q : (int)__umulhi((uint32_t)q, nbm);
#else
        i = nb == 1 ? q : (int)(((uint64_t)(uint32_t)q * nbm) >> 32);
#endif
        j = q - i * nb;
    }
    AI void which(int p, int& s, int& k) const {
        s = 0;
        if (p >= S[0].cnt) { p -= S[0].cnt; s = 1; if (p >= S[1].cnt) { p -= S[1].cnt; s = 2; } }
        k = p;
    }
    AI uint64_t hash(int p) const {
        if (kind == 0) {
            const int na = S[0].cnt, nb = S[1].cnt;
            if (p < na) return S[0].hash(p);
            if (p < na + nb) return S[1].hash(p - na);
            int i, j;
            split(p - na - nb, i, j);
            return S[0].hash(i) + S[1].hash(j);
        }
        int s, k;
        which(p, s, k);
        return s == 0 ? S[0].hash(k) : s == 1 ? S[1].hash(k) : S[2].hash(k);
    }
    AI void prod(const double* a, const double* b, double* out) const {
        const bool as = AR == 1 && AC == 1, bs = S[1].n == 1;
        if (as) { UNR for (int e = 0; e < 9; e++) out[e] = a[0] * b[e]; }
        else if (bs) { UNR for (int e = 0; e < 9; e++) out[e] = a[e] * b[0]; }
        else matmul(a, AR, AC, b, BC, out);
    }
    AI void coef(int p, double* out) const {
        if (kind == 0) {
            const int na = S[0].cnt, nb = S[1].cnt;
            double a[9], b[9];
            if (p < na) {
                S[0].read(p, false, a);
                UNR for (int e = 0; e < 9; e++) b[e] = Bc[e];
                prod(a, b, out);
                return;
            }
            if (p < na + nb) {
                S[1].read(p - na, false, b);
                UNR for (int e = 0; e < 9; e++) a[e] = Ac[e];
                prod(a, b, out);
                return;
            }
            int i, j;
            split(p - na - nb, i, j);
            S[0].read(i, false, a);
            S[1].read(j, false, b);
            prod(a, b, out);
            return;
        }
        int s, k;
        which(p, s, k);
        const bool ng = (negs >> s) & 1;
        if (s == 0) S[0].read(k, ng, out);
        else if (s == 1) S[1].read(k, ng, out);
        else S[2].read(k, ng, out);
        const int pl = ((places >> (4 * s)) & 15) - 1;
        if (pl >= 0) {
            const double v = out[0];
            UNR for (int e = 0; e < 9; e++) out[e] = (e == pl) ? v : 0.0;
        }
    }
    AI double in_bytes() const {
        double b = 0;
        UNR for (int s = 0; s < 3; s++) if (s < ns) b += (double)S[s].cnt * (8.0 + 8.0 * S[s].n);
        return b;
    }
    // number of sorted runs the term list is made of (rank merge cost)
    AI int runs() const {
        if (kind == 1) return ns;
        const int na = S[0].cnt, nb = S[1].cnt;
        return 2 + (na < nb ? na : nb);
    }
    // rank of term p (hash h) in the (hash, term index) order of the whole list
    AI int rank(int p, uint64_t h) const {
        // A run's equal key (at most one per run) precedes term p when its term index is lower,
        // which is decided by the run alone: earlier sources / T1 / T2 / earlier T3 rows precede,
        // later ones follow. So a preceding run counts keys <= h (a search for h + 1), a following
        // one keys < h, and the own run contributes the own index — no tie probe.
        const uint64_t h1 = h + 1;  // hashes stay below 2^63
        if (kind == 1) {
            int s, k;
            which(p, s, k);
            int r = k;
            UNR for (int t = 0; t < 3; t++)
                if (t < ns && t != s) r += lower_bound(S[t].h, S[t].cnt, t < s ? h1 : h);
            return r;
        }
        const int na = S[0].cnt, nb = S[1].cnt;
        const int base = na + nb;
        const int seg = p < na ? 0 : (p < base ? 1 : 2);
        int r = seg == 0 ? p : lower_bound(S[0].h, na, h1);             // T1
        r += seg == 1 ? p - na : lower_bound(S[1].h, nb, seg == 2 ? h1 : h);  // T2
        // the T3 runs, RK searches at a time (rows i: keys h[i] + b_j; columns j: keys a_i + h[j])
        if (na <= nb) {
            int i0 = -1, j0 = 0;
            if (seg == 2) split(p - base, i0, j0);
            for (int i = 0; i < na; i += RK) {
                uint64_t off[RK], key[RK];
                int lb[RK];
                UNR for (int u = 0; u < RK; u++) {
                    off[u] = S[0].h[i + u < na ? i + u : 0];
                    key[u] = i + u < i0 ? h1 : h;
                }
                lower_bounds(S[1].h, nb, off, key, lb);
                UNR for (int u = 0; u < RK; u++)
                    if (i + u < na) r += i + u == i0 ? j0 : lb[u];
            }
        } else {
            for (int j = 0; j < nb; j += RK) {
                uint64_t off[RK], key[RK];
                int lb[RK];
                UNR for (int u = 0; u < RK; u++) {
                    off[u] = S[1].h[j + u < nb ? j + u : 0];
                    key[u] = h;
                }
                lower_bounds(S[0].h, na, off, key, lb);
                uint64_t v[RK];
                UNR for (int u = 0; u < RK; u++) v[u] = S[0].h[lb[u] < na ? lb[u] : 0];
                UNR for (int u = 0; u < RK; u++) {
                    if (j + u >= nb) continue;
                    int l = lb[u];
                    if (l < na && v[u] + off[u] == h && base + l * nb + j + u < p) l++;
                    r += l;
                }
            }
        }
        return r;
    }
};

// copy the sources into LDS (hashes, then effective coefficient rows), if they fit; else the
// hashes alone, if they fit (the key order's searches are chains of dependent hash loads, the
// group passes' coefficient loads are independent). Uniform decision; the caller's barrier
// publishes the staged copy.
AI void stage_sources(Ctx& x, Terms& T) {
    int need = 0, need_h = 0;
    UNR for (int s = 0; s < 3; s++) if (s < T.ns) { need += T.S[s].cnt * (1 + T.S[s].n); need_h += T.S[s].cnt; }
    if (need_h > x.stage_cap) return;
    const bool full = need <= x.stage_cap;
    double* base = x.stage;
    UNR for (int s = 0; s < 3; s++) {
        if (s >= T.ns) continue;
        Src& S = T.S[s];
        uint64_t* hs = (uint64_t*)base;
        if (!full) {
            for (int k = x.g.tid; k < S.cnt; k += x.g.n) hs[k] = S.h[k];
            S.h = hs;
            base += S.cnt;
            continue;
        }
        double* cs = base + S.cnt;
        // two monomials per thread per round, every load of a round issued before its stores
        for (int k = x.g.tid; k < S.cnt; k += 2 * x.g.n) {
            const int k2 = k + x.g.n;
            const bool two = k2 < S.cnt;
            const uint64_t h1 = S.h[k], h2 = S.h[two ? k2 : k];
            double v1[9], v2[9];
            const double* s1 = S.c + (long)k * S.stride;
            const double* s2 = S.c + (long)(two ? k2 : k) * S.stride;
            UNR for (int e = 0; e < 9; e++) {
                if (e < S.n) {
                    v1[e] = s1[S.comp >= 0 ? S.comp : e];
                    v2[e] = s2[S.comp >= 0 ? S.comp : e];
                }
            }
            hs[k] = h1;
            UNR for (int e = 0; e < 9; e++) if (e < S.n) cs[k * S.n + e] = S.scaled ? S.scale * v1[e] : v1[e];
            if (two) {
                hs[k2] = h2;
                UNR for (int e = 0; e < 9; e++) if (e < S.n) cs[k2 * S.n + e] = S.scaled ? S.scale * v2[e] : v2[e];
            }
        }
        S.h = hs;
        S.c = cs;
        S.stride = S.n;
        S.comp = -1;
        S.scaled = 0;
        S.scale = 1.0;
        base += S.cnt * (1 + S.n);
    }
}

// shared counters of the workgroup, updated by one lane per op — or by several lanes at once in
// a lane-parallel group of thread-0 ops (reach.h), hence LDS atomics on the device
AI void err_or(const Ctx& x, int bits) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicOr(x.err, bits);
#else
    *x.err |= bits;
#endif
}
AI void bytes_add(const Ctx& x, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicAdd(&x.A->bytes, b);
#else
    x.A->bytes += b;
#endif
}
AI void int_add(int* p, int v) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicAdd(p, v);
#else
    *p += v;
#endif
}
AI void int_min(int* p, int v) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicMin(p, v);
#else
    *p = v < *p ? v : *p;
#endif
}
AI void arena_alloc_t0(Ctx& x, PZH& h, int K, int stride) {
    h.stride = stride;
#if defined(__HIP_DEVICE_COMPILE__)
    const long h0 = (long)atomicAdd((unsigned long long*)&x.A->hused, (unsigned long long)K);
    const long c0 = (long)atomicAdd((unsigned long long*)&x.A->cused, (unsigned long long)K * stride);
#else
    const long h0 = x.A->hused, c0 = x.A->cused;
    x.A->hused += K;
    x.A->cused += (long)K * stride;
#endif
    if (h0 + K > x.A->hcap || c0 + (long)K * stride > x.A->ccap) {
        err_or(x, ERR_ARENA);
        h.cnt = 0; h.hoff = 0; h.coff = 0;
    } else {
        h.hoff = h0;
        h.coff = c0;
        h.cnt = K;
    }
}

// output header finish (thread 0): pruned amount into both independent parts (PZsparse.cu:347-349)
AI void finish_t0(const Ctx& x, PZH& h, const double* red, const double* abs, int n) {
    if (frob_norm(red, n) != 0)
        UNR for (int v = 0; v < 2; v++)
            UNR for (int e = 0; e < 9; e++) if (e < n) ind(x, h, v)[e] = ind(x, h, v)[e] + red[e];
    UNR for (int e = 0; e < 9; e++) if (e < n) abs_(x, h)[e] = abs[e];
}

AI double frob1(double v) { return frob_norm(&v, 1); }
AI double pick3(const double* m, int i) { return i == 0 ? m[0] : (i == 1 ? m[1] : m[2]); }

// ---------------------------------------------------------------------------------------------
// group policies: what a simplify makes of an ordered term list. Per term a policy yields up to NV
// values; per equal-hash group it sums them in term order (the reference's merge) and decides
// keep / prune; NR reduction slots (a bit mask says which are live); finish() completes the
// output header from the reduced slots (thread 0).

// plain simplify (PZsparse.cu:284-350): group sum of coefficient blocks, prune by Frobenius norm.
// Instantiated per output class NN (1x1, 3x1, 3x3) so the frequent small blocks carry no 9-element
// arrays: the register budget of the common paths stays clear of the 3x3 one.
template <int NN>
struct PolBlock {
    static constexpr int NV = NN;
    static constexpr int NO = NN;
    static constexpr int NR = 2 * NN;   // [0, NN): pruned |sum|, [NN, 2NN): kept |sum| (absum)
    double thr;
    AI unsigned mask() const { return (1u << NR) - 1; }
    AI void term(const Terms& T, int p, double* v) const {
        double t[9];
        T.coef(p, t);
        UNR for (int e = 0; e < NN; e++) v[e] = t[e];
    }
    AI bool group(const double* s, double* out, double* red) const {
        const bool keep = frob_norm(s, NN) > thr;
        UNR for (int e = 0; e < NN; e++) {
            if (keep) { out[e] = s[e]; red[NN + e] = red[NN + e] + fabs(s[e]); }
            else red[e] = red[e] + fabs(s[e]);
        }
        return keep;
    }
    AI void finish(Ctx& x, int o, const double* red) const { finish_t0(x, x.H[o], red, red + NN, NN); }
};

// fused PZ x PZ cross product of two 3x1 PZs a, b (PZsparse.cu:1118-1167 composes it from element
// views): six 1x1 products P0 = a1 b2, P1 = a2 b1, P2 = a2 b0, P3 = a0 b2, P4 = a0 b1, P5 = a1 b0,
// each simplified; r_e = P_2e - P_2e+1, each simplified; stack(r0, r1, r2), simplified. All six
// products share one term list (T1 a_i, T2 b_j, T3 a_i + b_j), so one ordering serves them all;
// every intermediate prune is replicated per hash group.
struct PolCrossPP {
    static constexpr int NV = 6;
    static constexpr int NO = 3;
    static constexpr int NR = 15;   // [0,6) product prunes, [6,9) difference prunes, [9,12) stack prunes, [12,15) absum
    double thr;
    const double* ac;               // operand centres (LDS handles)
    const double* bc;
    int a, b;                       // operand handle slots
    AI unsigned mask() const { return (1u << NR) - 1; }
    AI static void prods(const double* u, const double* w, double* v) {
        v[0] = u[1] * w[2]; v[1] = u[2] * w[1]; v[2] = u[2] * w[0];
        v[3] = u[0] * w[2]; v[4] = u[0] * w[1]; v[5] = u[1] * w[0];
    }
    AI void term(const Terms& T, int p, double* v) const {
        const int na = T.S[0].cnt, nb = T.S[1].cnt;
        double u[9], w[9];
        if (p < na) {
            T.S[0].read(p, false, u);
            UNR for (int e = 0; e < 3; e++) w[e] = bc[e];
        } else if (p < na + nb) {
            UNR for (int e = 0; e < 3; e++) u[e] = ac[e];
            T.S[1].read(p - na, false, w);
        } else {
            int i, j;
            T.split(p - na - nb, i, j);
            T.S[0].read(i, false, u);
            T.S[1].read(j, false, w);
        }
        prods(u, w, v);
    }
    AI bool group(const double* s, double* out, double* red) const {
        bool pres[6];
        UNR for (int p = 0; p < 6; p++) {
            pres[p] = frob1(s[p]) > thr;
            if (!pres[p]) red[p] = red[p] + fabs(s[p]);
        }
        double vec[3];
        bool any = false;
        UNR for (int e = 0; e < 3; e++) {
            const int P = 2 * e, Q = 2 * e + 1;
            bool have = pres[P] || pres[Q];
            const double v = pres[P] ? (pres[Q] ? s[P] + (-s[Q]) : s[P]) : (pres[Q] ? -s[Q] : 0.0);
            if (have && !(frob1(v) > thr)) { red[6 + e] = red[6 + e] + fabs(v); have = false; }
            vec[e] = have ? v : 0.0;
            any = any || have;
        }
        if (!any) return false;
        if (!(frob_norm(vec, 3) > thr)) {
            UNR for (int e = 0; e < 3; e++) red[9 + e] = red[9 + e] + fabs(vec[e]);
            return false;
        }
        UNR for (int e = 0; e < 3; e++) { out[e] = vec[e]; red[12 + e] = red[12 + e] + fabs(vec[e]); }
        return true;
    }
    // headers of the whole composition: products (PZsparse.cu:944-990 for 1x1 operands), the
    // differences (:813-834) and the stack (:1087-1116), each plus its own pruned amount
    AI void finish(Ctx& x, int o, const double* red) const {
        const PZH& A = x.H[a];
        const PZH& B = x.H[b];
        PZH& h = x.H[o];
        const int ea[6] = {1, 2, 2, 0, 0, 1}, fb[6] = {2, 1, 0, 2, 1, 0};
        double pc[6], pi[2][6];
        UNR for (int p = 0; p < 6; p++) {
            const double ace = pick3(cen(x, A), ea[p]), bcf = pick3(cen(x, B), fb[p]);
            const double r2 = fabs(ace) + pick3(abs_(x, A), ea[p]);
            const double r3 = fabs(bcf) + pick3(abs_(x, B), fb[p]);
            pc[p] = ace * bcf;
            UNR for (int v = 0; v < 2; v++) {
                const double ai = pick3(ind(x, A, v), ea[p]), bi = pick3(ind(x, B, v), fb[p]);
                pi[v][p] = ai * bi + (r2 * bi + ai * r3);
                if (frob1(red[p]) != 0) pi[v][p] = pi[v][p] + red[p];
            }
        }
        double sred[3];
        UNR for (int e = 0; e < 3; e++) sred[e] = red[9 + e];
        const bool sadd = frob_norm(sred, 3) != 0;
        UNR for (int e = 0; e < 3; e++) {
            cen(x, h)[e] = pc[2 * e] - pc[2 * e + 1];
            UNR for (int v = 0; v < 2; v++) {
                double iv = pi[v][2 * e] + pi[v][2 * e + 1];
                if (frob1(red[6 + e]) != 0) iv = iv + red[6 + e];
                if (sadd) iv = iv + sred[e];
                ind(x, h, v)[e] = iv;
            }
            abs_(x, h)[e] = red[12 + e];
        }
    }
};

// deterministic reduction of the masked slots of an NR-block over the group
AI void block_sum_mask(const Ctx& x, double* v, int nr, unsigned mask) {
    const Grp& g = x.g;
#if defined(__HIP_DEVICE_COMPILE__)
    UNR for (int e = 0; e < 18; e++) if (e < nr && ((mask >> e) & 1)) v[e] = wsum(v[e]);
    const int wave = g.tid >> 6, nw = (g.n + 63) >> 6;
    if ((g.tid & 63) == 0)
        UNR for (int e = 0; e < 18; e++) if (e < nr && ((mask >> e) & 1)) x.red[wave * 18 + e] = v[e];
    g.sync();
    UNR for (int e = 0; e < 18; e++) {
        if (e < nr && ((mask >> e) & 1)) {
            double s = x.red[e];
            for (int w = 1; w < nw; w++) s = s + x.red[w * 18 + e];
            v[e] = s;
        }
    }
    g.sync();
#else
    block_sum(x, v, nr);
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
// ---- N <= 64: wave 0 alone, keys and term values in registers ---------------------------------
#define SPHASE(k)                                                                                  \
    if (x.phase && lane == 0) {                                                                    \
        const long long c_ = clock64();                                                            \
        x.phase[k] += (unsigned long long)(c_ - ph_t);                                             \
        ph_t = c_;                                                                                 \
    }
template <class Pol>
__device__ inline __attribute__((always_inline)) void simplify_small(Ctx& x, int o, const Terms& T, const Pol& pol, int N) {
    constexpr int NV = Pol::NV, n = Pol::NO;
    const int lane = x.g.tid & 63;
    long long ph_t = x.phase ? clock64() : 0;
    uint64_t h = ~(uint64_t)0;
    double c[NV];
    if (lane < N) {
        h = T.hash(lane);
        pol.term(T, lane, c);
    } else {
        UNR for (int e = 0; e < NV; e++) c[e] = 0.0;
    }
    if (x.phase) { UNR for (int e = 0; e < NV; e++) h ^= (c[e] != c[e]) ? 1 : 0; }  // force the loads before the stamp
    SPHASE(8)
    uint32_t id = (uint32_t)lane;
    int P = 1;
    while (P < N) P <<= 1;
    UNR for (int lk = 1; lk <= 6; lk++) {
        const int k = 1 << lk;
        if (k > P) break;
        UNR for (int lj = lk - 1; lj >= 0; lj--) {
            const int j = 1 << lj;
            const uint64_t oh = xor_u64(h, j);
            const uint32_t oi = xor_u32(id, j);
            const bool asc = (lane & k) == 0, lower = (lane & j) == 0;
            const bool other_less = key_less(oh, oi, h, id);
            if ((lower == asc) ? other_less : !other_less) { h = oh; id = oi; }
        }
    }
    SPHASE(9)
    // term values follow their keys
    UNR for (int e = 0; e < NV; e++) c[e] = __shfl(c[e], (int)id, 64);
    const uint64_t prev = prev_u64(h);
    const bool head = lane < N && (lane == 0 || h != prev);
    const unsigned long long hm = __ballot(head);
    const unsigned long long above = lane < 63 ? (hm & ~((2ull << lane) - 1)) : 0ull;
    const int next = above ? __builtin_ctzll(above) : N;
    const int size = head ? next - lane : 0;
    const int maxg = wave_max(size);
    double acc[NV], t[NV];
    UNR for (int e = 0; e < NV; e++) { acc[e] = c[e]; t[e] = c[e]; }
    for (int st = 1; st < maxg; st++) {
        // t <- value of lane + 1: after st shifts lane q holds the term at q + st
        UNR for (int e = 0; e < NV; e++) t[e] = next_f64(t[e]);
        if (head && st < size) UNR for (int e = 0; e < NV; e++) acc[e] = acc[e] + t[e];
    }
    SPHASE(10)
    double red[Pol::NR], out[n];
    UNR for (int e = 0; e < Pol::NR; e++) red[e] = 0.0;
    UNR for (int e = 0; e < n; e++) out[e] = 0.0;
    const bool keep = head && pol.group(acc, out, red);
    if (!head) UNR for (int e = 0; e < Pol::NR; e++) red[e] = 0.0;
    const unsigned long long km = __ballot(keep);
    const int K = __popcll(km);
    const int pos = __popcll(km & ((1ull << lane) - 1));
    long hoff = 0, coff = 0;
    int ok = 0;
    if (lane == 0) {
        PZH& oh = x.H[o];
        arena_alloc_t0(x, oh, K, n);
        hoff = oh.hoff;
        coff = oh.coff;
        ok = oh.cnt == K;
        x.A->bytes += T.in_bytes() + (double)K * (8.0 + 8.0 * n);
    }
    hoff = bcast0(hoff);
    coff = bcast0(coff);
    ok = __builtin_amdgcn_readlane(ok, 0);
    if (ok && keep) {
        x.ah[hoff + pos] = h;
        double* dst = x.ac + coff + (long)pos * n;
        UNR for (int e = 0; e < n; e++) dst[e] = out[e];
    }
    SPHASE(11)
    const unsigned mask = pol.mask();
    UNR for (int e = 0; e < Pol::NR; e++) if ((mask >> e) & 1) red[e] = wsum(red[e]);
    if (lane == 0) pol.finish(x, o, red);
    SPHASE(12)
}

#endif



// ---- N > 64: whole group. Key order first (independent of the policy), then the group passes.
// Keys live in LDS up to its capacity, else in the workgroup's global buffers. Returns false (and
// flags the error) when even those are too small. Sources staged, caller's barrier done.
struct KeyBufs {
    uint64_t* kh;
    uint32_t* ki;
    int* kp;
};
AI bool order_keys(Ctx& x, const Terms& T, int N, KeyBufs& K) {
    const Grp& g = x.g;
    K.kh = x.kh; K.ki = x.ki; K.kp = x.kp;
    const bool in_lds = N <= x.cap_lds;
    if (!in_lds) {
        K.kh = x.gkh; K.ki = x.gki; K.kp = x.gkp;
        if (N > x.cap_glb) return false;
    }
    uint64_t* kh = K.kh;
    uint32_t* ki = K.ki;
    // order the keys by rank merge of the sorted runs: a key's place is the sum of its lower
    // bounds in the runs (Terms::rank). Measured against a register bitonic (the earlier path for
    // more than 6 runs) it is faster at every run count the program produces, and it needs no
    // padding, exchange buffers or sort registers.
    for (int p = g.tid; p < N; p += g.n) {
        const uint64_t h = T.hash(p);
        const int r = T.rank(p, h);
        kh[r] = h;
        ki[r] = (uint32_t)p;
    }
    g.sync();
    return true;
}

#if defined(__HIP_DEVICE_COMPILE__)
#define PHASE(k)                                                                                   \
    if (x.phase && g.tid == 0) {                                                                   \
        const long long c_ = clock64();                                                            \
        x.phase[k] += (unsigned long long)(c_ - ph_t);                                             \
        ph_t = c_;                                                                                 \
    }
#else
#define PHASE(k)
#endif

// group sums in term order, keep flags and pruned amounts, compaction, output (keys ordered)
template <class Pol>
AI void simplify_groups(Ctx& x, int o, const Terms& T, const Pol& pol, int N, const KeyBufs& K) {
    const Grp& g = x.g;
#if defined(__HIP_DEVICE_COMPILE__)
    long long ph_t = x.phase ? clock64() : 0;
#endif
    constexpr int NV = Pol::NV, n = Pol::NO;
    const uint64_t* kh = K.kh;
    const uint32_t* ki = K.ki;
    int* kp = K.kp;
    // pass 1: each group head sums its group in term order and parks the NV sums in gout (HBM,
    // by key position); only the keep flag goes on. No reduction slots are live here — the sum
    // loop is the register-heavy part (a 3x3 block product per term).
    double acc[NV], tmp[NV];
    for (int q = g.tid; q < N; q += g.n) {
        const bool head = q == 0 || kh[q] != kh[q - 1];
        int keep = 0;
        if (head) {
            pol.term(T, ki[q], acc);
            for (int r = q + 1; r < N && kh[r] == kh[q]; r++) {
                pol.term(T, ki[r], tmp);
                UNR for (int e = 0; e < NV; e++) acc[e] = acc[e] + tmp[e];
            }
            double o1[n], r1[Pol::NR];  // dead: the decision only
            UNR for (int e = 0; e < Pol::NR; e++) r1[e] = 0.0;
            keep = pol.group(acc, o1, r1) ? 1 : 0;
            UNR for (int e = 0; e < NV; e++) x.gout[(long)q * NV + e] = acc[e];
        }
        kp[q] = keep;
    }
    g.sync();
    PHASE(2)
    const int K_ = block_scan(x, kp, N);
    if (g.tid == 0) {
        arena_alloc_t0(x, x.H[o], K_, n);
        x.A->bytes += T.in_bytes() + (double)K_ * (8.0 + 8.0 * n);
    }
    g.sync();
    PHASE(3)
    // pass 2, same thread and q order as pass 1: the group decision again from the parked sums,
    // its pruned / kept amounts into the reduction slots (the order pass 1 would have used), and
    // the kept rows written at their compacted position
    const long hoff = x.H[o].hoff, coff = x.H[o].coff;
    const bool ok = x.H[o].cnt == K_;
    double red[Pol::NR], out[n];
    UNR for (int e = 0; e < Pol::NR; e++) red[e] = 0.0;
    for (int q = g.tid; q < N; q += g.n) {
        const bool head = q == 0 || kh[q] != kh[q - 1];
        if (!head) continue;
        UNR for (int e = 0; e < NV; e++) acc[e] = x.gout[(long)q * NV + e];
        UNR for (int e = 0; e < n; e++) out[e] = 0.0;
        const bool keep = pol.group(acc, out, red);
        if (keep && ok) {
            const long pos = kp[q];
            x.ah[hoff + pos] = kh[q];
            double* dst = x.ac + coff + pos * n;
            UNR for (int e = 0; e < n; e++) dst[e] = out[e];
        }
    }
    PHASE(4)
    block_sum_mask(x, red, Pol::NR, pol.mask());
    PHASE(5)
    if (g.tid == 0) pol.finish(x, o, red);
}

// ---- fused PZ x constant / constant x PZ cross products (PZsparse.cu:1118-1167) -----------------
// r_e = sA_e * a[iA_e] - sB_e * a[iB_e] (two scaled element views of the 3x1 source, subtracted,
// simplified), then stack(r0, r1, r2) simplified. The source's monomials map one to one (its hash
// order is kept), so no ordering is needed.
struct CrossC {
    int iA[3], iB[3];
    double sA[3], sB[3];
};
// kind 0: a x v (PZ x const), kind 1: v x a (const x PZ), as the reference's two overloads
AI CrossC cross_const_table(int kind, const double* v) {
    CrossC C;
    if (kind == 0) {
        C.iA[0] = 1; C.sA[0] = v[2]; C.iB[0] = 2; C.sB[0] = v[1];
        C.iA[1] = 2; C.sA[1] = v[0]; C.iB[1] = 0; C.sB[1] = v[2];
        C.iA[2] = 0; C.sA[2] = v[1]; C.iB[2] = 1; C.sB[2] = v[0];
    } else {
        C.iA[0] = 2; C.sA[0] = v[1]; C.iB[0] = 1; C.sB[0] = v[2];
        C.iA[1] = 0; C.sA[1] = v[2]; C.iB[1] = 2; C.sB[1] = v[0];
        C.iA[2] = 1; C.sA[2] = v[0]; C.iB[2] = 0; C.sB[2] = v[1];
    }
    return C;
}
// one source monomial m -> output row; red: [0,3) difference prunes, [3,6) stack prunes, [6,9) absum
AI bool cross_const_mono(const CrossC& C, const double* m, double thr, double* out, double* red) {
    double vec[3];
    bool any = false;
    UNR for (int e = 0; e < 3; e++) {
        const double xa = C.sA[e] * pick3(m, C.iA[e]);
        const double xb = -(C.sB[e] * pick3(m, C.iB[e]));
        const double v = xa + xb;
        bool have = true;
        if (!(frob1(v) > thr)) { red[e] = red[e] + fabs(v); have = false; }
        vec[e] = have ? v : 0.0;
        any = any || have;
    }
    if (!any) return false;
    if (!(frob_norm(vec, 3) > thr)) {
        UNR for (int e = 0; e < 3; e++) red[3 + e] = red[3 + e] + fabs(vec[e]);
        return false;
    }
    UNR for (int e = 0; e < 3; e++) { out[e] = vec[e]; red[6 + e] = red[6 + e] + fabs(vec[e]); }
    return true;
}
// header: views (t0_view), differences (PZsparse.cu:813-834), stack, each plus its pruned amount
AI void cross_const_finish(const Ctx& x, PZH& h, const PZH& A, const CrossC& C, const double* red) {
    double sred[3];
    UNR for (int e = 0; e < 3; e++) sred[e] = red[3 + e];
    const bool sadd = frob_norm(sred, 3) != 0;
    UNR for (int e = 0; e < 3; e++) {
        cen(x, h)[e] = pick3(cen(x, A), C.iA[e]) * C.sA[e] - pick3(cen(x, A), C.iB[e]) * C.sB[e];
        UNR for (int v = 0; v < 2; v++) {
            double iv = pick3(ind(x, A, v), C.iA[e]) * fabs(C.sA[e]) + pick3(ind(x, A, v), C.iB[e]) * fabs(C.sB[e]);
            if (frob1(red[e]) != 0) iv = iv + red[e];
            if (sadd) iv = iv + sred[e];
            ind(x, h, v)[e] = iv;
        }
        abs_(x, h)[e] = red[6 + e];
    }
}

// the whole op; the header of o (3x1) is initialised by the caller's thread 0; ends without barrier
AI void cross_const(Ctx& x, int o, int a, const CrossC& C) {
    const Grp& g = x.g;
    const PZH& A = x.H[a];
    const int N = A.cnt;
    const Src S = src_of(x, A);
    double red[9], out[9], m[9];
    UNR for (int e = 0; e < 9; e++) { red[e] = 0.0; out[e] = 0.0; }
#if defined(__HIP_DEVICE_COMPILE__)
    if (N <= 64) {
        if (g.tid >= 64) return;
        const int lane = g.tid;
        bool keep = false;
        if (lane < N) {
            S.read(lane, false, m);
            keep = cross_const_mono(C, m, x.thr, out, red);
        }
        const unsigned long long km = __ballot(keep);
        const int K = __popcll(km);
        const int pos = __popcll(km & ((1ull << lane) - 1));
        long hoff = 0, coff = 0;
        int ok = 0;
        if (lane == 0) {
            PZH& oh = x.H[o];
            arena_alloc_t0(x, oh, K, 3);
            hoff = oh.hoff;
            coff = oh.coff;
            ok = oh.cnt == K;
            x.A->bytes += (double)N * 32.0 + (double)K * 32.0;
        }
        hoff = bcast0(hoff);
        coff = bcast0(coff);
        ok = __builtin_amdgcn_readlane(ok, 0);
        if (ok && keep) {
            x.ah[hoff + pos] = S.h[lane];
            double* dst = x.ac + coff + (long)pos * 3;
            UNR for (int e = 0; e < 3; e++) dst[e] = out[e];
        }
        UNR for (int e = 0; e < 9; e++) red[e] = wsum(red[e]);
        if (lane == 0) cross_const_finish(x, x.H[o], A, C, red);
        return;
    }
#endif
    int* kp = N <= x.cap_lds ? x.kp : x.gkp;
    if (N > x.cap_lds && N > x.cap_glb) {
        if (g.tid == 0) { *x.err |= ERR_SORTCAP; x.H[o].cnt = 0; }
        return;
    }
    for (int k = g.tid; k < N; k += g.n) {
        S.read(k, false, m);
        kp[k] = cross_const_mono(C, m, x.thr, out, red) ? 1 : 0;
    }
    g.sync();
    const int K = block_scan(x, kp, N);
    if (g.tid == 0) {
        arena_alloc_t0(x, x.H[o], K, 3);
        x.A->bytes += (double)N * 32.0 + (double)K * 32.0;
    }
    g.sync();
    const long hoff = x.H[o].hoff, coff = x.H[o].coff;
    if (x.H[o].cnt == K) {
        double dummy[9];
        for (int k = g.tid; k < N; k += g.n) {
            const bool keep = (k + 1 < N) ? (kp[k + 1] != kp[k]) : (kp[k] != K);
            if (!keep) continue;
            S.read(k, false, m);
            UNR for (int e = 0; e < 9; e++) dummy[e] = 0.0;
            cross_const_mono(C, m, x.thr, out, dummy);
            const long pos = kp[k];
            x.ah[hoff + pos] = S.h[k];
            double* dst = x.ac + coff + pos * 3;
            UNR for (int e = 0; e < 3; e++) dst[e] = out[e];
        }
    }
    block_sum_mask(x, red, 9, 0x1ff);
    if (g.tid == 0) cross_const_finish(x, x.H[o], A, C, red);
}

// header of an empty R x C PZ; the slot's payload class must be R*C (the program builder's shape
// classes guarantee it). Keeps `off`.
AI void hdr_init(const Ctx& x, PZH& h, int R, int C) {
    h.R = R; h.C = C; h.cnt = 0; h.stride = R * C; h.hoff = 0; h.coff = 0;
    h.comp = -1; h.scaled = 0; h.scale = 1.0;
    double* p = cen(x, h);
    const int n = R * C;
    UNR for (int e = 0; e < 36; e++) if (e < 4 * n) p[e] = 0.0;
}

// ---------------------------------------------------------------------------------------------
// operators: term list (all threads, uniform) and output header (thread 0: the operator's own
// centre / independent formula). Operands are never aliased by the output (the program builder
// allocates SSA-style slots).

// a + b (sign = +1) or a - b (sign = -1)  (PZsparse.cu:743-764, 813-834)
AI void terms_add(const Ctx& x, int a, int b, int sign, Terms& T) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    T.kind = 1; T.ns = 2;
    T.S[0] = src_of(x, A); T.S[1] = src_of(x, B);
    T.places = 0;
    T.negs = sign < 0 ? 2 : 0;
    T.nout = nel(A);
}
AI void header_add(Ctx& x, int o, int a, int b, int sign) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    PZH& h = x.H[o];
    hdr_init(x, h, A.R, A.C);
    const int n = nel(A);
    UNR for (int e = 0; e < 9; e++) {
        if (e < n) {
            cen(x, h)[e] = sign > 0 ? cen(x, A)[e] + cen(x, B)[e] : cen(x, A)[e] - cen(x, B)[e];
            ind(x, h, 0)[e] = ind(x, A, 0)[e] + ind(x, B, 0)[e];
            ind(x, h, 1)[e] = ind(x, A, 1)[e] + ind(x, B, 1)[e];
        }
    }
}

// a * b  (PZsparse.cu:864-994)
AI void terms_mul(const Ctx& x, int a, int b, Terms& T) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    T.kind = 0; T.ns = 2;
    T.places = 0; T.negs = 0;
    T.S[0] = src_of(x, A); T.S[1] = src_of(x, B);
    T.Ac = cen(x, A); T.Bc = cen(x, B);
    T.AR = A.R; T.AC = A.C; T.BC = B.C;
    T.nbm = B.cnt > 1 ? 0xFFFFFFFFu / (uint32_t)B.cnt + 1u : 0u;
    const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
    T.nout = as ? nel(B) : (bs ? nel(A) : A.R * B.C);
}
// centre, then the dual independent part
//   ind = A.ind B.ind + (|A.c| + sum|a_i|) B.ind + A.ind (|B.c| + sum|b_j|)
AI void header_mul(Ctx& x, int o, int a, int b, const Terms& T) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
    PZH& h = x.H[o];
    hdr_init(x, h, as ? B.R : A.R, as ? B.C : (bs ? A.C : B.C));
    const int na = nel(A), nb = nel(B), nr = nel(h);
    double cv[9], ac[9], bc[9], r2[9], r3[9];
    UNR for (int e = 0; e < 9; e++) {
        ac[e] = cen(x, A)[e];
        bc[e] = cen(x, B)[e];
        r2[e] = e < na ? fabs(cen(x, A)[e]) + abs_(x, A)[e] : 0.0;
        r3[e] = e < nb ? fabs(cen(x, B)[e]) + abs_(x, B)[e] : 0.0;
    }
    T.prod(ac, bc, cv);
    UNR for (int e = 0; e < 9; e++) if (e < nr) cen(x, h)[e] = cv[e];
    UNR for (int v = 0; v < 2; v++) {
        double ai[9], bi[9], t2[9], t3[9], ii[9];
        UNR for (int e = 0; e < 9; e++) { ai[e] = ind(x, A, v)[e]; bi[e] = ind(x, B, v)[e]; }
        if (as) {
            UNR for (int e = 0; e < 9; e++) { t2[e] = r2[0] * bi[e]; t3[e] = ai[0] * r3[e]; ii[e] = ai[0] * bi[e]; }
        } else if (bs) {
            UNR for (int e = 0; e < 9; e++) { t2[e] = r2[e] * bi[0]; t3[e] = ai[e] * r3[0]; ii[e] = ai[e] * bi[0]; }
        } else {
            matmul(r2, A.R, A.C, bi, B.C, t2);
            matmul(ai, A.R, A.C, r3, B.C, t3);
            matmul(ai, A.R, A.C, bi, B.C, ii);
        }
        UNR for (int e = 0; e < 9; e++) if (e < nr) ind(x, h, v)[e] = ii[e] + (t2[e] + t3[e]);
    }
    if (as && !bs && B.R != 1 && A.cnt > 0 && B.cnt > 0) *x.err |= ERR_HANDLES;  // Eigen assert in the reference
    if (!as && !bs && !(A.R == 3 && A.C == 3 && B.R == 3)) *x.err |= ERR_HANDLES;  // block shape outside matmul()
}

// ---- element-parallel headers: lane e < R*C of wave 0 computes output element e (the same
// arithmetic, element for element, as the serial formulas above); lane 0 also writes the meta.
AI void set_meta(PZH& h, int R, int C) {
    h.R = R; h.C = C; h.cnt = 0; h.stride = R * C; h.hoff = 0; h.coff = 0;
    h.comp = -1; h.scaled = 0; h.scale = 1.0;
}

AI void header_add_par(Ctx& x, int o, int a, int b, int sign, int e) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    PZH& h = x.H[o];
    const int n = nel(A);
    if (e == 0) set_meta(h, A.R, A.C);
    if (e >= n) return;
    const double* pa = x.pool + A.off;
    const double* pb = x.pool + B.off;
    double* ph = x.pool + h.off;
    ph[e] = sign > 0 ? pa[e] + pb[e] : pa[e] - pb[e];
    ph[n + e] = pa[n + e] + pb[n + e];
    ph[2 * n + e] = pa[2 * n + e] + pb[2 * n + e];
    ph[3 * n + e] = 0.0;
}

AI void header_mul_par(Ctx& x, int o, int a, int b, int e) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    PZH& h = x.H[o];
    const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
    const int R = as ? B.R : A.R, C = as ? B.C : (bs ? A.C : B.C), nr = R * C;
    const int na = nel(A), nb = nel(B);
    if (e == 0) {
        set_meta(h, R, C);
        if (as && !bs && B.R != 1 && A.cnt > 0 && B.cnt > 0) *x.err |= ERR_HANDLES;  // Eigen assert in the reference
        if (!as && !bs && !(A.R == 3 && A.C == 3 && B.R == 3)) *x.err |= ERR_HANDLES;  // block shape outside matmul()
    }
    if (e >= nr) return;
    const double* Ac = x.pool + A.off;
    const double* Bc = x.pool + B.off;
    const double* Aa = Ac + 3 * na;
    const double* Ba = Bc + 3 * nb;
    double* ph = x.pool + h.off;
    // centre (prod), then ind_v = A.ind B.ind + (|A.c| + sum|a_i|) B.ind + A.ind (|B.c| + sum|b_j|)
    if (as) {
        ph[e] = Ac[0] * Bc[e];
        const double r2 = fabs(Ac[0]) + Aa[0], r3 = fabs(Bc[e]) + Ba[e];
        UNR for (int v = 0; v < 2; v++) {
            const double ai = Ac[(1 + v) * na], bi = Bc[(1 + v) * nb + e];
            ph[(1 + v) * nr + e] = ai * bi + (r2 * bi + ai * r3);
        }
    } else if (bs) {
        ph[e] = Ac[e] * Bc[0];
        const double r2 = fabs(Ac[e]) + Aa[e], r3 = fabs(Bc[0]) + Ba[0];
        UNR for (int v = 0; v < 2; v++) {
            const double ai = Ac[(1 + v) * na + e], bi = Bc[(1 + v) * nb];
            ph[(1 + v) * nr + e] = ai * bi + (r2 * bi + ai * r3);
        }
    } else {
        // 3x3 times 3xC, column-major element (i, j), inner index summed in order (matmul())
        const int i = e % 3, j = e / 3;
        ph[e] = (Ac[i] * Bc[3 * j] + Ac[i + 3] * Bc[3 * j + 1]) + Ac[i + 6] * Bc[3 * j + 2];
        double r2[3], r3[3];
        UNR for (int k = 0; k < 3; k++) {
            r2[k] = fabs(Ac[i + 3 * k]) + Aa[i + 3 * k];
            r3[k] = fabs(Bc[k + 3 * j]) + Ba[k + 3 * j];
        }
        UNR for (int v = 0; v < 2; v++) {
            const double* Ai = Ac + (1 + v) * na;
            const double* Bi = Bc + (1 + v) * nb;
            const double t2 = (r2[0] * Bi[3 * j] + r2[1] * Bi[3 * j + 1]) + r2[2] * Bi[3 * j + 2];
            const double t3 = (Ai[i] * r3[0] + Ai[i + 3] * r3[1]) + Ai[i + 6] * r3[2];
            const double ii = (Ai[i] * Bi[3 * j] + Ai[i + 3] * Bi[3 * j + 1]) + Ai[i + 6] * Bi[3 * j + 2];
            ph[(1 + v) * nr + e] = ii + (t2 + t3);
        }
    }
    ph[3 * nr + e] = 0.0;
}

AI void header_stack3_par(Ctx& x, int o, int a0, int a1, int a2, int e) {
    PZH& h = x.H[o];
    if (e == 0) set_meta(h, 3, 1);
    if (e >= 3) return;
    const PZH& S = x.H[e == 0 ? a0 : (e == 1 ? a1 : a2)];
    const double* ps = x.pool + S.off;
    double* ph = x.pool + h.off;
    ph[e] = ps[0];
    ph[3 + e] = ps[1];
    ph[6 + e] = ps[2];
    ph[9 + e] = 0.0;
}

AI void header_add_one_dim_par(Ctx& x, int o, int self, int a, int pos, int e) {
    const PZH& A = x.H[self];
    const PZH& B = x.H[a];
    PZH& h = x.H[o];
    const int n = nel(A);
    if (e == 0) set_meta(h, A.R, A.C);
    if (e >= n) return;
    const double* pa = x.pool + A.off;
    const double* pb = x.pool + B.off;
    double* ph = x.pool + h.off;
    const bool at = e == pos;
    ph[e] = at ? pa[e] + pb[0] : pa[e];
    ph[n + e] = at ? pa[n + e] + pb[1] : pa[n + e];
    ph[2 * n + e] = at ? pa[2 * n + e] + pb[2] : pa[2 * n + e];
    ph[3 * n + e] = 0.0;
}

// fused PZ x PZ cross: the term list of the six 1x1 products is the product term list of the two
// full 3x1 operands (hashes only; PolCrossPP evaluates the coefficients)
AI void terms_cross_pp(const Ctx& x, int a, int b, Terms& T) {
    const PZH& A = x.H[a];
    const PZH& B = x.H[b];
    T.kind = 0; T.ns = 2;
    T.places = 0; T.negs = 0;
    T.S[0] = src_of(x, A); T.S[1] = src_of(x, B);
    T.Ac = cen(x, A); T.Bc = cen(x, B);
    T.AR = 3; T.AC = 1; T.BC = 1;
    T.nbm = B.cnt > 1 ? 0xFFFFFFFFu / (uint32_t)B.cnt + 1u : 0u;
    T.nout = 3;
}

// stack three 1x1 PZs into a 3x1 (PZsparse.cu:1087-1116)
AI void terms_stack3(const Ctx& x, int a0, int a1, int a2, Terms& T) {
    T.kind = 1; T.ns = 3;
    T.S[0] = src_of(x, x.H[a0]); T.S[1] = src_of(x, x.H[a1]); T.S[2] = src_of(x, x.H[a2]);
    T.places = 1 | (2 << 4) | (3 << 8);
    T.negs = 0;
    T.nout = 3;
}
AI void header_stack3(Ctx& x, int o, int a0, int a1, int a2) {
    const PZH& S0 = x.H[a0];
    const PZH& S1 = x.H[a1];
    const PZH& S2 = x.H[a2];
    PZH& h = x.H[o];
    hdr_init(x, h, 3, 1);
    cen(x, h)[0] = cen(x, S0)[0]; ind(x, h, 0)[0] = ind(x, S0, 0)[0]; ind(x, h, 1)[0] = ind(x, S0, 1)[0];
    cen(x, h)[1] = cen(x, S1)[0]; ind(x, h, 0)[1] = ind(x, S1, 0)[0]; ind(x, h, 1)[1] = ind(x, S1, 1)[0];
    cen(x, h)[2] = cen(x, S2)[0]; ind(x, h, 0)[2] = ind(x, S2, 0)[0]; ind(x, h, 1)[2] = ind(x, S2, 1)[0];
}

// self(e) += a (1x1)  (PZsparse.cu:1068-1085)
AI void terms_add_one_dim(const Ctx& x, int self, int a, int e, Terms& T) {
    const PZH& A = x.H[self];
    T.kind = 1; T.ns = 2;
    T.S[0] = src_of(x, A); T.S[1] = src_of(x, x.H[a]);
    T.places = (e + 1) << 4;
    T.negs = 0;
    T.nout = nel(A);
}
AI void header_add_one_dim(Ctx& x, int o, int self, int a, int e) {
    const PZH& A = x.H[self];
    const PZH& B = x.H[a];
    PZH& h = x.H[o];
    hdr_init(x, h, A.R, A.C);
    const int n = nel(A);
    UNR for (int q = 0; q < 9; q++) {
        if (q >= n) break;
        const bool at = q == e;
        cen(x, h)[q] = at ? cen(x, A)[q] + cen(x, B)[0] : cen(x, A)[q];
        ind(x, h, 0)[q] = at ? ind(x, A, 0)[q] + ind(x, B, 0)[0] : ind(x, A, 0)[q];
        ind(x, h, 1)[q] = at ? ind(x, A, 1)[q] + ind(x, B, 1)[0] : ind(x, A, 1)[q];
    }
}

}  // namespace armour
