// armour-mi355x — bundle engine: the reach program (reach.h) for 64 jobs at once, lane = job.
//
// The monomial *structure* of a PZ (which hashes it holds, in hash order) depends on the job only
// through the simplify() prunes (KPR/PZsparse.cu:284-350), and neighbouring jobs of a world prune
// almost alike: over 64 consecutive (world, interval) jobs the union of the hash lists is 1.2-1.5x
// one job's. So a bundle of 64 jobs carries one union hash list per handle plus a 64-bit presence
// mask per monomial (bit l: job l holds it), and coefficients as [row][64 lanes] doubles. A job that
// lacks a union monomial has zeros there, which every operator maps to exact zeros (x + 0 = x,
// 0 * y = 0): a group that no present term feeds sums to zero and is pruned with |0| = 0 added, so
// every lane computes exactly its own job's values, in its own job's term order (the union order
// restricted to one job's terms is that job's order). Presence masks only decide which monomials
// the link / torque emits hand on.
//
// Everything that the per-job engine (pz_engine.h) does once per job — term hashes, the rank-merge
// key order, group heads, compaction scans — happens once per bundle here; the coefficient
// arithmetic is lane-parallel with coalesced 512-byte row accesses, and the thread-0 ops of the
// per-job engine (1-D PZs, rotations, emits, torque radius) become plain lane code.
#pragma once
#include "reach.h"

namespace armour {
namespace lane {

constexpr int LG = 64;  // jobs per bundle = lanes per wave

#ifndef LANE_CFG_WAVES
#define LANE_CFG_WAVES 4
#endif
constexpr int LW = LANE_CFG_WAVES;        // waves per workgroup
constexpr int LT = LW * LG;               // threads per workgroup
constexpr int RCH = 6;                    // reduction slots combined per round across waves
// groups per wave round of each generator (round width LW x U; lane_variant experiments; DESIGN.md
// section 4 has the round-5 sweep: the defaults are the fastest measured)
#ifndef LANE_U99
#define LANE_U99 1                        // 3x3 x 3x3 product
#endif
#ifndef LANE_U93
#define LANE_U93 3                        // 3x3 x 3x1 product
#endif
#ifndef LANE_U13
#define LANE_U13 4                        // 1x1 x 3x1 product
#endif
#ifndef LANE_UX
#define LANE_UX 3                         // fused 3x1 x 3x1 cross product
#endif
#ifndef LANE_UC3
#define LANE_UC3 4                        // concatenations of 1- / 3-element blocks
#endif
#ifndef LANE_UC9
#define LANE_UC9 2                        // concatenations of 3x3 blocks
#endif

#define DI __device__ inline __attribute__((always_inline))
// Explicit address spaces for the simplify round loop: a pointer the
// compiler cannot prove to be LDS or global becomes a flat access, which counts in both vmcnt and
// lgkmcnt, so every LDS index read of a round waited for all of the wave's outstanding HBM loads and
// stores. Key and group-head reads are LDS-typed (ds_read, lgkmcnt only), coefficient rows
// global-typed (global_load / global_store, vmcnt only).
#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
template <class T>
DI GAS T* gas(T* p) { return (GAS T*)p; }
template <class T>
DI GAS const T* gas(const T* p) { return (GAS const T*)p; }

// bundle handle (LDS): union structure + where the lane data lives
struct LH {
    int R, C;
    int cnt;       // union monomials
    int stride;    // coefficient rows per monomial (parent's R*C for views)
    long hoff;     // hash / mask index
    long coff;     // first coefficient row; row r of lane l is c[r * LG + l]
    int comp;      // element view (>= 0) of the parent's block
    int scaled;
    double scale;
    int off;       // header payload rows in the pool: centre[n], ind0[n], ind1[n], absum[n]
};

struct LArena {
    uint64_t* h;   // union hashes
    uint64_t* m;   // presence masks
    double* c;     // coefficient rows [row][LG]
    long hcap, ccap;
    long hused, cused;
    long hmark, cmark;          // allocation marks of the simplify in flight
    unsigned long long bytes;  // algorithmic monomial bytes of the bundle's jobs
};

struct LCtx {
    int tid, wave, lane;
    LH* H;
    double* pool;          // HBM: [pool rows][LG]
    LArena* A;             // LDS
    uint64_t* kh;          // LDS keys (cap_lds), else the global buffers (cap_glb)
    uint32_t* ki;
    int* kp;
    int* gp;
    LAS uint64_t* lkh;     // the same LDS arrays, LDS-typed (the round loop's reads)
    LAS uint32_t* lki;
    LAS int* lgp;
    int cap_lds;
    uint64_t* gkh;
    uint32_t* gki;
    int* gkp;
    int* ggp;
    int cap_glb;
    double* gout;          // HBM [cap_out][9][LG]: kept group values between the two passes
    uint64_t* gm;          // HBM [cap_out]: group keep masks
    int cap_out;
    uint64_t* rmask;       // LDS [2][64]: keep masks of a simplify round (double-buffered)
    uint64_t* stage;       // LDS staged operand hashes
    int stage_cap;
    double* red;           // LDS [(LW - 1) * RCH][LG]
    double* scr;           // [2 * NF][LG] (pool rows): per-job disturbance / reduce radii
    int* iscan;            // LDS [LW]
    int* err;              // LDS
    int* occ;              // LDS [4]: largest operator term count, link / torque k-only monomials,
                           // arena coefficient rows in use
    double thr;
    const JrsJoint* jrs;   // this lane's job: jrs[i], i < NF
    unsigned long long* prof;  // optional per-op [cycles, terms] + phase cycles (null: off)
    int nops;
    int opcode;            // code of the op in flight (phase profile per code)
    long job;              // this lane's job index (clamped into range)
    bool valid;            // lane's job exists (the last bundle may be partial)
};

// Instrumentation (per-op cycles, simplify phase and round stamps, bundle wall clock) is compiled in
// only with -DLANE_PROF=1 (make lane_variant LW=4 LX=_prof EXTRA=-DLANE_PROF=1): its counters and
// time stamps otherwise stay live across the round loop and cost registers the product build needs.
#ifndef LANE_PROF
#define LANE_PROF 0
#endif

DI void sync() { __syncthreads(); }
// phase stamps (profiling): thread 0 adds the cycles since the last stamp to prof[2 * nops + k]
#define LPHASE(k)                                                                                  \
    if (x.prof && x.tid == 0) {                                                                    \
        const long long c_ = clock64();                                                            \
        atomicAdd(&x.prof[2 * x.nops + 16 + 8 * x.opcode + (k)], (unsigned long long)(c_ - ph_t));  \
        ph_t = c_;                                                                                 \
    }
DI long bcast0(long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (long)(((uint64_t)hi << 32) | lo);
}
DI unsigned long long ballot(bool p) { return __ballot(p); }
// wave-uniform copies (SGPRs) of values every lane holds alike (read from LDS tables)
DI int ui(int v) { return __builtin_amdgcn_readfirstlane(v); }
DI uint32_t uu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
DI double ud(double v) { return __builtin_bit_cast(double, bcast0(__builtin_bit_cast(long, v))); }
template <class T>
DI T* up(T* p) { return (T*)(uintptr_t)bcast0((long)(uintptr_t)p); }
// a wave-uniform value the optimiser cannot see through (readfirstlane, then an empty asm on the
// scalar register)
DI int opaque(int v) {
    int r = __builtin_amdgcn_readfirstlane(v);
    __asm__ volatile("" : "+s"(r));
    return r;
}
DI long opaque(long v) {
    long r = bcast0(v);
    __asm__ volatile("" : "+s"(r));
    return r;
}
DI double opaque(double v) { return __builtin_bit_cast(double, opaque(__builtin_bit_cast(long, v))); }
template <class T>
DI const T* opaque(const T* p) { return (const T*)(uintptr_t)opaque((long)(uintptr_t)p); }
template <class T>
DI GAS const T* opaque(GAS const T* p) { return (GAS const T*)(uintptr_t)opaque((long)(uintptr_t)p); }

// per-lane header rows
DI double& P(const LCtx& x, int row) { return x.pool[(long)row * LG + x.lane]; }
DI int nel(const LH& h) { return h.R * h.C; }
DI double& cen(const LCtx& x, const LH& h, int e) { return P(x, h.off + e); }
DI double& ind(const LCtx& x, const LH& h, int v, int e) { return P(x, h.off + (1 + v) * nel(h) + e); }
DI double& abs_(const LCtx& x, const LH& h, int e) { return P(x, h.off + 3 * nel(h) + e); }

DI void err_or(const LCtx& x, int bits) { atomicOr(x.err, bits); }

// meta of an empty R x C handle (one lane writes; the slot keeps its payload offset)
DI void set_meta(LH& h, int R, int C) {
    h.R = R; h.C = C; h.cnt = 0; h.stride = R * C; h.hoff = 0; h.coff = 0;
    h.comp = -1; h.scaled = 0; h.scale = 1.0;
}
// zero this lane's header of an R x C handle (payload rows of class R*C)
DI void hdr_zero(const LCtx& x, int off, int n) {
    for (int q = 0; q < 4 * n; q++) x.pool[(long)(off + q) * LG + x.lane] = 0.0;
}

// union monomial storage for K monomials of `stride` rows, allocated by one lane (atomics: lane
// ops of several waves allocate concurrently). Returns false on overflow (error flagged, cnt 0).
DI bool arena_alloc(const LCtx& x, LH& h, int K, int stride) {
    const long h0 = (long)atomicAdd((unsigned long long*)&x.A->hused, (unsigned long long)K);
    const long c0 = (long)atomicAdd((unsigned long long*)&x.A->cused, (unsigned long long)K * stride);
    h.stride = stride;
    atomicMax(&x.occ[3], (int)min(c0 + (long)K * stride, (long)INT_MAX));
    if (h0 + K > x.A->hcap || c0 + (long)K * stride > x.A->ccap) {
        err_or(x, ERR_ARENA);
        h.cnt = 0; h.hoff = 0; h.coff = 0;
        return false;
    }
    h.hoff = h0;
    h.coff = c0;
    h.cnt = K;
    return true;
}

// ---- operand view for term generation ------------------------------------------------------
struct LSrc {
    const uint64_t* h;   // hashes (LDS stage or arena)
    const uint64_t* m;   // presence masks (arena)
    const double* c;     // arena rows of monomial 0
    int cnt, n, stride, comp, scaled;
    double scale;
    DI uint64_t hash(int k) const { return h[k]; }
    // branch-free: nine loads from rows inside monomial k's block (clamped), then the selects
    DI void read(int k, bool neg, double* out, int lane) const {
        const double* base = c + (long)k * stride * LG + lane;
        double xs[9];
#pragma unroll
        for (int e = 0; e < 9; e++) xs[e] = base[(long)(comp >= 0 ? comp : (e < n ? e : 0)) * LG];
#pragma unroll
        for (int e = 0; e < 9; e++) {
            double v = xs[e];
            if (scaled) v = scale * v;
            if (neg) v = -v;
            out[e] = e < n ? v : 0.0;
        }
    }
};
DI LSrc src_of(const LCtx& x, const LH& p) {
    LSrc s;
    const long hoff = bcast0(p.hoff), coff = bcast0(p.coff);
    s.h = up(x.A->h) + hoff;
    s.m = up(x.A->m) + hoff;
    s.c = up(x.A->c) + coff * LG;
    s.cnt = ui(p.cnt);
    s.n = ui(p.R * p.C);
    s.stride = ui(p.stride);
    s.comp = ui(p.comp);
    s.scaled = ui(p.scaled);
    s.scale = ud(p.scale);
    return s;
}

// term list of an operator over the union lists (same layout as pz_engine.h Terms): kind 0 =
// product (T1 a_i x B.c, T2 A.c x b_j, T3 a_i x b_j), kind 1 = concatenation of up to 3 sources
struct LTerms {
    int kind, ns;
    LSrc S[3];
    int places, negs;
    int AR, AC, BC;
    int nout;
    uint32_t nbm;
    double Ac[9], Bc[9];  // this lane's operand centres (products)
    DI void split(int q, int& i, int& j) const {
        const int nb = S[1].cnt;
        i = nb == 1 ? q : (int)__umulhi((uint32_t)q, nbm);
        j = q - i * nb;
    }
    DI void which(int p, int& s, int& k) const {
        s = 0;
        if (p >= S[0].cnt) { p -= S[0].cnt; s = 1; if (p >= S[1].cnt) { p -= S[1].cnt; s = 2; } }
        k = p;
    }
    DI uint64_t hash(int p) const {
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
    DI void prod(const double* a, const double* b, double* out) const {
        const bool as = AR == 1 && AC == 1, bs = S[1].n == 1;
        if (as) {
#pragma unroll
            for (int e = 0; e < 9; e++) out[e] = a[0] * b[e];
        } else if (bs) {
#pragma unroll
            for (int e = 0; e < 9; e++) out[e] = a[e] * b[0];
        } else {
            matmul(a, AR, AC, b, BC, out);
        }
    }
    // operand rows of term p for this lane: u = left factor, w = right factor (products)
    DI void factors(int p, double* u, double* w, int lane) const {
        const int na = S[0].cnt, nb = S[1].cnt;
        if (p < na) {
            S[0].read(p, false, u, lane);
#pragma unroll
            for (int e = 0; e < 9; e++) w[e] = Bc[e];
        } else if (p < na + nb) {
#pragma unroll
            for (int e = 0; e < 9; e++) u[e] = Ac[e];
            S[1].read(p - na, false, w, lane);
        } else {
            int i, j;
            split(p - na - nb, i, j);
            S[0].read(i, false, u, lane);
            S[1].read(j, false, w, lane);
        }
    }
    DI void coef(int p, double* out, int lane) const {
        if (kind == 0) {
            double a[9], b[9];
            factors(p, a, b, lane);
            prod(a, b, out);
            return;
        }
        int s, k;
        which(p, s, k);
        const bool ng = (negs >> s) & 1;
        if (s == 0) S[0].read(k, ng, out, lane);
        else if (s == 1) S[1].read(k, ng, out, lane);
        else S[2].read(k, ng, out, lane);
        const int pl = ((places >> (4 * s)) & 15) - 1;
        if (pl >= 0) {
            const double v = out[0];
#pragma unroll
            for (int e = 0; e < 9; e++) out[e] = (e == pl) ? v : 0.0;
        }
    }
    DI int rank(int p, uint64_t h) const {
        // as pz_engine.h Terms::rank: preceding runs count keys <= h, following runs keys < h
        const uint64_t h1 = h + 1;
        if (kind == 1) {
            int s, k;
            which(p, s, k);
            int r = k;
#pragma unroll
            for (int t = 0; t < 3; t++)
                if (t < ns && t != s) r += lower_bound(S[t].h, S[t].cnt, t < s ? h1 : h);
            return r;
        }
        const int na = S[0].cnt, nb = S[1].cnt;
        const int base = na + nb;
        const int seg = p < na ? 0 : (p < base ? 1 : 2);
        int r = seg == 0 ? p : lower_bound(S[0].h, na, h1);
        r += seg == 1 ? p - na : lower_bound(S[1].h, nb, seg == 2 ? h1 : h);
        if (na <= nb) {
            int i0 = -1, j0 = 0;
            if (seg == 2) split(p - base, i0, j0);
            for (int i = 0; i < na; i++)
                r += i == i0 ? j0 : lower_bound_off(S[1].h, nb, S[0].h[i], i < i0 ? h1 : h);
        } else {
            for (int j = 0; j < nb; j++) {
                const uint64_t hbj = S[1].h[j];
                int lb = lower_bound_col(S[0].h, na, hbj, h);
                if (lb < na && S[0].h[lb] + hbj == h && base + lb * nb + j < p) lb++;
                r += lb;
            }
        }
        return r;
    }
};

// ---- block primitives (all LT threads) -------------------------------------------------------
// exclusive scan of kp[0..N) in place; returns the total; ends with a barrier
DI int block_scan(const LCtx& x, int* kp, int N) {
    const int chunk = (N + LT - 1) / LT;
    const int lo = x.tid * chunk, hi = (lo + chunk < N) ? lo + chunk : N;
    int s = 0;
    for (int i = lo; i < hi; i++) s += kp[i];
    const int inc = wave_incl_scan(s);
    if (x.lane == 63) x.iscan[x.wave] = inc;
    sync();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < LW; w++) {
        const int t = x.iscan[w];
        if (w < x.wave) base += t;
        total += t;
    }
    int run = base + inc - s;
    for (int i = lo; i < hi; i++) { const int v = kp[i]; kp[i] = run; run += v; }
    sync();
    return total;
}

// per-lane reduction slots of all waves into wave 0, in wave order (deterministic); wave 0's
// red[] holds the totals afterwards. Every thread must call it (barriers inside).
template <int NR>
DI void combine_red(const LCtx& x, double* red) {
#pragma unroll
    for (int r0 = 0; r0 < NR; r0 += RCH) {
        if (x.wave > 0) {
#pragma unroll
            for (int e = 0; e < RCH; e++)
                if (r0 + e < NR) x.red[((long)(x.wave - 1) * RCH + e) * LG + x.lane] = red[r0 + e];
        }
        sync();
        if (x.wave == 0) {
#pragma unroll
            for (int e = 0; e < RCH; e++)
                if (r0 + e < NR)
                    for (int w = 1; w < LW; w++) red[r0 + e] = red[r0 + e] + x.red[((long)(w - 1) * RCH + e) * LG + x.lane];
        }
        sync();
    }
}

// the sources' hashes into LDS when they fit (uniform decision); counts the operand bytes of the
// lanes' jobs (present monomials x (hash + row bytes)). The caller's barrier publishes the copy.
DI void stage_hashes(LCtx& x, LTerms& T) {
    int need = 0;
#pragma unroll
    for (int s = 0; s < 3; s++) if (s < T.ns) need += T.S[s].cnt;
    const bool fit = need <= x.stage_cap;
    uint64_t* base = x.stage;
    unsigned long long b = 0;
#pragma unroll
    for (int s = 0; s < 3; s++) {
        if (s >= T.ns) continue;
        LSrc& S = T.S[s];
        for (int k = x.tid; k < S.cnt; k += LT) {
            if (fit) base[k] = S.h[k];
            b += (unsigned long long)__popcll(S.m[k]) * (8ull + 8ull * S.n);
        }
        if (fit) {
            S.h = base;
            base += S.cnt;
        }
    }
    if (b) atomicAdd(&x.A->bytes, b);
}

// ---- per-lane headers (the per-job engine's element-parallel formulas) ------------------------
// Operand header rows are loaded into registers first, then the output rows are stored, so a
// header costs about one memory latency instead of one per element (the rows all live in the
// same pool, which the compiler cannot prove disjoint).
struct HRows {
    double c[9], i0[9], i1[9], ab[9];
};
DI void hdr_load(const LCtx& x, const LH& h, int n, HRows& r) {
    const double* __restrict__ p = x.pool + (long)h.off * LG + x.lane;
#pragma unroll
    for (int e = 0; e < 9; e++) {
        const bool in = e < n;
        r.c[e] = in ? p[(long)e * LG] : 0.0;
        r.i0[e] = in ? p[(long)(n + e) * LG] : 0.0;
        r.i1[e] = in ? p[(long)(2 * n + e) * LG] : 0.0;
        r.ab[e] = in ? p[(long)(3 * n + e) * LG] : 0.0;
    }
}
DI void hdr_store(const LCtx& x, const LH& h, int n, const double* c, const double* i0, const double* i1) {
    double* __restrict__ p = x.pool + (long)h.off * LG + x.lane;
#pragma unroll
    for (int e = 0; e < 9; e++)
        if (e < n) {
            p[(long)e * LG] = c[e];
            p[(long)(n + e) * LG] = i0[e];
            p[(long)(2 * n + e) * LG] = i1[e];
            p[(long)(3 * n + e) * LG] = 0.0;
        }
}
DI void header_add(const LCtx& x, const LH& A, const LH& B, const LH& h, int sign) {
    const int n = nel(A);
    HRows a, b;
    hdr_load(x, A, n, a);
    hdr_load(x, B, n, b);
    double c[9], i0[9], i1[9];
#pragma unroll
    for (int e = 0; e < 9; e++) {
        c[e] = sign > 0 ? a.c[e] + b.c[e] : a.c[e] - b.c[e];
        i0[e] = a.i0[e] + b.i0[e];
        i1[e] = a.i1[e] + b.i1[e];
    }
    hdr_store(x, h, n, c, i0, i1);
}
DI void header_mul(const LCtx& x, const LH& A, const LH& B, const LH& h) {
    const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
    const int nr = nel(h), na = nel(A), nb = nel(B);
    HRows a, b;
    hdr_load(x, A, na, a);
    hdr_load(x, B, nb, b);
    double c[9], iv[2][9];
    if (as) {
        const double r2 = fabs(a.c[0]) + a.ab[0];
#pragma unroll
        for (int e = 0; e < 9; e++) {
            c[e] = a.c[0] * b.c[e];
            const double r3 = fabs(b.c[e]) + b.ab[e];
            iv[0][e] = a.i0[0] * b.i0[e] + (r2 * b.i0[e] + a.i0[0] * r3);
            iv[1][e] = a.i1[0] * b.i1[e] + (r2 * b.i1[e] + a.i1[0] * r3);
        }
    } else if (bs) {
        const double r3 = fabs(b.c[0]) + b.ab[0];
#pragma unroll
        for (int e = 0; e < 9; e++) {
            c[e] = a.c[e] * b.c[0];
            const double r2 = fabs(a.c[e]) + a.ab[e];
            iv[0][e] = a.i0[e] * b.i0[0] + (r2 * b.i0[0] + a.i0[e] * r3);
            iv[1][e] = a.i1[e] * b.i1[0] + (r2 * b.i1[0] + a.i1[e] * r3);
        }
    } else {
        // 3x3 times 3xC, column-major element (i, j), inner index summed in order (matmul())
        double r2[9], r3[9];
#pragma unroll
        for (int e = 0; e < 9; e++) { r2[e] = fabs(a.c[e]) + a.ab[e]; r3[e] = fabs(b.c[e]) + b.ab[e]; }
#pragma unroll
        for (int e = 0; e < 9; e++) {
            const int i = e % 3, j = e / 3;
            c[e] = (a.c[i] * b.c[3 * j] + a.c[i + 3] * b.c[3 * j + 1]) + a.c[i + 6] * b.c[3 * j + 2];
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const double* Ai = v == 0 ? a.i0 : a.i1;
                const double* Bi = v == 0 ? b.i0 : b.i1;
                const double t2 = (r2[i] * Bi[3 * j] + r2[i + 3] * Bi[3 * j + 1]) + r2[i + 6] * Bi[3 * j + 2];
                const double t3 = (Ai[i] * r3[3 * j] + Ai[i + 3] * r3[3 * j + 1]) + Ai[i + 6] * r3[3 * j + 2];
                const double ii = (Ai[i] * Bi[3 * j] + Ai[i + 3] * Bi[3 * j + 1]) + Ai[i + 6] * Bi[3 * j + 2];
                iv[v][e] = ii + (t2 + t3);
            }
        }
    }
    hdr_store(x, h, nr, c, iv[0], iv[1]);
}
DI void header_stack3(const LCtx& x, const LH& S0, const LH& S1, const LH& S2, const LH& h) {
    HRows a, b, d;
    hdr_load(x, S0, 1, a);
    hdr_load(x, S1, 1, b);
    hdr_load(x, S2, 1, d);
    const double c[3] = {a.c[0], b.c[0], d.c[0]};
    const double i0[3] = {a.i0[0], b.i0[0], d.i0[0]};
    const double i1[3] = {a.i1[0], b.i1[0], d.i1[0]};
    hdr_store(x, h, 3, c, i0, i1);
}
DI void header_add_one_dim(const LCtx& x, const LH& A, const LH& B, const LH& h, int pos) {
    const int n = nel(A);
    HRows a, b;
    hdr_load(x, A, n, a);
    hdr_load(x, B, 1, b);
    double c[9], i0[9], i1[9];
#pragma unroll
    for (int e = 0; e < 9; e++) {
        const bool at = e == pos;
        c[e] = at ? a.c[e] + b.c[0] : a.c[e];
        i0[e] = at ? a.i0[e] + b.i0[0] : a.i0[e];
        i1[e] = at ? a.i1[e] + b.i1[0] : a.i1[e];
    }
    hdr_store(x, h, n, c, i0, i1);
}

// pruned amount into both independent parts, kept |sum| into absum (PZsparse.cu:347-349)
DI void finish_block(const LCtx& x, const LH& h, const double* red, const double* ab, int n) {
    if (frob_norm(red, n) != 0)
        for (int v = 0; v < 2; v++)
            for (int e = 0; e < n; e++) ind(x, h, v, e) = ind(x, h, v, e) + red[e];
    for (int e = 0; e < n; e++) abs_(x, h, e) = ab[e];
}

// ---- group policies (lane form of pz_engine.h PolBlock / PolCrossPP) --------------------------
template <int NN>
struct LPolBlock {
    static constexpr int NV = NN, NO = NN, NR = 2 * NN;
    PolBlock<NN> base;
    DI bool group(const double* s, double* out, double* red) const { return base.group(s, out, red); }
    DI void finish(const LCtx& x, int o, const double* red) const { finish_block(x, x.H[o], red, red + NN, NN); }
};

struct LPolCrossPP {
    static constexpr int NV = 6, NO = 3, NR = 15;
    PolCrossPP base;
    int a, b;
    DI bool group(const double* s, double* out, double* red) const { return base.group(s, out, red); }
    DI void finish(const LCtx& x, int o, const double* red) const {
        const LH& A = x.H[a];
        const LH& B = x.H[b];
        const LH& h = x.H[o];
        const int ea[6] = {1, 2, 2, 0, 0, 1}, fb[6] = {2, 1, 0, 2, 1, 0};
        double pc[6], pi[2][6];
#pragma unroll
        for (int p = 0; p < 6; p++) {
            const double ace = cen(x, A, ea[p]), bcf = cen(x, B, fb[p]);
            const double r2 = fabs(ace) + abs_(x, A, ea[p]);
            const double r3 = fabs(bcf) + abs_(x, B, fb[p]);
            pc[p] = ace * bcf;
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const double ai = ind(x, A, v, ea[p]), bi = ind(x, B, v, fb[p]);
                pi[v][p] = ai * bi + (r2 * bi + ai * r3);
                if (frob1(red[p]) != 0) pi[v][p] = pi[v][p] + red[p];
            }
        }
        double sred[3];
#pragma unroll
        for (int e = 0; e < 3; e++) sred[e] = red[9 + e];
        const bool sadd = frob_norm(sred, 3) != 0;
#pragma unroll
        for (int e = 0; e < 3; e++) {
            cen(x, h, e) = pc[2 * e] - pc[2 * e + 1];
#pragma unroll
            for (int v = 0; v < 2; v++) {
                double iv = pi[v][2 * e] + pi[v][2 * e + 1];
                if (frob1(red[6 + e]) != 0) iv = iv + red[6 + e];
                if (sadd) iv = iv + sred[e];
                ind(x, h, v, e) = iv;
            }
            abs_(x, h, e) = red[12 + e];
        }
    }
};


// ---- term value generators: this lane's value(s) of term p (p wave-uniform), operand shapes fixed
// at compile time so the pass-1 loop holds exactly the rows it needs; operand descriptors are
// wave-uniform (scalar registers)

// rows of a full (non-view) block of N elements, monomial k
template <int N>
DI void rows(GAS const double* c, int k, double* out, int lane) {
    GAS const double* base = c + (long)k * N * LG + lane;
#pragma unroll
    for (int e = 0; e < N; e++) out[e] = base[(long)e * LG];
}

// product a * b of full blocks (PZsparse.cu:864-994): a NA = 1 | 9 elements, b NB = 1 | 3 | 9
template <int NA, int NB>
struct GMul {
    static constexpr int NO = NA == 1 ? NB : (NB == 1 ? NA : 3 * (NB / 3));
    static constexpr int NV = NO;
    static constexpr int U = (NA == 9 && NB == 9) ? LANE_U99 : (NA == 9 ? LANE_U93 : LANE_U13);  // groups per wave round
    GAS const double* ca;   // arena rows of monomial 0
    GAS const double* cb;
    GAS const double* pa;   // header pool rows of the operands' centres ([e][LG], as a monomial block)
    GAS const double* pb;
    int na, nb;
    uint32_t nbm;
    DI void ra(int k, double* a, int lane) const { rows<NA>(ca, k, a, lane); }
    DI void rb(int k, double* b, int lane) const { rows<NB>(cb, k, b, lane); }
    // Branch-free (p is wave-uniform): each factor is read from one wave-uniform row block, a
    // monomial's in the arena or the operand's centre in the header pool (T1: a_i x B.c, T2:
    // A.c x b_j), chosen by a scalar select of the block address. A load inside a branch makes the
    // compiler wait for it where the branches meet, and centres held in registers across the round
    // loop cost 2 (NA + NB) VGPRs.
    DI void factors(int p, double* a, double* b, int lane) const {
        const bool ta = p < na, tb = !ta && p < na + nb;
        const int q = p - na - nb;
        const int iq = nb == 1 ? q : (int)__umulhi((uint32_t)(q > 0 ? q : 0), nbm);
        const int i = ta ? p : iq;
        const int j = tb ? p - na : q - iq * nb;
        GAS const double* ba = tb ? pa : ca + (long)(i > 0 ? i : 0) * NA * LG;
        GAS const double* bb = ta ? pb : cb + (long)(j > 0 ? j : 0) * NB * LG;
        rows<NA>(ba, 0, a, lane);
        rows<NB>(bb, 0, b, lane);
    }
    DI void term(int p, double* v, int lane) const {
        double a[NA], b[NB];
        factors(p, a, b, lane);
        if constexpr (NA == 1) {
#pragma unroll
            for (int e = 0; e < NB; e++) v[e] = a[0] * b[e];
        } else if constexpr (NB == 1) {
#pragma unroll
            for (int e = 0; e < NA; e++) v[e] = a[e] * b[0];
        } else {
#pragma unroll
            for (int j = 0; j < NB / 3; j++)
#pragma unroll
                for (int i = 0; i < 3; i++) v[i + 3 * j] = (a[i] * b[3 * j] + a[i + 3] * b[3 * j + 1]) + a[i + 6] * b[3 * j + 2];
        }
    }
};
template <int NA, int NB>
DI GMul<NA, NB> gen_mul(const LCtx& x, const LH& A, const LH& B) {
    GMul<NA, NB> G;
    G.na = ui(A.cnt);
    G.nb = ui(B.cnt);
    // an operand without monomials (a constant matrix) points at the arena's first rows, so the
    // branch-free factors() never reads past an allocation
    G.ca = gas(up(x.A->c)) + (G.na > 0 ? bcast0(A.coff) : 0) * LG;
    G.cb = gas(up(x.A->c)) + (G.nb > 0 ? bcast0(B.coff) : 0) * LG;
    G.pa = gas(up(x.pool)) + (long)ui(A.off) * LG;
    G.pb = gas(up(x.pool)) + (long)ui(B.off) * LG;
    G.nbm = G.nb > 1 ? 0xFFFFFFFFu / (uint32_t)G.nb + 1u : 0u;
    return G;
}

// fused PZ x PZ cross: the six 1x1 products of the term's factor rows (PolCrossPP)
struct GCross {
    static constexpr int NV = 6;
    static constexpr int U = LANE_UX;
    GMul<3, 3> M;  // factor rows only (3-element blocks both sides)
    DI void term(int p, double* v, int lane) const {
        double u[3], w[3];
        M.factors(p, u, w, lane);
        v[0] = u[1] * w[2]; v[1] = u[2] * w[1]; v[2] = u[2] * w[0];
        v[3] = u[0] * w[2]; v[4] = u[0] * w[1]; v[5] = u[1] * w[0];
    }
};

// concatenation of up to 3 sources into N-element terms (operator+/-, stack, addOneDimPZ): a
// source is a full N block or a 1x1 (possibly an element / scaled view) placed at a component
template <int N>
struct GCat {
    static constexpr int NV = N;
    static constexpr int U = N == 9 ? LANE_UC9 : LANE_UC3;
    // one descriptor per source, as plain scalars (an indexed member array would live in scratch)
    struct D {
        GAS const double* c;
        int stride, comp, one, place, neg, scaled;
        double scale;
    };
    D d0, d1, d2;
    int c0, c1;
    DI void term(int p, double* v, int lane) const {
        const int s = p < c0 ? 0 : (p < c0 + c1 ? 1 : 2);
        // Field-by-field value selects (all wave-uniform, so scalar registers). A reference to the
        // selected descriptor is a pointer select: the compiler then keeps d0..d2 in scratch and
        // every term pays a chain of dependent scratch loads (descriptor, row, flags, scale).
        // (opaque(): the optimiser would fold a select of two field loads back into one load from
        // a selected address)
        GAS const double* c = s == 0 ? opaque(d0.c) : (s == 1 ? opaque(d1.c) : opaque(d2.c));
        const int stride = s == 0 ? opaque(d0.stride) : (s == 1 ? opaque(d1.stride) : opaque(d2.stride));
        const int comp = s == 0 ? opaque(d0.comp) : (s == 1 ? opaque(d1.comp) : opaque(d2.comp));
        const int one = s == 0 ? opaque(d0.one) : (s == 1 ? opaque(d1.one) : opaque(d2.one));
        const int place = s == 0 ? opaque(d0.place) : (s == 1 ? opaque(d1.place) : opaque(d2.place));
        const int neg = s == 0 ? opaque(d0.neg) : (s == 1 ? opaque(d1.neg) : opaque(d2.neg));
        const int scaled = s == 0 ? opaque(d0.scaled) : (s == 1 ? opaque(d1.scaled) : opaque(d2.scaled));
        const double scale = s == 0 ? opaque(d0.scale) : (s == 1 ? opaque(d1.scale) : opaque(d2.scale));
        const int k = s == 0 ? p : (s == 1 ? p - c0 : p - c0 - c1);
        GAS const double* base = c + (long)k * stride * LG + lane;
        // branch-free: N loads either way (a 1x1 source reads its one element N times, the same
        // 512-byte row), then the same arithmetic as the per-element form
        const int e1 = comp >= 0 ? comp : 0;
        double xs[N];
#pragma unroll
        for (int e = 0; e < N; e++) xs[e] = base[(long)(one ? e1 : e) * LG];
#pragma unroll
        for (int e = 0; e < N; e++) {
            double x0 = xs[e];
            if (scaled) x0 = scale * x0;
            x0 = neg ? -x0 : x0;
            v[e] = one ? ((e == place) ? x0 : 0.0) : x0;
        }
    }
};
template <int N>
DI typename GCat<N>::D cat_desc(const LCtx& x, const LH& S, int neg, int place) {
    typename GCat<N>::D d;
    d.c = gas(up(x.A->c)) + bcast0(S.coff) * LG;
    d.stride = ui(S.stride);
    d.comp = ui(S.comp);
    d.scaled = ui(S.scaled);
    d.scale = ud(S.scale);
    d.one = ui(S.R * S.C) == 1 ? 1 : 0;
    d.neg = neg;
    d.place = place;
    return d;
}
template <int N>
DI GCat<N> gen_cat(const LCtx& x, const Op& op) {
    GCat<N> G;
    const bool st = op.code == OP_STACK3;
    G.d0 = cat_desc<N>(x, x.H[op.a], 0, 0);
    G.d1 = cat_desc<N>(x, x.H[op.b], op.code == OP_ADD && op.i < 0 ? 1 : 0, st ? 1 : (op.code == OP_ADD1D ? op.i : 0));
    G.d2 = cat_desc<N>(x, x.H[st ? op.c : op.b], 0, st ? 2 : 0);
    G.c0 = ui(x.H[op.a].cnt);
    G.c1 = ui(x.H[op.b].cnt);
    return G;
}

struct GAnyCross {
    static constexpr int NV = 6;
    static constexpr int U = 1;
    const LTerms* T;
    DI void term(int p, double* v, int lane) const {
        double u[9], w[9];
        T->factors(p, u, w, lane);
        PolCrossPP::prods(u, w, v);
    }
};
// any other shape: the runtime-shaped LTerms reader
template <int N>
struct GAny {
    static constexpr int NV = N;
    static constexpr int U = 1;
    const LTerms* T;
    DI void term(int p, double* v, int lane) const {
        double t[9];
        T->coef(p, t, lane);
#pragma unroll
        for (int e = 0; e < N; e++) v[e] = t[e];
    }
};

// ---- simplify over the union term list ----------------------------------------------------------
// keys ordered by rank merge (once per bundle), group heads, pass 1 (each wave sums whole groups,
// lane = job: per-lane sums, decisions, pruned amounts; the group's keep mask is the ballot),
// compaction scan over groups kept by any lane, pass 2 (copy), reduction, per-lane finish.
// Sources staged and published by the caller's barrier. Ends with a barrier.
// the end of the key window that starts at group g0 (operators beyond the LDS key capacity): the
// most whole rounds of RG groups (or up to NG) whose keys and group heads fit the LDS arrays;
// g0 itself when not even one round fits. Wave-uniform; gp is the global head array.
DI int key_window_end(const LCtx& x, const int* gp, int g0, int NG, int RG) {
    const int k0 = gp[g0];
    const int nr = (NG - g0 + RG - 1) / RG;
    // window of r rounds: groups [g0, min(g0 + r RG, NG)), fits when its groups and keys do
    const int e1 = min(g0 + RG, NG);
    if (e1 - g0 > x.cap_lds || gp[e1] - k0 > x.cap_lds) return g0;
    int lo = 1, hi = nr;  // lo rounds fit; find the largest r <= nr that does (monotone)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        const int g1 = min(g0 + mid * RG, NG);
        if (g1 - g0 <= x.cap_lds && gp[g1] - k0 <= x.cap_lds) lo = mid;
        else hi = mid - 1;
    }
    return min(g0 + lo * RG, NG);
}

// ---- simplify over the union term list ----------------------------------------------------------
// keys ordered by rank merge (once per bundle), group heads, pass 1 (each wave sums whole groups,
// lane = job: per-lane sums, decisions, pruned amounts; the group's keep mask is the ballot),
// compaction scan over groups kept by any lane, pass 2 (copy), reduction, per-lane finish.
// Sources staged and published by the caller's barrier. Ends with a barrier.
template <class Pol, class Gen>
DI void simplify(LCtx& x, int o, const LTerms& T, const Gen& G, const Pol& pol, int N) {
    constexpr int NV = Pol::NV, n = Pol::NO;
    static_assert(Gen::NV == Pol::NV, "generator / policy value count");
    const bool in_lds = N <= x.cap_lds;
    uint64_t* kh = in_lds ? x.kh : x.gkh;
    uint32_t* ki = in_lds ? x.ki : x.gki;
    int* kp = in_lds ? x.kp : x.gkp;
    int* gp = in_lds ? x.gp : x.ggp;
    double red[Pol::NR];
#pragma unroll
    for (int e = 0; e < Pol::NR; e++) red[e] = 0.0;
    if (x.tid == 0) atomicMax(&x.occ[0], N);
    if (N > x.cap_glb || N >= (1 << 16)) {
        if (x.tid == 0) { err_or(x, ERR_SORTCAP); x.H[o].cnt = 0; }
        combine_red<Pol::NR>(x, red);
        return;
    }
    long long ph_t = x.prof ? clock64() : 0;
    for (int p = x.tid; p < N; p += LT) {
        const uint64_t h = T.hash(p);
        const int r = T.rank(p, h);
        kh[r] = h;
        ki[r] = (uint32_t)p;
    }
    sync();
    LPHASE(1)
    for (int q = x.tid; q < N; q += LT) kp[q] = (q == 0 || kh[q] != kh[q - 1]) ? 1 : 0;
    sync();
    const int NG = block_scan(x, kp, N);
    for (int q = x.tid; q < N; q += LT)
        if (q == 0 || kh[q] != kh[q - 1]) gp[kp[q]] = q;
    if (x.tid == 0) gp[NG] = N;
    sync();
    LPHASE(2)
    // Rounds of LW x U groups: each wave sums U groups (their member loads issued together),
    // decides per lane and ballots the keep masks into LDS; after one barrier every wave knows the
    // round's kept prefix and writes its kept groups straight to their compacted rows. The output
    // reserves NG rows up front and gives back the unused tail at the end (no other allocation
    // runs during a simplify), so group values never leave registers.
    // The rounds read keys and group heads from LDS only: an operator with more keys than the LDS
    // arrays hold (sorted into the global buffers above) runs in windows of whole rounds, each
    // window's keys and rebased heads copied into the LDS arrays first. Windows do not change which
    // wave sums which group, or in what order, so the sums are those of one pass.
    constexpr int U = Gen::U;
    constexpr int RG = LW * U;
    static_assert(RG <= 64, "round masks fit one wave ballot");
    if (x.tid == 0) {
        x.A->hmark = x.A->hused;
        x.A->cmark = x.A->cused;
        arena_alloc(x, x.H[o], NG, n);
    }
    sync();
    LPHASE(3)
    const LH& ho = x.H[o];
    const bool ok = ui(ho.cnt) == NG;
    GAS double* const dst = gas(up(x.A->c)) + bcast0(ho.coff) * LG;  // wave-uniform; + lane at the store
    const long hoff = bcast0(ho.hoff);
    GAS uint64_t* const Ah = gas(up(x.A->h));
    GAS uint64_t* const Am = gas(up(x.A->m));
    LAS const uint64_t* const lkh = x.lkh;
    LAS const uint32_t* const lki = x.lki;
    LAS int* const lgp = x.lgp;
    int base = 0, par = 0;
    unsigned long long b = 0;
    unsigned long long sub[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long rt = x.prof ? clock64() : 0;
#define RSTAMP(k)                                                                                  \
    if (x.prof && x.tid == 0) {                                                                    \
        const long long c_ = clock64();                                                            \
        sub[k] += (unsigned long long)(c_ - rt);                                                   \
        rt = c_;                                                                                   \
    }
    for (int g0 = 0; g0 < NG;) {
        int g1 = NG;
        if (!in_lds) {
            g1 = key_window_end(x, gp, g0, NG, RG);
            if (g1 == g0) {  // not even one round's keys fit the LDS arrays
                if (x.tid == 0) err_or(x, ERR_SORTCAP);
                break;
            }
            const int k0 = gp[g0], k1 = gp[g1];
            for (int q = x.tid; q < k1 - k0; q += LT) {
                x.lki[q] = ki[k0 + q];
                x.lkh[q] = kh[k0 + q];
            }
            for (int g = x.tid; g <= g1 - g0; g += LT) x.lgp[g] = gp[g0 + g] - k0;
            sync();
        }
        const int ng = g1 - g0;  // groups of this window; lgp / lki / lkh indices are window-relative
        for (int r0 = 0; r0 < ng; r0 += RG, par ^= 1) {
            RSTAMP(7)
            // every index load of the round is issued before the first is used (clamped, no
            // branches), then every group's first-member loads, so the round costs one latency per phase
            int lo[U], sz[U];
            int maxsz = 0;
            {
                int l0[U], h0[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int g = min(r0 + x.wave * U + u, ng);
                    l0[u] = lgp[g];
                    h0[u] = lgp[min(g + 1, ng)];
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const bool in = r0 + x.wave * U + u < ng;
                    lo[u] = in ? ui(l0[u]) : 0;
                    sz[u] = in ? ui(h0[u]) - lo[u] : 0;
                    maxsz = sz[u] > maxsz ? sz[u] : maxsz;
                }
            }
            RSTAMP(0)
            if (LANE_PROF) {
                sub[5] += 1;
                sub[6] += maxsz;
            }
            double acc[U][NV];
            uint64_t hk[U];  // the groups' hashes, loaded with the first members (stored after the barrier)
            {
                int p0[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    p0[u] = (int)lki[lo[u]];
                    hk[u] = bcast0((long)lkh[lo[u]]);
                }
#pragma unroll
                for (int u = 0; u < U; u++) G.term(ui(p0[u]), acc[u], x.lane);
            }
            for (int r = 1; r < maxsz; r++) {
                double tmp[U][NV];
                int pr[U];
#pragma unroll
                for (int u = 0; u < U; u++) pr[u] = (int)lki[lo[u] + (r < sz[u] ? r : 0)];
#pragma unroll
                for (int u = 0; u < U; u++) G.term(ui(pr[u]), tmp[u], x.lane);
#pragma unroll
                for (int u = 0; u < U; u++)
                    if (r < sz[u])
#pragma unroll
                        for (int e = 0; e < NV; e++) acc[u][e] = acc[u][e] + tmp[u][e];
            }
            double out[U][n];
            unsigned long long mk[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
#pragma unroll
                for (int e = 0; e < n; e++) out[u][e] = 0.0;
                bool keep = false;
                if (sz[u] > 0) keep = pol.group(acc[u], out[u], red);
                mk[u] = ballot(keep);
                if (x.lane == 0) x.rmask[par * 64 + x.wave * U + u] = mk[u];
            }
            RSTAMP(1)
            sync();
            RSTAMP(2)
            const unsigned long long km = ballot(x.lane < RG && r0 + x.lane < ng && x.rmask[par * 64 + x.lane] != 0);
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (mk[u] == 0 || !ok) continue;
                const int idx = x.wave * U + u;
                const long pos = base + __popcll(km & ((1ull << idx) - 1));
#pragma unroll
                for (int e = 0; e < n; e++) dst[(pos * n + e) * LG + x.lane] = out[u][e];
                if (x.lane == 0) {
                    Ah[hoff + pos] = hk[u];
                    Am[hoff + pos] = mk[u];
                }
                b += (unsigned long long)__popcll(mk[u]) * (8ull + 8ull * n);  // wave-uniform
            }
            base += __popcll(km);
            RSTAMP(3)
        }
        g0 = g1;
        if (!in_lds) sync();  // every wave is done with this window's keys before the next copy
    }
#undef RSTAMP
    if (x.prof && x.tid == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&x.prof[2 * x.nops + k], sub[k]);
    if (b && x.lane == 0) atomicAdd(&x.A->bytes, b);
    LPHASE(4)
    sync();
    if (x.tid == 0 && ok) {
        // give back the rows of the groups no lane kept
        x.H[o].cnt = base;
        x.A->hused = x.A->hmark + base;
        x.A->cused = x.A->cmark + (long)base * n;
    }
    LPHASE(5)
    combine_red<Pol::NR>(x, red);
    if (x.wave == 0) pol.finish(x, o, red);
    sync();
    LPHASE(6)
}

// ---- fused PZ x constant crosses (pz_engine.h cross_const, lane form) ------------------------------
DI void cross_const_finish(const LCtx& x, const LH& h, const LH& A, const CrossC& C, const double* red) {
    double sred[3];
#pragma unroll
    for (int e = 0; e < 3; e++) sred[e] = red[3 + e];
    const bool sadd = frob_norm(sred, 3) != 0;
#pragma unroll
    for (int e = 0; e < 3; e++) {
        cen(x, h, e) = cen(x, A, C.iA[e]) * C.sA[e] - cen(x, A, C.iB[e]) * C.sB[e];
#pragma unroll
        for (int v = 0; v < 2; v++) {
            double iv = ind(x, A, v, C.iA[e]) * fabs(C.sA[e]) + ind(x, A, v, C.iB[e]) * fabs(C.sB[e]);
            if (frob1(red[e]) != 0) iv = iv + red[e];
            if (sadd) iv = iv + sred[e];
            ind(x, h, v, e) = iv;
        }
        abs_(x, h, e) = red[6 + e];
    }
}
// ends with a barrier
DI void cross_const(LCtx& x, int o, int a, const CrossC& C) {
    const LH& A = x.H[a];
    const int N = A.cnt;
    const LSrc S = src_of(x, A);
    double red[9], out[3], m[9];
#pragma unroll
    for (int e = 0; e < 9; e++) red[e] = 0.0;
    int* kp = N <= x.cap_lds ? x.kp : x.gkp;
    if (x.tid == 0) atomicMax(&x.occ[0], N);
    if (N > x.cap_glb || N > x.cap_out) {
        if (x.tid == 0) { err_or(x, ERR_SORTCAP); x.H[o].cnt = 0; }
        combine_red<9>(x, red);
        return;
    }
    unsigned long long b = 0;
    // two monomials per trip (k, k + LW: the wave's own order, so the pruned sums accumulate as
    // before), both monomials' rows loaded before either is used
    for (int k = x.wave; k < N; k += 2 * LW) {
        const int k2 = k + LW;
        const bool has2 = k2 < N;
        double m2[9];
        S.read(k, false, m, x.lane);
        S.read(has2 ? k2 : k, false, m2, x.lane);
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (q == 1 && !has2) break;
            const int kk = q == 0 ? k : k2;
#pragma unroll
            for (int e = 0; e < 3; e++) out[e] = 0.0;
            const bool keep = cross_const_mono(C, q == 0 ? m : m2, x.thr, out, red);
            double* go = x.gout + (long)kk * 3 * LG + x.lane;
#pragma unroll
            for (int e = 0; e < 3; e++) go[(long)e * LG] = keep ? out[e] : 0.0;
            const unsigned long long mk = ballot(keep);
            if (x.lane == 0) {
                x.gm[kk] = mk;
                kp[kk] = mk != 0 ? 1 : 0;
                b += (unsigned long long)__popcll(S.m[kk]) * 32ull + (unsigned long long)__popcll(mk) * 32ull;
            }
        }
    }
    if (b) atomicAdd(&x.A->bytes, b);
    sync();
    const int K = block_scan(x, kp, N);
    if (x.tid == 0) arena_alloc(x, x.H[o], K, 3);
    sync();
    const LH& ho = x.H[o];
    if (ho.cnt == K) {
        double* dst = x.A->c + ho.coff * LG + x.lane;
        // two monomials per trip, loads first (clamped), stores of the kept ones after
        for (int k = x.wave; k < N; k += 2 * LW) {
            int kk[2];
            kk[0] = k;
            kk[1] = k + LW < N ? k + LW : k;
            bool kept[2];
            long pos[2];
            double v[2][3];
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int j = kk[q];
                kept[q] = (q == 0 || k + LW < N) && ((j + 1 < N) ? kp[j + 1] != kp[j] : kp[j] != K);
                pos[q] = kp[j];
                const double* go = x.gout + (long)j * 3 * LG + x.lane;
#pragma unroll
                for (int e = 0; e < 3; e++) v[q][e] = go[(long)e * LG];
            }
#pragma unroll
            for (int q = 0; q < 2; q++) {
                if (!kept[q]) continue;
#pragma unroll
                for (int e = 0; e < 3; e++) dst[(pos[q] * 3 + e) * LG] = v[q][e];
                if (x.lane == 0) {
                    x.A->h[ho.hoff + pos[q]] = S.h[kk[q]];
                    x.A->m[ho.hoff + pos[q]] = x.gm[kk[q]];
                }
            }
        }
    }
    combine_red<9>(x, red);
    if (x.wave == 0) cross_const_finish(x, ho, A, C, red);
    sync();
}

// ---- lane ops (the per-job engine's thread-0 bodies; one wave, lane = job) ------------------------

// PZ from <= 4 raw candidate monomials with static hashes (PZsparse.cu:120-205), as t0_make_raw:
// per-lane merge / prune / pruned and |kept| sums in the same orders; the union keeps a monomial
// if any lane keeps it, at its rank among the union-kept hashes
DI void make_raw(const LCtx& x, int o, int R, int C, const double* center, int nc, const uint64_t* hs, const double (*cf)[9]) {
    constexpr int M = 4;
    const int n = R * C;
    uint64_t h[M];
#pragma unroll
    for (int m = 0; m < M; m++) h[m] = m < nc ? hs[m] : ~(uint64_t)0;
    bool head[M], keep[M];
    double acc[M][9];
#pragma unroll
    for (int m = 0; m < M; m++) {
        head[m] = m < nc;
#pragma unroll
        for (int m2 = 0; m2 < m; m2++) if (h[m2] == h[m]) head[m] = false;
#pragma unroll
        for (int e = 0; e < 9; e++) acc[m][e] = (m < nc && e < n) ? cf[m][e] : 0.0;
#pragma unroll
        for (int m2 = m + 1; m2 < M; m2++)
            if (m2 < nc && h[m2] == h[m])
#pragma unroll
                for (int e = 0; e < 9; e++) if (e < n) acc[m][e] = acc[m][e] + cf[m2][e];
        keep[m] = head[m] && !(frob_norm(acc[m], n) <= x.thr);
    }
    unsigned long long km[M];
    bool uk[M];
#pragma unroll
    for (int m = 0; m < M; m++) { km[m] = ballot(keep[m]); uk[m] = km[m] != 0; }
    int rk[M], pos[M], upos[M], K = 0;
#pragma unroll
    for (int m = 0; m < M; m++) {
        rk[m] = 0; pos[m] = 0; upos[m] = 0;
#pragma unroll
        for (int m2 = 0; m2 < M; m2++) {
            if (head[m2] && h[m2] < h[m]) rk[m]++;
            if (keep[m2] && h[m2] < h[m]) pos[m]++;
            if (uk[m2] && h[m2] < h[m]) upos[m]++;
        }
        K += uk[m] ? 1 : 0;
    }
    double red[9], ab[9];
#pragma unroll
    for (int e = 0; e < 9; e++) { red[e] = 0.0; ab[e] = 0.0; }
#pragma unroll
    for (int r = 0; r < M; r++)
#pragma unroll
        for (int m = 0; m < M; m++) {
            if (head[m] && !keep[m] && rk[m] == r)
#pragma unroll
                for (int e = 0; e < 9; e++) red[e] = red[e] + fabs(acc[m][e]);
            if (keep[m] && pos[m] == r)
#pragma unroll
                for (int e = 0; e < 9; e++) ab[e] = ab[e] + fabs(acc[m][e]);
        }
    LH& hd = x.H[o];
    const int off = hd.off;
    long hoff = 0, coff = 0;
    int ok = 0;
    if (x.lane == 0) {
        set_meta(hd, R, C);
        ok = arena_alloc(x, hd, K, n) ? 1 : 0;
        hoff = hd.hoff;
        coff = hd.coff;
    }
    hoff = bcast0(hoff);
    coff = bcast0(coff);
    ok = __builtin_amdgcn_readfirstlane(ok);
    // header rows of this lane's job
    for (int q = 0; q < 4 * n; q++) x.pool[(long)(off + q) * LG + x.lane] = 0.0;
    for (int e = 0; e < n; e++) x.pool[(long)(off + e) * LG + x.lane] = center[e];
    if (frob_norm(red, n) != 0)
        for (int e = 0; e < n; e++) {
            x.pool[(long)(off + n + e) * LG + x.lane] += red[e];
            x.pool[(long)(off + 2 * n + e) * LG + x.lane] += red[e];
        }
    for (int e = 0; e < n; e++) x.pool[(long)(off + 3 * n + e) * LG + x.lane] += ab[e];
    if (ok) {
#pragma unroll
        for (int m = 0; m < M; m++)
            if (uk[m]) {
                if (x.lane == 0) { x.A->h[hoff + upos[m]] = h[m]; x.A->m[hoff + upos[m]] = km[m]; }
#pragma unroll
                for (int e = 0; e < 9; e++)
                    if (e < n) x.A->c[(coff + (long)upos[m] * n + e) * LG + x.lane] = keep[m] ? acc[m][e] : 0.0;
            }
    }
}

DI void make_1d(const LCtx& x, int o, int i, int v) {
    const JrsJoint& J = x.jrs[i];
    const double c0 = v == 2 ? J.qdd_c : J.qd_c;
    uint64_t hh[2];
    double cf[2][9];
    hh[0] = slot_hash(SLOT_K + i);
    cf[0][0] = v == 2 ? J.qdd_k : J.qd_k;
    hh[1] = slot_hash((v == 0 ? SLOT_QDE : v == 1 ? SLOT_QDAE : SLOT_QDDAE) + i);
    cf[1][0] = v == 0 ? J.qd_e : v == 1 ? J.qda_e : J.qdd_e;
    make_raw(x, o, 1, 1, &c0, 2, hh, cf);
}

DI void make_rot(const LCtx& x, int o, const RobotParams& rp, int i) {
    const JrsJoint& J = x.jrs[i];
    const int ax = rp.axes[i];
    double cn[9], cf[4][9];
    uint64_t hh[4];
#pragma unroll
    for (int e = 0; e < 9; e++) cn[e] = (e % 4 == 0) ? 1.0 : 0.0;
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
        for (int e = 0; e < 9; e++) cf[m][e] = 0.0;
    auto put = [&](double* Rm, double c, double s) {
        const double ns = -1.0 * s;
        if (ax == 1) { Rm[1 + 3] = c; Rm[1 + 6] = ns; Rm[2 + 3] = s; Rm[2 + 6] = c; }
        else if (ax == 2) { Rm[0] = c; Rm[0 + 6] = s; Rm[2] = ns; Rm[2 + 6] = c; }
        else { Rm[0] = c; Rm[0 + 3] = ns; Rm[1] = s; Rm[1 + 3] = c; }
    };
    put(cn, J.cos_c, J.sin_c);
    put(cf[0], J.cos_k, 0.0); hh[0] = slot_hash(SLOT_K + i);
    put(cf[1], J.cos_e, 0.0); hh[1] = slot_hash(SLOT_COS + i);
    put(cf[2], 0.0, J.sin_k); hh[2] = slot_hash(SLOT_K + i);
    put(cf[3], 0.0, J.sin_e); hh[3] = slot_hash(SLOT_SIN + i);
    make_raw(x, o, 3, 3, cn, 4, hh, cf);
}

DI void make_box(const LCtx& x, int o, const RobotParams& rp, int i) {
    uint64_t hh[3];
    double cf[3][9];
#pragma unroll
    for (int m = 0; m < 3; m++) {
#pragma unroll
        for (int e = 0; e < 9; e++) cf[m][e] = 0.0;
        cf[m][m] = rp.link_g[i][m];
        hh[m] = slot_hash(NF * (m + 1));
    }
    make_raw(x, o, 3, 1, rp.link_c[i], 3, hh, cf);
}

DI void make_const(const LCtx& x, int o, int R, int C, const double* center, double unc_int) {
    LH& h = x.H[o];
    if (x.lane == 0) set_meta(h, R, C);
    const int n = R * C;
    hdr_zero(x, h.off, n);
    for (int e = 0; e < n; e++) {
        x.pool[(long)(h.off + e) * LG + x.lane] = center[e];
        x.pool[(long)(h.off + 2 * n + e) * LG + x.lane] = unc_int * fabs(center[e]);
    }
}

DI void make_view(const LCtx& x, int o, int a, int e, int scaled, double s) {
    const LH& Pp = x.H[a];
    LH& h = x.H[o];
    const int n = e >= 0 ? 1 : nel(Pp);
    if (x.lane == 0) {
        h.R = e >= 0 ? 1 : Pp.R;
        h.C = e >= 0 ? 1 : Pp.C;
        h.cnt = Pp.cnt; h.stride = Pp.stride; h.hoff = Pp.hoff; h.coff = Pp.coff;
        h.comp = e >= 0 ? e : Pp.comp;
        h.scaled = scaled;
        h.scale = scaled ? s : 1.0;
        if (Pp.comp >= 0 || Pp.scaled) err_or(x, ERR_HANDLES);
    }
    const int pn = nel(Pp);
    for (int q = 0; q < n; q++) {
        const int src = e >= 0 ? e : q;
        double c = P(x, Pp.off + src), i0 = P(x, Pp.off + pn + src), i1 = P(x, Pp.off + 2 * pn + src), ab = P(x, Pp.off + 3 * pn + src);
        if (scaled) { c = c * s; i0 = i0 * fabs(s); i1 = i1 * fabs(s); ab = ab * fabs(s); }
        P(x, h.off + q) = c; P(x, h.off + n + q) = i0; P(x, h.off + 2 * n + q) = i1; P(x, h.off + 3 * n + q) = ab;
    }
}

DI void make_transpose(const LCtx& x, int o, int a) {
    const LH& A = x.H[a];
    LH& h = x.H[o];
    const int n = nel(A);
    long hoff = 0, coff = 0;
    int ok = 0;
    if (x.lane == 0) {
        set_meta(h, A.C, A.R);
        ok = arena_alloc(x, h, A.cnt, n) ? 1 : 0;
        hoff = h.hoff;
        coff = h.coff;
    }
    hoff = bcast0(hoff);
    coff = bcast0(coff);
    ok = __builtin_amdgcn_readfirstlane(ok);
    for (int i = 0; i < A.R; i++)
        for (int j = 0; j < A.C; j++) {
            P(x, h.off + j + i * A.C) = P(x, A.off + i + j * A.R);
            P(x, h.off + n + j + i * A.C) = P(x, A.off + n + i + j * A.R);
            P(x, h.off + 2 * n + j + i * A.C) = P(x, A.off + 2 * n + i + j * A.R);
            P(x, h.off + 3 * n + j + i * A.C) = P(x, A.off + 3 * n + i + j * A.R);
        }
    if (!ok) return;
    const LSrc S = src_of(x, A);
    unsigned long long b = 0;
    for (int k = 0; k < A.cnt; k++) {
        double m[9];
        S.read(k, false, m, x.lane);
        if (x.lane == 0) {
            x.A->h[hoff + k] = S.h[k];
            x.A->m[hoff + k] = S.m[k];
            b += 2ull * __popcll(S.m[k]) * (8ull + 8ull * n);
        }
        for (int i = 0; i < A.R; i++)
            for (int jj = 0; jj < A.C; jj++) x.A->c[(coff + (long)k * n + jj + i * A.C) * LG + x.lane] = m[i + jj * A.R];
    }
    if (x.lane == 0 && b) atomicAdd(&x.A->bytes, b);
}

// reduce_link_PZ (PZsparse.cu:370-402) over this lane's monomials, then the k-only emit
DI void emit_link(const LCtx& x, const ReachOut& out, int a, int l) {
    const LH& h = x.H[a];
    const LSrc S = src_of(x, h);
    const long base = x.job * out.NJ + l;
    double gl[18];
#pragma unroll
    for (int e = 0; e < 18; e++) gl[e] = 0.0;
    int jg = 0, kk = 0, bad = 0;
    double rad[3] = {ind(x, h, 0, 0), ind(x, h, 0, 1), ind(x, h, 0, 2)};
    for (int k = 0; k < h.cnt; k++) {
        if (!((S.m[k] >> x.lane) & 1)) continue;
        const uint64_t hh = S.h[k];
        double c[9];
        S.read(k, false, c, x.lane);
        if (hh < HASH_K_ONLY) {
            if (kk < CAP_LM) {
                if (x.valid) {
                    out.link_hash[base * CAP_LM + kk] = (uint16_t)hh;
#pragma unroll
                    for (int e = 0; e < 3; e++) out.link_coef[(base * CAP_LM + kk) * 3 + e] = c[e];
                }
            } else {
                bad |= ERR_OUTCAP;
            }
            kk++;
        } else if (hh < HASH_K_LINKS_ONLY && (hh & K_MASK) == 0) {
            if (jg < 3) {
#pragma unroll
                for (int e = 0; e < 3; e++) gl[e + 3 * jg] = c[e];
            } else {
                bad |= ERR_LINKGEN;
            }
            jg++;
        } else {
#pragma unroll
            for (int e = 0; e < 3; e++) rad[e] += fabs(c[e]);
        }
    }
    if (bad && x.valid) err_or(x, bad);
    gl[0 + 3 * 3] = rad[0];
    gl[1 + 3 * 4] = rad[1];
    gl[2 + 3 * 5] = rad[2];
    if (!x.valid) return;
    double* gens = out.link_gens + base * 18;
#pragma unroll
    for (int e = 0; e < 18; e++) gens[e] = gl[e];
    atomicMax(&x.occ[1], kk);
    out.link_cnt[base] = kk < CAP_LM ? kk : CAP_LM;
#pragma unroll
    for (int e = 0; e < 3; e++) { out.link_center[base * 3 + e] = cen(x, h, e); out.link_rad[base * 3 + e] = rad[e]; }
}

DI void emit_torque(const LCtx& x, const ReachOut& out, int a, int i) {
    const LH& h = x.H[a];
    const LSrc S = src_of(x, h);
    const long base = x.job * NF + i;
    x.scr[(long)i * LG + x.lane] = ind(x, h, 1, 0) + ind(x, h, 0, 0);  // disturbance radius
    double rad = ind(x, h, 0, 0);
    int kk = 0, bad = 0;
    for (int k = 0; k < h.cnt; k++) {
        if (!((S.m[k] >> x.lane) & 1)) continue;
        const uint64_t hh = S.h[k];
        double c = S.c[((long)k * S.stride + (S.comp >= 0 ? S.comp : 0)) * LG + x.lane];
        if (S.scaled) c = S.scale * c;
        if (hh < HASH_K_ONLY) {
            if (kk < CAP_UM) {
                if (x.valid) {
                    out.tq_hash[base * CAP_UM + kk] = (uint16_t)hh;
                    out.tq_coef[base * CAP_UM + kk] = c;
                }
            } else {
                bad |= ERR_OUTCAP;
            }
            kk++;
        } else {
            rad += fabs(c);
        }
    }
    if (bad && x.valid) err_or(x, bad);
    x.scr[(long)(NF + i) * LG + x.lane] = rad;
    if (!x.valid) return;
    atomicMax(&x.occ[2], kk);
    out.tq_cnt[base] = kk < CAP_UM ? kk : CAP_UM;
    out.tq_center[base] = cen(x, h, 0);
    out.tq_rad[base] = rad;
}

DI void torque_radius(const LCtx& x, const RobotParams& rp, const ReachOut& out) {
    const double ubc = rp.alpha * (rp.M_max - rp.M_min) * rp.eps;
    double tr[NF];
    Ival rho = Ival{0.0, 0.0};
#pragma unroll
    for (int i = 0; i < NF; i++) {
        const double rd = x.scr[(long)i * LG + x.lane];
        const Ival tmp = iv(0.0 - rd, 0.0 + rd);
        rho = iadd(rho, imul(tmp, tmp));
        tr[i] = ubc + 0.5 * fmax(fabs(tmp.lo), fabs(tmp.hi));
    }
    rho = isqrt(rho);
#pragma unroll
    for (int i = 0; i < NF; i++) tr[i] += 0.5 * rho.hi;
#pragma unroll
    for (int i = 0; i < NF; i++) tr[i] += x.scr[(long)(NF + i) * LG + x.lane];
#pragma unroll
    for (int i = 0; i < NF; i++) tr[i] += rp.friction[i];
    if (x.valid)
#pragma unroll
        for (int i = 0; i < NF; i++) out.torque_radius[x.job * NF + i] = tr[i];
}

// ---- the program ----------------------------------------------------------------------------
DI void op_terms_of(const LCtx& x, const Op& op, LTerms& T) {
    const LH& A = x.H[op.a];
    const LH& B = x.H[op.b];
    T.ns = 2;
    T.places = 0;
    T.negs = 0;
    T.S[0] = src_of(x, A);
    T.S[1] = src_of(x, B);
    switch (op.code) {
        case OP_MUL:
        case OP_CROSS_PP: {
            T.kind = 0;
            T.AR = op.code == OP_CROSS_PP ? 3 : A.R;
            T.AC = op.code == OP_CROSS_PP ? 1 : A.C;
            T.BC = op.code == OP_CROSS_PP ? 1 : B.C;
            T.nbm = B.cnt > 1 ? 0xFFFFFFFFu / (uint32_t)B.cnt + 1u : 0u;
            const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
            T.nout = op.code == OP_CROSS_PP ? 3 : (as ? nel(B) : (bs ? nel(A) : A.R * B.C));
            break;
        }
        case OP_ADD:
            T.kind = 1;
            T.negs = op.i < 0 ? 2 : 0;
            T.nout = nel(A);
            break;
        case OP_STACK3:
            T.kind = 1;
            T.ns = 3;
            T.S[2] = src_of(x, x.H[op.c]);
            T.places = 1 | (2 << 4) | (3 << 8);
            T.nout = 3;
            break;
        default:  // OP_ADD1D: self = a, 1-D = b at component i
            T.kind = 1;
            T.places = (op.i + 1) << 4;
            T.nout = nel(A);
            break;
    }
}
// this lane's operand centres, for the runtime-shaped (GAny) product readers only
DI void terms_centres(const LCtx& x, const Op& op, LTerms& T) {
    const LH& A = x.H[op.a];
    const LH& B = x.H[op.b];
    const int na = nel(A), nb = nel(B);
#pragma unroll
    for (int e = 0; e < 9; e++) {
        T.Ac[e] = e < na ? cen(x, A, e) : 0.0;
        T.Bc[e] = e < nb ? cen(x, B, e) : 0.0;
    }
}
DI int op_terms(const LCtx& x, const Op& op) {
    const LH& A = x.H[op.a];
    const LH& B = x.H[op.b];
    if (op.code == OP_MUL || op.code == OP_CROSS_PP) return A.cnt + B.cnt + A.cnt * B.cnt;
    if (op.code == OP_STACK3) return A.cnt + B.cnt + x.H[op.c].cnt;
    return A.cnt + B.cnt;
}
// output header of a simplifying op for this lane's job (wave 0), meta by lane 0
DI void op_header(const LCtx& x, const Op& op) {
    const LH& A = x.H[op.a];
    const LH& B = x.H[op.b];
    LH& h = x.H[op.o];
    int R, C;
    switch (op.code) {
        case OP_MUL: {
            const bool as = A.R == 1 && A.C == 1, bs = B.R == 1 && B.C == 1;
            R = as ? B.R : A.R;
            C = as ? B.C : (bs ? A.C : B.C);
            if (x.lane == 0) {
                if (as && !bs && B.R != 1 && A.cnt > 0 && B.cnt > 0) err_or(x, ERR_HANDLES);
                if (!as && !bs && !(A.R == 3 && A.C == 3 && B.R == 3)) err_or(x, ERR_HANDLES);
            }
            break;
        }
        case OP_CROSS_PP:
        case OP_STACK3: R = 3; C = 1; break;
        default: R = A.R; C = A.C; break;
    }
    LH hv = h;
    set_meta(hv, R, C);  // local copy: the formulas read R, C through it
    if (x.lane == 0) set_meta(h, R, C);
    switch (op.code) {
        case OP_MUL: header_mul(x, A, B, hv); break;
        case OP_ADD: header_add(x, A, B, hv, op.i); break;
        case OP_STACK3: header_stack3(x, A, B, x.H[op.c], hv); break;
        case OP_ADD1D: header_add_one_dim(x, A, B, hv, op.i); break;
        default: hdr_zero(x, hv.off, 3); break;  // CROSS_PP: the policy's finish writes it all
    }
}

constexpr int LDUMP_W = DUMP_W;  // per op and lane: [cnt, R*C, centre[0..2], ind0[0], ind1[0], absum[0]]

DI void dump_op(const LCtx& x, const Op* prog, int pc, int par, double* dump) {
    sync();
    if (x.wave == 0)
        for (int mi = 0; mi < par; mi++) {
            const int mo = prog[pc + mi].o;
            if (mo < 0) continue;
            const LH& h = x.H[mo];
            int cnt = 0;
            for (int k = 0; k < h.cnt; k++) cnt += (x.A->m[h.hoff + k] >> x.lane) & 1;
            double* d = dump + ((long)(pc + mi) * LDUMP_W) * LG + x.lane;
            const int n = nel(h);
            d[0 * LG] = cnt; d[1 * LG] = n; d[2 * LG] = P(x, h.off); d[3 * LG] = n > 1 ? P(x, h.off + 1) : 0.0;
            d[4 * LG] = n > 2 ? P(x, h.off + 2) : 0.0;
            d[5 * LG] = P(x, h.off + n); d[6 * LG] = P(x, h.off + 2 * n); d[7 * LG] = P(x, h.off + 3 * n);
        }
    sync();
}

DI void run_program(LCtx& x, const RobotParams& rp, const Op* prog, int nops, const ReachOut& out, double* dump) {
    for (int pc = 0; pc < nops; pc++) {
        const Op op = prog[pc];
        const int par = op.par > 1 ? op.par : 1;
        const long long c0 = (x.prof && x.tid == 0) ? clock64() : 0;
        int nterms = 0;
        x.opcode = op.code;
        switch (op.code) {
            case OP_JRS: break;  // this lane's JRS scalars are read from jrs_kernel's output in place
            case OP_MAKE1D:
            case OP_MAKEROT:
            case OP_MAKEBOX:
            case OP_CONST:
            case OP_ZERO:
            case OP_VIEW:
            case OP_TRANSPOSE:
            case OP_EMIT_LINK:
            case OP_EMIT_TORQUE:
                for (int mi = x.wave; mi < par; mi += LW) {
                    const Op m = prog[pc + mi];
                    switch (m.code) {
                        case OP_MAKE1D: make_1d(x, m.o, m.i, m.b); break;
                        case OP_MAKEROT: make_rot(x, m.o, rp, m.i); break;
                        case OP_MAKEBOX: make_box(x, m.o, rp, m.i); break;
                        case OP_CONST:
                            if (m.a == CONST_RPY) make_const(x, m.o, 3, 3, rp.rpy[m.i], 0.0);
                            else if (m.a == CONST_TRANS) make_const(x, m.o, 3, 1, &rp.trans[3 * m.i], 0.0);
                            else if (m.a == CONST_MASS) make_const(x, m.o, 1, 1, &rp.mass[m.i], rp.mass_uncertainty);
                            else make_const(x, m.o, 3, 3, &rp.inertia[9 * m.i], rp.inertia_uncertainty);
                            break;
                        case OP_ZERO: {
                            LH& h = x.H[m.o];
                            if (x.lane == 0) set_meta(h, m.b, m.c);
                            hdr_zero(x, h.off, m.b * m.c);
                            if (m.i) P(x, h.off + 2) = rp.gravity;
                            break;
                        }
                        case OP_VIEW: make_view(x, m.o, m.a, m.i, m.b, m.s); break;
                        case OP_TRANSPOSE: make_transpose(x, m.o, m.a); break;
                        case OP_EMIT_LINK: emit_link(x, out, m.a, m.i); break;
                        default: emit_torque(x, out, m.a, m.i); break;
                    }
                }
                // lane ops chained without a barrier in the per-job program may read each other's
                // output on another wave here: always publish
                sync();
                break;
            case OP_TORQUE_RADIUS:
                if (x.wave == 0) torque_radius(x, rp, out);
                sync();
                break;
            case OP_CROSS_C: {
                const double* v = op.b == VEC_TRANS ? &rp.trans[3 * op.c] : &rp.com[3 * op.c];
                const CrossC C = cross_const_table(op.i, v);
                if (x.wave == 0) {
                    LH hv = x.H[op.o];
                    set_meta(hv, 3, 1);
                    if (x.lane == 0) set_meta(x.H[op.o], 3, 1);
                    hdr_zero(x, hv.off, 3);
                }
                sync();
                cross_const(x, op.o, op.a, C);
                break;
            }
            default: {
                LTerms T;
                op_terms_of(x, op, T);
                const int N = op_terms(x, op);
                nterms = N;
                long long ph_t = x.prof ? clock64() : 0;
                if (x.wave == 0) op_header(x, op);
                stage_hashes(x, T);
                sync();
                LPHASE(0)
                const LH& A = x.H[op.a];
                const LH& B = x.H[op.b];
                const int na = ui(A.R * A.C), nb = ui(B.R * B.C);
                const bool views = ui(A.comp) >= 0 || ui(A.scaled) || ui(B.comp) >= 0 || ui(B.scaled);
                if (op.code == OP_CROSS_PP && !views && na == 3 && nb == 3) {
                    LPolCrossPP pol;
                    pol.base.thr = x.thr;
                    pol.a = op.a;
                    pol.b = op.b;
                    GCross Gc;
                    Gc.M = gen_mul<3, 3>(x, A, B);
                    simplify(x, op.o, T, Gc, pol, N);
                } else if (op.code == OP_MUL && !views && na == 9 && nb == 3) {
                    simplify(x, op.o, T, gen_mul<9, 3>(x, A, B), LPolBlock<3>{PolBlock<3>{x.thr}}, N);
                } else if (op.code == OP_MUL && !views && na == 9 && nb == 9) {
                    simplify(x, op.o, T, gen_mul<9, 9>(x, A, B), LPolBlock<9>{PolBlock<9>{x.thr}}, N);
                } else if (op.code == OP_MUL && !views && na == 1 && nb == 3) {
                    simplify(x, op.o, T, gen_mul<1, 3>(x, A, B), LPolBlock<3>{PolBlock<3>{x.thr}}, N);
                } else if (op.code != OP_MUL && op.code != OP_CROSS_PP && T.nout == 3) {
                    simplify(x, op.o, T, gen_cat<3>(x, op), LPolBlock<3>{PolBlock<3>{x.thr}}, N);
                } else if (op.code != OP_MUL && op.code != OP_CROSS_PP && T.nout == 1) {
                    simplify(x, op.o, T, gen_cat<1>(x, op), LPolBlock<1>{PolBlock<1>{x.thr}}, N);
                } else if (op.code == OP_CROSS_PP) {
                    terms_centres(x, op, T);
                    LPolCrossPP pol;
                    pol.base.thr = x.thr;
                    pol.a = op.a;
                    pol.b = op.b;
                    GAnyCross Gc{&T};
                    simplify(x, op.o, T, Gc, pol, N);
                } else if (T.nout == 1) {
                    terms_centres(x, op, T);
                    simplify(x, op.o, T, GAny<1>{&T}, LPolBlock<1>{PolBlock<1>{x.thr}}, N);
                } else if (T.nout == 3) {
                    terms_centres(x, op, T);
                    simplify(x, op.o, T, GAny<3>{&T}, LPolBlock<3>{PolBlock<3>{x.thr}}, N);
                } else {
                    terms_centres(x, op, T);
                    simplify(x, op.o, T, GAny<9>{&T}, LPolBlock<9>{PolBlock<9>{x.thr}}, N);
                }
                break;
            }
        }
        if (x.prof && x.tid == 0) {
            atomicAdd(&x.prof[2 * pc], (unsigned long long)(clock64() - c0));
            atomicAdd(&x.prof[2 * pc + 1], (unsigned long long)nterms);
        }
        if (dump) dump_op(x, prog, pc, par, dump);
        pc += par - 1;
    }
}

}  // namespace lane
}  // namespace armour
