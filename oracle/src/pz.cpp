// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
// Restatement of KPR/PZsparse.cu (see pz.h for the contract).
#include "pz.h"
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace oracle {

// KPR/PZsparse.h:23-35
const uint64_t MOVE_BIT_INC[NF * 6] = {2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2};
const uint64_t DEGREE_MASK[NF * 6] = {3, 3, 3, 3, 3, 3, 3, 1, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                      3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3};

// PZsparse.cu:587-603
uint64_t convertDegreeToHash(const uint64_t* degreeArray) {
    uint64_t degree = 0, move_bit = 0;
    for (int i = 0; i < NF * 6; i++) {
        if (degreeArray[i] > 1) throw std::runtime_error("degree can not be larger than 1!");
        degree += (degreeArray[i] << move_bit);
        move_bit += MOVE_BIT_INC[i];
    }
    return degree;
}

// PZsparse.cu:578-585
void convertHashToDegree(uint64_t degree, uint64_t* degreeArray) {
    for (int i = 0; i < NF * 6; i++) {
        degreeArray[i] = degree & DEGREE_MASK[i];
        degree >>= MOVE_BIT_INC[i];
    }
}

// Eigen 3.3 MatrixXd::norm() = sqrt(cwiseAbs2().sum()); the sum is a LinearVectorizedTraversal
// redux with SSE2 Packet2d on a 16-byte aligned heap block (alignedStart = 0): two packet
// accumulators over blocks of 4, combined, horizontal add, then the scalar tail.
double frob_norm(const double* x, int n) {
    double s[9];
    for (int i = 0; i < n; i++) s[i] = x[i] * x[i];
    const int ps = 2;
    const int alignedSize2 = (n / (2 * ps)) * (2 * ps);
    const int alignedSize = (n / ps) * ps;
    double res;
    if (alignedSize) {
        double r0a = s[0], r0b = s[1];
        if (alignedSize > ps) {
            double r1a = s[2], r1b = s[3];
            for (int idx = 2 * ps; idx < alignedSize2; idx += 2 * ps) {
                r0a = r0a + s[idx];
                r0b = r0b + s[idx + 1];
                r1a = r1a + s[idx + 2];
                r1b = r1b + s[idx + 3];
            }
            r0a = r0a + r1a;
            r0b = r0b + r1b;
            if (alignedSize > alignedSize2) {
                r0a = r0a + s[alignedSize2];
                r0b = r0b + s[alignedSize2 + 1];
            }
        }
        res = r0a + r0b;
        for (int idx = alignedSize; idx < n; idx++) res = res + s[idx];
    } else {
        res = s[0];
        for (int idx = 1; idx < n; idx++) res = res + s[idx];
    }
    return std::sqrt(res);
}

// coefficient-based product (Eigen lazy product, inner index summed in order), column-major
static inline void matmul(const double* A, int ra, int ca, const double* B, int cb, double* out) {
    double tmp[9];
    for (int j = 0; j < cb; j++)
        for (int i = 0; i < ra; i++) {
            double acc = A[i] * B[j * ca];
            for (int k = 1; k < ca; k++) acc = acc + A[i + k * ra] * B[k + j * ca];
            tmp[i + j * ra] = acc;
        }
    std::memcpy(out, tmp, sizeof(double) * ra * cb);
}

PZ::PZ(int r, int c) : R(r), C(c) {}
PZ::PZ(double c0) : R(1), C(1) { center[0] = c0; }
PZ::PZ(int r, int c, const double* cm) : R(r), C(c) {
    for (int e = 0; e < r * c; e++) center[e] = cm[e];
}
PZ::PZ(int r, int c, const double* cm, double unc) : R(r), C(c) {
    for (int e = 0; e < r * c; e++) { center[e] = cm[e]; indep[e] = unc * std::fabs(cm[e]); }
}
PZ::PZ(double center_inp, const double* coeff, const uint64_t (*degree)[NF * 6], int num, double thr) : R(1), C(1) {
    center[0] = center_inp;
    poly.reserve(num);
    for (int i = 0; i < num; i++) {
        Mono m{};
        m.c[0] = coeff[i];
        m.h = convertDegreeToHash(degree[i]);
        poly.push_back(m);
    }
    simplify(thr);
}

PZ PZ::rpy(double roll, double pitch, double yaw) {
    PZ r(3, 3);
    double* c = r.center;  // col-major: (i,j) -> i + 3j
    c[0 + 0] = std::cos(pitch) * std::cos(yaw);
    c[0 + 3] = -std::cos(pitch) * std::sin(yaw);
    c[0 + 6] = std::sin(pitch);
    c[1 + 0] = std::cos(roll) * std::sin(yaw) + std::cos(yaw) * std::sin(pitch) * std::sin(roll);
    c[1 + 3] = std::cos(roll) * std::cos(yaw) - std::sin(pitch) * std::sin(roll) * std::sin(yaw);
    c[1 + 6] = -std::cos(pitch) * std::sin(roll);
    c[2 + 0] = std::sin(roll) * std::sin(yaw) - std::cos(roll) * std::cos(yaw) * std::sin(pitch);
    c[2 + 3] = std::cos(yaw) * std::sin(roll) + std::cos(roll) * std::sin(pitch) * std::sin(yaw);
    c[2 + 6] = std::cos(pitch) * std::cos(roll);
    return r;
}

// PZsparse.cu:211-250
static void makeRotationMatrix(double* R, double cosElt, double sinElt, int axis, bool startFromZero) {
    for (int e = 0; e < 9; e++) R[e] = 0.0;
    if (!startFromZero) { R[0] = 1.0; R[4] = 1.0; R[8] = 1.0; }
    const double negSinElt = -1.0 * sinElt;
    switch (axis) {
        case 0: return;
        case 1: R[1 + 3] = cosElt; R[1 + 6] = negSinElt; R[2 + 3] = sinElt; R[2 + 6] = cosElt; break;
        case 2: R[0 + 0] = cosElt; R[0 + 6] = sinElt; R[2 + 0] = negSinElt; R[2 + 6] = cosElt; break;
        case 3: R[0 + 0] = cosElt; R[0 + 3] = negSinElt; R[1 + 0] = sinElt; R[1 + 3] = cosElt; break;
        default: throw std::runtime_error("Undefined axis");
    }
}

PZ PZ::rot(double cos_c, const double* cos_coeff, const uint64_t (*cos_deg)[NF * 6], int ncos,
           double sin_c, const double* sin_coeff, const uint64_t (*sin_deg)[NF * 6], int nsin,
           int axis, double thr) {
    PZ r(3, 3);
    makeRotationMatrix(r.center, cos_c, sin_c, axis, false);
    r.poly.reserve(ncos + nsin);
    for (int i = 0; i < ncos; i++) {
        Mono m{};
        makeRotationMatrix(m.c, cos_coeff[i], 0, axis, true);
        m.h = convertDegreeToHash(cos_deg[i]);
        r.poly.push_back(m);
    }
    for (int i = 0; i < nsin; i++) {
        Mono m{};
        makeRotationMatrix(m.c, 0, sin_coeff[i], axis, true);
        m.h = convertDegreeToHash(sin_deg[i]);
        r.poly.push_back(m);
    }
    r.simplify(thr);
    return r;
}

// PZsparse.cu:284-350. The reference's std::sort leaves the order of equal hashes unspecified,
// and with it the summation order of a merged group (rounding only). Here equal hashes keep their
// generation order (stable sort), the order the HIP engines sum in (term index).
void PZ::simplify(double thr) {
    const int n = R * C;
    std::stable_sort(poly.begin(), poly.end(), [](const Mono& l, const Mono& r) { return l.h < r.h; });
    double red[9] = {0};
    std::vector<Mono> out;
    out.reserve(poly.size());
    size_t i = 0;
    while (i < poly.size()) {
        size_t j;
        const uint64_t h = poly[i].h;
        for (j = i + 1; j < poly.size(); j++) {
            if (poly[j].h != h) break;
            for (int e = 0; e < n; e++) poly[i].c[e] = poly[i].c[e] + poly[j].c[e];
        }
        if (frob_norm(poly[i].c, n) <= thr) {
            for (int e = 0; e < n; e++) red[e] = red[e] + std::fabs(poly[i].c[e]);
        } else {
            out.push_back(poly[i]);
        }
        i = j;
    }
    poly.swap(out);
    if (frob_norm(red, n) != 0)
        for (int e = 0; e < n; e++) indep[e] = indep[e] + red[e];
}

// PZsparse.cu:352-368
void PZ::reduce() {
    const int n = R * C;
    std::vector<Mono> out;
    out.reserve(poly.size());
    for (const Mono& m : poly) {
        if (m.h < HASH_K_ONLY) out.push_back(m);
        else for (int e = 0; e < n; e++) indep[e] += std::fabs(m.c[e]);
    }
    poly.swap(out);
}

// PZsparse.cu:370-402 ; out is Eigen::Matrix<double,3,6> in column-major
void PZ::reduce_link_PZ(double out[18]) {
    assert(R == 3 && C == 1);
    for (int e = 0; e < 18; e++) out[e] = 0.0;
    std::vector<Mono> keep;
    keep.reserve(poly.size());
    int j = 0;
    for (const Mono& m : poly) {
        if (m.h < HASH_K_ONLY) {
            keep.push_back(m);
        } else if (m.h < HASH_K_LINKS_ONLY && (m.h & K_MASK) == 0) {
            if (j >= 3) throw std::runtime_error("reduce_link_PZ: more than 3 link generators");
            for (int r = 0; r < 3; r++) out[r + 3 * j] = m.c[r];
            j++;
        } else {
            for (int e = 0; e < 3; e++) indep[e] += std::fabs(m.c[e]);
        }
    }
    poly.swap(keep);
    out[0 + 3 * 3] = indep[0];
    out[1 + 3 * 4] = indep[1];
    out[2 + 3 * 5] = indep[2];
}

// PZsparse.cu:404-435
void PZ::slice(const double* x, double* rc, double* rr) const {
    const int n = R * C;
    for (int e = 0; e < n; e++) { rc[e] = center[e]; rr[e] = indep[e]; }
    uint64_t deg[NF * 6];
    for (const Mono& m : poly) {
        double tmp[9];
        for (int e = 0; e < n; e++) tmp[e] = m.c[e];
        if (m.h < ((uint64_t)1 << (2 * NF))) {
            convertHashToDegree(m.h, deg);
            for (int j = 0; j < NF; j++) {
                const double p = std::pow(x[j], (double)deg[j]);
                for (int e = 0; e < n; e++) tmp[e] = tmp[e] * p;
            }
            for (int e = 0; e < n; e++) rc[e] = rc[e] + tmp[e];
        } else {
            for (int e = 0; e < n; e++) rr[e] = rr[e] + std::fabs(tmp[e]);
        }
    }
}

// PZsparse.cu:437-555 (all three overloads share this arithmetic); grad[k * n + e]
void PZ::slice_grad(const double* x, double* grad) const {
    const int n = R * C;
    for (int k = 0; k < NF * n; k++) grad[k] = 0.0;
    uint64_t deg[NF * 6];
    double tmp[NF][9];
    for (const Mono& m : poly) {
        if (m.h <= ((uint64_t)1 << (2 * NF))) {
            for (int k = 0; k < NF; k++)
                for (int e = 0; e < n; e++) tmp[k][e] = m.c[e];
            convertHashToDegree(m.h, deg);
            for (int j = 0; j < NF; j++) {
                for (int k = 0; k < NF; k++) {
                    if (j == k) {
                        if (deg[j] == 0) {
                            for (int e = 0; e < n; e++) tmp[k][e] = 0.0;
                        } else {
                            const double f = (double)deg[j] * std::pow(x[j], (double)(deg[j] - 1));
                            for (int e = 0; e < n; e++) tmp[k][e] = tmp[k][e] * f;
                        }
                    } else {
                        const double p = std::pow(x[j], (double)deg[j]);
                        for (int e = 0; e < n; e++) tmp[k][e] = tmp[k][e] * p;
                    }
                }
            }
            for (int k = 0; k < NF; k++)
                for (int e = 0; e < n; e++) grad[k * n + e] = grad[k * n + e] + tmp[k][e];
        }
    }
}

// PZsparse.cu:557-576 ; the Interval(l,u) constructor's checking is applied by the caller
void PZ::toInterval(double* lo, double* hi) const {
    const int n = R * C;
    double rad[9];
    for (int e = 0; e < n; e++) rad[e] = indep[e];
    for (const Mono& m : poly)
        for (int e = 0; e < n; e++) rad[e] = rad[e] + std::fabs(m.c[e]);
    for (int e = 0; e < n; e++) { lo[e] = center[e] - rad[e]; hi[e] = center[e] + rad[e]; }
}

// PZsparse.cu:678-697
PZ PZ::elem(int r, int c) const {
    PZ res(1, 1);
    const int idx = r + c * R;
    res.center[0] = center[idx];
    res.poly.reserve(poly.size());
    for (const Mono& m : poly) {
        Mono q{};
        q.c[0] = m.c[idx];
        q.h = m.h;
        res.poly.push_back(q);
    }
    res.indep[0] = indep[idx];
    return res;
}

static inline void transpose_block(const double* a, int R, int C, double* out) {
    double tmp[9];
    for (int i = 0; i < R; i++)
        for (int j = 0; j < C; j++) tmp[j + i * C] = a[i + j * R];
    std::memcpy(out, tmp, sizeof(double) * R * C);
}

// PZsparse.cu:1050-1066
PZ PZ::transpose() const {
    PZ res(C, R);
    transpose_block(center, R, C, res.center);
    res.poly.reserve(poly.size());
    for (const Mono& m : poly) {
        Mono q{};
        transpose_block(m.c, R, C, q.c);
        q.h = m.h;
        res.poly.push_back(q);
    }
    transpose_block(indep, R, C, res.indep);
    return res;
}

// PZsparse.cu:1068-1085
void PZ::addOneDimPZ(const PZ& a, int r, int c, double thr) {
    const int idx = r + c * R;
    center[idx] += a.center[0];
    for (const Mono& m : a.poly) {
        Mono q{};
        q.c[idx] = m.c[0];
        q.h = m.h;
        poly.push_back(q);
    }
    indep[idx] += a.indep[0];
    simplify(thr);
}

// PZsparse.cu:743-764
PZ add(const PZ& a, const PZ& b, double thr) {
    PZ res(a.R, a.C);
    const int n = a.R * a.C;
    for (int e = 0; e < n; e++) res.center[e] = a.center[e] + b.center[e];
    res.poly.reserve(a.poly.size() + b.poly.size());
    res.poly.insert(res.poly.end(), a.poly.begin(), a.poly.end());
    for (const Mono& m : b.poly) res.poly.push_back(m);
    for (int e = 0; e < n; e++) res.indep[e] = a.indep[e] + b.indep[e];
    res.simplify(thr);
    return res;
}

// PZsparse.cu:813-834
PZ sub(const PZ& a, const PZ& b, double thr) {
    PZ res(a.R, a.C);
    const int n = a.R * a.C;
    for (int e = 0; e < n; e++) res.center[e] = a.center[e] - b.center[e];
    res.poly.reserve(a.poly.size() + b.poly.size());
    res.poly.insert(res.poly.end(), a.poly.begin(), a.poly.end());
    for (const Mono& m : b.poly) {
        Mono q{};
        for (int e = 0; e < n; e++) q.c[e] = -m.c[e];
        q.h = m.h;
        res.poly.push_back(q);
    }
    for (int e = 0; e < n; e++) res.indep[e] = a.indep[e] + b.indep[e];
    res.simplify(thr);
    return res;
}

// PZsparse.cu:864-994
PZ mul(const PZ& a, const PZ& b, double thr) {
    const bool as = (a.R == 1 && a.C == 1);
    const bool bs = (b.R == 1 && b.C == 1);
    PZ res;
    if (as) { res.R = b.R; res.C = b.C; }
    else if (bs) { res.R = a.R; res.C = a.C; }
    else { res.R = a.R; res.C = b.C; }
    const int na = a.R * a.C, nb = b.R * b.C, nr = res.R * res.C;
    // the reference forms `it1.coeff * it2.coeff` before branching (:926); Eigen's live
    // eigen_assert aborts on a (1x1)*(Rx C) product with R != 1 — mirror that failure.
    if (as && !bs && b.R != 1 && !a.poly.empty() && !b.poly.empty())
        throw std::runtime_error("invalid matrix product (Eigen assert in PZsparse::operator*)");

    // center * center
    if (as) for (int e = 0; e < nb; e++) res.center[e] = a.center[0] * b.center[e];
    else if (bs) for (int e = 0; e < na; e++) res.center[e] = a.center[e] * b.center[0];
    else matmul(a.center, a.R, a.C, b.center, b.C, res.center);

    res.poly.reserve(a.poly.size() + b.poly.size() + a.poly.size() * b.poly.size());
    for (const Mono& m : a.poly) {
        Mono q{};
        q.h = m.h;
        if (as) for (int e = 0; e < nb; e++) q.c[e] = m.c[0] * b.center[e];
        else if (bs) for (int e = 0; e < na; e++) q.c[e] = m.c[e] * b.center[0];
        else matmul(m.c, a.R, a.C, b.center, b.C, q.c);
        res.poly.push_back(q);
    }
    for (const Mono& m : b.poly) {
        Mono q{};
        q.h = m.h;
        if (as) for (int e = 0; e < nb; e++) q.c[e] = a.center[0] * m.c[e];
        else if (bs) for (int e = 0; e < na; e++) q.c[e] = a.center[e] * m.c[0];
        else matmul(a.center, a.R, a.C, m.c, b.C, q.c);
        res.poly.push_back(q);
    }
    for (const Mono& m1 : a.poly) {
        for (const Mono& m2 : b.poly) {
            Mono q{};
            if (as) for (int e = 0; e < nb; e++) q.c[e] = m1.c[0] * m2.c[e];
            else if (bs) for (int e = 0; e < na; e++) q.c[e] = m1.c[e] * m2.c[0];
            else matmul(m1.c, a.R, a.C, m2.c, b.C, q.c);
            q.h = m1.h + m2.h;  // carry-less by design (:938-940)
            res.poly.push_back(q);
        }
    }

    // a.independent * (center + polynomial)
    double r2[9];
    for (int e = 0; e < na; e++) r2[e] = std::fabs(a.center[e]);
    for (const Mono& m : a.poly)
        for (int e = 0; e < na; e++) r2[e] = r2[e] + std::fabs(m.c[e]);
    if (as) { const double s = r2[0]; for (int e = 0; e < nb; e++) r2[e] = s * b.indep[e]; }
    else if (bs) { for (int e = 0; e < na; e++) r2[e] = r2[e] * b.indep[0]; }
    else matmul(r2, a.R, a.C, b.indep, b.C, r2);

    // independent * (a.center + a.polynomial)
    double r3[9];
    for (int e = 0; e < nb; e++) r3[e] = std::fabs(b.center[e]);
    for (const Mono& m : b.poly)
        for (int e = 0; e < nb; e++) r3[e] = r3[e] + std::fabs(m.c[e]);
    if (as) { for (int e = 0; e < nb; e++) r3[e] = a.indep[0] * r3[e]; }
    else if (bs) { const double s = r3[0]; for (int e = 0; e < na; e++) r3[e] = a.indep[e] * s; }
    else matmul(a.indep, a.R, a.C, r3, b.C, r3);

    double red[9];
    for (int e = 0; e < nr; e++) red[e] = r2[e] + r3[e];
    if (as) for (int e = 0; e < nr; e++) res.indep[e] = a.indep[0] * b.indep[e] + red[e];
    else if (bs) for (int e = 0; e < nr; e++) res.indep[e] = a.indep[e] * b.indep[0] + red[e];
    else {
        double ii[9];
        matmul(a.indep, a.R, a.C, b.indep, b.C, ii);
        for (int e = 0; e < nr; e++) res.indep[e] = ii[e] + red[e];
    }
    res.simplify(thr);
    return res;
}

// PZsparse.cu:996-1030 (no simplify)
PZ scale(double s, const PZ& b) {
    PZ res(b.R, b.C);
    const int n = b.R * b.C;
    for (int e = 0; e < n; e++) res.center[e] = b.center[e] * s;
    res.poly.reserve(b.poly.size());
    for (const Mono& m : b.poly) {
        Mono q{};
        for (int e = 0; e < n; e++) q.c[e] = s * m.c[e];
        q.h = m.h;
        res.poly.push_back(q);
    }
    for (int e = 0; e < n; e++) res.indep[e] = b.indep[e] * std::fabs(s);
    return res;
}

// PZsparse.cu:725-741 — note: the reference leaves `independent` at zero here
PZ neg(const PZ& a) {
    PZ res(a.R, a.C);
    const int n = a.R * a.C;
    for (int e = 0; e < n; e++) res.center[e] = -a.center[e];
    for (const Mono& m : a.poly) {
        Mono q{};
        for (int e = 0; e < n; e++) q.c[e] = -m.c[e];
        q.h = m.h;
        res.poly.push_back(q);
    }
    return res;
}

// PZsparse.cu:1087-1116
PZ stack3(const PZ& a0, const PZ& a1, const PZ& a2, double thr) {
    const PZ* a[3] = {&a0, &a1, &a2};
    PZ res(3, 1);
    for (int i = 0; i < 3; i++) res.center[i] = a[i]->center[0];
    res.poly.reserve(3 * a0.poly.size());
    for (int i = 0; i < 3; i++)
        for (const Mono& m : a[i]->poly) {
            Mono q{};
            q.c[i] = m.c[0];
            q.h = m.h;
            res.poly.push_back(q);
        }
    for (int i = 0; i < 3; i++) res.indep[i] = a[i]->indep[0];
    res.simplify(thr);
    return res;
}

// PZsparse.cu:1118-1132
PZ cross_mp(const double* a, const PZ& b, double thr) {
    PZ b0 = b.elem(0, 0), b1 = b.elem(1, 0), b2 = b.elem(2, 0);
    PZ r0 = sub(scale(a[1], b2), scale(a[2], b1), thr);
    PZ r1 = sub(scale(a[2], b0), scale(a[0], b2), thr);
    PZ r2 = sub(scale(a[0], b1), scale(a[1], b0), thr);
    return stack3(r0, r1, r2, thr);
}

// PZsparse.cu:1134-1151
PZ cross_pp(const PZ& a, const PZ& b, double thr) {
    PZ a0 = a.elem(0, 0), a1 = a.elem(1, 0), a2 = a.elem(2, 0);
    PZ b0 = b.elem(0, 0), b1 = b.elem(1, 0), b2 = b.elem(2, 0);
    PZ r0 = sub(mul(a1, b2, thr), mul(a2, b1, thr), thr);
    PZ r1 = sub(mul(a2, b0, thr), mul(a0, b2, thr), thr);
    PZ r2 = sub(mul(a0, b1, thr), mul(a1, b0, thr), thr);
    return stack3(r0, r1, r2, thr);
}

// PZsparse.cu:1153-1167
PZ cross_pm(const PZ& a, const double* b, double thr) {
    PZ a0 = a.elem(0, 0), a1 = a.elem(1, 0), a2 = a.elem(2, 0);
    PZ r0 = sub(scale(b[2], a1), scale(b[1], a2), thr);
    PZ r1 = sub(scale(b[0], a2), scale(b[2], a0), thr);
    PZ r2 = sub(scale(b[1], a0), scale(b[0], a1), thr);
    return stack3(r0, r1, r2, thr);
}

}  // namespace oracle
