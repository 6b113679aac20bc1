// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product.
//
// Restatement of the reference's sparse polynomial zonotope, class PZsparse
// (KPR/PZsparse.h:50-183, KPR/PZsparse.cu:50-1167), with identical semantics:
//   * 63-bit monomial hash over 42 factors (KPR/PZsparse.h:23-40), carry-less addition on products;
//   * simplify() (KPR/PZsparse.cu:284-350): std::sort by hash (same libstdc++ introsort, so the
//     same permutation as the reference), merge equal hashes in sorted order, prune merged
//     coefficients with Frobenius norm <= SIMPLIFY_THRESHOLD into `independent`;
//   * every operator calls simplify() exactly where the reference does;
//   * Eigen's arithmetic order is reproduced: coefficient-based products sum the inner index
//     sequentially; MatrixXd::norm() uses the SSE2 packet redux order (see frob_norm()).
// Coefficients are stored column-major in a fixed 9-double block (the largest PZ is 3x3).
#pragma once
#include <cstdint>
#include <vector>
#include "interval.h"
#include "robot.h"

namespace oracle {

// KPR/PZsparse.h:23-40
extern const uint64_t MOVE_BIT_INC[NF * 6];
extern const uint64_t DEGREE_MASK[NF * 6];
constexpr uint64_t HASH_K_ONLY = (uint64_t)1 << (2 * NF);        // max_hash_dependent_k_only
constexpr uint64_t HASH_K_LINKS_ONLY = (uint64_t)1 << (5 * NF);  // max_hash_dependent_k_links_only
constexpr uint64_t K_MASK = HASH_K_ONLY - 1;                      // dependent_k_mask

uint64_t convertDegreeToHash(const uint64_t* degreeArray);
void convertHashToDegree(uint64_t degree, uint64_t* degreeArray);

struct Mono {
    double c[9];
    uint64_t h;
};

double frob_norm(const double* x, int n);

struct PZ {
    int R = 1, C = 1;
    double center[9] = {0};
    std::vector<Mono> poly;
    double indep[9] = {0};

    PZ() {}
    PZ(int r, int c);                                  // PZsparse.cu:50-55 (zeros)
    explicit PZ(double c0);                            // :66-72
    PZ(int r, int c, const double* center_cm);         // :75-80 (Eigen matrix ctor)
    PZ(int r, int c, const double* center_cm, double uncertainty);  // :93-98
    // 1x1 PZ from monomials (:120-136) and with independent interval (:139-157)
    PZ(double center_inp, const double* coeff, const uint64_t (*degree)[NF * 6], int num, double thr);
    // RPY rotation (:160-176)
    static PZ rpy(double roll, double pitch, double yaw);
    // rotation about axis from cos/sin 1-D PZ data (:179-205)
    static PZ rot(double cos_c, const double* cos_coeff, const uint64_t (*cos_deg)[NF * 6], int ncos,
                  double sin_c, const double* sin_coeff, const uint64_t (*sin_deg)[NF * 6], int nsin,
                  int axis, double thr);

    int size() const { return R * C; }
    void simplify(double thr);
    void reduce();                                     // :352-368
    void reduce_link_PZ(double out36[18]);             // :370-402 (3x6 col-major)
    // slice value (:404-435): returns center and radius arrays (size R*C)
    void slice(const double* x, double* res_center, double* res_radius) const;
    // slice gradient (:437-555): grad[k*R*C + e]
    void slice_grad(const double* x, double* grad) const;
    // toInterval (:557-576)
    void toInterval(double* lo, double* hi) const;

    PZ elem(int r, int c) const;                       // operator()(r,c) :678-697
    PZ transpose() const;                              // :1050-1066
    void addOneDimPZ(const PZ& a, int r, int c, double thr);  // :1068-1085
};

PZ add(const PZ& a, const PZ& b, double thr);            // operator+ :743-764
PZ sub(const PZ& a, const PZ& b, double thr);            // operator- :813-834
PZ mul(const PZ& a, const PZ& b, double thr);            // operator* :864-994
PZ scale(double s, const PZ& b);                         // double * PZ  :1014-1030 / PZ * double :996-1012
PZ neg(const PZ& a);                                     // unary - :725-741 (drops independent)
PZ stack3(const PZ& a0, const PZ& a1, const PZ& a2, double thr);  // stack :1087-1116
PZ cross_mp(const double* a, const PZ& b, double thr);   // cross(MatrixXd, PZ) :1118-1132
PZ cross_pp(const PZ& a, const PZ& b, double thr);       // cross(PZ, PZ) :1134-1151
PZ cross_pm(const PZ& a, const double* b, double thr);   // cross(PZ, MatrixXd) :1153-1167

}  // namespace oracle
