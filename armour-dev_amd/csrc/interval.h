// armour-mi355x — outward-rounded interval arithmetic for the JRS (KPR/Trajectory.cu:97-134) and
// the torque bound (KPR/armour_main.cu:180-191). Same operation set and case analysis as the
// reference's boost::numeric::interval policy (KPR/Headers.h:30-36); directed rounding uses the
// gfx950 round-toward-(-inf / +inf) ocml primitives on the device. The host side of these
// functions exists only for the sequential emulation used by the CPU tests.
#pragma once
#include "common.h"
#if !defined(__HIP_DEVICE_COMPILE__)
#include <cfenv>
#include <cmath>
#endif

namespace armour {

#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline double add_dn(double a, double b) { return __ocml_add_rtn_f64(a, b); }
__device__ inline double add_up(double a, double b) { return __ocml_add_rtp_f64(a, b); }
__device__ inline double sub_dn(double a, double b) { return __ocml_sub_rtn_f64(a, b); }
__device__ inline double sub_up(double a, double b) { return __ocml_sub_rtp_f64(a, b); }
__device__ inline double mul_dn(double a, double b) { return __ocml_mul_rtn_f64(a, b); }
__device__ inline double mul_up(double a, double b) { return __ocml_mul_rtp_f64(a, b); }
// division / square root rounded toward -inf / +inf from the round-to-nearest result and its
// exact fma residual (ocml ships no directed-rounding div/sqrt for f64)
__device__ inline double div_dn(double a, double b) {
    const double q = a / b;
    const double r = fma(-q, b, a);  // a - q*b exactly
    return (r != 0 && ((r < 0) != (b < 0))) ? nextafter(q, -__builtin_inf()) : q;
}
__device__ inline double sqrt_dn(double a) {
    const double s = sqrt(a);
    return fma(-s, s, a) < 0 ? nextafter(s, -__builtin_inf()) : s;
}
__device__ inline double sqrt_up(double a) {
    const double s = sqrt(a);
    return fma(-s, s, a) > 0 ? nextafter(s, __builtin_inf()) : s;
}
#else
inline double rnd_op(int mode, int op, double a, double b) {
    std::fesetround(mode);
    volatile double r;
    switch (op) {
        case 0: r = a + b; break;
        case 1: r = a - b; break;
        case 2: r = a * b; break;
        case 3: r = a / b; break;
        default: r = std::sqrt(a); break;
    }
    std::fesetround(FE_TONEAREST);
    return r;
}
inline double add_dn(double a, double b) { return rnd_op(FE_DOWNWARD, 0, a, b); }
inline double add_up(double a, double b) { return rnd_op(FE_UPWARD, 0, a, b); }
inline double sub_dn(double a, double b) { return rnd_op(FE_DOWNWARD, 1, a, b); }
inline double sub_up(double a, double b) { return rnd_op(FE_UPWARD, 1, a, b); }
inline double mul_dn(double a, double b) { return rnd_op(FE_DOWNWARD, 2, a, b); }
inline double mul_up(double a, double b) { return rnd_op(FE_UPWARD, 2, a, b); }
inline double div_dn(double a, double b) { return rnd_op(FE_DOWNWARD, 3, a, b); }
inline double sqrt_dn(double a) { return rnd_op(FE_DOWNWARD, 4, a, 0); }
inline double sqrt_up(double a) { return rnd_op(FE_UPWARD, 4, a, 0); }
#endif

// boost/numeric/interval/constants.hpp (exact binary fractions)
constexpr double PI_D_L = (3373259426.0 + 273688.0 / (1 << 21)) / (1 << 30);
constexpr double PI_D_U = (3373259426.0 + 273689.0 / (1 << 21)) / (1 << 30);

struct Ival {
    double lo, hi;
};

AD Ival iv(double l, double u) {
    // checking_base constructor: empty (NaN) unless l <= u
    if (!(l <= u)) { const double nan = __builtin_nan(""); return Ival{nan, nan}; }
    return Ival{l, u};
}
AD Ival ineg(Ival x) { return Ival{-x.hi, -x.lo}; }
AD Ival iadd(Ival x, Ival y) { return Ival{add_dn(x.lo, y.lo), add_up(x.hi, y.hi)}; }
AD Ival iadd(double x, Ival y) { return Ival{add_dn(x, y.lo), add_up(x, y.hi)}; }
AD Ival isub(Ival x, Ival y) { return Ival{sub_dn(x.lo, y.hi), sub_up(x.hi, y.lo)}; }
AD Ival isub(Ival x, double y) { return Ival{sub_dn(x.lo, y), sub_up(x.hi, y)}; }
AD Ival imul(double x, Ival y) {
    if (x < 0) return Ival{mul_dn(x, y.hi), mul_up(x, y.lo)};
    if (x == 0) return Ival{0.0, 0.0};
    return Ival{mul_dn(x, y.lo), mul_up(x, y.hi)};
}
AD Ival imul(Ival x, Ival y) {
    const double xl = x.lo, xu = x.hi, yl = y.lo, yu = y.hi;
    if (xl < 0) {
        if (xu > 0) {
            if (yl < 0) {
                if (yu > 0) return Ival{fmin(mul_dn(xl, yu), mul_dn(xu, yl)), fmax(mul_up(xl, yl), mul_up(xu, yu))};
                return Ival{mul_dn(xu, yl), mul_up(xl, yl)};
            }
            if (yu > 0) return Ival{mul_dn(xl, yu), mul_up(xu, yu)};
            return Ival{0.0, 0.0};
        }
        if (yl < 0) {
            if (yu > 0) return Ival{mul_dn(xl, yu), mul_up(xl, yl)};
            return Ival{mul_dn(xu, yu), mul_up(xl, yl)};
        }
        if (yu > 0) return Ival{mul_dn(xl, yu), mul_up(xu, yl)};
        return Ival{0.0, 0.0};
    }
    if (xu > 0) {
        if (yl < 0) {
            if (yu > 0) return Ival{mul_dn(xu, yl), mul_up(xu, yu)};
            return Ival{mul_dn(xu, yl), mul_up(xl, yu)};
        }
        if (yu > 0) return Ival{mul_dn(xl, yl), mul_up(xu, yu)};
        return Ival{0.0, 0.0};
    }
    return Ival{0.0, 0.0};
}
AD Ival isqr(Ival x) {  // pow(x, 2) (power.hpp, square-and-multiply with directed products)
    if (x.hi < 0) return Ival{mul_dn(-x.hi, -x.hi), mul_up(-x.lo, -x.lo)};
    if (x.lo < 0) { const double m = fmax(-x.lo, x.hi); return Ival{0.0, mul_up(m, m)}; }
    return Ival{mul_dn(x.lo, x.lo), mul_up(x.hi, x.hi)};
}
AD Ival isqrt(Ival x) {
    const double l = !(x.lo > 0) ? 0.0 : sqrt_dn(x.lo);
    return Ival{l, sqrt_up(x.hi)};
}
AD double iwidth(Ival x) { return sub_up(x.hi, x.lo); }
AD double icenter(Ival a) { return (a.lo + a.hi) * 0.5; }
AD double iradius(Ival a) { return (a.hi - a.lo) * 0.5; }

// transc.hpp cos(interval): fmod by [2 pi], then monotone pieces; the reference's one-level
// recursion `-cos(tmp - pi)` is unrolled into a sign flag
AD Ival icos(Ival x) {
    bool negate = false;
    const Ival pi2{PI_D_L * 2, PI_D_U * 2};
    for (int depth = 0; depth < 4; depth++) {
        const double yb = (x.lo < 0) ? pi2.lo : pi2.hi;
        const double nq = floor(div_dn(x.lo, yb));
        const Ival tmp = isub(x, imul(nq, pi2));
        Ival r;
        if (iwidth(tmp) >= pi2.lo) {
            r = Ival{-1.0, 1.0};
        } else if (tmp.lo >= PI_D_U) {
            x = isub(tmp, Ival{PI_D_L, PI_D_U});
            negate = !negate;
            continue;
        } else {
            const double l = tmp.lo, u = tmp.hi;
            if (u <= PI_D_L) r = Ival{cos(u), cos(l)};
            else if (u <= pi2.lo) r = Ival{-1.0, cos(fmin(sub_dn(pi2.lo, u), l))};
            else r = Ival{-1.0, 1.0};
        }
        return negate ? ineg(r) : r;
    }
    return Ival{-1.0, 1.0};
}
AD Ival isin(Ival x) { return icos(isub(x, Ival{PI_D_L / 2, PI_D_U / 2})); }

}  // namespace armour
