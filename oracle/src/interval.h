// ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into the product (libarmour_hip.so).
//
// Restatement of the interval type the reference uses:
//   boost::numeric::interval<double, policies<save_state<rounded_transc_std<double>>,
//                                             checking_base<double>>>      (KPR/Headers.h:30-36)
// Boost 1.71 is not present in this image; this file restates the published
// algorithms of boost/numeric/interval/{arith,arith2,transc,rounded_arith,rounded_transc,
// constants}.hpp for the operations the reference actually calls:
//   + - * (interval/interval, interval/double), unary -, +=, pow(I,int), sqrt(I), cos(I), sin(I),
//   width, and the (l,u) constructor with checking_base (empty == NaN bounds).
// Directed rounding is done the way rounded_arith_std does it: switch the FPU rounding mode
// around every elementary operation (fesetround), restoring round-to-nearest afterwards
// (save_state). Requires -frounding-math.
#pragma once
#include <cfenv>
#include <cmath>
#include <limits>
#include <algorithm>

namespace oracle {

struct Rnd {
    static double add_dn(double a, double b) { std::fesetround(FE_DOWNWARD); volatile double r = a + b; std::fesetround(FE_TONEAREST); return r; }
    static double add_up(double a, double b) { std::fesetround(FE_UPWARD);   volatile double r = a + b; std::fesetround(FE_TONEAREST); return r; }
    static double sub_dn(double a, double b) { std::fesetround(FE_DOWNWARD); volatile double r = a - b; std::fesetround(FE_TONEAREST); return r; }
    static double sub_up(double a, double b) { std::fesetround(FE_UPWARD);   volatile double r = a - b; std::fesetround(FE_TONEAREST); return r; }
    static double mul_dn(double a, double b) { std::fesetround(FE_DOWNWARD); volatile double r = a * b; std::fesetround(FE_TONEAREST); return r; }
    static double mul_up(double a, double b) { std::fesetround(FE_UPWARD);   volatile double r = a * b; std::fesetround(FE_TONEAREST); return r; }
    static double div_dn(double a, double b) { std::fesetround(FE_DOWNWARD); volatile double r = a / b; std::fesetround(FE_TONEAREST); return r; }
    static double sqrt_dn(double a) { std::fesetround(FE_DOWNWARD); volatile double r = std::sqrt(a); std::fesetround(FE_TONEAREST); return r; }
    static double sqrt_up(double a) { std::fesetround(FE_UPWARD);   volatile double r = std::sqrt(a); std::fesetround(FE_TONEAREST); return r; }
    // rounded_transc_std: libm cos evaluated with the FPU in the directed mode (glibc returns
    // its round-to-nearest result regardless; we call it the same way).
    static double cos_dn(double a) { std::fesetround(FE_DOWNWARD); volatile double r = std::cos(a); std::fesetround(FE_TONEAREST); return r; }
    static double cos_up(double a) { std::fesetround(FE_UPWARD);   volatile double r = std::cos(a); std::fesetround(FE_TONEAREST); return r; }
    // int_down: downward(); rint(x)  == floor
    static double int_dn(double a) { std::fesetround(FE_DOWNWARD); volatile double r = std::rint(a); std::fesetround(FE_TONEAREST); return r; }
};

// boost/numeric/interval/constants.hpp
static const double PI_D_L = (3373259426.0 + 273688.0 / (1 << 21)) / (1 << 30);
static const double PI_D_U = (3373259426.0 + 273689.0 / (1 << 21)) / (1 << 30);

struct Interval {
    double lo, hi;
    Interval() : lo(0), hi(0) {}
    explicit Interval(double v) : lo(v), hi(v) {}
    // checking_base: !(l <= u) or NaN -> empty (quiet NaN bounds)
    Interval(double l, double u) : lo(l), hi(u) {
        if (std::isnan(l) || std::isnan(u) || !(l <= u)) {
            lo = std::numeric_limits<double>::quiet_NaN();
            hi = std::numeric_limits<double>::quiet_NaN();
        }
    }
    // the 'checked == true' constructor used inside Boost's operators (no test)
    static Interval raw(double l, double u) { Interval r; r.lo = l; r.hi = u; return r; }
    double lower() const { return lo; }
    double upper() const { return hi; }
    bool empty() const { return std::isnan(lo); }
    Interval& operator+=(const Interval& r) { lo = Rnd::add_dn(lo, r.lo); hi = Rnd::add_up(hi, r.hi); return *this; }
};

inline Interval operator-(const Interval& x) { return Interval::raw(-x.hi, -x.lo); }
inline Interval operator+(const Interval& x, const Interval& y) { return Interval::raw(Rnd::add_dn(x.lo, y.lo), Rnd::add_up(x.hi, y.hi)); }
inline Interval operator+(double x, const Interval& y) { return Interval::raw(Rnd::add_dn(x, y.lo), Rnd::add_up(x, y.hi)); }
inline Interval operator+(const Interval& x, double y) { return Interval::raw(Rnd::add_dn(x.lo, y), Rnd::add_up(x.hi, y)); }
inline Interval operator-(const Interval& x, const Interval& y) { return Interval::raw(Rnd::sub_dn(x.lo, y.hi), Rnd::sub_up(x.hi, y.lo)); }
inline Interval operator-(const Interval& x, double y) { return Interval::raw(Rnd::sub_dn(x.lo, y), Rnd::sub_up(x.hi, y)); }
inline Interval operator-(double x, const Interval& y) { return Interval::raw(Rnd::sub_dn(x, y.hi), Rnd::sub_up(x, y.lo)); }

// arith.hpp: operator*(const T& x, const interval& y)
inline Interval operator*(double x, const Interval& y) {
    if (x < 0) return Interval::raw(Rnd::mul_dn(x, y.hi), Rnd::mul_up(x, y.lo));
    if (x == 0) return Interval::raw(0.0, 0.0);
    return Interval::raw(Rnd::mul_dn(x, y.lo), Rnd::mul_up(x, y.hi));
}
// operator*(const interval& x, const T& y) { return y * x; }
inline Interval operator*(const Interval& x, double y) { return y * x; }

// arith.hpp: operator*(interval, interval), full sign-case analysis
inline Interval operator*(const Interval& x, const Interval& y) {
    const double xl = x.lo, xu = x.hi, yl = y.lo, yu = y.hi;
    if (xl < 0) {
        if (xu > 0) {
            if (yl < 0) {
                if (yu > 0)  // M * M
                    return Interval::raw(std::min(Rnd::mul_dn(xl, yu), Rnd::mul_dn(xu, yl)),
                                         std::max(Rnd::mul_up(xl, yl), Rnd::mul_up(xu, yu)));
                return Interval::raw(Rnd::mul_dn(xu, yl), Rnd::mul_up(xl, yl));  // M * N
            }
            if (yu > 0) return Interval::raw(Rnd::mul_dn(xl, yu), Rnd::mul_up(xu, yu));  // M * P
            return Interval::raw(0.0, 0.0);  // M * Z
        }
        if (yl < 0) {
            if (yu > 0) return Interval::raw(Rnd::mul_dn(xl, yu), Rnd::mul_up(xl, yl));  // N * M
            return Interval::raw(Rnd::mul_dn(xu, yu), Rnd::mul_up(xl, yl));  // N * N
        }
        if (yu > 0) return Interval::raw(Rnd::mul_dn(xl, yu), Rnd::mul_up(xu, yl));  // N * P
        return Interval::raw(0.0, 0.0);  // N * Z
    }
    if (xu > 0) {
        if (yl < 0) {
            if (yu > 0) return Interval::raw(Rnd::mul_dn(xu, yl), Rnd::mul_up(xu, yu));  // P * M
            return Interval::raw(Rnd::mul_dn(xu, yl), Rnd::mul_up(xl, yu));  // P * N
        }
        if (yu > 0) return Interval::raw(Rnd::mul_dn(xl, yl), Rnd::mul_up(xu, yu));  // P * P
        return Interval::raw(0.0, 0.0);  // P * Z
    }
    return Interval::raw(0.0, 0.0);  // Z * ?
}

inline double width(const Interval& x) { return Rnd::sub_up(x.hi, x.lo); }

// detail::pow_dn / pow_up (x, pwr positive), square-and-multiply with directed products
inline double pow_dn_(double x, int pwr) {
    double y = (pwr & 1) ? x : 1.0;
    pwr >>= 1;
    while (pwr > 0) { x = Rnd::mul_dn(x, x); if (pwr & 1) y = Rnd::mul_dn(x, y); pwr >>= 1; }
    return y;
}
inline double pow_up_(double x, int pwr) {
    double y = (pwr & 1) ? x : 1.0;
    pwr >>= 1;
    while (pwr > 0) { x = Rnd::mul_up(x, x); if (pwr & 1) y = Rnd::mul_up(x, y); pwr >>= 1; }
    return y;
}
// transc.hpp-adjacent power.hpp: pow(interval, int), pwr > 0 branch
inline Interval pow(const Interval& x, int pwr) {
    if (pwr == 0) return Interval(1.0);
    if (x.hi < 0) {
        double yl = pow_dn_(-x.hi, pwr), yu = pow_up_(-x.lo, pwr);
        if (pwr & 1) return Interval::raw(-yu, -yl);
        return Interval::raw(yl, yu);
    } else if (x.lo < 0) {
        if (pwr & 1) return Interval::raw(-pow_up_(-x.lo, pwr), pow_up_(x.hi, pwr));
        return Interval::raw(0.0, pow_up_(std::max(-x.lo, x.hi), pwr));
    }
    return Interval::raw(pow_dn_(x.lo, pwr), pow_up_(x.hi, pwr));
}

inline Interval sqrt(const Interval& x) {
    if (x.hi < 0) return Interval(std::numeric_limits<double>::quiet_NaN());
    double l = !(x.lo > 0) ? 0.0 : Rnd::sqrt_dn(x.lo);
    return Interval::raw(l, Rnd::sqrt_up(x.hi));
}

// transc.hpp: fmod(interval x, interval y)
inline Interval fmod(const Interval& x, const Interval& y) {
    const double yb = (x.lo < 0) ? y.lo : y.hi;
    const double n = Rnd::int_dn(Rnd::div_dn(x.lo, yb));
    return x - n * y;
}

inline Interval pi_I() { return Interval::raw(PI_D_L, PI_D_U); }
inline Interval pi_half_I() { return Interval::raw(PI_D_L / 2, PI_D_U / 2); }
inline Interval pi_twice_I() { return Interval::raw(PI_D_L * 2, PI_D_U * 2); }

// transc.hpp: cos(interval)
inline Interval cos(const Interval& x) {
    const Interval pi2 = pi_twice_I();
    Interval tmp = fmod(x, pi2);
    if (width(tmp) >= pi2.lo) return Interval::raw(-1.0, 1.0);
    if (tmp.lo >= PI_D_U) return -cos(tmp - pi_I());
    const double l = tmp.lo, u = tmp.hi;
    if (u <= PI_D_L) return Interval::raw(Rnd::cos_dn(u), Rnd::cos_up(l));
    if (u <= pi2.lo) return Interval::raw(-1.0, Rnd::cos_up(std::min(Rnd::sub_dn(pi2.lo, u), l)));
    return Interval::raw(-1.0, 1.0);
}

// transc.hpp: sin(x) = cos(x - pi/2)
inline Interval sin(const Interval& x) { return cos(x - pi_half_I()); }

// KPR/PZsparse.cu:10-16
inline double getCenter(const Interval& a) { return (a.lo + a.hi) * 0.5; }
inline double getRadius(const Interval& a) { return (a.hi - a.lo) * 0.5; }

}  // namespace oracle
