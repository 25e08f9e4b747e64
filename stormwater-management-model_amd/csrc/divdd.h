// divdd.h -- correctly rounded division by a divisor known in advance.
//
// a / b with b's reciprocal held as a double-double (rh = RN(1/b), rl =
// RN(1/b - rh)): q0 = RN(a*rh + RN(a*rl)) is within one ulp of a/b (its error
// is one rounding plus ~2^-104 relative), the remainder r = a - b*q0 is exact
// in one FMA, and q0 + r*rh rounded once is RN(a/b) (Markstein's theorem: y
// within half an ulp of 1/b, q faithful => RN(q + (a - bq) y) = RN(a/b); no
// underflow or overflow in the kernels' ranges).  Four FMA-class operations
// instead of the ~10 of a general fp64 division (v_div_scale x2, v_rcp,
// Newton steps, v_div_fmas, v_div_fixup), with the identical result -- the
// kernels' table lookups divide by the same few divisors (the table step,
// a section's full depth) millions of times per step.
// tests/test_divdd.py checks the identity against plain division.
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SWX_DIV_HD __host__ __device__ __forceinline__
#else
#define SWX_DIV_HD inline
#endif

namespace swx {

SWX_DIV_HD double divDD(double a, double b, double rh, double rl)
{
    double q0 = fma(a, rh, a * rl);
    double r = fma(-b, q0, a);
    return fma(r, rh, q0);
}

// the reciprocal pair of b computed in place (device and host): one division
// and an FMA; rl = (1 - b*rh) * rh carries 1/b - rh to ~2^-105 relative, so
// divDD's q0 stays within one ulp and its result is RN(a/b) (Markstein);
// for a divisor several quotients share (tests/c/divdd_check.cpp)
SWX_DIV_HD void recipDDFast(double b, double* rh, double* rl)
{
    const double h = 1.0 / b;
    *rh = h;
    *rl = fma(-b, h, 1.0) * h;
}

// the reciprocal pair of b (host side, at set-up)
inline void recipDD(double b, double* rh, double* rl)
{
    double h = 1.0 / b;
    double e = fma(-b, h, 1.0);        // 1 - b*h, exact
    *rh = h;
    *rl = e / b;                       // (1/b - h) to 53 bits
}

// the circular tables' step (xsect.c:1481, n = 51) and its square, with their
// reciprocal pairs (exact values: tools/ derivation in tests/test_divdd.py)
constexpr double kCircDelta = 0x1.47ae147ae147bp-6;      // 1.0 / 50.0
constexpr double kCircDeltaRh = 0x1.9000000000000p+5;    // RN(1 / kCircDelta) = 50
constexpr double kCircDeltaRl = -0x1.2c00000000000p-50;
constexpr double kCircDelta2 = 0x1.a36e2eb1c432dp-12;    // kCircDelta * kCircDelta
constexpr double kCircDelta2Rh = 0x1.3880000000000p+11;  // 2500
constexpr double kCircDelta2Rl = -0x1.0dc6800000000p-43;

}  // namespace swx
