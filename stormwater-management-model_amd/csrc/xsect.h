// xsect.h -- cross-section geometry shared by the host initialiser and the
// gfx950 kernels (one definition, compiled for both sides).
//
// Semantics are those of the reference's xsect.c (line refs per function);
// arithmetic is written in the reference's evaluation order and everything is
// compiled with -ffp-contract=off, so host results equal the reference
// bit-for-bit and device results differ only through libm ulps (OCML vs
// glibc pow/exp/sin/cos).
//
// Table-driven lookups take the 5x51 circular geometry block as a pointer:
// host code passes SWX_CIRC_TABLES, kernels pass their LDS copy (the block is
// staged once per workgroup; see dw_kernels.hip).
#pragma once

#include <math.h>
#include "xsect_tables.h"
#include "shape_tables.h"
#include "divdd.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SWX_HD __host__ __device__ __forceinline__
// rarely taken iterative paths (root finders) stay out of line so they do not
// inflate the register budget of the streaming kernels
#define SWX_HD_COLD __host__ __device__ __attribute__((noinline)) inline
#else
#define SWX_HD inline
#define SWX_HD_COLD inline
#endif

namespace swx {

struct Geom {                 // TXsect (objects.h:581-599), packed per link
    int type;
    double yFull, wMax, ywMax, aFull, rFull, sFull, sMax, yBot, aBot, sBot, rBot;
    // tabulated shapes: the shape's table block (SWX_SHAPE_TAB, or a
    // transect's own tables); unused by the closed-form shapes
    const double* tb = nullptr;
    // reciprocal pair of yFull (divdd.h) when the kernels' section table
    // supplies one; 0: y / yFull is a plain division
    double rYh = 0.0, rYl = 0.0;
};
// y / yFull, the normalised depth of every geometry relation
SWX_HD double normDepth(const Geom& x, double y)
{
    if (x.rYh != 0.0) return divDD(y, x.yFull, x.rYh, x.rYl);
    return y / x.yFull;
}

// xsection types in the reference's enum order (enums.h)
enum GeomType {
    G_DUMMY = 0, G_CIRCULAR = 1, G_FILLED_CIRCULAR = 2, G_RECT_CLOSED = 3, G_RECT_OPEN = 4,
    G_TRAPEZOIDAL = 5, G_TRIANGULAR = 6, G_PARABOLIC = 7, G_POWERFUNC = 8, G_RECT_TRIANG = 9,
    G_RECT_ROUND = 10, G_MOD_BASKET = 11, G_HORIZ_ELLIPSE = 12, G_VERT_ELLIPSE = 13, G_ARCH = 14,
    G_EGGSHAPED = 15, G_HORSESHOE = 16, G_GOTHIC = 17, G_CATENARY = 18, G_SEMIELLIPTICAL = 19,
    G_BASKETHANDLE = 20, G_SEMICIRCULAR = 21, G_IRREGULAR = 22, G_CUSTOM = 23, G_FORCE_MAIN = 24,
    G_STREET = 25
};
// the shapes the streaming link kernels handle inline; every other shape
// (tabulated, composite, transect-based, force main) is routed to the cold
// conduit kernel, so the streaming kernels' code is unchanged by them
SWX_HD bool isBasicShape(int t)
{
    return t == G_DUMMY || t == G_CIRCULAR || t == G_RECT_CLOSED || t == G_RECT_OPEN ||
           t == G_TRAPEZOIDAL || t == G_TRIANGULAR;
}

SWX_HD double gmin(double x, double y) { return (x <= y) ? x : y; }   // macros.h:28
SWX_HD double gmax(double x, double y) { return (x >= y) ? x : y; }   // macros.h:29
SWX_HD int gsgn(double x) { return (x < 0) ? -1 : 1; }               // macros.h:33

// xsect.c:55-81 -- area at max. flow / full area (1 for open shapes)
SWX_HD double amaxRatio(int t)
{
    switch (t) {
    case G_CIRCULAR: case 2: case G_FORCE_MAIN: return 0.9756;
    case G_RECT_CLOSED: return 0.97;
    case 9: case 10: return 0.98;
    case 11: case 12: case 13: case 15: case 16: case 17: case 20: case 21: case 23: return 0.96;
    case 14: return 0.92;
    case 18: case 19: return 0.98;
    default: return 1.0;
    }
}
SWX_HD int isOpen(int t) { return amaxRatio(t) >= 1.0 ? 1 : 0; }     // xsect.c:204-212

// lookup on the circular tables (n = 51) in two parts: the index part at x
// (CircIdx: the entry, x - x0 and the quadratic term's factor), which every
// table evaluated at the same depth shares, and the table part.  The two
// divisions by the step are divisions by a known constant (divdd.h),
// bit-identical; on the device lookup() below is circLookup(circIdx(x), t).
struct CircIdx {
    int i;
    double dx;                // x - x0
    double q;                 // (x - x0)(x - x1) / delta^2 (i < 2)
};
SWX_HD CircIdx circIdx(double x)
{
    const double delta = kCircDelta;
    CircIdx c;
    c.i = (int)divDD(x, delta, kCircDeltaRh, kCircDeltaRl);
    const double x0 = c.i * delta;
    const double x1 = ((double)c.i + 1) * delta;
    c.dx = x - x0;
    c.q = (c.i < 2) ? divDD((x - x0) * (x - x1), kCircDelta2, kCircDelta2Rh, kCircDelta2Rl) : 0.0;
    return c;
}
SWX_HD double circLookup(const CircIdx& c, const double* t)
{
    const int n = SWX_CIRC_N, i = c.i;
    if (i >= n - 1) return t[n - 1];
    double y = t[i] + divDD(c.dx * (t[i + 1] - t[i]), kCircDelta, kCircDeltaRh, kCircDeltaRl);
    if (i < 2) {
        double y2 = y + c.q * (t[i] / 2.0 - t[i + 1] + t[i + 2] / 2.0);
        if (y2 > 0.0) y = y2;
    }
    if (y < 0.0) y = 0.0;
    return y;
}

// xsect.c:1474-1507 -- uniform table lookup, quadratic near the origin
SWX_HD double lookup(double x, const double* t, int n)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if (n == SWX_CIRC_N) return circLookup(circIdx(x), t);
#endif

    double delta = 1.0 / ((double)n - 1);
    int i = (int)(x / delta);
    if (i >= n - 1) return t[n - 1];
    double x0 = i * delta;
    double x1 = ((double)i + 1) * delta;
    double y = t[i] + (x - x0) * (t[i + 1] - t[i]) / delta;
    if (i < 2) {
        double y2 = y + (x - x0) * (x - x1) / (delta * delta) *
                        (t[i] / 2.0 - t[i + 1] + t[i + 2] / 2.0);
        if (y2 > 0.0) y = y2;
    }
    if (y < 0.0) y = 0.0;
    return y;
}

// xsect.c:1571-1608 -- bisection for the bracketing entry
SWX_HD int locate(double y, const double* t, int jLast)
{
    int j1 = 0, j2 = jLast;
    if (y <= t[0]) return 0;
    if (y >= t[jLast]) return jLast;
    while (j2 - j1 > 1) {
        int j = (j1 + j2) >> 1;
        if (y >= t[j]) j1 = j; else j2 = j;
    }
    return j1;
}

// xsect.c:1511-1567 -- inverse lookup (handles the S-table's interior maximum)
SWX_HD double invLookup(double y, const double* t, int nItems)
{
    double dx = 1.0 / (double)((double)nItems - 1);
    int n = nItems, i;
    if (t[n - 3] > t[n - 1]) n = n - 2;
    if (n < nItems && y > t[nItems - 1]) {
        if (y >= t[nItems - 3]) return ((double)n - 1) * dx;
        if (y <= t[nItems - 2]) i = nItems - 2; else i = nItems - 3;
    } else {
        i = locate(y, t, n - 1);
    }
    if (i >= n - 1) return ((double)n - 1) * dx;
    double x0 = i * dx, x;
    double dy = t[i + 1] - t[i];
    if (dy == 0.0) x = x0; else x = x0 + (y - t[i]) * dx / dy;
    if (x < 0.0) x = 0.0;
    if (x > 1.0) x = 1.0;
    return x;
}

// Device forms of the Newton solves' transcendentals.  A single lane runs
// these solves (the outfall prologue's normal depth), so their instruction
// count is their latency: on the device sin and cos share one argument
// reduction (sincos) and x^(1/3), x^(2/3) are taken from cbrt rather than
// the general pow (a log and an exp in extended precision).  The results
// differ from glibc's by a few ulp, as OCML's sin, cos and pow already do;
// the host keeps the reference's calls, bit-identical.
SWX_HD void swxSinCos(double t, double* s, double* c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    sincos(t, s, c);
#else
    *s = sin(t);
    *c = cos(t);
#endif
}
SWX_HD double swxPowThird(double x)           // pow(x, 1/3) (NaN below 0, as pow)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return x < 0.0 ? __builtin_nan("") : cbrt(x);
#else
    return pow(x, 1. / 3.);
#endif
}
SWX_HD double swxPowTwoThirds(double x)       // pow(x, 2/3) (NaN below 0, as pow)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const double c = cbrt(x);
    return x < 0.0 ? __builtin_nan("") : c * c;
#else
    return pow(x, 2. / 3.);
#endif
}

// pow(r, 1.33333), the friction term of the momentum update (dwflow.c:210):
// on the device exp2(1.33333 log2 r) -- OCML's pow carries its logarithm in
// extended precision for every exponent, about a hundred instructions more
// per conduit in the streaming link kernels; this form stays within a few
// ulp of it for the hydraulic radii that occur (|1.33333 log2 r| < 64), far
// inside the 1e-6 contract.  r = 0 gives 0 and r < 0 NaN, as pow does.
SWX_HD double swxPowFriction(double r)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return r < 0.0 ? __builtin_nan("") : exp2(1.33333 * log2(r));
#else
    return pow(r, 1.33333);
#endif
}

// xsect.c:2573-2591 -- Newton solve of theta - sin(theta) = 2 pi alpha
SWX_HD_COLD double thetaOfAlpha(double alpha)
{
    double theta;
    if (alpha > 0.04) theta = 1.2 + 5.08 * (alpha - 0.04) / 0.96;
    else theta = 0.031715 - 12.79384 * alpha + 8.28479 * sqrt(alpha);
    double theta1 = theta;
    double ap = (2.0 * 3.141592654) * alpha;
    #pragma unroll 1
    for (int k = 1; k <= 40; k++) {
        double st, cth;
        swxSinCos(theta, &st, &cth);
        double d = -(ap - theta + st) / (1.0 - cth);
        if (d > 1.0) d = (d >= 0.0 ? fabs(1.0) : -fabs(1.0));
        theta = theta - d;
        if (fabs(d) <= 0.0001) return theta;
    }
    return theta1;
}

// xsect.c:2593-2618
SWX_HD_COLD double thetaOfPsi(double psi)
{
    double theta;
    if (psi > 0.90) theta = 4.17 + 1.12 * (psi - 0.90) / 0.176;
    else if (psi > 0.5) theta = 3.14 + 1.03 * (psi - 0.5) / 0.4;
    else if (psi > 0.015) theta = 1.2 + 1.94 * (psi - 0.015) / 0.485;
    else theta = 0.12103 - 55.5075 * psi + 15.62254 * sqrt(psi);
    double theta1 = theta;
    double ap = (2.0 * 3.141592654) * psi;
    #pragma unroll 1
    for (int k = 1; k <= 40; k++) {
        theta = fabs(theta);
        double st, cth;
        swxSinCos(theta, &st, &cth);
        double tt = theta - st;
        double tt23 = swxPowTwoThirds(tt);
        double t3 = swxPowThird(theta);
        double d = ap * theta / t3 - tt * tt23;
        d = d / (ap * (2. / 3.) / t3 - (5. / 3.) * tt23 * (1.0 - cth));
        theta = theta - d;
        if (fabs(d) <= 0.0001) return theta;
    }
    return theta1;
}

// xsect.c:2531-2571 -- small-area circular closed forms
SWX_HD double yCircular(double alpha)
{
    if (alpha >= 1.0) return 1.0;
    if (alpha <= 0.0) return 0.0;
    if (alpha <= 1.0e-5) {
        double theta = pow(37.6911 * alpha, 1. / 3.);
        return theta * theta / 16.0;
    }
    double theta = thetaOfAlpha(alpha);
    return (1.0 - cos(theta / 2.)) / 2.0;
}
SWX_HD double sCircular(double alpha)
{
    if (alpha >= 1.0) return 1.0;
    if (alpha <= 0.0) return 0.0;
    if (alpha <= 1.0e-5) {
        double theta = pow(37.6911 * alpha, 1. / 3.);
        return pow(theta, 13. / 3.) / 124.4797;
    }
    double theta = thetaOfAlpha(alpha);
    return pow((theta - sin(theta)), 5. / 3.) / (2.0 * 3.141592654) / pow(theta, 2. / 3.);
}
SWX_HD double aCircular(double psi)
{
    if (psi >= 1.0) return 1.0;
    if (psi <= 0.0) return 0.0;
    if (psi <= 1.0e-6) {
        double theta = pow(124.4797 * psi, 3. / 13.);
        return theta * theta * theta / 37.6911;
    }
    double theta = thetaOfPsi(psi);
    return (theta - sin(theta)) / (2.0 * 3.141592654);
}

#define SWX_TA(ct) ((ct) + SWX_CIRC_A * SWX_CIRC_N)
#define SWX_TR(ct) ((ct) + SWX_CIRC_R * SWX_CIRC_N)
#define SWX_TY(ct) ((ct) + SWX_CIRC_Y * SWX_CIRC_N)
#define SWX_TS(ct) ((ct) + SWX_CIRC_S * SWX_CIRC_N)
#define SWX_TW(ct) ((ct) + SWX_CIRC_W * SWX_CIRC_N)

// xsect.c:1793-1803
SWX_HD double rectClosedRofA(const Geom& x, double a)
{
    if (a <= 0.0) return 0.0;
    double p = x.wMax + 2. * a / x.wMax;
    if (a / x.aFull > 0.97) p += (a / x.aFull - 0.97) / (1.0 - 0.97) * x.wMax;
    return a / p;
}
// xsect.c:2184-2189
SWX_HD double trapYofA(const Geom& x, double a)
{
    if (x.sBot == 0.0) return a / x.yBot;
    return (sqrt(x.yBot * x.yBot + 4. * x.sBot * a) - x.yBot) / (2. * x.sBot);
}


// ---------------------------------------------------------------------------
// Tabulated shapes.  The reference selects, per shape, which xsect.dat table
// each relation interpolates (xsect_getAofY/YofA/WofY/RofY/RofA/SofA/AofS/
// dSdA, xsect.c:714-1253): e.g. A(y) of the gothic shape is the inverse of its
// Y(A) table, the ellipses have no S table.  TabDesc records that choice.
struct TabDesc {
    short a, nA, y, nY, w, nW, r, nR, s, nS;   // offset / length in the block (0 = absent)
    bool aInv;   // A(y) = invLookup of the Y(A) table
    bool yInv;   // Y(A) = invLookup of the A(y) table
    bool rOfY;   // R(A) = R(Y(A)) (xsect.c:1112-1119) instead of (S(A)/A)^1.5
};
#define SWX_TD5(S) TabDesc{SWX_TAB_##S##_A, SWX_TAB_##S##_A_N, SWX_TAB_##S##_Y, SWX_TAB_##S##_Y_N, \
    SWX_TAB_##S##_W, SWX_TAB_##S##_W_N, SWX_TAB_##S##_R, SWX_TAB_##S##_R_N, \
    SWX_TAB_##S##_S, SWX_TAB_##S##_S_N, false, false, false}
#define SWX_TD3(S) TabDesc{0, 0, SWX_TAB_##S##_Y, SWX_TAB_##S##_Y_N, SWX_TAB_##S##_W, SWX_TAB_##S##_W_N, \
    0, 0, SWX_TAB_##S##_S, SWX_TAB_##S##_S_N, true, false, false}
#define SWX_TDE(S) TabDesc{SWX_TAB_##S##_A, SWX_TAB_##S##_A_N, 0, 0, SWX_TAB_##S##_W, SWX_TAB_##S##_W_N, \
    SWX_TAB_##S##_R, SWX_TAB_##S##_R_N, 0, 0, false, true, true}
SWX_HD bool isTabShape(int t)
{
    return (t >= G_HORIZ_ELLIPSE && t <= G_CUSTOM) || t == G_STREET;
}
SWX_HD TabDesc tabDesc(const Geom& x)
{
    switch (x.type) {
    case G_EGGSHAPED: return SWX_TD5(EGG);
    case G_HORSESHOE: return SWX_TD5(HORSESHOE);
    case G_BASKETHANDLE: return SWX_TD5(BASKETHANDLE);
    case G_GOTHIC: return SWX_TD3(GOTHIC);
    case G_CATENARY: return SWX_TD3(CATENARY);
    case G_SEMIELLIPTICAL: return SWX_TD3(SEMIELLIP);
    case G_SEMICIRCULAR: return SWX_TD3(SEMICIRC);
    case G_HORIZ_ELLIPSE: return SWX_TDE(HORIZ_ELLIPSE);
    case G_VERT_ELLIPSE: return SWX_TDE(VERT_ELLIPSE);
    case G_ARCH: return SWX_TDE(ARCH);
    default: {
        // transect / custom-shape / street tables: [n][A n][W n][R n]
        short n = (short)x.tb[0];
        return TabDesc{1, n, 0, 0, (short)(1 + n), n, (short)(1 + 2 * n), n, 0, 0, false, true, true};
    }
    }
}
// block offset of a built-in tabulated shape in SWX_SHAPE_TAB (-1: none)
SWX_HD int shapeTabOffset(int t)
{
    switch (t) {
    case G_EGGSHAPED: return SWX_TAB_EGG;
    case G_HORSESHOE: return SWX_TAB_HORSESHOE;
    case G_GOTHIC: return SWX_TAB_GOTHIC;
    case G_CATENARY: return SWX_TAB_CATENARY;
    case G_SEMIELLIPTICAL: return SWX_TAB_SEMIELLIP;
    case G_BASKETHANDLE: return SWX_TAB_BASKETHANDLE;
    case G_SEMICIRCULAR: return SWX_TAB_SEMICIRC;
    case G_HORIZ_ELLIPSE: return SWX_TAB_HORIZ_ELLIPSE;
    case G_VERT_ELLIPSE: return SWX_TAB_VERT_ELLIPSE;
    case G_ARCH: return SWX_TAB_ARCH;
    default: return -1;
    }
}

#define SWX_RECT_TRIANG_ALFMAX 0.98   // xsect.c:45-46
#define SWX_RECT_ROUND_ALFMAX 0.98

// xsect.c:2284-2289, 2323-2344 -- wetted perimeters
SWX_HD double parabPofY(const Geom& x, double y)
{
    double xx = 2. * sqrt(y) / x.rBot;
    double t = sqrt(1.0 + xx * xx);
    return 0.5 * x.rBot * x.rBot * (xx * t + log(xx + t));
}
SWX_HD double powerPofY(const Geom& x, double y)
{
    double dy1 = 0.02 * x.yFull;
    double h = (x.sBot + 1.0) * x.rBot / 2.0;
    double m = x.sBot;
    double p = 0.0, y1 = 0.0, x1 = 0.0, x2, y2, dx, dy;
    #pragma unroll 1
    do {
        y2 = y1 + dy1;
        if (y2 > y) y2 = y;
        x2 = h * pow(y2, m);
        dx = x2 - x1;
        dy = y2 - y1;
        p += sqrt(dx * dx + dy * dy);
        x1 = x2;
        y1 = y2;
    } while (y2 < y);
    return 2.0 * p;
}
// xsect.c:1837-1844, 2038-2049, 2082-2099 etc.
SWX_HD double rectTriangYofA(const Geom& x, double a)
{
    if (a <= x.aBot) return sqrt(a / x.sBot);
    return x.yBot + (a - x.aBot) / x.wMax;
}
SWX_HD double rectTriangRofA(const Geom& x, double a)             // xsect.c:1846-1864
{
    if (a <= 0.0) return 0.0;
    double y = rectTriangYofA(x, a);
    if (y <= x.yBot) return a / (2. * y * x.rBot);
    double p = 2. * x.yBot * x.rBot + 2. * (y - x.yBot);
    double alf = (a / x.aFull) - SWX_RECT_TRIANG_ALFMAX;
    if (alf > 0.0) p += alf / (1.0 - SWX_RECT_TRIANG_ALFMAX) * x.wMax;
    return a / p;
}
SWX_HD double rectRoundAofY(const Geom& x, double y)              // xsect.c:2038-2049
{
    if (y > x.yBot) return x.aBot + (y - x.yBot) * x.wMax;
    double theta1 = 2.0 * acos(1.0 - y / x.rBot);
    return 0.5 * x.rBot * x.rBot * (theta1 - sin(theta1));
}
SWX_HD double rectRoundYofA(const Geom& x, double a, const double* ct)   // xsect.c:1938-1950
{
    if (a > x.aBot) return x.yBot + (a - x.aBot) / x.wMax;
    double alpha = a / (3.141592654 * x.rBot * x.rBot);
    if (alpha < 0.04) return (2.0 * x.rBot) * yCircular(alpha);
    return (2.0 * x.rBot) * lookup(alpha, SWX_TY(ct), SWX_CIRC_N);
}
SWX_HD double rectRoundRofA(const Geom& x, double a, const double* ct)   // xsect.c:1952-1976
{
    if (a <= 0.0) return 0.0;
    if (a > x.aBot) {
        double y1 = (a - x.aBot) / x.wMax;
        double theta1 = 2.0 * asin(x.wMax / 2.0 / x.rBot);
        double p = x.rBot * theta1 + 2.0 * y1;
        double arg = (a / x.aFull) - SWX_RECT_ROUND_ALFMAX;
        if (arg > 0.0) p += arg / (1.0 - SWX_RECT_ROUND_ALFMAX) * x.wMax;
        return a / p;
    }
    double y1 = rectRoundYofA(x, a, ct);
    double theta1 = 2.0 * acos(1.0 - y1 / x.rBot);
    double p = x.rBot * theta1;
    return a / p;
}
SWX_HD double modBasketYofA(const Geom& x, double a, const double* ct)   // xsect.c:2082-2099
{
    if (a <= x.aFull - x.aBot) return a / x.wMax;
    double alpha = (x.aFull - a) / (3.141592654 * x.rBot * x.rBot);
    double y1;
    if (alpha < 0.04) y1 = yCircular(alpha);
    else y1 = lookup(alpha, SWX_TY(ct), SWX_CIRC_N);
    y1 = 2.0 * x.rBot * y1;
    return x.yFull - y1;
}
SWX_HD double modBasketRofA(const Geom& x, double a, const double* ct)   // xsect.c:2101-2126
{
    if (a <= x.aFull - x.aBot) return a / (x.wMax + 2.0 * a / x.wMax);
    double y1 = x.yFull - modBasketYofA(x, a, ct);
    double theta1 = 2.0 * acos(1.0 - y1 / x.rBot);
    double p = (x.sBot - theta1) * x.rBot;
    y1 = x.yFull - x.yBot;
    p = p + 2.0 * y1 + x.wMax;
    return a / p;
}
// FILLED_CIRCULAR: the reference widens the section to the unfilled circle,
// evaluates the circular relation and narrows it again (xsect.c:2462-2524)
SWX_HD double filledCircAofY(const Geom& x, double y, const double* ct)
{
    double yF = x.yFull + x.yBot, aF = x.aFull + x.aBot;
    y += x.yBot;
    double a = aF * lookup(y / yF, SWX_TA(ct), SWX_CIRC_N);
    return a - x.aBot;
}
SWX_HD double filledCircYofA(const Geom& x, double a, const double* ct)
{
    double yF = x.yFull + x.yBot, aF = x.aFull + x.aBot;
    a += x.aBot;
    double alpha = a / aF, y;
    if (alpha < 0.04) y = yF * yCircular(alpha);
    else y = yF * lookup(alpha, SWX_TY(ct), SWX_CIRC_N);
    return y - x.yBot;
}
SWX_HD double filledCircRofY(const Geom& x, double y, const double* ct)
{
    double yF = x.yFull + x.yBot, aF = x.aFull + x.aBot;
    y += x.yBot;
    double a = aF * lookup(y / yF, SWX_TA(ct), SWX_CIRC_N);
    double r = 0.25 * yF * lookup(y / yF, SWX_TR(ct), SWX_CIRC_N);
    double p = (a / r);
    a = a - x.aBot;
    p = p - x.rBot + x.sBot;
    return a / p;
}

// the non-basic shapes' A(y), W(y), R(y) and Y(A) (xsect.c:773-1096)
SWX_HD double exAofY(const Geom& x, double y, const double* ct)
{
    switch (x.type) {
    case G_FILLED_CIRCULAR: return filledCircAofY(x, y, ct);
    case G_RECT_TRIANG:
        if (y <= x.yBot) return y * y * x.sBot;
        return x.aBot + (y - x.yBot) * x.wMax;
    case G_RECT_ROUND: return rectRoundAofY(x, y);
    case G_MOD_BASKET: {
        if (y <= x.yFull - x.yBot) return y * x.wMax;
        double y1 = x.yFull - y;
        double theta1 = 2.0 * acos(1.0 - y1 / x.rBot);
        double a1 = 0.5 * x.rBot * x.rBot * (theta1 - sin(theta1));
        return x.aFull - a1;
    }
    case G_PARABOLIC: return (4. / 3. * x.rBot * y * sqrt(y));
    case G_POWERFUNC: return x.rBot * pow(y, x.sBot + 1.0);
    default: {
        if (!isTabShape(x.type)) return 0.0;
        TabDesc d = tabDesc(x);
        double yNorm = y / x.yFull;
        if (d.aInv) return x.aFull * invLookup(yNorm, x.tb + d.y, d.nY);
        return x.aFull * lookup(yNorm, x.tb + d.a, d.nA);
    }
    }
}
SWX_HD double exWofY(const Geom& x, double y, const double* ct)
{
    switch (x.type) {
    case G_FILLED_CIRCULAR: {
        double yNorm = (y + x.yBot) / (x.yFull + x.yBot);
        return x.wMax * lookup(yNorm, SWX_TW(ct), SWX_CIRC_N);
    }
    case G_RECT_TRIANG:
        if (y <= x.yBot) return 2.0 * x.sBot * y;
        return x.wMax;
    case G_RECT_ROUND:
        if (y > x.yBot) return x.wMax;
        return 2.0 * sqrt(y * (2.0 * x.rBot - y));
    case G_MOD_BASKET: {
        if (y <= 0.0) return 0.0;
        if (y <= x.yFull - x.yBot) return x.wMax;
        double y1 = x.yFull - y;
        return 2.0 * sqrt(y1 * (2.0 * x.rBot - y1));
    }
    case G_PARABOLIC: return 2.0 * x.rBot * sqrt(y);
    case G_POWERFUNC: return (x.sBot + 1.0) * x.rBot * pow(y, x.sBot);
    default: {
        if (!isTabShape(x.type)) return 0.0;
        TabDesc d = tabDesc(x);
        return x.wMax * lookup(y / x.yFull, x.tb + d.w, d.nW);
    }
    }
}
SWX_HD double exYofA(const Geom& x, double a, const double* ct)
{
    switch (x.type) {
    case G_FILLED_CIRCULAR: return filledCircYofA(x, a, ct);
    case G_RECT_TRIANG: return rectTriangYofA(x, a);
    case G_RECT_ROUND: return rectRoundYofA(x, a, ct);
    case G_MOD_BASKET: return modBasketYofA(x, a, ct);
    case G_PARABOLIC: return pow((3. / 4.) * a / x.rBot, 2. / 3.);
    case G_POWERFUNC: return pow(a / x.rBot, 1.0 / (x.sBot + 1.0));
    default: {
        if (!isTabShape(x.type)) return 0.0;
        TabDesc d = tabDesc(x);
        double alpha = a / x.aFull;
        if (d.yInv) return x.yFull * invLookup(alpha, x.tb + d.a, d.nA);
        return x.yFull * lookup(alpha, x.tb + d.y, d.nY);
    }
    }
}

// kAll: the relations for every shape.  The streaming link kernels, which
// only see the basic shapes, pass false so the other shapes' code is not
// compiled into them; everything else uses the default.
// xsect.c:857-939
template <bool kAll = true>
SWX_HD double getAofY(const Geom& x, double y, const double* ct)
{
    double yNorm = normDepth(x, y);
    if (y <= 0.0) return 0.0;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: return x.aFull * lookup(yNorm, SWX_TA(ct), SWX_CIRC_N);
    case G_RECT_CLOSED: return y * x.wMax;
    case G_RECT_OPEN:   return y * x.wMax;
    case G_TRAPEZOIDAL: return (x.yBot + x.sBot * y) * y;
    case G_TRIANGULAR:  return y * y * x.sBot;
    default:
        if (kAll) return exAofY(x, y, ct);
        return 0.0;
    }
}

// xsect.c:943-1027
template <bool kAll = true>
SWX_HD double getWofY(const Geom& x, double y, const double* ct)
{
    double yNorm = normDepth(x, y);
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: return x.wMax * lookup(yNorm, SWX_TW(ct), SWX_CIRC_N);
    case G_RECT_CLOSED: if (yNorm == 1.0) return 0.0; return x.wMax;
    case G_RECT_OPEN:   return x.wMax;
    case G_TRAPEZOIDAL: return x.yBot + 2.0 * y * x.sBot;
    case G_TRIANGULAR:  return 2.0 * x.sBot * y;
    default:
        if (kAll) return exWofY(x, y, ct);
        return 0.0;
    }
}

template <bool kAll = true>
SWX_HD_COLD double getSofA(const Geom& x, double a, const double* ct);
SWX_HD_COLD double getRofYAll(const Geom& x, double y, const double* ct);

// R(A) of every shape whose relation does not go through the section factor
// (xsect.c:1112-1138); false for the shapes whose R(A) is (S(A)/A)^1.5.  Never
// calls back into getSofA, so the cold call graph stays acyclic.
template <bool kAll = true>
SWX_HD bool rOfADirect(const Geom& x, double a, const double* ct, double* r)
{
    switch (x.type) {
    case G_RECT_CLOSED: { *r = rectClosedRofA(x, a); return true; }
    case G_RECT_OPEN:   { *r = a / (x.wMax + (2. - x.sBot) * a / x.wMax); return true; }
    case G_TRAPEZOIDAL: { *r = a / (x.yBot + trapYofA(x, a) * x.rBot); return true; }
    case G_TRIANGULAR:  { *r = a / (2. * sqrt(a / x.sBot) * x.rBot); return true; }
    default: break;
    }
    if (!kAll) return false;
    switch (x.type) {
    case G_RECT_TRIANG: { *r = rectTriangRofA(x, a); return true; }
    case G_RECT_ROUND: { *r = rectRoundRofA(x, a, ct); return true; }
    case G_MOD_BASKET: { *r = modBasketRofA(x, a, ct); return true; }
    case G_PARABOLIC: { *r = a / parabPofY(x, exYofA(x, a, ct)); return true; }
    case G_POWERFUNC: { *r = a / powerPofY(x, exYofA(x, a, ct)); return true; }
    case G_FILLED_CIRCULAR: {                 // R(Y(A)) (xsect.c:1116, 1046-1049)
        double y = filledCircYofA(x, a, ct);
        if (x.yBot == 0.0) { *r = x.rFull * lookup(y / x.yFull, SWX_TR(ct), SWX_CIRC_N); return true; }
        { *r = filledCircRofY(x, y, ct); return true; }
    }
    default:
        if (isTabShape(x.type)) {
            TabDesc d = tabDesc(x);
            if (d.rOfY) { *r = x.rFull * lookup(exYofA(x, a, ct) / x.yFull, x.tb + d.r, d.nR); return true; }
        }
        return false;
    }
}

// xsect.c:1100-1145
template <bool kAll = true>
SWX_HD double getRofA(const Geom& x, double a, const double* ct)
{
    if (a <= 0.0) return 0.0;
    switch (x.type) {
    case G_RECT_CLOSED: return rectClosedRofA(x, a);
    case G_RECT_OPEN:   return a / (x.wMax + (2. - x.sBot) * a / x.wMax);
    case G_TRAPEZOIDAL: return a / (x.yBot + trapYofA(x, a) * x.rBot);
    case G_TRIANGULAR:  return a / (2. * sqrt(a / x.sBot) * x.rBot);
    default: {
        if (kAll && !isBasicShape(x.type)) {
            double r;
            if (rOfADirect<kAll>(x, a, ct, &r)) return r;
        }
        double cathy = getSofA<kAll>(x, a, ct);
        if (cathy < 1.E-6 || a < 1.E-6) return 0.0;
        return pow(cathy / a, 3. / 2.);
    }
    }
}

// xsect.c:1031-1096
template <bool kAll = true>
SWX_HD double getRofY(const Geom& x, double y, const double* ct)
{
    double yNorm = normDepth(x, y);
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: return x.rFull * lookup(yNorm, SWX_TR(ct), SWX_CIRC_N);
    case G_TRAPEZOIDAL:
        if (y == 0.0) return 0.0;
        return ((x.yBot + x.sBot * y) * y) / (x.yBot + y * x.rBot);
    case G_TRIANGULAR: return (y * x.sBot) / (2. * x.rBot);
    // xsect.c:1094 default branch R(A(y)); written out for the two table-free
    // basic shapes so the streaming kernels' hydraulic-radius path has no call
    case G_RECT_CLOSED: return rectClosedRofA(x, getAofY<false>(x, y, ct));
    case G_RECT_OPEN: {
        double a = getAofY<false>(x, y, ct);
        if (a <= 0.0) return 0.0;
        return a / (x.wMax + (2. - x.sBot) * a / x.wMax);
    }
    default:
        if (kAll) return getRofYAll(x, y, ct);
        return 0.0;
    }
}

// xsect.c:773-853
template <bool kAll = true>
SWX_HD double getYofA(const Geom& x, double a, const double* ct)
{
    double alpha = a / x.aFull;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN:
        if (alpha < 0.04) return x.yFull * yCircular(alpha);
        return x.yFull * lookup(alpha, SWX_TY(ct), SWX_CIRC_N);
    case G_RECT_CLOSED: return a / x.wMax;
    case G_RECT_OPEN:   return a / x.wMax;
    case G_TRAPEZOIDAL: return trapYofA(x, a);
    case G_TRIANGULAR:  return sqrt(a / x.sBot);
    default:
        if (kAll) return exYofA(x, a, ct);
        return 0.0;
    }
}

// R(y) of the non-basic shapes (xsect.c:1046-1094)
SWX_HD_COLD double getRofYAll(const Geom& x, double y, const double* ct)
{
    double yNorm = y / x.yFull;
    switch (x.type) {
    case G_FILLED_CIRCULAR:
        if (x.yBot == 0.0) return x.rFull * lookup(yNorm, SWX_TR(ct), SWX_CIRC_N);
        return filledCircRofY(x, y, ct);
    case G_RECT_TRIANG: {                                          // xsect.c:1908-1925
        if (y <= x.yBot) return y * x.sBot / (2. * x.rBot);
        double a = x.aBot + (y - x.yBot) * x.wMax;
        double p = 2. * x.yBot * x.rBot + 2. * (y - x.yBot);
        double alf = (a / x.aFull) - SWX_RECT_TRIANG_ALFMAX;
        if (alf > 0.0) p += alf / (1.0 - SWX_RECT_TRIANG_ALFMAX) * x.wMax;
        return a / p;
    }
    case G_RECT_ROUND: {                                           // xsect.c:2051-2063
        if (y <= 0.0) return 0.0;
        if (y > x.yBot) return rectRoundRofA(x, rectRoundAofY(x, y), ct);
        double theta1 = 2.0 * acos(1.0 - y / x.rBot);
        return 0.5 * x.rBot * (1.0 - sin(theta1)) / theta1;
    }
    case G_PARABOLIC:
        if (y <= 0.0) return 0.0;
        return exAofY(x, y, ct) / parabPofY(x, y);
    case G_POWERFUNC:
        if (y <= 0.0) return 0.0;
        return exAofY(x, y, ct) / powerPofY(x, y);
    default:
        if (isTabShape(x.type)) {
            TabDesc d = tabDesc(x);
            if (d.nR) return x.rFull * lookup(yNorm, x.tb + d.r, d.nR);
        }
        return getRofA<true>(x, getAofY<true>(x, y, ct), ct);
    }
}

// xsect.c:714-769 (+1755-1768, 1810-1815, 1866-1877, 1978-2011, 2391-2401)
template <bool kAll>
SWX_HD_COLD double getSofA(const Geom& x, double a, const double* ct)
{
    double alpha = a / x.aFull;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN:
        if (alpha < 0.04) return x.sFull * sCircular(alpha);
        return x.sFull * lookup(alpha, SWX_TS(ct), SWX_CIRC_N);
    case G_RECT_CLOSED:
        if (a / x.aFull > 0.97)
            return x.sMax + (x.sFull - x.sMax) * (a / x.aFull - 0.97) / (1.0 - 0.97);
        return a * pow(rectClosedRofA(x, a), 2. / 3.);
    case G_RECT_OPEN: {
        double y = a / x.wMax;
        double r = a / ((2.0 - x.sBot) * y + x.wMax);
        return a * pow(r, 2. / 3.);
    }
    case G_RECT_TRIANG:
        if (!kAll) return 0.0;
        if (a / x.aFull > SWX_RECT_TRIANG_ALFMAX)
            return x.sMax + (x.sFull - x.sMax) * (a / x.aFull - SWX_RECT_TRIANG_ALFMAX) /
                                (1.0 - SWX_RECT_TRIANG_ALFMAX);
        return a * pow(rectTriangRofA(x, a), 2. / 3.);
    case G_RECT_ROUND: {
        if (!kAll) return 0.0;
        if (a / x.aFull > SWX_RECT_ROUND_ALFMAX)
            return x.sMax + (x.sFull - x.sMax) * (a / x.aFull - SWX_RECT_ROUND_ALFMAX) /
                                (1.0 - SWX_RECT_ROUND_ALFMAX);
        if (a > x.aBot) return a * pow(rectRoundRofA(x, a, ct), 2. / 3.);
        double aF = 3.141592654 * x.rBot * x.rBot;
        double al = a / aF;
        if (al < 0.04) return x.sBot * sCircular(al);
        return x.sBot * lookup(al, SWX_TS(ct), SWX_CIRC_N);
    }
    default: {
        if (kAll && isTabShape(x.type)) {
            TabDesc d = tabDesc(x);
            if (d.nS) return x.sFull * lookup(alpha, x.tb + d.s, d.nS);
        }
        if (a == 0.0) return 0.0;
        if (a <= 0.0) return 0.0;                  // xsect_getRofA's a <= 0 test
        double r = 0.0;                            // no shape reaching here has an S table
        if (!rOfADirect<kAll>(x, a, ct, &r)) r = 0.0;
        if (r < 1.E-6) return 0.0;
        return a * pow(r, 2. / 3.);
    }
    }
}

// xsect_getAmax (xsect.c:700-710)
SWX_HD double areaMax(const Geom& x)
{
    if (x.type == G_IRREGULAR || x.type == G_CUSTOM) return x.aBot;
    return amaxRatio(x.type) * x.aFull;
}

// xsect.c:1453-1470
template <bool kAll = true>
SWX_HD_COLD double genericdSdA(const Geom& x, double a, const double* ct)
{
    double alpha = a / x.aFull, alpha1 = alpha - 0.001, alpha2 = alpha + 0.001;
    if (alpha1 < 0.0) alpha1 = 0.0;
    double a1 = alpha1 * x.aFull;
    double a2 = alpha2 * x.aFull;
    return (getSofA<kAll>(x, a2, ct) - getSofA<kAll>(x, a1, ct)) / (a2 - a1);
}

// xsect.c:1424-1449
SWX_HD double tabulardSdA(const Geom& x, double a, const double* t, int n)
{
    double alpha = a / x.aFull;
    double delta = 1.0 / ((double)n - 1);
    int i = (int)(alpha / delta);
    if (i >= n - 1) i = n - 2;
    double dSdA = (t[i + 1] - t[i]) / delta;
    return dSdA * x.sFull / x.aFull;
}

// xsect.c:1194-1253 with the shape-specific derivatives
template <bool kAll = true>
SWX_HD_COLD double getdSdA(const Geom& x, double a, const double* ct)
{
    double alpha, r, dPdA;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: {                 // xsect.c:2403-2423
        alpha = a / x.aFull;
        if (alpha <= 1.0e-30) return 1.0e-30;
        if (alpha < 0.04) {
            double theta = thetaOfAlpha(alpha);
            double p = theta * x.yFull / 2.0;
            r = a / p;
            dPdA = 4.0 / x.yFull / (1. - cos(theta));
            return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
        }
        return tabulardSdA(x, a, SWX_TS(ct), SWX_CIRC_N);
    }
    case G_RECT_CLOSED:                                     // xsect.c:1770-1791
        alpha = a / x.aFull;
        if (alpha > 0.97) return (x.sFull - x.sMax) / ((1.0 - 0.97) * x.aFull);
        if (alpha <= 1.0e-30) return genericdSdA<kAll>(x, a, ct);
        r = getRofA<kAll>(x, a, ct);
        return (5. / 3. - (2. / 3.) * (2.0 / x.wMax) * r) * pow(r, 2. / 3.);
    case G_RECT_OPEN:                                       // xsect.c:1818-1830
        if (a / x.aFull <= 1.0e-30) return genericdSdA<kAll>(x, a, ct);
        r = getRofA<kAll>(x, a, ct);
        dPdA = (2.0 - x.sBot) / x.wMax;
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    case G_TRAPEZOIDAL:                                     // xsect.c:2196-2208
        if (a / x.aFull <= 1.0e-30) return genericdSdA<kAll>(x, a, ct);
        r = getRofA<kAll>(x, a, ct);
        dPdA = x.rBot / sqrt(x.yBot * x.yBot + 4. * x.sBot * a);
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    case G_TRIANGULAR:                                      // xsect.c:2241-2251
        if (a / x.aFull <= 1.0e-30) return genericdSdA<kAll>(x, a, ct);
        r = getRofA<kAll>(x, a, ct);
        dPdA = x.rBot / sqrt(a * x.sBot);
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    case G_RECT_TRIANG:                                     // xsect.c:1879-1900
        if (!kAll) return 0.0;
        alpha = a / x.aFull;
        if (alpha > SWX_RECT_TRIANG_ALFMAX)
            return (x.sFull - x.sMax) / ((1.0 - SWX_RECT_TRIANG_ALFMAX) * x.aFull);
        if (alpha <= 1.0e-30) return genericdSdA<kAll>(x, a, ct);
        if (a > x.aBot) dPdA = 2.0 / x.wMax;
        else dPdA = x.rBot / sqrt(a * x.sBot);
        r = rectTriangRofA(x, a);
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    case G_RECT_ROUND:                                      // xsect.c:2013-2036
        if (!kAll) return 0.0;
        if (a / x.aFull > SWX_RECT_ROUND_ALFMAX)
            return (x.sFull - x.sMax) / ((1.0 - SWX_RECT_ROUND_ALFMAX) * x.aFull);
        if (a > x.aBot) {
            r = rectRoundRofA(x, a, ct);
            dPdA = 2.0 / x.wMax;
            return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
        }
        return genericdSdA<kAll>(x, a, ct);
    case G_MOD_BASKET:                                      // xsect.c:2128-2143
        if (!kAll) return 0.0;
        if (a <= x.aFull - x.aBot && a / x.aFull > 1.0e-30) {
            r = a / (x.wMax + 2.0 * a / x.wMax);
            dPdA = 2.0 / x.wMax;
            return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
        }
        return genericdSdA<kAll>(x, a, ct);
    default:
        if (kAll && isTabShape(x.type)) {
            TabDesc d = tabDesc(x);
            if (d.nS) return tabulardSdA(x, a, x.tb + d.s, d.nS);
        }
        return genericdSdA<kAll>(x, a, ct);
    }
}

// findroot.c:19-87 on f(a) = S(a) - s, used by generic_getAofS (xsect.c:1359-1400)
template <bool kAll = true>
SWX_HD_COLD double genericAofS(const Geom& x, double s, const double* ct)
{
    if (s <= 0.0) return 0.0;
    double x1, x2;
    if ((s <= x.sMax && s >= x.sFull) && x.sMax != x.sFull) {
        x1 = x.aFull;
        x2 = areaMax(x);
    } else {
        x1 = 0.0;
        x2 = areaMax(x);
    }
    double xx = 0.5 * (x1 + x2), xacc = 0.0001 * x.aFull;
    double xlo = x1, xhi = x2;
    double dxold = fabs(x2 - x1), dx = dxold;
    double f = getSofA<kAll>(x, xx, ct) - s;
    double df = getdSdA<kAll>(x, xx, ct);
    #pragma unroll 1
    for (int j = 1; j <= 60; j++) {
        if ((((xx - xhi) * df - f) * ((xx - xlo) * df - f) >= 0.0 ||
             (fabs(2.0 * f) > fabs(dxold * df)))) {
            dxold = dx;
            dx = 0.5 * (xhi - xlo);
            xx = xlo + dx;
            if (xlo == xx) break;
        } else {
            dxold = dx;
            dx = f / df;
            double temp = xx;
            xx -= dx;
            if (temp == xx) break;
        }
        if (fabs(dx) < xacc) break;
        f = getSofA<kAll>(x, xx, ct) - s;
        df = getdSdA<kAll>(x, xx, ct);
        if (f < 0.0) xlo = xx; else xhi = xx;
    }
    return xx;
}

// xsect.c:1149-1190 (+ circ_getAofS 2378-2389)
template <bool kAll = true>
SWX_HD double getAofS(const Geom& x, double s, const double* ct)
{
    double psi = s / x.sFull;          // of the unclamped s (xsect.c:1157)
    if (s <= 0.0) return 0.0;
    if (s > x.sMax) s = x.sMax;
    if (x.type == G_CIRCULAR || x.type == G_FORCE_MAIN) {
        psi = s / x.sFull;
        if (psi == 0.0) return 0.0;
        if (psi >= 1.0) return x.aFull;
        if (psi <= 0.015) return x.aFull * aCircular(psi);
        return x.aFull * invLookup(psi, SWX_TS(ct), SWX_CIRC_N);
    }
    if (x.type == G_DUMMY) return 0.0;
    if (kAll && isTabShape(x.type)) {
        TabDesc d = tabDesc(x);
        if (d.nS) return x.aFull * invLookup(psi, x.tb + d.s, d.nS);
    }
    return genericAofS<kAll>(x, s, ct);
}

// xsect.c:1612-1630
template <bool kAll = true>
SWX_HD double qCritical(const Geom& x, double yc, double qTarget, const double* ct)
{
    double a = getAofY<kAll>(x, yc, ct);
    double w = getWofY<kAll>(x, yc, ct);
    double qc = -qTarget;
    if (w > 0.0) qc = a * sqrt(32.2 * a / w) - qTarget;
    return qc;
}

// xsect.c:1634-1696
template <bool kAll = true>
SWX_HD_COLD double yCritEnum(const Geom& x, double q, double y0, const double* ct)
{
    double dy = x.yFull / 25., yc, qc;
    int i1 = (int)(y0 / dy);
    double q0 = qCritical<kAll>(x, i1 * dy, 0.0, ct);
    if (q0 < q) {
        yc = x.yFull;
        #pragma unroll 1
        for (int i = i1 + 1; i <= 25; i++) {
            qc = qCritical<kAll>(x, i * dy, 0.0, ct);
            if (qc >= q) {
                yc = ((q - q0) / (qc - q0) + ((double)i - 1)) * dy;
                break;
            }
            q0 = qc;
        }
    } else {
        yc = 0.0;
        #pragma unroll 1
        for (int i = i1 - 1; i >= 0; i--) {
            qc = qCritical<kAll>(x, i * dy, 0.0, ct);
            if (qc < q) {
                yc = ((q - qc) / (q0 - qc) + (double)i) * dy;
                break;
            }
            q0 = qc;
        }
    }
    return yc;
}

// yCritEnum's search (xsect.c:1634-1696) over the critical flows qcs[i] =
// qCritical(i * yFull / 25) of all 26 depth increments, evaluated beforehand
// (in parallel, one lane per increment): the same operations on the same
// values, so the same critical depth
SWX_HD double yCritEnumScan(const Geom& x, double q, double y0, const double* qcs)
{
    double dy = x.yFull / 25., yc, qc;
    int i1 = (int)(y0 / dy);
    double q0 = qcs[i1];
    if (q0 < q) {
        yc = x.yFull;
        for (int i = i1 + 1; i <= 25; i++) {
            qc = qcs[i];
            if (qc >= q) {
                yc = ((q - q0) / (qc - q0) + ((double)i - 1)) * dy;
                break;
            }
            q0 = qc;
        }
    } else {
        yc = 0.0;
        for (int i = i1 - 1; i >= 0; i--) {
            qc = qcs[i];
            if (qc < q) {
                yc = ((q - qc) / (q0 - qc) + (double)i) * dy;
                break;
            }
            q0 = qc;
        }
    }
    return yc;
}
// getYcrit takes the enumeration branch (xsect.c:1297-1312): its starting
// estimate y0 is returned in *y0
SWX_HD bool yCritByEnum(const Geom& x, double q, double* y0)
{
    double q2g = (q * q) / 32.2;
    if (q2g == 0.0) return false;
    switch (x.type) {
    case G_DUMMY: case G_RECT_OPEN: case G_RECT_CLOSED: case G_TRIANGULAR: case G_PARABOLIC: case G_POWERFUNC:
        return false;
    default: break;
    }
    double y = 1.01 * pow(q2g / x.yFull, 1. / 4.);
    if (y >= x.yFull) y = 0.97 * x.yFull;
    double r = x.aFull / (3.141592654 / 4.0 * (x.yFull * x.yFull));
    *y0 = y;
    return r >= 0.5 && r <= 2.0;
}

// xsect.c:1700-1748 with findroot_Ridder (findroot.c:90-138)
template <bool kAll = true>
SWX_HD_COLD double yCritRidder(const Geom& x, double q, double y0, const double* ct)
{
    double y1 = 0.0, y2 = 0.99 * x.yFull;
    double q2 = qCritical<kAll>(x, y2, 0.0, ct);
    if (q2 < q) return x.yFull;
    double q0 = qCritical<kAll>(x, y0, 0.0, ct);
    double q1 = qCritical<kAll>(x, 0.5 * x.yFull, 0.0, ct);
    if (q0 > q) { y2 = y0; if (q1 < q) y1 = 0.5 * x.yFull; }
    else        { y1 = y0; if (q1 > q) y2 = 0.5 * x.yFull; }
    double flo = qCritical<kAll>(x, y1, q, ct), fhi = qCritical<kAll>(x, y2, q, ct);
    if (flo == 0.0) return y1;
    if (fhi == 0.0) return y2;
    double ans = 0.5 * (y1 + y2);
    if ((flo > 0.0 && fhi < 0.0) || (flo < 0.0 && fhi > 0.0)) {
        double xlo = y1, xhi = y2;
        #pragma unroll 1
        for (int j = 1; j <= 60; j++) {
            double xm = 0.5 * (xlo + xhi);
            double fm = qCritical<kAll>(x, xm, q, ct);
            double s = sqrt(fm * fm - flo * fhi);
            if (s == 0.0) return ans;
            double xnew = xm + (xm - xlo) * ((flo >= fhi ? 1.0 : -1.0) * fm / s);
            if (fabs(xnew - ans) <= 0.001) break;
            ans = xnew;
            double fnew = qCritical<kAll>(x, ans, q, ct);
            if ((fnew >= 0.0 ? fabs(fm) : -fabs(fm)) != fm) { xlo = xm; flo = fm; xhi = ans; fhi = fnew; }
            else if ((fnew >= 0.0 ? fabs(flo) : -fabs(flo)) != flo) { xhi = ans; fhi = fnew; }
            else if ((fnew >= 0.0 ? fabs(fhi) : -fabs(fhi)) != fhi) { xlo = ans; flo = fnew; }
            else return ans;
            if (fabs(xhi - xlo) <= 0.001) return ans;
        }
        return ans;
    }
    return -1.e20;
}

// xsect.c:1257-1319
template <bool kAll = true>
SWX_HD_COLD double getYcrit(const Geom& x, double q, const double* ct)
{
    double q2g = (q * q) / 32.2, y;
    if (q2g == 0.0) return 0.0;
    switch (x.type) {
    case G_DUMMY: return 0.0;
    case G_RECT_OPEN:
    case G_RECT_CLOSED:
        y = pow(q2g / (x.wMax * x.wMax), 1. / 3.);
        break;
    case G_TRIANGULAR:
        y = pow(2.0 * q2g / (x.sBot * x.sBot), 1. / 5.);
        break;
    case G_PARABOLIC:
        y = pow(27. / 32. * q2g / (x.rBot * x.rBot), 1. / 4.);
        break;
    case G_POWERFUNC:
        y = 1. / (2.0 * x.sBot + 3.0);
        y = pow(q2g * (x.sBot + 1.0) / (x.rBot * x.rBot), y);
        break;
    default: {
        y = 1.01 * pow(q2g / x.yFull, 1. / 4.);
        if (y >= x.yFull) y = 0.97 * x.yFull;
        double r = x.aFull / (3.141592654 / 4.0 * (x.yFull * x.yFull));
        if (r >= 0.5 && r <= 2.0) y = yCritEnum<kAll>(x, q, y, ct);
        else y = yCritRidder<kAll>(x, q, y, ct);
    }
    }
    return gmin(y, x.yFull);
}

// link.c:783-804 (conduits)
template <bool kAll = true>
SWX_HD_COLD double linkYnorm(const Geom& x, double q, double qMax, double beta, const double* ct)
{
    if (x.type == G_DUMMY) return 0.0;
    q = fabs(q);
    if (q > qMax) q = qMax;
    if (q <= 0.0) return 0.0;
    double s = q / beta;
    double a = getAofS<kAll>(x, s, ct);
    return getYofA<kAll>(x, a, ct);
}

// link.c:847-871 (conduits)
template <bool kAll = true>
SWX_HD double linkFroude(const Geom& x, double v, double y, const double* ct)
{
    if (y <= 0.0001) return 0.0;
    if (!isOpen(x.type) && x.yFull - y <= 0.0001) return 0.0;
    y = getAofY<kAll>(x, y, ct) / getWofY<kAll>(x, y, ct);
    return fabs(v) / sqrt(32.2 * y);
}


// ---------------------------------------------------------------------------
// Force mains (forcmain.c).  rBot holds the Hazen-Williams C-factor or the
// Darcy-Weisbach roughness height; sBot the full-flow roughness factor.
enum { FM_H_W = 0, FM_D_W = 1 };
// forcemain_getFricFactor (forcmain.c:128-157), the 2000 < Re < 4000 blend's
// recursion on Re = 4000 written out
SWX_HD double fmFricFactor(double e, double hrad, double re)
{
    if (re < 10.0) re = 10.0;
    if (re <= 2000.0) return 64.0 / re;
    double r = (re < 4000.0) ? 4000.0 : re;
    double f = e / 3.7 / (4.0 * hrad);
    if (r < 1.0e10) f += 5.74 / pow(r, 0.9);
    f = log10(f);
    f = 0.25 / f / f;
    if (re < 4000.0) f = 0.032 + (f - 0.032) * (re - 2000.0) / 2000.0;
    return f;
}
// forcemain_getFricSlope (forcmain.c:93-115)
SWX_HD double fmFricSlope(int eqn, const Geom& x, double v, double hrad)
{
    if (eqn == FM_H_W) return x.sBot * pow(v, 0.852) / pow(hrad, 1.1667);
    double re = 4.0 * hrad * v / 1.1E-5;
    double f = fmFricFactor(x.rBot, hrad, re);
    return f * x.sBot * v / hrad;
}

// Geometry evaluation for the known-answer tests (swmmx_xsect): fn 1 A(y),
// 2 W(y), 3 R(y), 4 Y(A), 5 R(A), 6 S(A), 7 A(S), 8 dS/dA, 9 critical depth
// at flow x (xsect_getAofY ... xsect_getYcrit, xsect.c:714-1319)
SWX_HD_COLD double evalXsect(const Geom& g, int fn, double v, const double* ct)
{
    switch (fn) {
    case 1: return getAofY(g, v, ct);
    case 2: return getWofY(g, v, ct);
    case 3: return getRofY(g, v, ct);
    case 4: return getYofA(g, v, ct);
    case 5: return getRofA(g, v, ct);
    case 6: return getSofA(g, v, ct);
    case 7: return getAofS(g, v, ct);
    case 8: return getdSdA(g, v, ct);
    case 9: return getYcrit(g, v, ct);
    default: return 0.0;
    }
}

}  // namespace swx

