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
};

enum GeomType {
    G_DUMMY = 0, G_CIRCULAR = 1, G_RECT_CLOSED = 3, G_RECT_OPEN = 4, G_TRAPEZOIDAL = 5,
    G_TRIANGULAR = 6, G_FORCE_MAIN = 24
};

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

// xsect.c:1474-1507 -- uniform table lookup, quadratic near the origin
SWX_HD double lookup(double x, const double* t, int n)
{
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
        double d = -(ap - theta + sin(theta)) / (1.0 - cos(theta));
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
        double tt = theta - sin(theta);
        double tt23 = pow(tt, 2. / 3.);
        double t3 = pow(theta, 1. / 3.);
        double d = ap * theta / t3 - tt * tt23;
        d = d / (ap * (2. / 3.) / t3 - (5. / 3.) * tt23 * (1.0 - cos(theta)));
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

// xsect.c:857-939
SWX_HD double getAofY(const Geom& x, double y, const double* ct)
{
    double yNorm = y / x.yFull;
    if (y <= 0.0) return 0.0;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: return x.aFull * lookup(yNorm, SWX_TA(ct), SWX_CIRC_N);
    case G_RECT_CLOSED: return y * x.wMax;
    case G_RECT_OPEN:   return y * x.wMax;
    case G_TRAPEZOIDAL: return (x.yBot + x.sBot * y) * y;
    case G_TRIANGULAR:  return y * y * x.sBot;
    default: return 0.0;
    }
}

// xsect.c:943-1027
SWX_HD double getWofY(const Geom& x, double y, const double* ct)
{
    double yNorm = y / x.yFull;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: return x.wMax * lookup(yNorm, SWX_TW(ct), SWX_CIRC_N);
    case G_RECT_CLOSED: if (yNorm == 1.0) return 0.0; return x.wMax;
    case G_RECT_OPEN:   return x.wMax;
    case G_TRAPEZOIDAL: return x.yBot + 2.0 * y * x.sBot;
    case G_TRIANGULAR:  return 2.0 * x.sBot * y;
    default: return 0.0;
    }
}

SWX_HD_COLD double getSofA(const Geom& x, double a, const double* ct);

// xsect.c:1100-1145
SWX_HD double getRofA(const Geom& x, double a, const double* ct)
{
    if (a <= 0.0) return 0.0;
    switch (x.type) {
    case G_RECT_CLOSED: return rectClosedRofA(x, a);
    case G_RECT_OPEN:   return a / (x.wMax + (2. - x.sBot) * a / x.wMax);
    case G_TRAPEZOIDAL: return a / (x.yBot + trapYofA(x, a) * x.rBot);
    case G_TRIANGULAR:  return a / (2. * sqrt(a / x.sBot) * x.rBot);
    default: {
        double cathy = getSofA(x, a, ct);
        if (cathy < 1.E-6 || a < 1.E-6) return 0.0;
        return pow(cathy / a, 3. / 2.);
    }
    }
}

// xsect.c:1031-1096
SWX_HD double getRofY(const Geom& x, double y, const double* ct)
{
    double yNorm = y / x.yFull;
    switch (x.type) {
    case G_CIRCULAR: case G_FORCE_MAIN: return x.rFull * lookup(yNorm, SWX_TR(ct), SWX_CIRC_N);
    case G_TRAPEZOIDAL:
        if (y == 0.0) return 0.0;
        return ((x.yBot + x.sBot * y) * y) / (x.yBot + y * x.rBot);
    case G_TRIANGULAR: return (y * x.sBot) / (2. * x.rBot);
    // xsect.c:1091 default branch R(A(y)); written out for the two table-free
    // shapes that reach it so the kernels' hydraulic-radius path has no call
    case G_RECT_CLOSED: return rectClosedRofA(x, getAofY(x, y, ct));
    case G_RECT_OPEN: {
        double a = getAofY(x, y, ct);
        if (a <= 0.0) return 0.0;
        return a / (x.wMax + (2. - x.sBot) * a / x.wMax);
    }
    default: return 0.0;     // no other shape is accepted by the reader
    }
}

// xsect.c:773-853
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
    default: return 0.0;
    }
}

// xsect.c:714-769 (+1755-1768, 1810-1815, 2391-2401)
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
        return a * pow(getRofA(x, a, ct), 2. / 3.);
    case G_RECT_OPEN: {
        double y = a / x.wMax;
        double r = a / ((2.0 - x.sBot) * y + x.wMax);
        return a * pow(r, 2. / 3.);
    }
    default: {
        if (a == 0.0) return 0.0;
        double r = getRofA(x, a, ct);
        if (r < 1.E-6) return 0.0;
        return a * pow(r, 2. / 3.);
    }
    }
}

// xsect.c:1453-1470
SWX_HD_COLD double genericdSdA(const Geom& x, double a, const double* ct)
{
    double alpha = a / x.aFull, alpha1 = alpha - 0.001, alpha2 = alpha + 0.001;
    if (alpha1 < 0.0) alpha1 = 0.0;
    double a1 = alpha1 * x.aFull;
    double a2 = alpha2 * x.aFull;
    return (getSofA(x, a2, ct) - getSofA(x, a1, ct)) / (a2 - a1);
}

// xsect.c:1194-1253 with the shape-specific derivatives
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
        const double* t = SWX_TS(ct);                     // xsect.c:1424-1449
        double delta = 1.0 / ((double)SWX_CIRC_N - 1);
        int i = (int)(alpha / delta);
        if (i >= SWX_CIRC_N - 1) i = SWX_CIRC_N - 2;
        double dSdA = (t[i + 1] - t[i]) / delta;
        return dSdA * x.sFull / x.aFull;
    }
    case G_RECT_CLOSED:                                     // xsect.c:1770-1791
        alpha = a / x.aFull;
        if (alpha > 0.97) return (x.sFull - x.sMax) / ((1.0 - 0.97) * x.aFull);
        if (alpha <= 1.0e-30) return genericdSdA(x, a, ct);
        r = getRofA(x, a, ct);
        return (5. / 3. - (2. / 3.) * (2.0 / x.wMax) * r) * pow(r, 2. / 3.);
    case G_RECT_OPEN:                                       // xsect.c:1818-1830
        if (a / x.aFull <= 1.0e-30) return genericdSdA(x, a, ct);
        r = getRofA(x, a, ct);
        dPdA = (2.0 - x.sBot) / x.wMax;
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    case G_TRAPEZOIDAL:                                     // xsect.c:2196-2208
        if (a / x.aFull <= 1.0e-30) return genericdSdA(x, a, ct);
        r = getRofA(x, a, ct);
        dPdA = x.rBot / sqrt(x.yBot * x.yBot + 4. * x.sBot * a);
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    case G_TRIANGULAR:                                      // xsect.c:2241-2251
        if (a / x.aFull <= 1.0e-30) return genericdSdA(x, a, ct);
        r = getRofA(x, a, ct);
        dPdA = x.rBot / sqrt(a * x.sBot);
        return (5. / 3. - (2. / 3.) * dPdA * r) * pow(r, 2. / 3.);
    default: return genericdSdA(x, a, ct);
    }
}

// findroot.c:19-87 on f(a) = S(a) - s, used by generic_getAofS (xsect.c:1359-1400)
SWX_HD_COLD double genericAofS(const Geom& x, double s, const double* ct)
{
    if (s <= 0.0) return 0.0;
    double x1, x2;
    if ((s <= x.sMax && s >= x.sFull) && x.sMax != x.sFull) {
        x1 = x.aFull;
        x2 = amaxRatio(x.type) * x.aFull;
    } else {
        x1 = 0.0;
        x2 = amaxRatio(x.type) * x.aFull;
    }
    double xx = 0.5 * (x1 + x2), xacc = 0.0001 * x.aFull;
    double xlo = x1, xhi = x2;
    double dxold = fabs(x2 - x1), dx = dxold;
    double f = getSofA(x, xx, ct) - s;
    double df = getdSdA(x, xx, ct);
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
        f = getSofA(x, xx, ct) - s;
        df = getdSdA(x, xx, ct);
        if (f < 0.0) xlo = xx; else xhi = xx;
    }
    return xx;
}

// xsect.c:1149-1190 (+ circ_getAofS 2378-2389)
SWX_HD double getAofS(const Geom& x, double s, const double* ct)
{
    if (s <= 0.0) return 0.0;
    if (s > x.sMax) s = x.sMax;
    if (x.type == G_CIRCULAR || x.type == G_FORCE_MAIN) {
        double psi = s / x.sFull;
        if (psi == 0.0) return 0.0;
        if (psi >= 1.0) return x.aFull;
        if (psi <= 0.015) return x.aFull * aCircular(psi);
        return x.aFull * invLookup(psi, SWX_TS(ct), SWX_CIRC_N);
    }
    if (x.type == G_DUMMY) return 0.0;
    return genericAofS(x, s, ct);
}

// xsect.c:1612-1630
SWX_HD double qCritical(const Geom& x, double yc, double qTarget, const double* ct)
{
    double a = getAofY(x, yc, ct);
    double w = getWofY(x, yc, ct);
    double qc = -qTarget;
    if (w > 0.0) qc = a * sqrt(32.2 * a / w) - qTarget;
    return qc;
}

// xsect.c:1634-1696
SWX_HD_COLD double yCritEnum(const Geom& x, double q, double y0, const double* ct)
{
    double dy = x.yFull / 25., yc, qc;
    int i1 = (int)(y0 / dy);
    double q0 = qCritical(x, i1 * dy, 0.0, ct);
    if (q0 < q) {
        yc = x.yFull;
        #pragma unroll 1
        for (int i = i1 + 1; i <= 25; i++) {
            qc = qCritical(x, i * dy, 0.0, ct);
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
            qc = qCritical(x, i * dy, 0.0, ct);
            if (qc < q) {
                yc = ((q - qc) / (q0 - qc) + (double)i) * dy;
                break;
            }
            q0 = qc;
        }
    }
    return yc;
}

// xsect.c:1700-1748 with findroot_Ridder (findroot.c:90-138)
SWX_HD_COLD double yCritRidder(const Geom& x, double q, double y0, const double* ct)
{
    double y1 = 0.0, y2 = 0.99 * x.yFull;
    double q2 = qCritical(x, y2, 0.0, ct);
    if (q2 < q) return x.yFull;
    double q0 = qCritical(x, y0, 0.0, ct);
    double q1 = qCritical(x, 0.5 * x.yFull, 0.0, ct);
    if (q0 > q) { y2 = y0; if (q1 < q) y1 = 0.5 * x.yFull; }
    else        { y1 = y0; if (q1 > q) y2 = 0.5 * x.yFull; }
    double flo = qCritical(x, y1, q, ct), fhi = qCritical(x, y2, q, ct);
    if (flo == 0.0) return y1;
    if (fhi == 0.0) return y2;
    double ans = 0.5 * (y1 + y2);
    if ((flo > 0.0 && fhi < 0.0) || (flo < 0.0 && fhi > 0.0)) {
        double xlo = y1, xhi = y2;
        #pragma unroll 1
        for (int j = 1; j <= 60; j++) {
            double xm = 0.5 * (xlo + xhi);
            double fm = qCritical(x, xm, q, ct);
            double s = sqrt(fm * fm - flo * fhi);
            if (s == 0.0) return ans;
            double xnew = xm + (xm - xlo) * ((flo >= fhi ? 1.0 : -1.0) * fm / s);
            if (fabs(xnew - ans) <= 0.001) break;
            ans = xnew;
            double fnew = qCritical(x, ans, q, ct);
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
    default: {
        y = 1.01 * pow(q2g / x.yFull, 1. / 4.);
        if (y >= x.yFull) y = 0.97 * x.yFull;
        double r = x.aFull / (3.141592654 / 4.0 * (x.yFull * x.yFull));
        if (r >= 0.5 && r <= 2.0) y = yCritEnum(x, q, y, ct);
        else y = yCritRidder(x, q, y, ct);
    }
    }
    return gmin(y, x.yFull);
}

// link.c:783-804 (conduits)
SWX_HD_COLD double linkYnorm(const Geom& x, double q, double qMax, double beta, const double* ct)
{
    if (x.type == G_DUMMY) return 0.0;
    q = fabs(q);
    if (q > qMax) q = qMax;
    if (q <= 0.0) return 0.0;
    double s = q / beta;
    double a = getAofS(x, s, ct);
    return getYofA(x, a, ct);
}

// link.c:847-871 (conduits)
SWX_HD double linkFroude(const Geom& x, double v, double y, const double* ct)
{
    if (y <= 0.0001) return 0.0;
    if (!isOpen(x.type) && x.yFull - y <= 0.0001) return 0.0;
    y = getAofY(x, y, ct) / getWofY(x, y, ct);
    return fabs(v) / sqrt(32.2 * y);
}

}  // namespace swx
