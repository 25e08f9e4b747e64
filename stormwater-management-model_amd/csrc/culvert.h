// culvert.h -- inlet-controlled culvert flow (the reference's culvert.c,
// FHWA HDS-5 inlet control equations), shared by host and device.
//
// A conduit with a culvert code (7th [XSECTIONS] parameter) runs in the cold
// conduit kernel; after the momentum update, while its barrel is not full, its
// flow is limited to the inlet's capacity at the upstream head
// (dwflow.c:250-252, culvert_getInflow culvert.c:190-259).
#pragma once

#include "xsect.h"

namespace swx {

// FHWA inlet-control coefficients per culvert code 1..57 (HDS-5 Table 9;
// the reference's culvert.c:40-99): equation form, K, M, c, Y
struct CulvertCoef { double form, k, m, c, y; };
// rows: form, K, M, c, Y
static constexpr double kCulvertTable[58][5] = {
    {0, 0, 0, 0, 0},   // code 0: none
    {1, 0.0098, 2.00, 0.0398, 0.67}, {1, 0.0018, 2.00, 0.0292, 0.74}, {1, 0.0045, 2.00, 0.0317, 0.69},   // codes 1-3
    {1, 0.0078, 2.00, 0.0379, 0.69}, {1, 0.0210, 1.33, 0.0463, 0.75}, {1, 0.0340, 1.50, 0.0553, 0.54},   // codes 4-6
    {1, 0.0018, 2.50, 0.0300, 0.74}, {1, 0.0018, 2.50, 0.0243, 0.83},   // codes 7-8
    {1, 0.026, 1.0, 0.0347, 0.81}, {1, 0.061, 0.75, 0.0400, 0.80}, {1, 0.061, 0.75, 0.0423, 0.82},   // codes 9-11
    {2, 0.510, 0.667, 0.0309, 0.80}, {2, 0.486, 0.667, 0.0249, 0.83},   // codes 12-13
    {2, 0.515, 0.667, 0.0375, 0.79}, {2, 0.495, 0.667, 0.0314, 0.82}, {2, 0.486, 0.667, 0.0252, 0.865},   // codes 14-16
    {2, 0.545, 0.667, 0.04505, 0.73}, {2, 0.533, 0.667, 0.0425, 0.705}, {2, 0.522, 0.667, 0.0402, 0.68},   // codes 17-19
    {2, 0.498, 0.667, 0.0327, 0.75},   // code 20
    {2, 0.497, 0.667, 0.0339, 0.803}, {2, 0.493, 0.667, 0.0361, 0.806}, {2, 0.495, 0.667, 0.0386, 0.71},   // codes 21-23
    {2, 0.497, 0.667, 0.0302, 0.835}, {2, 0.495, 0.667, 0.0252, 0.881}, {2, 0.493, 0.667, 0.0227, 0.887},   // codes 24-26
    {1, 0.0083, 2.00, 0.0379, 0.69}, {1, 0.0145, 1.75, 0.0419, 0.64}, {1, 0.0340, 1.50, 0.0496, 0.57},   // codes 27-29
    {1, 0.0100, 2.00, 0.0398, 0.67}, {1, 0.0018, 2.50, 0.0292, 0.74}, {1, 0.0045, 2.00, 0.0317, 0.69},   // codes 30-32
    {1, 0.0100, 2.00, 0.0398, 0.67}, {1, 0.0018, 2.50, 0.0292, 0.74}, {1, 0.0095, 2.00, 0.0317, 0.69},   // codes 33-35
    {1, 0.0083, 2.00, 0.0379, 0.69}, {1, 0.0300, 1.00, 0.0463, 0.75}, {1, 0.0340, 1.50, 0.0496, 0.57},   // codes 36-38
    {1, 0.0300, 1.50, 0.0496, 0.57}, {1, 0.0088, 2.00, 0.0368, 0.68}, {1, 0.0030, 2.00, 0.0269, 0.77},   // codes 39-41
    {1, 0.0300, 1.50, 0.0496, 0.57}, {1, 0.0088, 2.00, 0.0368, 0.68}, {1, 0.0030, 2.00, 0.0269, 0.77},   // codes 42-44
    {1, 0.0083, 2.00, 0.0379, 0.69}, {1, 0.0300, 1.00, 0.0473, 0.75}, {1, 0.0340, 1.50, 0.0496, 0.57},   // codes 45-47
    {2, 0.534, 0.555, 0.0196, 0.90}, {2, 0.519, 0.640, 0.0210, 0.90}, {2, 0.536, 0.622, 0.0368, 0.83},   // codes 48-50
    {2, 0.5035, 0.719, 0.0478, 0.80}, {2, 0.547, 0.800, 0.0598, 0.75}, {2, 0.475, 0.667, 0.0179, 0.97},   // codes 51-53
    {2, 0.560, 0.667, 0.0446, 0.85}, {2, 0.560, 0.667, 0.0378, 0.87}, {2, 0.500, 0.667, 0.0446, 0.65},   // codes 54-56
    {2, 0.500, 0.667, 0.0378, 0.71}};   // code 57
SWX_HD CulvertCoef culvertCoef(int code)
{
    const double* r = kCulvertTable[code];
    return CulvertCoef{r[0], r[1], r[2], r[3], r[4]};
}

struct CulvertState {          // TCulvert (culvert.c:111-121)
    double yFull, scf, dQdH, qc, kk, mm, ad, hPlus;
};

// form1Eqn (culvert.c:375-392): the unsubmerged form-1 energy balance at a
// trial critical depth; sets qc
SWX_HD double culvertForm1Eqn(const Geom& x, CulvertState& c, double yc, const double* ct)
{
    double ac = getAofY(x, yc, ct);
    double wc = getWofY(x, yc, ct);
    double yh = ac / wc;
    c.qc = ac * sqrt(32.2 * yh);
    return c.hPlus - yc / c.yFull - yh / 2.0 / c.yFull - c.kk * pow(c.qc / c.ad, c.mm);
}

// getForm1Flow (culvert.c:350-371): Ridder's method (findroot.c:90-138) on
// form1Eqn; the flow is the qc of the last evaluation
SWX_HD_COLD double culvertForm1Flow(const Geom& x, CulvertState& c, double h, const double* ct)
{
    c.hPlus = h / c.yFull + c.scf;
    const double x1 = 0.01 * h, x2 = h, xacc = 0.001;
    double flo = culvertForm1Eqn(x, c, x1, ct);
    double fhi = culvertForm1Eqn(x, c, x2, ct);
    if (flo == 0.0 || fhi == 0.0) return c.qc;
    double ans = 0.5 * (x1 + x2);
    if ((flo > 0.0 && fhi < 0.0) || (flo < 0.0 && fhi > 0.0)) {
        double xlo = x1, xhi = x2;
        #pragma unroll 1
        for (int j = 1; j <= 60; j++) {
            double xm = 0.5 * (xlo + xhi);
            double fm = culvertForm1Eqn(x, c, xm, ct);
            double s = sqrt(fm * fm - flo * fhi);
            if (s == 0.0) return c.qc;
            double xnew = xm + (xm - xlo) * ((flo >= fhi ? 1.0 : -1.0) * fm / s);
            if (fabs(xnew - ans) <= xacc) break;
            ans = xnew;
            double fnew = culvertForm1Eqn(x, c, ans, ct);
            if ((fnew >= 0.0 ? fabs(fm) : -fabs(fm)) != fm) { xlo = xm; flo = fm; xhi = ans; fhi = fnew; }
            else if ((fnew >= 0.0 ? fabs(flo) : -fabs(flo)) != flo) { xhi = ans; fhi = fnew; }
            else if ((fnew >= 0.0 ? fabs(fhi) : -fabs(fhi)) != fhi) { xlo = ans; flo = fnew; }
            else return c.qc;
            if (fabs(xhi - xlo) <= xacc) return c.qc;
        }
    }
    return c.qc;
}

// getUnsubmergedFlow / getSubmergedFlow (culvert.c:263-322)
SWX_HD double culvertUnsubmerged(const Geom& x, const CulvertCoef& P, CulvertState& c, double h,
                                 const double* ct)
{
    c.kk = P.k;
    c.mm = P.m;
    double arg = h / c.yFull / c.kk;
    double q;
    if (P.form == 1.0) q = culvertForm1Flow(x, c, h, ct);
    else q = c.ad * pow(arg, 1.0 / c.mm);
    c.dQdH = q / h / c.mm;
    return q;
}
SWX_HD double culvertSubmerged(const CulvertCoef& P, CulvertState& c, double h)
{
    double arg = (h / c.yFull - P.y + c.scf) / P.c;
    if (arg <= 0.0) {
        c.dQdH = 0.0;
        return 1.E10;
    }
    double q = sqrt(arg) * c.ad;
    c.dQdH = 0.5 * q / arg / c.yFull / P.c;
    return q;
}

// culvert_getInflow (culvert.c:190-259): the inlet-controlled flow for a
// computed flow q0 at water depth y = h1 - (node1 invert + offset1) above
// the inlet.  Returns q0 unless inlet control governs, then sets *dqdh
// (not multiplied by barrels, as in the reference) and *inlet.
SWX_HD_COLD double culvertInflow(const Geom& x, int code, double slope, double q0, double y, double* dqdh,
                                 int* inlet, const double* ct)
{
    if (code <= 0 || code > 57) return q0;
    const CulvertCoef P = culvertCoef(code);
    CulvertState c;
    c.dQdH = 0.0;
    c.qc = 0.0;
    c.kk = c.mm = c.hPlus = 0.0;
    c.yFull = x.yFull;
    c.ad = x.aFull * sqrt(c.yFull);
    if (code == 5 || code == 37 || code == 46) c.scf = -7.0 * slope;
    else c.scf = 0.5 * slope;
    double y2 = c.yFull * (16.0 * P.c + P.y - c.scf), q;
    if (y >= y2) q = culvertSubmerged(P, c, y);
    else {
        double y1 = 0.95 * c.yFull;
        if (y <= y1) q = culvertUnsubmerged(x, P, c, y, ct);
        else {                                              // getTransitionFlow culvert.c:326-346
            double q1 = culvertUnsubmerged(x, P, c, y1, ct);
            double q2 = culvertSubmerged(P, c, y2);
            q = q1 + (q2 - q1) * (y - y1) / (y2 - y1);
            c.dQdH = (q2 - q1) / (y2 - y1);
        }
    }
    if (q < q0) {
        *inlet = 1;
        *dqdh = c.dQdH;
        return q;
    }
    return q0;
}

}  // namespace swx
