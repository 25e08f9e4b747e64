// regulators.h -- pumps, orifices, weirs and outlets (link.c:1406-2692,
// dynwave.c:423-524), shared by the host (validation: orifice / weir
// coefficients) and the device (k_nc, the non-conduit phase of every Picard
// iteration).  Restated from the reference's equations in its order of
// operations; roadway weirs and control-rule settings are out of scope.
#pragma once

#include <cmath>

#include "storage.h"   // table lookups
#include "xsect.h"

namespace swx {

enum LinkTypeNC { LK_CONDUIT = 0, LK_PUMP = 1, LK_ORIFICE = 2, LK_WEIR = 3, LK_OUTLET = 4 };
enum PumpTypeNC { PT_TYPE1 = 0, PT_TYPE2, PT_TYPE3, PT_TYPE4, PT_TYPE5, PT_IDEAL };
enum OrificeTypeNC { OR_SIDE = 0, OR_BOTTOM = 1 };
enum WeirTypeNC { WR_TRANSVERSE = 0, WR_SIDEFLOW, WR_VNOTCH, WR_TRAPEZOIDAL, WR_ROADWAY };
enum OutletCurveNC { OC_DEPTH = 0, OC_HEAD = 1 };
// flow classes (enums.h FlowClassType)
enum { FC_DRY = 0, FC_UP_DRY, FC_DN_DRY, FC_SUBCRITICAL, FC_SUPCRITICAL, FC_UP_CRITICAL, FC_DN_CRITICAL };

// static description of one non-conduit link
struct NcLink {
    int type, sub;              // LinkTypeNC; orifice / weir / pump / outlet-curve type
    int flap, canSurcharge;
    int cOff, cN;               // curve slice (pump curve, rating curve, weir Cd curve)
    double offset1, yFull;
    double c1, c2;              // orifice cDisch / orate; weir cDisch1 / cDisch2; outlet qCoeff / qExpon
    double endCon, slope, length;
    double yOn, yOff, xMin, xMax, qFull;   // pumps
    double ucfL, ucfQ;          // UCF(LENGTH), UCF(FLOW)
    int si;                     // UnitSystem == SI
    double roadWidth;           // roadway weirs: road width (ft), surface 1 paved / 2 gravel
    int roadSurf;
    double qLimit;              // DUMMY conduits: Link.qLimit (0: none)
};

// setting-dependent coefficients (orifice_setSetting, weir_setSetting)
struct NcCoef {
    double cOrif, cWeir, hCrit, cSurcharge;
};

// one evaluation's outputs besides the flow
struct NcOut {
    double dqdh, depth, surfArea;
    int flowClass;
};

// link_setFlapGate (link.c:643-670); dir is the sign of the flow
SWX_HD bool ncFlapClosed(int flap, bool n1OutfallFlap, bool n2OutfallFlap, double dir)
{
    if (flap && dir * 1.0 < 0.0) return true;           // NC links keep direction +1
    if (dir < 0.0 && n2OutfallFlap) return true;
    if (dir > 0.0 && n1OutfallFlap) return true;
    return false;
}

// orifice_getWeirCoeff (link.c:1769-1806): returns cDisch*sqrt(h) and hCrit
SWX_HD double orificeWeirCoeff(const NcLink& L, const Geom& g, double h, double* hCrit)
{
    if (L.sub == OR_BOTTOM) {
        double aOverL;
        if (g.type == G_CIRCULAR) aOverL = h / 4.0;
        else {
            double w = g.wMax;
            aOverL = (h * w) / (2.0 * (h + w));
        }
        h = L.c1 / 0.414 * aOverL;
        *hCrit = h;
    } else {
        *hCrit = h;
        h = h / 2.0;
    }
    return L.c1 * sqrt(h);
}

// orifice_setSetting (link.c:1729-1765) for an already adjusted setting
SWX_HD void orificeCoefs(const NcLink& L, const Geom& g, double setting, const double* ct, NcCoef* c)
{
    double h = setting * g.yFull;
    double f = getAofY(g, h, ct) * sqrt(2.0 * 32.2);
    c->cOrif = L.c1 * f;
    double hc;
    c->cWeir = orificeWeirCoeff(L, g, h, &hc) * f;
    c->hCrit = hc;
}

// orifice_getFlow (link.c:1921-2003)
SWX_HD double orificeFlow(const NcLink& L, const Geom& g, const NcCoef& c, double setting, double head,
                          double f, int hasFlapGate, double* dqdh, const double* ct)
{
    double q;
    if (head == 0.0 || f <= 0.0) { *dqdh = 0.0; return 0.0; }
    else if (f < 1.0) {
        q = c.cWeir * pow(f, 1.5);
        *dqdh = 1.5 * q / (f * c.hCrit);
    } else {
        q = c.cOrif * sqrt(head);
        *dqdh = q / (2.0 * head);
    }
    if (hasFlapGate) {
        double area = getAofY(g, setting * g.yFull, ct);
        double veloc = q / area;
        double hLoss = (4.0 / 32.2) * veloc * veloc * exp(-1.15 * veloc / sqrt(head));
        if (f < 1.0) {
            f = f - hLoss / c.hCrit;
            if (f < 0.0) f = 0.0;
        } else {
            head = head - hLoss;
            if (head < 0.0) head = 0.0;
        }
        q = orificeFlow(L, g, c, setting, head, f, 0, dqdh, ct);
    }
    return q;
}

// orifice_getInflow (link.c:1810-1917), dynamic wave
SWX_HD double orificeInflow(const NcLink& L, const Geom& g, const NcCoef& c, double setting, double y1n,
                            double y2n, double inv1, double inv2, bool of1, bool of2, NcOut* o,
                            const double* ct)
{
    double h1 = y1n + inv1, h2 = y2n + inv2;
    double dir = (h1 >= h2) ? +1.0 : -1.0;
    double y1 = y1n, head, f, hcrest, hcrown, hmidpt;
    if (dir < 0.0) {
        head = h1;
        h1 = h2;
        h2 = head;
        y1 = y2n;
    }
    hcrest = inv1 + L.offset1;
    if (L.sub == OR_BOTTOM) {
        if (h1 < hcrest) head = 0.0;
        else if (h2 > hcrest) head = h1 - h2;
        else head = h1 - hcrest;
        f = head / c.hCrit;
        f = gmin(f, 1.0);
    } else {
        hcrown = hcrest + g.yFull * setting;
        hmidpt = (hcrest + hcrown) / 2.0;
        if (h1 < hcrown && hcrown > hcrest) f = (h1 - hcrest) / (hcrown - hcrest);
        else f = 1.0;
        if (f < 1.0) head = h1 - hcrest;
        else if (h2 < hmidpt) head = h1 - hmidpt;
        else head = h1 - h2;
    }
    if (head <= 0.0001 || y1 <= 0.0001 || ncFlapClosed(L.flap, of1, of2, dir)) {
        o->depth = 0.0;
        o->flowClass = FC_DRY;
        o->surfArea = 0.0001 * L.length;
        o->dqdh = 0.0;
        return 0.0;
    }
    o->flowClass = FC_SUBCRITICAL;
    if (hcrest > h2) o->flowClass = (dir == 1.0) ? FC_DN_CRITICAL : FC_UP_CRITICAL;
    y1 = g.yFull * setting;
    if (L.sub == OR_SIDE) {
        o->depth = y1 * f;
        o->surfArea = getWofY(g, o->depth, ct) * L.length;
    } else {
        o->depth = y1;
        o->surfArea = getAofY(g, y1, ct);
    }
    double q = dir * orificeFlow(L, g, c, setting, head, f, L.flap, &o->dqdh, ct);
    if (f < 1.0 && h2 > hcrest) {
        double ratio = (h2 - hcrest) / (h1 - hcrest);
        q *= pow((1.0 - pow(ratio, 1.5)), 0.385);
    }
    return q;
}

// weir_getOpenArea (link.c:2466-2484)
SWX_HD double weirOpenArea(const Geom& g, double setting, double y, const double* ct)
{
    double z = (1.0 - setting) * g.yFull;
    double zy = z + y;
    zy = gmin(zy, g.yFull);
    return getAofY(g, zy, ct) - getAofY(g, z, ct);
}

// weir_getdqdh (link.c:2488-2514)
SWX_HD double weirdQdH(int type, double dir, double h, double q1, double q2)
{
    if (fabs(h) < 0.0001) return 0.0;
    double q1h = fabs(q1 / h), q2h = fabs(q2 / h);
    switch (type) {
    case WR_TRANSVERSE: return 1.5 * q1h;
    case WR_SIDEFLOW: return (dir < 0.0) ? 1.5 * q1h : 1.67 * q1h;
    case WR_VNOTCH: return (q2h == 0.0) ? 2.5 * q1h : 1.5 * q1h + 2.5 * q2h;
    case WR_TRAPEZOIDAL: return 1.5 * q1h + 2.5 * q2h;
    }
    return 0.0;
}

// weir_getFlow (link.c:2316-2428)
SWX_HD void weirFlow(const NcLink& L, const Geom& g, const double* cx, const double* cy, double setting,
                     double head, double dir, int hasFlapGate, double* q1, double* q2, double* dqdh,
                     const double* ct)
{
    *q1 = 0.0;
    *q2 = 0.0;
    *dqdh = 0.0;
    if (head <= 0.0) return;
    double length = g.wMax * L.ucfL;
    double h = head * L.ucfL;
    double cDisch1 = L.c1;
    if (L.cN > 0) cDisch1 = tableLookup(cx, cy, L.cN, h);
    int wType = L.sub;
    if (wType == WR_VNOTCH && setting < 1.0) wType = WR_TRAPEZOIDAL;
    switch (wType) {
    case WR_TRANSVERSE:
        length -= 0.1 * L.endCon * h;
        length = gmax(length, 0.0);
        *q1 = cDisch1 * length * pow(h, 1.5);
        break;
    case WR_SIDEFLOW:
        length -= 0.1 * L.endCon * h;
        length = gmax(length, 0.0);
        if (dir < 0.0) *q1 = cDisch1 * length * pow(h, 1.5);
        else *q1 = cDisch1 * pow(length, 0.83) * pow(h, 1.67);
        break;
    case WR_VNOTCH:
        *q1 = cDisch1 * L.slope * pow(h, 2.5);
        break;
    case WR_TRAPEZOIDAL: {
        double y = (1.0 - setting) * g.yFull;
        length = getWofY(g, y, ct) * L.ucfL;
        *q1 = cDisch1 * length * pow(h, 1.5);
        *q2 = L.c2 * L.slope * pow(h, 2.5);
        break;
    }
    }
    if (L.si) {
        *q1 /= 0.028317;
        *q2 /= 0.028317;
    }
    if (hasFlapGate) {
        double area = weirOpenArea(g, setting, head, ct);
        if (area > 1.0e-6) {
            double veloc = (*q1 + *q2) / area;
            double hLoss = (4.0 / 32.2) * veloc * veloc * exp(-1.15 * veloc / sqrt(head));
            head = head - hLoss;
            if (head < 0.0) head = 0.0;
            weirFlow(L, g, cx, cy, setting, head, dir, 0, q1, q2, dqdh, ct);
        }
    }
    *dqdh = weirdQdH(L.sub, dir, head, *q1, *q2);
}

// weir_setSetting's surcharge coefficient (link.c:2156-2186) / weir_validate
SWX_HD double weirSurchargeCoef(const NcLink& L, const Geom& g, const double* cx, const double* cy,
                                double setting, const double* ct)
{
    if (setting == 0.0) return 0.0;
    double q1, q2, dq;
    double h = setting * g.yFull;
    weirFlow(L, g, cx, cy, setting, h, 1.0, 0, &q1, &q2, &dq, ct);
    double q = q1 + q2;
    h = h / 2.0;
    return q / sqrt(h);
}

// weir_getOrificeFlow (link.c:2432-2462)
SWX_HD double weirOrificeFlow(const NcLink& L, const Geom& g, double setting, double head, double y,
                              double cOrif, double* dqdh, const double* ct)
{
    double q = cOrif * sqrt(head);
    if (L.flap) {
        double a = weirOpenArea(g, setting, y, ct);
        if (a > 0.0) {
            double v = q / a;
            double hloss = (4.0 / 32.2) * v * v * exp(-1.15 * v / sqrt(y));
            head -= hloss;
            head = gmax(head, 0.0);
            q = cOrif * sqrt(head);
        }
    }
    if (head > 0.0) *dqdh = q / (2.0 * head);
    else *dqdh = 0.0;
    return q;
}

// Roadway overflow (roadway.c, FHWA HDS-5 roadway discharge coefficients and
// submergence factors, as (x, y) tables)
static constexpr double kCrLowPaved[4][2] = {{0.0, 2.85}, {0.2, 2.95}, {0.7, 3.03}, {4.0, 3.05}};
static constexpr double kCrLowGravel[8][2] = {{0.0, 2.5}, {0.5, 2.7}, {1.0, 2.8}, {1.5, 2.9},
                                              {2.0, 2.98}, {2.5, 3.02}, {3.0, 3.03}, {4.0, 3.05}};
static constexpr double kCrHighPaved[2][2] = {{0.15, 3.05}, {0.25, 3.10}};
static constexpr double kCrHighGravel[2][2] = {{0.15, 2.95}, {0.30, 3.10}};
static constexpr double kKtPaved[9][2] = {{0.8, 1.0}, {0.85, 0.98}, {0.90, 0.92}, {0.93, 0.85}, {0.95, 0.80},
                                          {0.97, 0.70}, {0.98, 0.60}, {0.99, 0.50}, {1.00, 0.40}};
static constexpr double kKtGravel[12][2] = {{0.75, 1.00}, {0.80, 0.985}, {0.83, 0.97}, {0.86, 0.93},
                                            {0.89, 0.90}, {0.90, 0.87}, {0.92, 0.80}, {0.94, 0.70},
                                            {0.96, 0.60}, {0.98, 0.50}, {0.99, 0.40}, {1.00, 0.24}};
// getY (roadway.c:176-194)
SWX_HD double roadwayY(double x, const double (*t)[2], int n)
{
    if (x <= t[0][0]) return t[0][1];
    if (x >= t[n - 1][0]) return t[n - 1][1];
    for (int i = 1; i < n; i++) {
        if (x <= t[i][0]) {
            double x1 = t[i - 1][0], dx = t[i][0] - x1;
            double y1 = t[i - 1][1], dy = t[i][1] - y1;
            return y1 + (x - x1) * dy / dx;
        }
    }
    return t[n - 1][1];
}
// getCd (roadway.c:146-172)
SWX_HD double roadwayCd(double hWr, double ht, double roadWidth, int roadSurf)
{
    double kT = 1.0, cR;
    if (hWr <= 0.0) return 0.0;
    double hL = hWr / roadWidth;
    if (hL <= 0.15) {
        if (roadSurf == 1) cR = roadwayY(hWr, kCrLowPaved, 4);
        else cR = roadwayY(hWr, kCrLowGravel, 8);
    } else {
        if (roadSurf == 1) cR = roadwayY(hL, kCrHighPaved, 2);
        else cR = roadwayY(hL, kCrHighGravel, 2);
    }
    if (ht > 0.0) {
        double htH = ht / hWr;
        if (roadSurf == 1) kT = roadwayY(htH, kKtPaved, 9);
        else kT = roadwayY(htH, kKtGravel, 12);
    }
    return cR * kT;
}
// roadway_getInflow (roadway.c:85-142): h1 / h2 already ordered by dir
SWX_HD double roadwayInflow(const NcLink& L, const Geom& g, double dir, double hRoad, double h1, double h2,
                            NcOut* o)
{
    double cD = L.c1;
    if (L.si) cD = cD / 0.552;
    bool useVariableCd = L.roadWidth > 0.0 && L.roadSurf >= 1;
    double hWr = h1 - hRoad, ht = h2 - hRoad, q = 0.0, dqdh = 0.0;
    if (hWr > 0.0001) {
        if (useVariableCd) cD = roadwayCd(hWr, ht, L.roadWidth, L.roadSurf);
        double length = g.wMax;
        q = cD * length * pow(hWr, 1.5);
        dqdh = 1.5 * q / hWr;
    }
    o->dqdh = dqdh;
    o->depth = gmax(h1 - hRoad, 0.0);
    o->flowClass = FC_SUBCRITICAL;
    if (hRoad > h2) o->flowClass = (dir == 1.0) ? FC_DN_CRITICAL : FC_UP_CRITICAL;
    return dir * q;
}

// weir_getInflow (link.c:2190-2312), dynamic wave
SWX_HD double weirInflow(const NcLink& L, const Geom& g, const NcCoef& c, const double* cx,
                         const double* cy, double setting, double y1n, double y2n, double inv1,
                         double inv2, bool of1, bool of2, NcOut* o, const double* ct)
{
    const double weirPower[] = {1.5, 5. / 3., 2.5, 1.5};
    double h1 = y1n + inv1, h2 = y2n + inv2, head, q1, q2;
    double dir = (h1 > h2) ? +1.0 : -1.0;
    if (dir < 0.0) {
        head = h1;
        h1 = h2;
        h2 = head;
    }
    double hcrest = inv1 + L.offset1;
    double hcrown = hcrest + g.yFull;
    if (L.sub == WR_ROADWAY) return roadwayInflow(L, g, dir, hcrest, h1, h2, o);
    hcrest += (1.0 - setting) * g.yFull;
    head = h1 - hcrest;
    o->dqdh = 0.0;
    if (head <= 0.0001 || hcrest >= hcrown || ncFlapClosed(L.flap, of1, of2, dir)) {
        o->depth = 0.0;
        o->flowClass = FC_DRY;
        return 0.0;
    }
    o->flowClass = FC_SUBCRITICAL;
    if (hcrest > h2) o->flowClass = (dir == 1.0) ? FC_DN_CRITICAL : FC_UP_CRITICAL;
    double y = g.yFull - (hcrown - gmin(h1, hcrown));
    o->surfArea = getWofY(g, y, ct) * L.length;
    if (h1 >= hcrown) {
        if (L.canSurcharge) {
            y = (hcrest + hcrown) / 2.0;
            if (h2 < y) head = h1 - y;
            else head = h1 - h2;
            y = hcrown - hcrest;
            q1 = weirOrificeFlow(L, g, setting, head, y, c.cSurcharge, &o->dqdh, ct);
            o->depth = y;
            return dir * q1;
        }
        head = hcrown - hcrest;
    }
    weirFlow(L, g, cx, cy, setting, head, dir, L.flap, &q1, &q2, &o->dqdh, ct);
    if (h2 > hcrest) {
        double ratio = (h2 - hcrest) / (h1 - hcrest);
        q1 *= pow((1.0 - pow(ratio, weirPower[L.sub])), 0.385);
        if (q2 > 0.0) q2 *= pow((1.0 - pow(ratio, weirPower[WR_VNOTCH])), 0.385);
    }
    o->depth = gmin((h1 - hcrest), g.yFull);
    return dir * (q1 + q2);
}

// outlet_getInflow + outlet_getFlow (link.c:2600-2692), dynamic wave
SWX_HD double outletInflow(const NcLink& L, const double* cx, const double* cy, double setting,
                           double y1n, double y2n, double inv1, double inv2, bool of1, bool of2,
                           NcOut* o)
{
    double h1 = y1n + inv1, h2 = y2n + inv2;
    double dir = (h1 >= h2) ? +1.0 : -1.0;
    double y1 = y1n, head;
    if (dir < 0.0) {
        y1 = h1;
        h1 = h2;
        h2 = y1;
        y1 = y2n;
    }
    double hcrest = inv1 + L.offset1;
    if (L.sub == OC_HEAD) head = h1 - gmax(h2, hcrest);
    else head = h1 - hcrest;
    if (head <= 0.0001 || y1 <= 0.0001 || ncFlapClosed(L.flap, of1, of2, dir)) {
        o->depth = 0.0;
        o->flowClass = FC_DRY;
        return 0.0;
    }
    o->depth = head;
    o->flowClass = FC_SUBCRITICAL;
    double h = head * L.ucfL, q;
    if (L.cN > 0) q = tableLookup(cx, cy, L.cN, h) / L.ucfQ;
    else q = L.c1 * pow(h, L.c2) / L.ucfQ;
    return dir * setting * q;
}

// pump_getInflow (link.c:1548-1637) for curve pumps (ideal pumps need the
// inlet node's running inflow: handled by the caller).  vol1 = inlet node
// volume; returns the flow and sets dqdh / flowClass.
SWX_HD double pumpInflow(const NcLink& L, const double* cx, const double* cy, double setting,
                         double y1, double y2, double inv1, double inv2, double vol1, double ucfV,
                         NcOut* o)
{
    double qIn = 0.0, s = 1.0, head, depth, vol, qIn1, dh = 0.001;
    o->flowClass = 0;                  // NO
    switch (L.sub) {
    case PT_TYPE1:
        vol = vol1 * ucfV;
        qIn = tableIntervalLookup(cx, cy, L.cN, vol) / L.ucfQ;
        if (vol < L.xMin || vol > L.xMax) o->flowClass = 1;   // YES
        break;
    case PT_TYPE2:
        depth = y1 * L.ucfL;
        qIn = tableIntervalLookup(cx, cy, L.cN, depth) / L.ucfQ;
        if (depth < L.xMin || depth > L.xMax) o->flowClass = 1;
        break;
    case PT_TYPE3:
    case PT_TYPE5:
        if (L.sub == PT_TYPE5) s = setting;
        head = ((y2 + inv2) - (y1 + inv1)) / s / s;
        head = gmax(head, 0.0) * L.ucfL;
        qIn = tableLookup(cx, cy, L.cN, head) / L.ucfQ;
        o->dqdh = -tableSlope(cx, cy, L.cN, head) * L.ucfL / L.ucfQ / s;
        if (head < L.xMin || head > L.xMax) o->flowClass = 1;
        break;
    case PT_TYPE4:
        depth = y1;
        qIn = tableLookup(cx, cy, L.cN, depth * L.ucfL) / L.ucfQ;
        qIn1 = tableLookup(cx, cy, L.cN, (depth + dh) * L.ucfL) / L.ucfQ;
        o->dqdh = (qIn1 - qIn) / dh;
        depth *= L.ucfL;
        if (depth < L.xMin) o->flowClass = FC_DN_DRY;
        if (depth > L.xMax) o->flowClass = FC_UP_DRY;
        break;
    default: qIn = 0.0;
    }
    if (qIn < 0.0) qIn = 0.0;
    return qIn * setting;
}

}  // namespace swx
