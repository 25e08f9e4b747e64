// storage.h -- storage unit geometry (node.c:813-1050, table.c:395-650),
// shared by the host (initial state, hot start) and the device (node update,
// step-end losses).  Everything is evaluated in the reference's order of
// operations, including its unit conversions (user units inside the shape
// functions, UCF(LENGTH) / UCF(VOLUME) at the boundary).
#pragma once

#include <cmath>

#include "xsect.h"   // SWX_HD

namespace swx {

// RelationWords order (keywords.c:108-110)
enum StorageShape { ST_TABULAR = 0, ST_FUNCTIONAL, ST_CYLINDRICAL, ST_CONICAL, ST_PARABOLOID, ST_PYRAMIDAL };

struct StorageGeom {
    int shape;
    double a0, a1, a2;
    const double* cx;      // area curve (TABULAR): depth, area in user units
    const double* cy;
    int cn;
    double fullDepth, fullVolume;   // ft, ft3
    double ucfL, ucfV;              // UCF(LENGTH), UCF(VOLUME)
};

// table_interpolate (table.c:51-58)
SWX_HD double tableInterp(double x, double x1, double y1, double x2, double y2)
{
    double dx = x2 - x1;
    if (fabs(dx) < 1.0e-20) return (y1 + y2) / 2.;
    return y1 + (x - x1) * (y2 - y1) / dx;
}

// table_lookup (table.c:395-426): clamped at both ends
SWX_HD double tableLookup(const double* tx, const double* ty, int n, double x)
{
    if (n <= 0) return 0.0;
    double x1 = tx[0], y1 = ty[0];
    if (x <= x1) return y1;
    for (int i = 1; i < n; i++) {
        double x2 = tx[i], y2 = ty[i];
        if (x <= x2) return tableInterp(x, x1, y1, x2, y2);
        x1 = x2;
        y1 = y2;
    }
    return y1;
}

// table_lookupEx (table.c:464-499): linear extrapolation beyond the table
SWX_HD double tableLookupEx(const double* tx, const double* ty, int n, double x)
{
    if (n <= 0) return 0.0;
    double x1 = tx[0], y1 = ty[0], s = 0.0;
    if (x <= x1) {
        if (x1 > 0.0) return x / x1 * y1;
        return y1;
    }
    for (int i = 1; i < n; i++) {
        double x2 = tx[i], y2 = ty[i];
        if (x2 != x1) s = (y2 - y1) / (x2 - x1);
        if (x <= x2) return tableInterp(x, x1, y1, x2, y2);
        x1 = x2;
        y1 = y2;
    }
    if (s < 0.0) s = 0.0;
    return y1 + s * (x - x1);
}

// table_getSlope (table.c:430-460)
SWX_HD double tableSlope(const double* tx, const double* ty, int n, double x)
{
    if (n <= 0) return 0.0;
    double x1 = tx[0], y1 = ty[0], x2 = x1, y2 = y1;
    for (int i = 1; i < n; i++) {
        x2 = tx[i];
        y2 = ty[i];
        if (x <= x2) break;
        x1 = x2;
        y1 = y2;
    }
    double dx = x2 - x1;
    if (dx == 0.0) return 0.0;
    return (y2 - y1) / dx;
}

// table_intervalLookup (table.c:503-523)
SWX_HD double tableIntervalLookup(const double* tx, const double* ty, int n, double x)
{
    if (n <= 0) return 0.0;
    if (x < tx[0]) return ty[0];
    for (int i = 1; i < n; i++)
        if (x < tx[i]) return ty[i];
    return ty[n - 1];
}

// table_getStorageVolume (table.c:587-647): end-area integration of the curve
SWX_HD double tableStorageVolume(const double* tx, const double* ty, int n, double x)
{
    double a, v = 0.0, dx = 0.0, dy = 0.0, s;
    if (n <= 0) return 0.0;
    double x1 = tx[0], a1 = ty[0];
    if (x <= x1) {
        if (x1 < 1.e-6) return 0.0;
        return (a1 / x1) * x * x / 2.0;
    }
    for (int i = 1; i < n; i++) {
        if (tx[i] >= x) {
            a = tableInterp(x, x1, a1, tx[i], ty[i]);
            return v + (a1 + a) / 2.0 * (x - x1);
        }
        dx = tx[i] - x1;
        dy = ty[i] - a1;
        v = v + (a1 + ty[i]) / 2.0 * dx;
        x1 = tx[i];
        a1 = ty[i];
    }
    if (dx > 1.0e-6) {
        s = dy / dx;
        a = a1 + s * (x - x1);
        if (a < 0.0) v = v - a1 * a1 / s / 2.0;
        else v = v + (a1 + a) / 2.0 * (x - x1);
    }
    return v;
}

// storage_getVolume (node.c:930-975)
SWX_HD double storageVolume(const StorageGeom& s, double d)
{
    if (d == 0.0) return 0.0;
    if (d >= s.fullDepth && s.fullVolume > 0.0) return s.fullVolume;
    double n, v;
    switch (s.shape) {
    case ST_TABULAR:
        if (s.cn > 0) return tableStorageVolume(s.cx, s.cy, s.cn, d * s.ucfL) / s.ucfV;
        return 0.0;
    case ST_FUNCTIONAL:
        d *= s.ucfL;
        n = s.a2 + 1.0;
        v = (s.a0 * d) + s.a1 / n * pow(d, n);
        return v / s.ucfV;
    case ST_CYLINDRICAL: case ST_CONICAL: case ST_PARABOLOID: case ST_PYRAMIDAL:
        d *= s.ucfL;
        v = d * (s.a0 + d * (s.a1 / 2.0 + d * s.a2 / 3.0));
        return v / s.ucfV;
    default: return 0.0;
    }
}

// storage_getSurfArea (node.c:979-1018)
SWX_HD double storageSurfArea(const StorageGeom& s, double d)
{
    double area = 0.0;
    switch (s.shape) {
    case ST_TABULAR:
        if (s.cn > 0) area = tableLookupEx(s.cx, s.cy, s.cn, d * s.ucfL);
        break;
    case ST_FUNCTIONAL:
        area = s.a0 + s.a1 * pow(d * s.ucfL, s.a2);
        break;
    case ST_CYLINDRICAL: case ST_CONICAL: case ST_PARABOLOID: case ST_PYRAMIDAL:
        d *= s.ucfL;
        area = s.a0 + d * (s.a1 + d * s.a2);
        break;
    default: return 0.0;
    }
    return area / s.ucfL / s.ucfL;
}

// storage_getLosses (node.c:1052-1105) without exfiltration (seepage with a
// non-zero Ksat is rejected by the reader).  evapRate: Evap.rate (ft/s);
// returns the loss rate (cfs) and the step's evaporated volume in *evapVol.
// The reference's quirk is kept: below FUDGE stored volume the rate stays
// the per-area rate.
SWX_HD double storageLosses(const StorageGeom& s, double fEvap, double evapRate, double depth,
                            double volume, double tStep, double* evapVol)
{
    double rate = evapRate * fEvap;
    if (rate > 0.0) {
        double area = storageSurfArea(s, depth);
        if (volume > 0.0001) rate = area * rate;
        double total = rate * tStep;
        if (total > volume) rate *= volume / total;
    }
    *evapVol = rate * tStep;
    return rate;
}

}  // namespace swx
