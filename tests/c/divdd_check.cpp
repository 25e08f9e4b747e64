// divdd_check.cpp -- host check of divdd.h: divDD(a, b, recip(b)) == a / b bitwise
// (tests/test_divdd.py builds and runs it).  Inputs: uniform values, values
// within a few ulps of every table knot k*delta (where the lookup index
// floor(x / delta) is decided), and random divisors with their own pairs.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include "divdd.h"

using namespace swx;

static uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }

int main(int argc, char** argv)
{
    long n = argc > 1 ? atol(argv[1]) : 10000000;
    long bad = 0, tried = 0;
    // constants
    double rh, rl;
    recipDD(kCircDelta, &rh, &rl);
    if (kCircDelta != 1.0 / 50.0 || rh != kCircDeltaRh || rl != kCircDeltaRl) { printf("delta constants\n"); return 2; }
    recipDD(kCircDelta2, &rh, &rl);
    if (kCircDelta2 != kCircDelta * kCircDelta || rh != kCircDelta2Rh || rl != kCircDelta2Rl) { printf("delta2 constants\n"); return 2; }
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> u01(0.0, 1.2);
    auto check = [&](double a, double b, double h, double l) {
        tried++;
        double q = divDD(a, b, h, l), r = a / b;
        if (bits(q) != bits(r)) {
            if (bad < 10) printf("mismatch a=%a b=%a q=%a ref=%a\n", a, b, q, r);
            bad++;
        }
    };
    for (long i = 0; i < n; i++) {
        double a = u01(g);
        check(a, kCircDelta, kCircDeltaRh, kCircDeltaRl);
        check(a * a, kCircDelta2, kCircDelta2Rh, kCircDelta2Rl);
    }
    // knots: k*delta and its neighbours
    for (int k = 0; k <= 60; k++) {
        double x = k * kCircDelta;
        for (int s = -64; s <= 64; s++) {
            double y = x;
            for (int t = 0; t < (s < 0 ? -s : s); t++) y = nextafter(y, s < 0 ? -1.0 : 2.0);
            check(y, kCircDelta, kCircDeltaRh, kCircDeltaRl);
            check(y * y, kCircDelta2, kCircDelta2Rh, kCircDelta2Rl);
        }
    }
    // random divisors (section full depths 0.05 .. 40 ft) with their pairs
    std::uniform_real_distribution<double> ub(0.05, 40.0);
    for (long i = 0; i < n / 4; i++) {
        double b = ub(g);
        recipDD(b, &rh, &rl);
        for (int m = 0; m < 4; m++) check(u01(g) * b * 1.1, b, rh, rl);
        check(b, b, rh, rl);
        check(0.5 * b, b, rh, rl);
    }
    // the in-kernel pair (recipDDFast) for the momentum terms' shared
    // divisors -- conduit lengths and the momentum denominator -- with
    // numerators of either sign over many decades
    std::uniform_real_distribution<double> le(-3.0, 7.0), ae(-30.0, 12.0);
    for (long i = 0; i < n / 2; i++) {
        double b = std::pow(10.0, le(g));
        recipDDFast(b, &rh, &rl);
        if (rh != 1.0 / b) { printf("recipDDFast rh\n"); return 2; }
        for (int m = 0; m < 3; m++) {
            double a = std::pow(10.0, ae(g)) * ((g() & 1) ? -1.0 : 1.0);
            check(a, b, rh, rl);
        }
        check(b * 0.999, b, rh, rl);
        check(1.0, b, rh, rl);
    }
    printf("checked %ld quotients, %ld mismatches\n", tried, bad);
    return bad ? 1 : 0;
}
