// Markstein division check (CPU): q = RN(a*y), y = RN(1/b), one and two corrections
// q <- fma(fma(-q, b, a), y, q) against the IEEE quotient a / b (sptrsv_grid_kernel's div_markstein).
// gcc -O2 -mfma tools/markstein_check.c -lm -o /tmp/mk && /tmp/mk 200000000
// Ranges: (1) the original sample (a: 2^-30..2^30, b: 2^-10..2^10); (2) the full range the kernel
// admits: a in [2^-900, 2^900], b (dictionary diagonal) in [2^-100, 2^100], exponents drawn uniformly,
// plus both ends of each range; (3) the guard the kernel applies (device-side fallback to a / b for
// |a| outside [2^-900, 2^901) or not finite, a == 0 keeps q0) on zeros, subnormals, infinities.
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double rd(int emin, int erange) {
    uint64_t m = xr() & ((1ull << 52) - 1);
    int e = emin + (int)(xr() % erange);
    uint64_t b = ((uint64_t)(e + 1023) << 52) | m;
    if (xr() & 1) b |= 1ull << 63;
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static inline double mk2(double a, double b, double y) {   // div_markstein as the kernel computes it
    double q0 = a * y;
    double q1 = fma(fma(-q0, b, a), y, q0);
    double q2 = fma(fma(-q1, b, a), y, q1);
    int ex = 0;
    if (isfinite(a)) frexp(a, &ex);                          // the kernel's frexp exponent: 0 for 0 / inf / NaN
    if ((unsigned)(ex + 899) > 1800u || !isfinite(a)) return a / b;   // the conditional IEEE re-solve
    return a == 0.0 ? q0 : q2;
}
static inline int same(double u, double v) { return memcmp(&u, &v, 8) == 0 || (isnan(u) && isnan(v)); }
int main(int argc, char **argv) {
    long N = argc > 1 ? atol(argv[1]) : 20000000;
    long bad1 = 0, bad2 = 0, badfull = 0, badedge = 0;
    for (long i = 0; i < N; i++) {
        double a = rd(-30, 60), b = rd(-10, 20);
        double q = a / b, y = 1.0 / b;
        double q0 = a * y, r0 = fma(-q0, b, a), q1 = fma(r0, y, q0);
        if (q1 != q) bad1++;
        double r1 = fma(-q1, b, a), q2 = fma(r1, y, q1);
        if (q2 != q) bad2++;
        double A = rd(-900, 1801), B = rd(-100, 201);   // exponents -900..900 and -100..100
        if (!same(mk2(A, B, 1.0 / B), A / B)) badfull++;
    }
    // range ends and special values of the right-hand side against ends of the diagonal range
    const double bs[] = {0x1p-100, -0x1p-100, 0x1.fffffffffffffp+100, 0x1p+100, 3.0, -7.25, 0x1.8p-99};
    const double as[] = {0.0, -0.0, 0x1p-900, -0x1p-900, 0x1.fffffffffffffp+900, 0x1p+900, 0x1p+901, 0x1.fffffffffffffp-901, 0x1p-1074, 0x1p-1022,
                         0x1.8p-1000, 1e300, -1e308, INFINITY, -INFINITY, NAN, 1.0, 0x1.fffffffffffffp-1};
    long nedge = 0;
    for (unsigned i = 0; i < sizeof bs / sizeof *bs; ++i)
        for (unsigned j = 0; j < sizeof as / sizeof *as; ++j) {
            ++nedge;
            if (!same(mk2(as[j], bs[i], 1.0 / bs[i]), as[j] / bs[i])) {
                badedge++;
                printf("edge mismatch a=%a b=%a: %a vs %a\n", as[j], bs[i], mk2(as[j], bs[i], 1.0 / bs[i]), as[j] / bs[i]);
            }
        }
    printf("N=%ld one-step mismatches %ld, two-step %ld; full kernel range (a 2^-900..2^900, b 2^-100..2^100) "
           "with the guard: %ld; %ld edge pairs: %ld mismatches\n", N, bad1, bad2, badfull, nedge, badedge);
    return (bad2 || badfull || badedge) ? 1 : 0;
}
