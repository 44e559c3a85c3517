/* CPU check of sq_qm1d.hip's udiv: the compiler's fp64 division with the
   divisor's refined reciprocal shared, for initial reciprocals up to +-4 ulp
   off (v_rcp_f64's result is an approximation), against IEEE a / b. */
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double ulp_step(double x, int k) { while (k > 0) { x = nextafter(x, INFINITY); --k; } while (k < 0) { x = nextafter(x, -INFINITY); ++k; } return x; }
int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : 2000000, bad = 0;
    for (long i = 0; i < n; ++i) {
        /* divisor in [2^-60, 2^60]; numerator 2^-960 < |a| < 2^700 (udiv's fast range) */
        double b = ldexp(1.0 + (nxt() >> 11) * 0x1p-53, (int)(nxt() % 121) - 60);
        if (i % 3 == 0) b = (double)(1 + nxt() % 100000000ull);   /* den: integers */
        double a = ldexp(1.0 + (nxt() >> 11) * 0x1p-53, (int)(nxt() % 1659) - 959);
        if (i % 4 == 1) a = ldexp(1.0 + (nxt() >> 11) * 0x1p-53, (int)(nxt() % 64) - 40);
        if (nxt() & 1) a = -a;
        double r0 = ulp_step(1.0 / b, (int)(nxt() % 9) - 4);
        double r1 = fma(r0, fma(-b, r0, 1.0), r0);
        double R = fma(r1, fma(-b, r1, 1.0), r1);
        double m = a * R;
        double q = fma(fma(-b, m, a), R, m);
        double t = a / b;
        if (memcmp(&q, &t, 8) != 0) { if (bad < 5) printf("a=%a b=%a q=%a t=%a\n", a, b, q, t); ++bad; }
    }
    printf("checked %ld bad %ld\n", n, bad);
    return bad != 0;
}
