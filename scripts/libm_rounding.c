/* How often glibc's float logf / cosf / tanhf differ from the correctly rounded
 * value (fp64 evaluation rounded once) on the arguments the reference's
 * random() and x_cl produce.  gcc -O2 -ffp-contract=off libm_rounding.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

int main(void)
{
    uint64_t s = 88172645463325252ull;
    long n = 20000000, bc = 0, bl = 0, bt = 0;
    for (long k = 0; k < n; k++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        double u2 = (double)((s >> 16) & 0xffffffffull) / 4294967296.0;
        float x = (float)(2 * 3.1415 * u2);
        if (cosf(x) != (float)cos((double)x)) bc++;
        double u1 = (double)(((s >> 20) & 0xffffffffull) | 1) / 4294967296.0;
        float y = (float)u1;
        if (logf(y) != (float)log((double)y)) bl++;
        float z = (float)(((double)(s & 0xffffff) / 16777216.0 - 0.5) * 8);
        if (tanhf(z) != (float)tanh((double)z)) bt++;
    }
    printf("of %ld arguments: cosf %ld (%.2f%%), logf %ld (%.2f%%), tanhf %ld (%.2f%%) differ from correct rounding\n",
           n, bc, 100.0 * bc / n, bl, 100.0 * bl / n, bt, 100.0 * bt / n);
    return 0;
}
