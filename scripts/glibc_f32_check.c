// Exhaustive check of the device restatement of glibc 2.35's logf and cosf
// (stochquant_amd/csrc/sq_glibcf.h) against this host's libm, bit for bit,
// over every float argument the reference's random() can pass
// (tau_kernel.cl:269-284: log of a uniform in (0, 1], cos of 2*3.1415*u).
//
//   gcc -O2 -fopenmp -ffp-contract=off -o /tmp/glibc_f32_check scripts/glibc_f32_check.c -lm
//   /tmp/glibc_f32_check [stride]   -> mismatch counts (0 = bit-identical);
//   stride > 1 checks every stride-th argument (tests/test_glibcf.py)
//
// glibc selects its x86-64 FMA builds of logf / cosf (ifunc) on CPUs with
// FMA (this container's Xeon and the GPU box's EPYC both have it), so the
// restatement contracts exactly where GCC contracted those builds.
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define SQ_GLIBCF_HOST 1
#include "../stochquant_amd/csrc/sq_glibcf.h"

static float as_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t as_u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    const long long st = argc > 1 ? atoll(argv[1]) : 1;
    // logf: every float in [0, 2) (v1 is 0 or >= 2^-32 in the reference;
    // subnormals and zero for completeness) and the specials below
    const uint32_t lo_l = 0, hi_l = as_u(2.0f);
    long long bad_l = 0, n_l = 0;
    uint32_t first_l = 0;
#pragma omp parallel for reduction(+ : bad_l, n_l) schedule(static)
    for (long long u = lo_l; u < (long long)hi_l; u += st) {
        const float x = as_f((uint32_t)u);
        const float a = logf(x), b = sq_glibc_logf(x);
        ++n_l;
        if (as_u(a) != as_u(b)) {
            ++bad_l;
            if (!first_l) first_l = (uint32_t)u;
        }
    }
    const float spec[] = {-0.0f, -1.0f, INFINITY, -INFINITY, NAN, 3.0e38f};
    for (int k = 0; k < 6; ++k) {
        const float a = logf(spec[k]), b = sq_glibc_logf(spec[k]);
        if (!(as_u(a) == as_u(b) || (isnan(a) && isnan(b)))) ++bad_l;
        ++n_l;
    }
    // cosf: every float in [0, 6.3] (2 * 3.1415 * u < 6.283) and the negatives
    const uint32_t hi_c = as_u(6.3f);
    long long bad_c = 0, n_c = 0;
    uint32_t first_c = 0;
#pragma omp parallel for reduction(+ : bad_c, n_c) schedule(static)
    for (long long u = 0; u <= (long long)hi_c; u += st) {
        for (int sgn = 0; sgn < 2; ++sgn) {
            const float x = as_f((uint32_t)u | (sgn ? 0x80000000u : 0u));
            const float a = cosf(x), b = sq_glibc_cosf(x);
            ++n_c;
            if (as_u(a) != as_u(b)) {
                ++bad_c;
                if (!first_c) first_c = (uint32_t)u;
            }
        }
    }
    // tanhf: every float (both signs; x_cl's argument s (t - w) / eta spans the chain)
    long long bad_t = 0, n_t = 0;
    uint32_t first_t = 0;
#pragma omp parallel for reduction(+ : bad_t, n_t) schedule(static)
    for (long long u = 0; u <= 0xffffffffLL; u += st) {
        const float x = as_f((uint32_t)u);
        const float a = tanhf(x), b = sq_glibc_tanhf(x);
        ++n_t;
        if (as_u(a) != as_u(b) && !(isnan(a) && isnan(b))) {
            ++bad_t;
            if (!first_t) first_t = (uint32_t)u;
        }
    }
    printf("tanhf: %lld of %lld arguments differ (first 0x%08x)\n", bad_t, n_t, first_t);
    printf("logf: %lld of %lld arguments differ (first 0x%08x)\n", bad_l, n_l, first_l);
    printf("cosf: %lld of %lld arguments differ (first 0x%08x)\n", bad_c, n_c, first_c);
    return (bad_l || bad_c || bad_t) ? 1 : 0;
}
