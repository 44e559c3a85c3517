/*
 * orc_rng.c -- oracle RNGs (TEST INFRASTRUCTURE ONLY, see sq_oracle.h).
 *
 *  - orc_philox4x32_10: Philox4x32-10 as published by Salmon, Moraes, Dror,
 *    Shaw, "Parallel random numbers: as easy as 1, 2, 3" (SC'11), the
 *    Random123 reference algorithm.  Third-party algorithm, not vendored in
 *    /root/reference; pinned by the Random123 known-answer vectors recorded
 *    in SURVEY.md Appendix D (tests/golden/philox_kat.json).
 *  - orc_normals4: the build's counter layout + Box-Muller,
 *    evaluated in double and rounded once to float (the "ideal" value the
 *    GPU's hardware transcendentals are compared against).
 *  - orc_ref_random: restatement of the reference's random(),
 *    tau_kernel.cl:269-284 (Java-style 48-bit LCG on one shared seed,
 *    Box-Muller with the literal 3.1415 and float log/sqrt/cos).
 */
#include <math.h>
#include <stdint.h>
#include "sq_oracle.h"

#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Box-Muller pair from two 32-bit words:
 *   u = 1 - (w0 & 0x7FFFFF) * 2^-23   in (0,1], exact in fp32
 *   t = (w1 & 0x7FFFFF) * 2^-23       in [0,1) revolutions, exact in fp32
 *   n_cos = sqrt(-2 ln u) cos(2 pi t),  n_sin = sqrt(-2 ln u) sin(2 pi t) */
/* Device-transcendental mode (orc_set_bm_tables): the MI355X's Box-Muller
 * factors for every 23-bit argument, as sq_selftest_bm_tables returns them
 * (radius sqrt(-2 ln u), radius_q sqrt(-log2 u), cos, sin; 2^23 each).  A
 * device normal is then one fp32 product of two entries, so the oracle gives
 * the GPU's bits; the entries themselves are checked against the
 * double-evaluated values (tests/test_gpu_selftest.py). */
#define BM_N ((size_t)1 << 23)
static const float *g_bm = NULL;

void orc_set_bm_tables(const float *tab) { g_bm = tab; }
int orc_bm_tables_on(void) { return g_bm != NULL; }

static void bm_pair(uint32_t w0, uint32_t w1, float *nc, float *ns)
{
    if (g_bm) {
        const float r = g_bm[w0 & 0x7FFFFFu];
        *nc = r * g_bm[2 * BM_N + (w1 & 0x7FFFFFu)];
        *ns = r * g_bm[3 * BM_N + (w1 & 0x7FFFFFu)];
        return;
    }
    const double u = 1.0 - (double)(w0 & 0x7FFFFFu) * 0x1p-23;
    const double t = (double)(w1 & 0x7FFFFFu) * 0x1p-23;
    const double r = sqrt(-2.0 * log(u));
    const double ang = 2.0 * M_PI * t;
    *nc = (float)(r * cos(ang));
    *ns = (float)(r * sin(ang));
}

/* The phi^4 kernels' field noise in device-transcendental mode: the pairs
 * without the sqrt(2 ln 2) factor (box_muller_q), which sigq carries. */
static void bm_pair_q(uint32_t w0, uint32_t w1, float *nc, float *ns)
{
    const float r = g_bm[BM_N + (w0 & 0x7FFFFFu)];
    *nc = r * g_bm[2 * BM_N + (w1 & 0x7FFFFFu)];
    *ns = r * g_bm[3 * BM_N + (w1 & 0x7FFFFFu)];
}

void orc_normals4_q(uint64_t seed, uint32_t stream, uint64_t quad, uint64_t step, float out[4])
{
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)quad,
                       ((uint32_t)(quad >> 32) & 0x00FFFFFFu) | (stream << 24),
                       (uint32_t)step, (uint32_t)(step >> 32)};
    uint32_t o[4];
    orc_philox4x32_10(ctr, key, o);
    bm_pair_q(o[0], o[1], &out[0], &out[1]);
    bm_pair_q(o[2], o[3], &out[2], &out[3]);
}

void orc_normals4(uint64_t seed, uint32_t stream, uint64_t quad, uint64_t step, float out[4])
{
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)quad,
                       ((uint32_t)(quad >> 32) & 0x00FFFFFFu) | (stream << 24),
                       (uint32_t)step, (uint32_t)(step >> 32)};
    uint32_t o[4];
    orc_philox4x32_10(ctr, key, o);
    bm_pair(o[0], o[1], &out[0], &out[1]);
    bm_pair(o[2], o[3], &out[2], &out[3]);
}

/* OpenCL isinf() on a scalar returns exactly 1 for +-inf (the reference
 * compares `== 1`, tau_kernel.cl:130,282). */
static int cl_isinf(float v) { return isinf(v) ? 1 : 0; }

/* One call of random(); w1, w2 (if non-NULL) get the 32-bit words t1>>16,
 * t2>>16 of the accepted (non-retried) draw. */
static double ref_random_words(uint64_t *seed, int gid, uint32_t *w1, uint32_t *w2)
{
    const uint64_t mask48 = (((uint64_t)1) << 48) - 1;
    const uint64_t two31 = (uint64_t)2147483648.0f;   /* (ulong)pown((float)2,31) */
    const double two32 = (double)4294967296.0f;       /* (double)pown((float)2,32) */
    double result;
    uint64_t t;
    do {
        t = ((*seed + (uint64_t)gid) * 0x5DEECE66DULL + 0xBULL) & mask48;
        const uint32_t a1 = (uint32_t)(t >> 16);
        double v1 = (double)(t >> 16) / two32;
        t = ((t + (uint64_t)gid) * 0x5DEECE66DULL + 0xBULL) & mask48;
        double v2 = (double)(t >> 16) / two32;
        if (w1) *w1 = a1;
        if (w2) *w2 = (uint32_t)(t >> 16);
        float lg = logf((float)v1);
        float cs = cosf((float)(2. * 3.1415 * v2));
        float sq = sqrtf((float)(-2. * (double)lg));
        result = (double)cs * (double)sq;
        if (*seed < two31 && t < two31)
            *seed += t;
        else
            *seed = t - two31;
    } while (cl_isinf((float)result) == 1);
    return result;
}

double orc_ref_random(uint64_t *seed, int gid) { return ref_random_words(seed, gid, 0, 0); }

void orc_libm_f32(int fn, const float *x, float *y, long long n)
{
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < n; ++i)
        y[i] = fn == 0 ? logf(x[i]) : fn == 1 ? cosf(x[i]) : tanhf(x[i]);
}

/* The draws of one full launch in call order: rounds 0..loops-1, items
 * 0..N in id order, k = r*(N+1) + g.  seeds[k] is the
 * shared seed after call k, so a launch that breaks after call k leaves the
 * seed at seeds[k]. */
void orc_ref_noise_stream(uint64_t seed, int N, int loops, double *xi, uint32_t *w1, uint32_t *w2,
                          uint64_t *seeds)
{
    size_t k = 0;
    for (int r = 0; r < loops; ++r)
        for (int g = 0; g <= N; ++g, ++k) {
            xi[k] = ref_random_words(&seed, g, &w1[k], &w2[k]);
            seeds[k] = seed;
        }
}
