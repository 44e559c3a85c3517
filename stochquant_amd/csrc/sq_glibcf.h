// sq_glibcf.h -- glibc 2.35's single-precision logf and cosf, restated for the
// device, so the reference's random() (tau_kernel.cl:269-284: float log / cos
// of its LCG uniforms) draws the same bits on the GPU as the oracle and the
// reference do on the host (glibc libm).
//
// Algorithm (glibc sysdeps/ieee754/flt-32/e_logf.c, s_cosf.c + sincosf.h,
// from Arm's optimized-routines; the host's libm.so.6 holds the same tables):
//   logf: x = 2^k z, z in [OFF, 2 OFF); log x = log1p(z/c - 1) + log c + k ln2
//         with (1/c, log c) from a 16-entry table and a degree-4 polynomial in
//         double;
//   cosf: |x| < pi/4 the cosine polynomial; |x| < 120 one multiply-subtract
//         reduction by pi/2 (2/pi pre-scaled by 2^24) and the sine or cosine
//         polynomial of the quadrant, in double.
// glibc selects its FMA builds of both (x86-64 ifunc) on CPUs with FMA; the
// a*b+c that GCC contracts there are explicit fma here (the uncontracted
// order rounds to the same floats over the checked ranges too).  Pinned by
// scripts/glibc_f32_check.c: bit-identical to the host's libm over every
// argument the reference can pass and more (logf on every float of [0, 2)
// and the specials, cosf on [-6.3, 6.3]).  cosf beyond |x| >= 120 (glibc's
// Payne-Hanek branch) is not restated: the callers pass 2 * 3.1415 * u < 6.3.
//
// Provenance and licences (see also THIRD_PARTY_NOTICES.md at the repo root):
// the 16-entry log table, the logf/cosf polynomial coefficients and the
// 2/pi reduction constants below are numeric data reproduced from GNU C
// Library 2.35, sysdeps/ieee754/flt-32/{e_logf_data.c, s_sincosf_data.c,
// sincosf.h}.  glibc is licensed LGPL-2.1-or-later; these files were
// contributed to it by Arm Ltd from Arm's optimized-routines project
// (Copyright (c) 2017-2018 Arm Ltd, today distributed under MIT OR
// Apache-2.0 WITH LLVM-exception).  The flt-32 directory's older routines
// carry Sun Microsystems' fdlibm notice, reproduced here because glibc's
// single-precision reduction derives from it:
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this software is freely
//   granted, provided that this notice is preserved.
// The code in this header is a restatement (written for this project), not a
// copy of glibc's sources; the constants are what make it bit-identical.
#pragma once

#include <stdint.h>

#ifdef SQ_GLIBCF_HOST
#include <math.h>
#include <string.h>
#define SQ_GF_FN static inline
#define SQ_GF_FMA(a, b, c) fma((a), (b), (c))
#define SQ_GF_CONST static const
static inline uint32_t sq_gf_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float sq_gf_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
#else
#include <hip/hip_runtime.h>
#define SQ_GF_FN __device__ __forceinline__
#define SQ_GF_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define SQ_GF_CONST __device__ static const
__device__ __forceinline__ uint32_t sq_gf_asuint(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float sq_gf_asfloat(uint32_t u) { return __builtin_bit_cast(float, u); }
#endif

// (1/c, log c) per 1/16 of the mantissa range, e_logf_data.c
SQ_GF_CONST double sq_gf_logf_tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};

SQ_GF_FN float sq_glibc_logf(float x) {
    const double ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = sq_gf_asuint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {  // subnormal, zero, negative, inf or NaN
        if (ix * 2 == 0) return -__builtin_inff();           // log(+-0) = -inf (the caller retries)
        if (ix == 0x7f800000u) return x;                      // log(inf) = inf
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
        ix = sq_gf_asuint(x * 0x1p23f) - (23u << 23);         // subnormal: normalise
    }
    const uint32_t tmp = ix - 0x3f330000u;  // OFF
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = sq_gf_logf_tab[i][0], logc = sq_gf_logf_tab[i][1];
    const double z = (double)sq_gf_asfloat(iz);
    const double r = SQ_GF_FMA(z, invc, -1.0);
    const double y0 = SQ_GF_FMA((double)k, ln2, logc);
    const double r2 = r * r;
    double y = SQ_GF_FMA(A1, r, A2);
    y = SQ_GF_FMA(A0, r2, y);
    y = SQ_GF_FMA(y, r2, y0 + r);
    return (float)y;
}

// sincosf.h's sinf_poly: n odd the cosine polynomial, even the sine one;
// q selects the sign-flipped cosine coefficients of quadrants 2 and 3.
SQ_GF_FN float sq_gf_sinf_poly(double x, double x2, int q, int n) {
    const double c0 = q ? -1.0 : 1.0;
    const double c1 = q ? 0x1.ffffffd0c621cp-2 : -0x1.ffffffd0c621cp-2;
    const double c2 = q ? -0x1.55553e1068f19p-5 : 0x1.55553e1068f19p-5;
    const double c3 = q ? 0x1.6c087e89a359dp-10 : -0x1.6c087e89a359dp-10;
    const double c4 = q ? -0x1.99343027bf8c3p-16 : 0x1.99343027bf8c3p-16;
    const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double t1 = SQ_GF_FMA(x2, s3, s2);
        const double x7 = x3 * x2;
        const double s = SQ_GF_FMA(x3, s1, x);
        return (float)SQ_GF_FMA(x7, t1, s);
    }
    const double x4 = x2 * x2;
    const double t2 = SQ_GF_FMA(x2, c4, c3);
    const double t1 = SQ_GF_FMA(x2, c1, c0);
    const double x6 = x4 * x2;
    const double c = SQ_GF_FMA(x4, c2, t1);
    return (float)SQ_GF_FMA(x6, t2, c);
}

SQ_GF_FN float sq_glibc_cosf(float y) {
    const uint32_t top = (sq_gf_asuint(y) >> 20) & 0x7ff;
    double x = (double)y;
    if (top < ((sq_gf_asuint(0x1.921FB6p-1f) >> 20) & 0x7ff)) {  // |y| < pi/4
        if (top < ((sq_gf_asuint(0x1p-12f) >> 20) & 0x7ff)) return 1.0f;
        return sq_gf_sinf_poly(x, x * x, 0, 1);
    }
    // |y| < 120: reduce_fast without the toint intrinsics (2/pi * 2^24, the
    // quadrant in bits 24..31 of the truncated product)
    const double r = x * 0x1.45f306dc9c883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = SQ_GF_FMA(-(double)n, 0x1.921fb54442d18p+0, x);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;  // sign[n & 3] = {1, -1, -1, 1}
    return sq_gf_sinf_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
}

// glibc 2.35's tanhf (sysdeps/ieee754/flt-32/s_tanhf.c) and the expm1f it
// calls (s_expm1f.c): fdlibm's float algorithms, every operation a float
// operation in source order (no FMA builds of these exist in glibc).
SQ_GF_FN float sq_glibc_expm1f(float x) {
    const float o_threshold = 8.8721679688e+01f, ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f,
                invln2 = 1.4426950216e+00f, Q1 = -3.3333335072e-02f, Q2 = 1.5873016091e-03f,
                Q3 = -7.9365076090e-05f, Q4 = 4.0082177293e-06f, Q5 = -2.0109921195e-07f;
    uint32_t hx = sq_gf_asuint(x);
    const uint32_t xsb = hx & 0x80000000u;
    hx &= 0x7fffffffu;
    if (hx >= 0x4195b844u) {  // |x| >= 27 ln2
        if (hx >= 0x42b17218u) {
            if (hx > 0x7f800000u) return x + x;
            if (hx == 0x7f800000u) return xsb == 0 ? x : -1.0f;
            if (x > o_threshold) return __builtin_inff();
        }
        if (xsb != 0) return -1.0f;  // tiny - one
    }
    float hi, lo, c = 0.0f, t;
    int k;
    if (hx > 0x3eb17218u) {  // |x| > 0.5 ln2
        if (hx < 0x3F851592u) {
            if (xsb == 0) {
                hi = x - ln2_hi;
                lo = ln2_lo;
                k = 1;
            } else {
                hi = x + ln2_hi;
                lo = -ln2_lo;
                k = -1;
            }
        } else {
            k = (int)(invln2 * x + ((xsb == 0) ? 0.5f : -0.5f));
            t = (float)k;
            hi = x - t * ln2_hi;
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (hx < 0x33000000u) {  // |x| < 2^-25
        return x;
    } else {
        k = 0;
    }
    const float hfx = 0.5f * x;
    const float hxs = x * hfx;
    const float r1 = 1.0f + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    t = 3.0f - r1 * hfx;
    float e = hxs * ((r1 - t) / (6.0f - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5f * (x - e) - 0.5f;
    if (k == 1) {
        if (x < -0.25f) return -2.0f * (e - (x + 0.5f));
        return 1.0f + 2.0f * (x - e);
    }
    float y;
    if (k <= -2 || k > 56) {
        y = 1.0f - (e - x);
        y = sq_gf_asfloat(sq_gf_asuint(y) + ((uint32_t)k << 23));
        return y - 1.0f;
    }
    if (k < 23) {
        t = sq_gf_asfloat(0x3f800000u - (0x1000000u >> k));  // 1 - 2^-k
        y = t - (e - x);
        y = sq_gf_asfloat(sq_gf_asuint(y) + ((uint32_t)k << 23));
    } else {
        t = sq_gf_asfloat((uint32_t)(0x7f - k) << 23);  // 2^-k
        y = x - (e + t);
        y += 1.0f;
        y = sq_gf_asfloat(sq_gf_asuint(y) + ((uint32_t)k << 23));
    }
    return y;
}

SQ_GF_FN float sq_glibc_tanhf(float x) {
    const uint32_t jx = sq_gf_asuint(x), ix = jx & 0x7fffffffu;
    if (ix >= 0x7f800000u) return (int32_t)jx >= 0 ? 1.0f / x + 1.0f : 1.0f / x - 1.0f;
    float z;
    if (ix < 0x41b00000u) {  // |x| < 22
        if (ix == 0) return x;
        if (ix < 0x24000000u) return x * (1.0f + x);  // |x| < 2^-55
        if (ix >= 0x3f800000u) {                      // |x| >= 1
            const float t = sq_glibc_expm1f(2.0f * __builtin_fabsf(x));
            z = 1.0f - 2.0f / (t + 2.0f);
        } else {
            const float t = sq_glibc_expm1f(-2.0f * __builtin_fabsf(x));
            z = -t / (t + 2.0f);
        }
    } else {
        z = 1.0f;  // one - tiny
    }
    return (int32_t)jx >= 0 ? z : -z;
}
