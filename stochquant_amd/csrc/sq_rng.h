// sq_rng.h -- counter-based noise for the Langevin kernels (gfx950 device code).
//
// Replaces the reference's random() (tau_kernel.cl:269-284): a 48-bit LCG on
// ONE shared seed that every work-item read-modify-writes, i.e. a serial
// dependency chain across all sites and a data race under any parallel
// execution.  Here every site draws from Philox4x32-10 keyed by the run seed
// with the counter {quad, stream|quad_hi, step_lo, step_hi}, so a normal
// depends only on (seed, stream, site, step): no shared state, any execution
// order and any slab decomposition give the same numbers.
//
// Box-Muller on hardware transcendentals:
//   u = 1 - (w0 & 0x7FFFFF)*2^-23 in (0,1],  t = (w1 & 0x7FFFFF)*2^-23 (both exact)
//   r = sqrt(-2 ln2 * log2 u)   v_log_f32 + v_sqrt_f32
//   n = r*cos(2 pi t), r*sin(2 pi t)   v_cos_f32 / v_sin_f32 take revolutions,
//   so no range reduction is needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sq {

constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;

// Noise streams (bits 24..31 of counter word 1).
constexpr uint32_t kStreamField = 0;  // per-site field noise
constexpr uint32_t kStreamOmega = 1;  // QM1D collective coordinate
constexpr uint32_t kStreamInit = 2;   // initial field

struct u32x4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += kPhiloxW0;
            k1 += kPhiloxW1;
        }
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c.x;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    }
    return c;
}

__device__ __forceinline__ u32x4 philox_counter(uint64_t quad, uint32_t stream, uint32_t step_lo,
                                                uint32_t step_hi) {
    return u32x4{(uint32_t)quad, ((uint32_t)(quad >> 32) & 0x00FFFFFFu) | (stream << 24), step_lo,
                 step_hi};
}

// The four factors of a pair, each a function of 23 bits of one word (so
// sq_selftest_bm_tables can tabulate them, and the oracle reproduce a
// device normal bit for bit as one fp32 product of two table entries):
//   u = 2 - [1.m0] in (0,1] (exact, Sterbenz), t = [1.m1] in [1,2) revolutions
//   (one v_and_or_b32 each; cos/sin have period 1 revolution, so t needs no "- 1").
__device__ __forceinline__ float bm_u(uint32_t w0) { return 2.0f - __uint_as_float(0x3F800000u | (w0 & 0x007FFFFFu)); }
__device__ __forceinline__ float bm_t(uint32_t w1) { return __uint_as_float(0x3F800000u | (w1 & 0x007FFFFFu)); }
__device__ __forceinline__ float bm_radius(uint32_t w0) {  // sqrt(-2 ln u) = sqrt(-2 ln 2 * log2 u)
    return __builtin_amdgcn_sqrtf(__builtin_amdgcn_logf(bm_u(w0)) * -1.38629436111989061f);
}
__device__ __forceinline__ float bm_radius_q(uint32_t w0) {  // sqrt(-log2 u)
    return __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(bm_u(w0)));
}
__device__ __forceinline__ float bm_cos(uint32_t w1) { return __builtin_amdgcn_cosf(bm_t(w1)); }
__device__ __forceinline__ float bm_sin(uint32_t w1) { return __builtin_amdgcn_sinf(bm_t(w1)); }

__device__ __forceinline__ void box_muller(uint32_t w0, uint32_t w1, float &nc, float &ns) {
    const float r = bm_radius(w0);
    nc = r * bm_cos(w1);
    ns = r * bm_sin(w1);
}

// Box-Muller without the sqrt(2 ln 2) factor: r' = sqrt(-log2 u), so the pair
// is (r' cos, r' sin) = (nc, ns) / sqrt(2 ln 2).  The Langevin kernels fold the
// factor into their noise amplitude (Phi4StepArgs::sigq = sigma sqrt(2 ln 2)),
// which saves one multiply per pair; the sign flip is a free source modifier.
__device__ __forceinline__ void box_muller_q(uint32_t w0, uint32_t w1, float &nc, float &ns) {
    const float r = bm_radius_q(w0);
    nc = r * bm_cos(w1);
    ns = r * bm_sin(w1);
}

struct f32x4n {
    float a, b, c, d;
};

__device__ __forceinline__ f32x4n normals4(uint64_t quad, uint32_t stream, uint32_t step_lo,
                                           uint32_t step_hi, uint32_t k0, uint32_t k1) {
    const u32x4 o = philox4x32_10(philox_counter(quad, stream, step_lo, step_hi), k0, k1);
    f32x4n n;
    box_muller(o.x, o.y, n.a, n.b);
    box_muller(o.z, o.w, n.c, n.d);
    return n;
}

}  // namespace sq
