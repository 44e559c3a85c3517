// sq_selftest.hip -- small device kernels used by tests and bench.py: the
// Philox/Box-Muller normals exactly as the step kernels draw them (for the
// RNG parity test), a DPP lane-rotation probe (the x-neighbour exchange of the
// phi^4 kernel relies on wave_ror/wave_rol semantics), and a float4 streaming
// copy that measures the attainable HBM rate on the box.
#include <algorithm>

#include "sq_glibcf.h"
#include "sq_dpp.h"
#include "sq_internal.h"
#include "sq_rng.h"

namespace sq {

namespace {

__global__ __launch_bounds__(256) void normals_kernel(float *out, size_t nquads,
                                                     unsigned long long quad0, uint32_t stream,
                                                     unsigned long long step, uint32_t k0,
                                                     uint32_t k1) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nquads) return;
    const f32x4n n = normals4(quad0 + q, stream, (uint32_t)step, (uint32_t)(step >> 32), k0, k1);
    out[4 * q] = n.a;
    out[4 * q + 1] = n.b;
    out[4 * q + 2] = n.c;
    out[4 * q + 3] = n.d;
}

__global__ void dpp_kernel(float *out) {
    const int lane = threadIdx.x & 63;
    const int v = lane;
    out[lane] = (float)__builtin_amdgcn_update_dpp(0, v, 0x13C, 0xF, 0xF, false);       // wave_ror:1
    out[64 + lane] = (float)__builtin_amdgcn_update_dpp(0, v, 0x134, 0xF, 0xF, false);  // wave_rol:1
}

// glibc's logf / cosf / tanhf as the serial-order QM1D kernels evaluate them
// (sq_glibcf.h), for the bitwise test against the host libm.
__global__ __launch_bounds__(256) void libm_kernel(int fn, const float *x, float *y, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        y[i] = fn == 0 ? sq_glibc_logf(x[i]) : fn == 1 ? sq_glibc_cosf(x[i]) : sq_glibc_tanhf(x[i]);
}

// The Box-Muller factors of every 23-bit argument (sq_rng.h): radius
// sqrt(-2 ln u), radius_q sqrt(-log2 u), cos and sin of t revolutions.
__global__ __launch_bounds__(256) void bm_tables_kernel(float *rad, float *radq, float *cs, float *sn) {
    const uint32_t m = blockIdx.x * 256u + threadIdx.x;
    if (m >= (1u << 23)) return;
    rad[m] = bm_radius(m);
    radq[m] = bm_radius_q(m);
    cs[m] = bm_cos(m);
    sn[m] = bm_sin(m);
}

__global__ void philox_kernel(const uint32_t *ck, uint32_t *out) {
    const u32x4 o = philox4x32_10(u32x4{ck[0], ck[1], ck[2], ck[3]}, ck[4], ck[5]);
    out[0] = o.x;
    out[1] = o.y;
    out[2] = o.z;
    out[3] = o.w;
}

// Streaming copy used as the measured HBM ceiling: every thread moves 4
// float4 (all four loads issued before the stores), one pass, no grid-stride;
// NT = non-temporal loads/stores.  sq_copy_bandwidth reports the faster.
typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const f4v *__restrict__ in, f4v *__restrict__ out,
                                                   size_t n4) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
    f4v v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t i = base + 256 * k;
        if (i < n4) v[k] = NT ? __builtin_nontemporal_load(in + i) : in[i];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t i = base + 256 * k;
        if (i < n4) {
            if (NT) __builtin_nontemporal_store(v[k], out + i);
            else out[i] = v[k];
        }
    }
}

}  // namespace

// DPP cross-wave stress (the round-3 frame-record finding): the
// waves of a 16-wave block either run the frame records' wave-max scan
// (row_shr 1/2/4/8 + row_bcast 15/31 with row masks, sq_dpp.h dpp_all_max_f)
// or the stencil's x-neighbour rotation (wave_ror:1 / wave_rol:1 DPP fused into
// an add), checking every rotated value against the exact lane-1 / lane+1
// value; errs[lane] counts the lanes that got a wrong one.  mode 0: every wave
// rotates (control); 1: even waves scan, odd waves rotate; 2: every wave scans
// and rotates in turn; 3: as 1 with the scan's row_bcast steps left out.
__device__ __forceinline__ float mix_val(int lane, int wave, int it) {
    return (float)((lane * 131 + wave * 17 + it * 7) & 1023) * 0.25f + 1.0f;
}
template <int M>
__device__ __forceinline__ float mix_scan(float v) {
    const float id = -__builtin_inff();
    v = fmaxf(v, dpp_f<0x111, 0xf, 0xf>(v, id));
    v = fmaxf(v, dpp_f<0x112, 0xf, 0xf>(v, id));
    v = fmaxf(v, dpp_f<0x114, 0xf, 0xf>(v, id));
    v = fmaxf(v, dpp_f<0x118, 0xf, 0xf>(v, id));
    if constexpr (M != 3) {
        v = fmaxf(v, dpp_f<0x142, 0xa, 0xf>(v, id));
        v = fmaxf(v, dpp_f<0x143, 0xc, 0xf>(v, id));
    }
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
template <int M>
__global__ __launch_bounds__(1024) void dpp_mix_kernel(int iters, unsigned *errs, float *sink) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool scanner = (M == 1 || M == 3) ? (wave & 1) == 0 : M == 2;
    const bool rotator = M == 0 || M == 2 || (wave & 1) == 1;
    float acc = 0.f;
    unsigned bad = 0;
    for (int it = 0; it < iters; ++it) {
        const float v = mix_val(lane, wave, it), w = mix_val(lane, wave, it + 1);
        if (scanner) {
            // the records' shape: a ballot, a divergent per-lane update, the scan
            if (__ballot(v > 200.f) != 0ull) {
                if (v > acc) acc = v;
                acc = fmaxf(acc, mix_scan<M>(acc + v));
            }
        }
        if (rotator) {
            const float l = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x13C, 0xF, 0xF, true));
            const float r = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x134, 0xF, 0xF, true));
            const float sl = l + w, sr = r + w;  // fused into v_add_f32_dpp like the stencil's x-sums
            const float el = mix_val((lane + 63) & 63, wave, it) + w, er = mix_val((lane + 1) & 63, wave, it) + w;
            bad += (sl != el) + (sr != er);
        }
    }
    if (bad) atomicAdd(errs + lane, bad);
    if (acc == 12345.f) sink[threadIdx.x] = acc;  // keeps the scans alive
}

hipError_t selftest_normals_launch(float *out, size_t nquads, unsigned long long quad0,
                                   uint32_t stream, unsigned long long step, uint32_t k0,
                                   uint32_t k1, hipStream_t s) {
    const unsigned grid = (unsigned)((nquads + 255) / 256);
    hipLaunchKernelGGL(normals_kernel, dim3(grid), dim3(256), 0, s, out, nquads, quad0, stream, step,
                       k0, k1);
    return hipGetLastError();
}

hipError_t selftest_dpp_mix_launch(int mode, int blocks, int iters, unsigned *errs, float *sink, hipStream_t s) {
    switch (mode) {
    case 0: hipLaunchKernelGGL(dpp_mix_kernel<0>, dim3(blocks), dim3(1024), 0, s, iters, errs, sink); break;
    case 1: hipLaunchKernelGGL(dpp_mix_kernel<1>, dim3(blocks), dim3(1024), 0, s, iters, errs, sink); break;
    case 2: hipLaunchKernelGGL(dpp_mix_kernel<2>, dim3(blocks), dim3(1024), 0, s, iters, errs, sink); break;
    default: hipLaunchKernelGGL(dpp_mix_kernel<3>, dim3(blocks), dim3(1024), 0, s, iters, errs, sink); break;
    }
    return hipGetLastError();
}

hipError_t selftest_dpp_launch(float *out, hipStream_t s) {
    hipLaunchKernelGGL(dpp_kernel, dim3(1), dim3(64), 0, s, out);
    return hipGetLastError();
}

hipError_t selftest_libm_launch(int fn, const float *x, float *y, long long n, hipStream_t s) {
    const unsigned grid = (unsigned)std::min<long long>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(libm_kernel, dim3(grid), dim3(256), 0, s, fn, x, y, n);
    return hipGetLastError();
}

hipError_t selftest_bm_tables_launch(float *t, hipStream_t s) {
    const size_t n = (size_t)1 << 23;
    hipLaunchKernelGGL(bm_tables_kernel, dim3((unsigned)(n / 256)), dim3(256), 0, s, t, t + n, t + 2 * n, t + 3 * n);
    return hipGetLastError();
}

hipError_t selftest_philox_launch(const uint32_t *ck, uint32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(philox_kernel, dim3(1), dim3(1), 0, s, ck, out);
    return hipGetLastError();
}

hipError_t copy_launch(const float4 *in, float4 *out, size_t n4, bool nt, hipStream_t s) {
    const unsigned grid = (unsigned)((n4 + 1023) / 1024);
    const f4v *i4 = reinterpret_cast<const f4v *>(in);
    f4v *o4 = reinterpret_cast<f4v *>(out);
    if (nt) hipLaunchKernelGGL(copy_kernel<true>, dim3(grid), dim3(256), 0, s, i4, o4, n4);
    else hipLaunchKernelGGL(copy_kernel<false>, dim3(grid), dim3(256), 0, s, i4, o4, n4);
    return hipGetLastError();
}

}  // namespace sq
