// sq_fields.hip -- deterministic initial fields that need no random-number
// generator shared with a checker: phi(site) = amp * u(site), u the top 24 bits
// of splitmix64(global site index ^ key) mapped to [-1, 1).  Integer arithmetic
// and one exact power-of-two scaling, so a host restatement (numpy,
// stochquant_amd/verify.py hash_field) produces the same bits, and every
// decomposition (slabs, ranks) the same field.  bench.py's oracle_check starts
// the noise-off protocol from it (sq_init_field_hash).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sq_internal.h"

namespace sq {
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One float4 per thread and iteration: sites i0 .. i0+3 of the slab (global
// index gi0 + 4 q .. +3); amp / 2^23 scales the centred 24-bit integer exactly.
__global__ __launch_bounds__(256) void phi4_init_hash_kernel(float *slab, size_t nq, uint64_t gi0, uint64_t key,
                                                             double scale) {
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (size_t)gridDim.x * blockDim.x) {
        const uint64_t g = gi0 + 4 * (uint64_t)q;
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t h = splitmix64((g + (uint64_t)k) ^ key) >> 40;  // [0, 2^24)
            v[k] = (float)(((double)h - 8388608.0) * scale);
        }
        *reinterpret_cast<float4 *>(slab + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
    }
}

}  // namespace

hipError_t phi4_init_hash_launch(float *slab, int Lx, int Ly, int nz, long long zg0, unsigned long long key,
                                 double amp, hipStream_t s) {
    const size_t plane = (size_t)Lx * Ly, n = (size_t)nz * plane;
    if (n % 4 != 0) return hipErrorInvalidValue;
    const size_t nq = n / 4;
    const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>((nq + 255) / 256, 8192));
    hipLaunchKernelGGL(phi4_init_hash_kernel, dim3(grid), dim3(256), 0, s, slab, nq, (uint64_t)zg0 * plane,
                       (uint64_t)key, amp / 8388608.0);
    return hipGetLastError();
}

}  // namespace sq
