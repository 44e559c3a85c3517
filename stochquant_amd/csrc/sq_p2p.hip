// sq_p2p.hip -- device halves of the peer-pointer transport (SQ_COMM_P2P,
// DESIGN.md §8): the collectives' fold (every rank has copied its
// contribution into slot r of each rank's gather buffer; the kernel folds the
// nranks slots of the local buffer in rank order, so every rank computes the
// same result bit for bit, the sums included, without RCCL) and the
// exchange's two-range copies.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sq_internal.h"

namespace sq {
namespace {

template <typename T, bool SUM>
__global__ void __launch_bounds__(256) p2p_fold_kernel(const unsigned char *__restrict__ slots, int nranks,
                                                       size_t cap, T *__restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T acc = reinterpret_cast<const T *>(slots)[i];
        for (int q = 1; q < nranks; ++q) {
            const T v = reinterpret_cast<const T *>(slots + (size_t)q * cap)[i];
            if constexpr (SUM)
                acc = acc + v;
            else
                acc = v > acc ? v : acc;
        }
        out[i] = acc;
    }
}

template <typename T, bool SUM>
hipError_t fold(const unsigned char *slots, int nranks, size_t cap, void *out, size_t n, hipStream_t s) {
    const int blocks = (int)std::min<size_t>(1024, (n + 255) / 256);
    p2p_fold_kernel<T, SUM><<<blocks, 256, 0, s>>>(slots, nranks, cap, static_cast<T *>(out), n);
    return hipGetLastError();
}

// Two equal ranges copied by one launch: the exchange's staged copy of both
// edge ranges, and its pull of both neighbours' staged planes (either range
// may be peer memory mapped through IPC).  One kernel instead of two blit
// copies: on this stack every copy and every stream-ordered flag is a launch
// of 4-6 us on the exchange stream.
template <bool V4>
__global__ void __launch_bounds__(256) p2p_copy2_kernel(float *__restrict__ d0, const float *__restrict__ s0,
                                                        float *__restrict__ d1, const float *__restrict__ s1,
                                                        size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    if constexpr (V4) {
        const size_t n4 = n / 4;
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n4; i += stride) {
            const bool hi = i >= n4;
            const size_t k = hi ? i - n4 : i;
            const float4 v = reinterpret_cast<const float4 *>(hi ? s1 : s0)[k];
            reinterpret_cast<float4 *>(hi ? d1 : d0)[k] = v;
        }
    } else {
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n; i += stride) {
            const bool hi = i >= n;
            const size_t k = hi ? i - n : i;
            (hi ? d1 : d0)[k] = (hi ? s1 : s0)[k];
        }
    }
}

// The exchange's hand-shake in one launch of one wave (it replaces two
// stream-ordered flag writes and two waits, each a 4-6 us launch of its own on
// this stack): release the staged copy the launch before wrote (system scope:
// the neighbours may be other GPUs), tell both neighbours exchange e is
// staged, and wait until both have told us the same.  Sequence numbers only
// grow.  Bounded: after `polls` polls the wave gives up and sets bit 1 of
// *err (the host reports it, sticky, as a failed exchange) -- the pull that
// follows then copies whatever is there, and the field is void.
__global__ void __launch_bounds__(64) p2p_handshake_kernel(unsigned int *up_from_dn, unsigned int *dn_from_up,
                                                          const unsigned int *from_dn, const unsigned int *from_up,
                                                          unsigned int e, unsigned int polls, int *err,
                                                          const unsigned int *pre, unsigned int pre_n) {
    if (threadIdx.x != 0) return;
    // pre: the staging slot is written by the block's last pair on the
    // interior stream (phi4_tb2_stage_kernel, write-through stores drained
    // before each block's count): wait until all its blocks have counted
    if (pre != nullptr) {
        for (unsigned int k = 0;; ++k) {
            if ((int)(__hip_atomic_load(pre, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - pre_n) >= 0) break;
            if (k >= polls) {
                if (err) __hip_atomic_fetch_or(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __threadfence_system();
    __hip_atomic_store(up_from_dn, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dn_from_up, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (unsigned int k = 0;; ++k) {
        const unsigned int a = __hip_atomic_load(from_dn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned int b = __hip_atomic_load(from_up, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a >= e && b >= e) break;
        if (k >= polls) {
            if (err) __hip_atomic_fetch_or(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

}  // namespace

hipError_t p2p_handshake_launch(unsigned int *up_from_dn, unsigned int *dn_from_up, const unsigned int *from_dn,
                                const unsigned int *from_up, unsigned int e, unsigned int polls, int *err,
                                hipStream_t s, const unsigned int *pre, unsigned int pre_n) {
    p2p_handshake_kernel<<<1, 64, 0, s>>>(up_from_dn, dn_from_up, from_dn, from_up, e, polls, err, pre, pre_n);
    return hipGetLastError();
}

hipError_t p2p_copy2_launch(float *d0, const float *s0, float *d1, const float *s1, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const bool v4 = n % 4 == 0 && ((reinterpret_cast<uintptr_t>(d0) | reinterpret_cast<uintptr_t>(s0) |
                                    reinterpret_cast<uintptr_t>(d1) | reinterpret_cast<uintptr_t>(s1)) & 15) == 0;
    const size_t items = v4 ? n / 2 : 2 * n;  // float4s or floats over both ranges
    const unsigned blocks = (unsigned)std::min<size_t>(1024, (items + 255) / 256);
    if (v4)
        p2p_copy2_kernel<true><<<blocks, 256, 0, s>>>(d0, s0, d1, s1, n);
    else
        p2p_copy2_kernel<false><<<blocks, 256, 0, s>>>(d0, s0, d1, s1, n);
    return hipGetLastError();
}

hipError_t p2p_fold_launch(const unsigned char *slots, int nranks, size_t cap, void *out, size_t n, P2pRed red,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    switch (red) {
    case P2pRed::kMaxU32: return fold<unsigned int, false>(slots, nranks, cap, out, n, s);
    case P2pRed::kMaxI32: return fold<int, false>(slots, nranks, cap, out, n, s);
    case P2pRed::kMaxU64: return fold<unsigned long long, false>(slots, nranks, cap, out, n, s);
    case P2pRed::kMaxF64: return fold<double, false>(slots, nranks, cap, out, n, s);
    case P2pRed::kSumF64: return fold<double, true>(slots, nranks, cap, out, n, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace sq
