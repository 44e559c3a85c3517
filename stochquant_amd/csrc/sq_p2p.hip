// sq_p2p.hip -- the reduction half of the peer-pointer transport's
// collectives (SQ_COMM_P2P): every rank has copied its
// contribution into slot r of each rank's gather buffer; this kernel folds the
// nranks slots of the local buffer in rank order, so every rank computes the
// same result bit for bit (the sums included) without RCCL.
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

}  // namespace

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
