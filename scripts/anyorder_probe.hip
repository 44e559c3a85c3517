// Does hipExtAnyOrderLaunch let a kernel start before the previous kernel on
// the same stream has finished (gfx950)?  Kernel A: `nb` blocks, block b spins
// for (b % 4 + 1) * spin_us on the 100 MHz constant clock, recording its start
// and end; kernel B: `nb` blocks recording their start.  Printed: A's last
// end, B's first start (constant-clock ticks, 10 ns) for an ordinary launch of
// B and for B launched with hipExtAnyOrderLaunch.
//   hipcc --offload-arch=gfx950 -O2 scripts/anyorder_probe.hip -o scripts/bin/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ void spin_kernel(unsigned long long *t, unsigned long long spin_ticks) {
    __shared__ unsigned long long t0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long stop = t0 + spin_ticks * (blockIdx.x % 4 + 1);
        while (__builtin_amdgcn_s_memrealtime() < stop) __builtin_amdgcn_s_sleep(2);
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ void stamp_kernel(unsigned long long *t) {
    if (threadIdx.x == 0) t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

int main(int argc, char **argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 512;
    unsigned long long spin = argc > 2 ? strtoull(argv[2], nullptr, 10) : 2000;  // 20 us
    unsigned long long *ta, *tb;
    CK(hipMalloc(&ta, 2 * sizeof(unsigned long long) * nb));
    CK(hipMalloc(&tb, sizeof(unsigned long long) * nb));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<unsigned long long> ha(2 * nb), hb(nb);
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            void *aa[] = {&ta, &spin};
            void *ab[] = {&tb};
            CK(hipExtLaunchKernel((const void *)spin_kernel, dim3(nb), dim3(640), aa, 0, s, nullptr, nullptr, 0));
            CK(hipExtLaunchKernel((const void *)stamp_kernel, dim3(nb), dim3(640), ab, 0, s, nullptr, nullptr,
                                  mode ? hipExtAnyOrderLaunch : 0));
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(ha.data(), ta, ha.size() * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hb.data(), tb, hb.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long a0 = ~0ull, a1 = 0, b0 = ~0ull, b1 = 0;
            for (int b = 0; b < nb; ++b) {
                a0 = std::min(a0, ha[2 * b]);
                a1 = std::max(a1, ha[2 * b + 1]);
                b0 = std::min(b0, hb[b]);
                b1 = std::max(b1, hb[b]);
            }
            int early = 0;
            for (int b = 0; b < nb; ++b) early += hb[b] < a1;
            printf("%s rep %d: A span %.2f us, B first start - A last end %.2f us, B blocks started before A ended: %d/%d\n",
                   mode ? "any-order" : "ordinary ", rep, (a1 - a0) * 1e-2, ((double)b0 - (double)a1) * 1e-2, early,
                   nb);
        }
    }
    return 0;
}
