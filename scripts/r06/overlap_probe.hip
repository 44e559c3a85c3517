// Do two kernels launched back to back on one HIP stream overlap on gfx950?
// Kernel A: 512 blocks of 640 threads; block b busy-waits (2 + b % 5) us on
// the 100 MHz constant clock, then thread 0 stores its end stamp.  Kernel B:
// the same grid; thread 0 stores its start stamp.  If B's earliest start
// precedes A's latest end, the second launch's blocks ran while the first's
// were still running.  Also: A then B with B reading a value every A block
// wrote (a counter A's blocks increment last), to see whether B ever saw an
// unfinished A.  Prints the overlap in us for 20 trials of each.
//   hipcc --offload-arch=gfx950 -O2 -o overlap_probe overlap_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(640) void ka(unsigned long long *end, unsigned int *ctr, int spin_base) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long wait = (unsigned long long)(spin_base + (blockIdx.x % 5)) * 100ull;  // 100 MHz ticks
    while (__builtin_amdgcn_s_memrealtime() - t0 < wait) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        end[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ __launch_bounds__(640) void kb(unsigned long long *start, const unsigned int *ctr, unsigned int *seen) {
    if (threadIdx.x == 0) {
        start[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        seen[blockIdx.x] = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main() {
    const int nb = 512;
    unsigned long long *end, *start;
    unsigned int *ctr, *seen;
    hipMalloc(&end, nb * 8);
    hipMalloc(&start, nb * 8);
    hipMalloc(&ctr, 4);
    hipMalloc(&seen, nb * 4);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<unsigned long long> he(nb), hs(nb);
    std::vector<unsigned int> hseen(nb);
    int early = 0;
    for (int t = 0; t < 20; ++t) {
        hipMemsetAsync(ctr, 0, 4, s);
        for (int w = 0; w < 8; ++w) hipLaunchKernelGGL(ka, dim3(nb), dim3(640), 0, s, end, ctr, 25);  // queue depth
        hipMemsetAsync(ctr, 0, 4, s);
        hipLaunchKernelGGL(ka, dim3(nb), dim3(640), 0, s, end, ctr, 25);
        hipLaunchKernelGGL(kb, dim3(nb), dim3(640), 0, s, start, ctr, seen);
        hipStreamSynchronize(s);
        hipMemcpy(he.data(), end, nb * 8, hipMemcpyDeviceToHost);
        hipMemcpy(hs.data(), start, nb * 8, hipMemcpyDeviceToHost);
        hipMemcpy(hseen.data(), seen, nb * 4, hipMemcpyDeviceToHost);
        const unsigned long long last_end = *std::max_element(he.begin(), he.end());
        const unsigned long long first_start = *std::min_element(hs.begin(), hs.end());
        const unsigned int min_seen = *std::min_element(hseen.begin(), hseen.end());
        if (min_seen < (unsigned)nb) ++early;
        printf("trial %2d: B first start - A last end = %+8.2f us; min A blocks seen done by a B block: %u / %d\n", t,
               ((double)first_start - (double)last_end) / 100.0, min_seen, nb);
    }
    printf("trials where a B block saw an unfinished A: %d / 20\n", early);
    return 0;
}
