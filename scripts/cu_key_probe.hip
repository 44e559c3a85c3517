// Probe: do the two 10-wave blocks a CU holds read the same hardware ids?
// 512 blocks x 640 threads, 60 KB of LDS each (two blocks per CU, as the fused
// phi^4 kernel), each block spins ~50 us so all are resident together; block b
// stores HW_REG_HW_ID and HW_REG_XCC_ID of its wave 0 and its start clock.
//   hipcc --offload-arch=gfx950 -O2 scripts/cu_key_probe.hip -o scripts/bin/cu_key_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(640) void probe(unsigned *out, int spin) {
    __shared__ float lds[15360];
    lds[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x] = hw;
        out[3 * blockIdx.x + 1] = xcc;
        out[3 * blockIdx.x + 2] = (unsigned)t0;
    }
    if (lds[(threadIdx.x * 7) % 15360] < -1.f) out[0] = 0;
}

int main() {
    const int nb = 512;
    unsigned *d;
    if (hipMalloc(&d, 3 * nb * sizeof(unsigned)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(nb), dim3(640), 0, 0, d, 5000);  // 50 us at 100 MHz
    std::vector<unsigned> h(3 * nb);
    if (hipMemcpy(h.data(), d, 3 * nb * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::map<unsigned, std::vector<int>> byk;
    for (int b = 0; b < nb; ++b) {
        const unsigned hw = h[3 * b], xcc = h[3 * b + 1];
        const unsigned key = ((xcc & 7u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
        byk[key].push_back(b);
    }
    std::map<size_t, int> hist;
    for (auto &kv : byk) hist[kv.second.size()]++;
    printf("distinct keys %zu;", byk.size());
    for (auto &kv : hist) printf(" %d keys with %zu blocks;", kv.second, kv.first);
    printf("\n");
    int shown = 0;
    for (auto &kv : byk) {
        if (shown++ >= 8) break;
        printf("key %4u:", kv.first);
        for (int b : kv.second) printf(" b%d(hw %08x xcc %u)", b, h[3 * b], h[3 * b + 1]);
        printf("\n");
    }
    unsigned smin = ~0u, smax = 0;
    for (int b = 0; b < nb; ++b) { smin = std::min(smin, h[3 * b + 2]); smax = std::max(smax, h[3 * b + 2]); }
    printf("start spread %.2f us\n", (smax - smin) * 0.01);
    return 0;
}
