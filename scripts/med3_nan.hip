// Probe: does v_med3_f32(v, -c, c) implement the reference's guard
// (tau_kernel.cl:119-133: > c -> c, < -c -> -c, NaN -> c) on gfx950?
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
__global__ void k(const float *in, float *out, float c, int n) {
    int i = threadIdx.x;
    if (i < n) {
        float v = in[i];
        out[2 * i] = __builtin_amdgcn_fmed3f(v, -c, c);
        out[2 * i + 1] = fmaxf(fminf(v, c), -c);
    }
}
int main() {
    const float c = 1000.f;
    float h[8] = {NAN, -NAN, INFINITY, -INFINITY, 5e3f, -5e3f, 3.5f, -0.0f};
    float *d, *o, r[16];
    hipMalloc(&d, sizeof h);
    hipMalloc(&o, sizeof r);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, c, 8);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int i = 0; i < 8; ++i) {
        printf("in %-10g med3 %-10g minmax %-10g\n", h[i], r[2 * i], r[2 * i + 1]);
        unsigned a, b;
        memcpy(&a, &r[2 * i], 4);
        memcpy(&b, &r[2 * i + 1], 4);
        ok &= a == b;
    }
    printf(ok ? "IDENTICAL\n" : "DIFFERENT\n");
    return 0;
}
