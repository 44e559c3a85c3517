// Probe: which operand order of v_med3_f32 implements the reference's guard
// (tau_kernel.cl:119-133: > c -> c, < -c -> -c, NaN -> +c) on gfx950?
// Compared bitwise with fmaxf(fminf(v, c), -c), the product's two-instruction form.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
__global__ void k(const float *in, float *out, float c, int n) {
    int i = threadIdx.x;
    if (i < n) {
        float v = in[i];
        out[7 * i + 0] = fmaxf(fminf(v, c), -c);
        out[7 * i + 1] = __builtin_amdgcn_fmed3f(v, -c, c);
        out[7 * i + 2] = __builtin_amdgcn_fmed3f(v, c, -c);
        out[7 * i + 3] = __builtin_amdgcn_fmed3f(-c, v, c);
        out[7 * i + 4] = __builtin_amdgcn_fmed3f(c, v, -c);
        out[7 * i + 5] = __builtin_amdgcn_fmed3f(-c, c, v);
        out[7 * i + 6] = __builtin_amdgcn_fmed3f(c, -c, v);
    }
}
int main() {
    const float c = 1000.f;
    float h[8] = {NAN, -NAN, INFINITY, -INFINITY, 5e3f, -5e3f, 3.5f, -0.0f};
    float *d, *o, r[56];
    if (hipMalloc(&d, sizeof h) || hipMalloc(&o, sizeof r)) return 1;
    if (hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice)) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, c, 8);
    if (hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost)) return 1;
    int ok[7] = {1, 1, 1, 1, 1, 1, 1};
    for (int i = 0; i < 8; ++i) {
        printf("in %-6g minmax %-6g med3 orders:", h[i], r[7 * i]);
        for (int j = 1; j < 7; ++j) {
            printf(" %-6g", r[7 * i + j]);
            ok[j] &= memcmp(&r[7 * i + j], &r[7 * i], 4) == 0;
        }
        printf("\n");
    }
    const char *nm[7] = {"", "(v,-c,c)", "(v,c,-c)", "(-c,v,c)", "(c,v,-c)", "(-c,c,v)", "(c,-c,v)"};
    for (int j = 1; j < 7; ++j) printf("%s %s\n", nm[j], ok[j] ? "IDENTICAL" : "different");
    return 0;
}
