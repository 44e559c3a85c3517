// Microbenchmark: issue cost of the VALU instructions the phi^4 step uses,
// relative to v_add_f32 (8 independent chains per lane, 8 waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 256;

#define BODY8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

__global__ void k_add(float *o, float s) {
    float a[8]; for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_fma(float *o, float s) {
    float a[8]; for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_pkfma(float *o, float s) {
    f2 a[8]; f2 b = {s, s};
    for (int i = 0; i < 8; ++i) a[i] = f2{(float)threadIdx.x, (float)i};
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i].x + a[i].y; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_pkadd(float *o, float s) {
    f2 a[8]; f2 b = {s, s};
    for (int i = 0; i < 8; ++i) a[i] = f2{(float)threadIdx.x, (float)i};
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i].x + a[i].y; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_mad64(float *o, float s) {
    uint64_t a[8]; uint32_t m = __float_as_uint(s) | 1u;
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) { uint64_t c; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(a[i]), "=s"(c) : "v"((uint32_t)a[i]), "v"(m)); }
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += (float)a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_mulhi(float *o, float s) {
    uint32_t a[8]; uint32_t m = __float_as_uint(s) | 1u;
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += (float)a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_mulu24(float *o, float s) {
    uint32_t a[8]; uint32_t m = __float_as_uint(s) | 1u;
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(m));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += (float)a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_bitop3(float *o, float s) {
    uint32_t a[8]; uint32_t m = __float_as_uint(s) | 1u;
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[i]) : "v"(m));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += (float)a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_log(float *o, float s) {
    float a[8]; for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i + 2.f;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_log_f32 %0, %0" : "+v"(a[i]));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_med3(float *o, float s) {
    float a[8]; for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_med3_f32 %0, %0, %1, -%1" : "+v"(a[i]) : "v"(s));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
__global__ void k_dpp(float *o, float s) {
    float a[8]; for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#define S(i) asm volatile("v_mov_b32_dpp %0, %0 wave_ror:1 row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
            BODY8(S)
#undef S
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i]; o[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

// NaN semantics of v_med3_f32(x, c, -c) and of the min/max pair
__global__ void k_nan(float *o, float c) {
    const float x[4] = {__int_as_float(0x7fc00000), 5e3f, -5e3f, 0.5f};
    for (int i = 0; i < 4; ++i) {
        float r;
        asm volatile("v_med3_f32 %0, %1, %2, -%2" : "=v"(r) : "v"(x[i]), "v"(c));
        o[i] = r;
        o[4 + i] = fmaxf(fminf(x[i], c), -c);
    }
}

typedef void (*kfn)(float *, float);
int main() {
    float *o;
    hipMalloc(&o, 2048 * 256 * sizeof(float));
    struct { const char *n; kfn f; } ks[] = {{"v_add_f32", k_add}, {"v_fma_f32", k_fma}, {"v_pk_fma_f32", k_pkfma},
        {"v_pk_add_f32", k_pkadd}, {"v_mad_u64_u32", k_mad64}, {"v_mul_hi_u32", k_mulhi},
        {"v_mul_u32_u24", k_mulu24}, {"v_bitop3_b32", k_bitop3}, {"v_log_f32", k_log},
        {"v_med3_f32", k_med3}, {"v_mov_b32_dpp", k_dpp}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    double base = 0;
    for (auto &k : ks) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            k.f<<<2048, 256>>>(o, 1.0001f);
            hipEventRecord(b);
            hipEventSynchronize(b);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double ins = 2048.0 * 4 * ITER * 16 * 8;  // wave-instructions
        const double per_simd_ns = ins / 1024 / (ms * 1e6);
        if (base == 0) base = per_simd_ns;
        printf("%-16s %8.3f ms  %.3f wave-instr/ns/SIMD  cost %.2f x v_add_f32\n", k.n, ms, per_simd_ns, base / per_simd_ns);
    }
    k_nan<<<1, 1>>>(o, 1000.f);
    float h[8];
    hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
    printf("med3(NaN,5e3,-5e3,0.5) = %g %g %g %g ; minmax = %g %g %g %g\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    return 0;
}
