// sq_phi4.hip -- 3-D phi^4 Langevin step on gfx950 (the north-star hot path).
//
// Per-site update (the reference's tau_kernel.cl:111-117 + guard :119-133,
// generalised to a periodic 3-D lattice with the non-linear phi^4 force):
//   nb    = ((phi[x-1]+phi[x+1]) + (phi[y-1]+phi[y+1])) + (phi[z-1]+phi[z+1])
//   drift = fma(-phi, fma(lam/6, phi*phi, m2), fma(-6, phi, nb))
//   phi'  = guard(fma(sigma, xi, fma(dtau, drift, phi)))
// Memory-bound: 8 algorithmic bytes per site update (read phi, write phi').
//
// Mapping: a wave owns an x-segment of 4*QX sites (each
// lane a float4 = 16-B coalesced access) by R consecutive y-rows per lane and
// marches along z over a chunk of planes, holding planes z-1, z, z+1 in a
// register queue.  x-neighbours come from the adjacent lane (DPP wave_ror /
// wave_rol when a wave spans 256 sites, ds_bpermute for narrower rows),
// interior y-neighbours from the lane's own registers, the two y-halo rows of
// plane z+1 are prefetched one plane ahead.  No LDS, no barriers: the waves of
// a block are independent, so a block's 4 waves take 4 y-adjacent units and
// consecutive logical blocks are dealt to one XCD (T1 swizzle) so that the
// halo rows and chunk-boundary planes they share hit that XCD's L2.
#include "sq_internal.h"
#include "sq_rng.h"

namespace sq {

namespace {

__device__ __forceinline__ float from_left_lane(float v) {  // lane i <- lane i-1 (mod 64)
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x13C, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_right_lane(float v) {  // lane i <- lane i+1 (mod 64)
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x134, 0xF, 0xF, false));
}

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

__device__ __forceinline__ const float *plane_ptr(const Phi4StepArgs &A, int zl, size_t plane) {
    int p = zl + 1;  // padded index
    if (A.periodic) {
        if (zl < 0) p = A.nz;
        else if (zl >= A.nz) p = 1;
    }
    return A.in + (size_t)p * plane;
}

__device__ __forceinline__ float site_update(float phi, float xm, float xp, float ym, float yp,
                                             float zm, float zp, float xi, const Phi4StepArgs &A,
                                             int &bad) {
    const float nb = ((xm + xp) + (ym + yp)) + (zm + zp);
    const float lap = __builtin_fmaf(-6.0f, phi, nb);
    const float g = __builtin_fmaf(A.lam6, phi * phi, A.m2);
    const float drift = __builtin_fmaf(-phi, g, lap);
    const float v = __builtin_fmaf(A.sig, xi, __builtin_fmaf(A.h, drift, phi));
    const bool out = !(__builtin_fabsf(v) <= A.clampv);  // > clamp or NaN
    bad |= (int)out;
    const float gv = v < 0.0f ? -A.clampv : A.clampv;
    return out ? gv : v;
}

template <int QX, int R>
__global__ __launch_bounds__(256) void phi4_step_kernel(const Phi4StepArgs A) {
    constexpr int RS = 64 / QX;  // row sets per wave
    const int lane = threadIdx.x & 63;
    const int nb = gridDim.x, b = blockIdx.x;
    const int lb = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;
    const int unit = lb * 4 + (int)(threadIdx.x >> 6);
    if (unit >= A.nunits) return;
    const int yg = unit % A.nyg;
    const int rest = unit / A.nyg;
    const int xs = rest % A.nxseg;
    const int zk = rest / A.nxseg;
    const int zbeg = A.zlo + zk * A.zstep;
    const int zend = min(zbeg + A.zc, A.zhi);

    const int Lx = A.Lx, Ly = A.Ly;
    const size_t plane = (size_t)Lx * (size_t)Ly;
    const int xq = lane & (QX - 1);
    const int rsid = lane / QX;
    const int x = xs * (4 * QX) + 4 * xq;
    // lanes whose rows fall past Ly (narrow lattices: a wave covers more rows
    // than Ly has) read row 0 and store nothing; shuffles stay inside their
    // x-segment group, which is idle as a whole.
    const int y0r = yg * (RS * R) + rsid * R;
    const bool rows_ok = y0r < Ly;
    const int y0 = rows_ok ? y0r : 0;
    const int ym = y0 == 0 ? Ly - 1 : y0 - 1;
    const int yp = (y0 + R == Ly) ? 0 : y0 + R;
    const bool multiseg = A.nxseg > 1;  // only for QX == 64
    const int xl = (x == 0 ? Lx : x) - 1;
    const int xr = (x + 4 == Lx) ? 0 : x + 4;
    const int seg_base = lane & ~(QX - 1);
    const int src_l = seg_base | ((xq + QX - 1) & (QX - 1));
    const int src_r = seg_base | ((xq + 1) & (QX - 1));

    float4 pv[R], cv[R], nv[R];
    float4 hm, hp, hm_n = make_float4(0, 0, 0, 0), hp_n = make_float4(0, 0, 0, 0);
    {
        const float *P = plane_ptr(A, zbeg - 1, plane);
        const float *C = plane_ptr(A, zbeg, plane);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            pv[r] = ld4(P + (size_t)(y0 + r) * Lx + x);
            cv[r] = ld4(C + (size_t)(y0 + r) * Lx + x);
        }
        hm = ld4(C + (size_t)ym * Lx + x);
        hp = ld4(C + (size_t)yp * Lx + x);
    }
    const uint64_t qplane = (uint64_t)(plane >> 2);
    int bad = 0;
    for (int z = zbeg; z < zend; ++z) {
        const float *Np = plane_ptr(A, z + 1, plane);
        const float *Cp = plane_ptr(A, z, plane);
#pragma unroll
        for (int r = 0; r < R; ++r) nv[r] = ld4(Np + (size_t)(y0 + r) * Lx + x);
        const bool more = z + 1 < zend;
        if (more) {
            hm_n = ld4(Np + (size_t)ym * Lx + x);
            hp_n = ld4(Np + (size_t)yp * Lx + x);
        }
        float el[R], er[R];
        if (multiseg) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                el[r] = 0.f;
                er[r] = 0.f;
                if (lane == 0) el[r] = Cp[(size_t)(y0 + r) * Lx + xl];
                if (lane == 63) er[r] = Cp[(size_t)(y0 + r) * Lx + xr];
            }
        }
        // noise for the R float4s of plane z (independent of the loads above)
        const uint64_t pq = (uint64_t)(A.zg0 + z) * qplane;
        f32x4n xi[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t off = (uint32_t)(((size_t)(y0 + r) * Lx + x) >> 2);
            xi[r] = normals4(pq + off, kStreamField, A.s_lo, A.s_hi, A.k0, A.k1);
        }
        float *O = A.out + (size_t)(z + 1) * plane;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float4 c = cv[r];
            const float4 up = r > 0 ? cv[r > 0 ? r - 1 : 0] : hm;
            const float4 dn = r < R - 1 ? cv[r < R - 1 ? r + 1 : 0] : hp;
            float lft, rgt;
            if constexpr (QX == 64) {
                lft = from_left_lane(c.w);
                rgt = from_right_lane(c.x);
            } else {
                lft = __shfl(c.w, src_l, 64);
                rgt = __shfl(c.x, src_r, 64);
            }
            if (multiseg) {
                if (lane == 0) lft = el[r];
                if (lane == 63) rgt = er[r];
            }
            float4 o;
            o.x = site_update(c.x, lft, c.y, up.x, dn.x, pv[r].x, nv[r].x, xi[r].a, A, bad);
            o.y = site_update(c.y, c.x, c.z, up.y, dn.y, pv[r].y, nv[r].y, xi[r].b, A, bad);
            o.z = site_update(c.z, c.y, c.w, up.z, dn.z, pv[r].z, nv[r].z, xi[r].c, A, bad);
            o.w = site_update(c.w, c.z, rgt, up.w, dn.w, pv[r].w, nv[r].w, xi[r].d, A, bad);
            if (rows_ok) st4(O + (size_t)(y0 + r) * Lx + x, o);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            pv[r] = cv[r];
            cv[r] = nv[r];
        }
        hm = hm_n;
        hp = hp_n;
    }
    if (!rows_ok) bad = 0;
    if (A.flag != nullptr) {
        if (__ballot(bad) != 0ull && lane == 0) atomicOr(A.flag, 1);
    }
}

__global__ __launch_bounds__(256) void phi4_init_kernel(float *slab, int Lx, int Ly, int nz,
                                                        long long zg0, uint32_t k0, uint32_t k1,
                                                        float amp) {
    const size_t plane = (size_t)Lx * Ly;
    const size_t nq = (size_t)nz * plane / 4;
    const uint64_t q0 = (uint64_t)zg0 * (uint64_t)(plane >> 2);
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq;
         q += (size_t)gridDim.x * blockDim.x) {
        const f32x4n n = normals4(q0 + q, kStreamInit, 0u, 0u, k0, k1);
        st4(slab + plane + 4 * q, make_float4(amp * n.a, amp * n.b, amp * n.c, amp * n.d));
    }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ __launch_bounds__(256) void phi4_moments_kernel(const float *p, long long n4,
                                                           double *acc, unsigned int *acc_max) {
    double s1 = 0, s2 = 0;
    float mx = 0;
    const float4 *q = reinterpret_cast<const float4 *>(p);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
        const float4 v = q[i];
        s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    __shared__ double sh1[4], sh2[4];
    __shared__ float shm[4];
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    mx = wave_max(mx);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh1[w] = s1;
        sh2[w] = s2;
        shm[w] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t1 = 0, t2 = 0;
        float tm = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
            t1 += sh1[k];
            t2 += sh2[k];
            tm = fmaxf(tm, shm[k]);
        }
        atomicAdd(&acc[0], t1);
        atomicAdd(&acc[1], t2);
        atomicMax(acc_max, __float_as_uint(tm));
    }
}

__global__ __launch_bounds__(256) void phi4_slices_kernel(const float *slab, long long plane4,
                                                          double *out) {
    const float4 *q = reinterpret_cast<const float4 *>(slab) + (size_t)(blockIdx.x + 1) * plane4;
    double s = 0;
    for (long long i = threadIdx.x; i < plane4; i += blockDim.x) {
        const float4 v = q[i];
        s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
    }
    __shared__ double sh[4];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

}  // namespace

bool phi4_geometry(int Lx, int Ly, Phi4Geom *g) {
    if (Lx <= 0 || Ly <= 0 || (Lx & 3)) return false;
    int qx;
    if (Lx % 256 == 0) qx = 64;
    else if (Lx < 256 && Lx >= 8 && 64 % (Lx / 4) == 0) qx = Lx / 4;
    else return false;
    const int rs = 64 / qx;
    static const int rcand[3] = {4, 2, 1};
    for (int r : rcand) {  // a full wave tile that divides Ly
        if (Ly % (rs * r) == 0) {
            *g = Phi4Geom{qx, r, rs * r};
            return true;
        }
    }
    for (int r : rcand) {  // otherwise a partial last tile (rows past Ly idle)
        if (Ly % r == 0) {
            *g = Phi4Geom{qx, r, rs * r};
            return true;
        }
    }
    return false;
}

void phi4_fill_units(Phi4StepArgs &a, const Phi4Geom &g) {
    a.nxseg = a.Lx / (4 * g.qx);
    a.nyg = (a.Ly + g.wy - 1) / g.wy;
    a.nunits = a.nxseg * a.nyg * a.nzc;
}

template <int QX>
static hipError_t launch_qx(const Phi4StepArgs &a, int r, dim3 grid, hipStream_t s) {
    switch (r) {
    case 4: hipLaunchKernelGGL((phi4_step_kernel<QX, 4>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((phi4_step_kernel<QX, 2>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((phi4_step_kernel<QX, 1>), grid, dim3(256), 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t phi4_step_launch(const Phi4StepArgs &a, const Phi4Geom &g, hipStream_t s) {
    if (a.nunits <= 0) return hipSuccess;
    const dim3 grid((unsigned)((a.nunits + 3) / 4));
    switch (g.qx) {
    case 64: return launch_qx<64>(a, g.r, grid, s);
    case 32: return launch_qx<32>(a, g.r, grid, s);
    case 16: return launch_qx<16>(a, g.r, grid, s);
    case 8: return launch_qx<8>(a, g.r, grid, s);
    case 4: return launch_qx<4>(a, g.r, grid, s);
    case 2: return launch_qx<2>(a, g.r, grid, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t phi4_init_launch(float *slab, int Lx, int Ly, int nz, long long zg0, uint32_t k0,
                            uint32_t k1, float amp, hipStream_t s) {
    const size_t nq = (size_t)nz * Lx * Ly / 4;
    const unsigned grid = (unsigned)std::min<size_t>((nq + 255) / 256, 8192);
    hipLaunchKernelGGL(phi4_init_kernel, dim3(grid), dim3(256), 0, s, slab, Lx, Ly, nz, zg0, k0, k1,
                       amp);
    return hipGetLastError();
}

hipError_t phi4_moments_launch(const float *slab, long long n, double *acc, unsigned int *acc_max,
                               hipStream_t s) {
    const long long n4 = n / 4;
    const unsigned grid = (unsigned)std::min<long long>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(phi4_moments_kernel, dim3(grid), dim3(256), 0, s, slab, n4, acc, acc_max);
    return hipGetLastError();
}

hipError_t phi4_slices_launch(const float *slab, int Lx, int Ly, int nz, double *out,
                              hipStream_t s) {
    hipLaunchKernelGGL(phi4_slices_kernel, dim3((unsigned)nz), dim3(256), 0, s, slab,
                       (long long)Lx * Ly / 4, out);
    return hipGetLastError();
}

}  // namespace sq
