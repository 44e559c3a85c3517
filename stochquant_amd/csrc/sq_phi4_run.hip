// sq_phi4_run.hip -- the two-step march as ONE resident launch per sq_step call.
//
// phi4_tb2_kernel (sq_phi4.hip) runs one pair of steps per launch.  Launches on
// one stream do not overlap on this stack: the next launch's first block starts
// ~2.5 us after the previous launch's last block ends
// (profiles/r06/c10/overlap_probe.log), and each launch has its ramp and tail
// (busy fraction 0.92), together ~5 us of every ~34 us pair at 256^3
// (DESIGN.md §10).  Here the grid stays resident for all the call's pairs and
// a block starts pair t+1 as soon as the 3 x 3 neighbourhood of blocks around
// it (y-bands x z-chunks, periodic in both) has finished pair t: those blocks
// wrote every input site it reads (rows y0-2 .. y0+9, planes z0-2 .. z1+1, the
// two-step light cone) and have finished reading every site it overwrites
// (the buffers alternate, so pair t+1 writes the buffer pair t read).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility;
// cdna_hip_programming.md Guideline 16, form R1): the outputs are write-through
// stores (sc0 sc1, tb_plane's bstore4<17>), every wave of the block drains them
// (s_waitcnt vmcnt(0)), one block barrier, then one lane stores the block's
// epoch with an agent-scope relaxed store.  A waiting block's lane 0 polls its
// 8 neighbours' epochs with agent-scope relaxed loads; then either (LAUX = 0)
// one agent-scope acquire (this CU's L1 may hold lines of the buffer from two
// pairs ago) and a block barrier before the plain loads of the pair, or
// (LAUX = 16) no acquire, every load of the march being an sc1 load, which
// bypasses L1.  Every wait is bounded (kRunSpinMax polls); a block that gives
// up sets bit 2 of *err and stops, and every other block's wait ends at its
// next poll when it sees *err, so the grid always drains; the host reports the
// error and the field is then corrupt (sq_api.cpp, gate_check).
//
// The site arithmetic is tb_plane's, so a call of n pairs is bit-identical to
// n phi4_tb2_kernel launches (tests/test_gpu_phi4.py, test_run_kernel_*).
#define SQ_PHI4_KERNELS_ONLY
#include "sq_phi4.hip"

namespace sq {

namespace {

constexpr unsigned int kRunSpinMax = 1u << 20;  // ~1 s of polls under load
constexpr int kRunErrBit = 4;                   // *err: a march wait gave up

// Lane 0 of the block: wait until the 8 blocks around logical block lb (the
// 3 x 3 neighbourhood of y-bands x z-chunks, periodic) have published `need`.
__device__ __forceinline__ bool run_wait(const Tb2RunArgs &R, int lb, int nyg, int nzc, unsigned int need) {
    int nbr[8];
    {
        const int yb = lb % nyg, zk = lb / nyg;
        int k = 0;
#pragma unroll
        for (int dz = -1; dz <= 1; ++dz)
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy) {
                if (dz == 0 && dy == 0) continue;
                const int zz = zk + dz < 0 ? zk + dz + nzc : (zk + dz >= nzc ? zk + dz - nzc : zk + dz);
                const int yy = yb + dy < 0 ? yb + dy + nyg : (yb + dy >= nyg ? yb + dy - nyg : yb + dy);
                nbr[k++] = zz * nyg + yy;
            }
    }
    for (unsigned int n = 0;; ++n) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            ok &= (int)(__hip_atomic_load(R.flags + nbr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - need) >= 0;
        if (ok) return true;
        if (n >= kRunSpinMax || __hip_atomic_load(R.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            __hip_atomic_fetch_or(R.err, kRunErrBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// phi4_tb2_kernel<NZ, false, 1, false, true, false> with the pairs looped
// inside: 256-site rows, whole-buffer descriptors, no frame records.
template <bool NZ, int LAUX>
__global__ __launch_bounds__(kTbWaves * 64) __attribute__((amdgpu_waves_per_eu(1)))
void phi4_tb2_run_kernel(const Phi4StepArgs A0, const Tb2RunArgs R0) {
    Phi4StepArgs A = A0;
    const int nb = gridDim.x, b = blockIdx.x;
    const TbBlock tbk = tb_block<false>(A, b, nb);
    const int lb = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;  // tb_block's logical block
    const int Lx = A.Lx, Ly = A.Ly;
    TbCtx K;
    K.w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    K.lane = threadIdx.x & 63;
    K.outw = K.w >= 1 && K.w <= kTbRows;
    K.z0 = tbk.z0;
    K.z1 = tbk.z1;
    K.snapw = 0;
    K.plane = (size_t)Lx * (size_t)Ly;
    K.pbytes = (uint32_t)(K.plane * sizeof(float));
    K.qplane = (uint32_t)(K.plane >> 2);
    K.qwrap = (uint32_t)A.Lzg * K.qplane;
    K.m2v = f32x2{A.m2, A.m2};
    asm volatile("" : "+v"(K.m2v));
    K.swrap_at = A.nz - 2;  // periodic (phi4_tb2_run_ok)
    {
        auto wrapy = [Ly](int y) { return y < 0 ? y + Ly : (y >= Ly ? y - Ly : y); };
        const int y = wrapy(tbk.yb * kTbRows - 1 + K.w);
        const int ym = wrapy(y - 1), yp = wrapy(y + 1);
        K.voff = (uint32_t)((y * Lx + 4 * K.lane) * 4);
        K.vm = (uint32_t)((ym * Lx + 4 * K.lane) * 4);
        K.vp = (uint32_t)((yp * Lx + 4 * K.lane) * 4);
        K.vex = 0;
        K.vx2 = 0;
        K.qoff = (uint32_t)((y * Lx + 4 * K.lane) >> 2);
    }
    __shared__ float4 lds[3][kTbWaves][64];
    __shared__ float tx[1][kTbWaves][2];
    __shared__ int s_ok;
    const int nbytes = (int)((uint32_t)(A.nz + 2 * A.gz) * K.pbytes);  // < 2^31 (phi4_tb2_run_ok)
    const unsigned long long sbase = ((unsigned long long)A0.s_hi << 32) | A0.s_lo;
    const PrioQ pq(K.z0, K.z1 - K.z0 + 2);
    for (int t = 0; t < R0.npairs; ++t) {
        A.in = (t & 1) ? A0.out : A0.in;
        A.out = (t & 1) ? const_cast<float *>(A0.in) : A0.out;
        if (t > 0) A.fin = 1;  // the previous pair's guarded output
        K.rin = __builtin_amdgcn_make_buffer_rsrc((void *)A.in, (short)0, nbytes, 0x00020000);
        K.rout = __builtin_amdgcn_make_buffer_rsrc((void *)A.out, (short)0, nbytes, 0x00020000);
        const unsigned long long s0 = sbase + 2ull * (unsigned long long)t, s1 = s0 + 1;
        K.slo = (uint32_t)s0;
        K.shi = (uint32_t)(s0 >> 32);
        K.slo1 = (uint32_t)s1;
        K.shi1 = (uint32_t)(s1 >> 32);
        if (t > 0) {
            if (threadIdx.x == 0) {
                const bool ok = run_wait(R0, lb, A0.nyg, A0.nzc, R0.base + (unsigned int)t);
                if constexpr (LAUX == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                s_ok = ok ? 1 : 0;
            }
            __syncthreads();
            if (s_ok == 0) return;  // block-uniform: every wave leaves
        }
        if (R0.stamps != nullptr && threadIdx.x == 0) {
            R0.stamps[2 * ((size_t)t * nb + b)] = __builtin_amdgcn_s_memrealtime();
            if (t == 0)
                R0.stamps[2 * (size_t)R0.npairs * nb + b] =
                    ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 16) |
                    __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        }
        TbIn I0, I1, I2;
        {
            const __amdgpu_buffer_rsrc_t r0 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 2), K.plane, K.pbytes);
            const __amdgpu_buffer_rsrc_t r1 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 1), K.plane, K.pbytes);
            I0.row = bload4<LAUX>(r0, K.voff);
            I0.hm = I0.hp = I0.row;
            I1.row = bload4<LAUX>(r1, K.voff);
            I1.hm = bload4<LAUX>(r1, K.vm);
            I1.hp = bload4<LAUX>(r1, K.vp);
        }
        float4 T0 = make_float4(0.f, 0.f, 0.f, 0.f), T1 = T0, T2 = T0;
        FrameAcc f1 = frame_acc(), f2 = frame_acc();  // unused (no records)
        TbRun R;
        R.scur = (uint32_t)tb_pidx(A, K.z0 - 1) * K.pbytes;
        R.snext = (uint32_t)tb_pidx(A, K.z0) * K.pbytes;
        R.qz = (uint32_t)global_z(A, K.z0 - 1) * K.qplane;
        R.qzm = 0;
        const int z1 = K.z1;
        for (int p = K.z0 - 1; p <= z1; p += 3) {
            if (A.prio) prio_by_progress(pq.q(p));
            tb_plane<NZ, false, false, true, 0, false, LAUX>(A, K, R, p, I0, I1, I2, T0, T1, T2, lds, tx, f1, f2,
                                                             nullptr);
            if (p + 1 > z1) break;
            tb_plane<NZ, false, false, true, 1, false, LAUX>(A, K, R, p + 1, I1, I2, I0, T1, T2, T0, lds, tx, f1, f2,
                                                             nullptr);
            if (p + 2 > z1) break;
            tb_plane<NZ, false, false, true, 2, false, LAUX>(A, K, R, p + 2, I2, I0, I1, T2, T0, T1, lds, tx, f1, f2,
                                                             nullptr);
        }
        // publish pair t: every wave's write-through stores drained, then one flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (R0.stamps != nullptr && threadIdx.x == 0)
            R0.stamps[2 * ((size_t)t * nb + b) + 1] = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0)
            __hip_atomic_store(R0.flags + lb, R0.base + (unsigned int)t + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

// phi4_tb2_kernel<NZ, false, 1, false, true, false> for the last pair of a
// P2P deep-halo block (one range of a slab with ghost zones): its edge output
// planes also go to the staging slot, and every block counts itself done.
template <bool NZ>
__global__ __launch_bounds__(kTbWaves * 64) __attribute__((amdgpu_waves_per_eu(1)))
void phi4_tb2_stage_kernel(const Phi4StepArgs A, const Tb2StageArgs S) {
    const int nb = gridDim.x, b = blockIdx.x;
    const TbBlock tbk = tb_block<false>(A, b, nb);
    const int Lx = A.Lx, Ly = A.Ly;
    TbCtx K;
    K.w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    K.lane = threadIdx.x & 63;
    K.outw = K.w >= 1 && K.w <= kTbRows;
    K.z0 = tbk.z0;
    K.z1 = tbk.z1;
    K.snapw = 0;
    K.plane = (size_t)Lx * (size_t)Ly;
    K.pbytes = (uint32_t)(K.plane * sizeof(float));
    K.qplane = (uint32_t)(K.plane >> 2);
    const int nbytes = (int)((uint32_t)(A.nz + 2 * A.gz) * K.pbytes);  // < 2^31 (phi4_tb2_stage_ok)
    K.rin = __builtin_amdgcn_make_buffer_rsrc((void *)A.in, (short)0, nbytes, 0x00020000);
    K.rout = __builtin_amdgcn_make_buffer_rsrc((void *)A.out, (short)0, nbytes, 0x00020000);
    K.rstg = __builtin_amdgcn_make_buffer_rsrc((void *)S.stage, (short)0, (int)(2u * (uint32_t)S.G * K.pbytes),
                                               0x00020000);
    K.stg_g = S.G;
    K.stg_hi = A.nz - S.G;
    K.qwrap = (uint32_t)A.Lzg * K.qplane;
    K.m2v = f32x2{A.m2, A.m2};
    asm volatile("" : "+v"(K.m2v));
    K.swrap_at = INT_MIN;  // a slab: p < 0 in ghost zones
    const unsigned long long s0 = ((unsigned long long)A.s_hi << 32) | A.s_lo, s1 = s0 + 1;
    K.slo = (uint32_t)s0;
    K.shi = (uint32_t)(s0 >> 32);
    K.slo1 = (uint32_t)s1;
    K.shi1 = (uint32_t)(s1 >> 32);
    {
        auto wrapy = [Ly](int y) { return y < 0 ? y + Ly : (y >= Ly ? y - Ly : y); };
        const int y = wrapy(tbk.yb * kTbRows - 1 + K.w);
        const int ym = wrapy(y - 1), yp = wrapy(y + 1);
        K.voff = (uint32_t)((y * Lx + 4 * K.lane) * 4);
        K.vm = (uint32_t)((ym * Lx + 4 * K.lane) * 4);
        K.vp = (uint32_t)((yp * Lx + 4 * K.lane) * 4);
        K.vex = 0;
        K.vx2 = 0;
        K.qoff = (uint32_t)((y * Lx + 4 * K.lane) >> 2);
    }
    __shared__ float4 lds[3][kTbWaves][64];
    __shared__ float tx[1][kTbWaves][2];
    TbIn I0, I1, I2;
    {
        const __amdgpu_buffer_rsrc_t r0 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 2), K.plane, K.pbytes);
        const __amdgpu_buffer_rsrc_t r1 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 1), K.plane, K.pbytes);
        I0.row = bload4(r0, K.voff);
        I0.hm = I0.hp = I0.row;
        I1.row = bload4(r1, K.voff);
        I1.hm = bload4(r1, K.vm);
        I1.hp = bload4(r1, K.vp);
    }
    float4 T0 = make_float4(0.f, 0.f, 0.f, 0.f), T1 = T0, T2 = T0;
    FrameAcc f1 = frame_acc(), f2 = frame_acc();  // unused (no records)
    TbRun R;
    R.scur = (uint32_t)tb_pidx(A, K.z0 - 1) * K.pbytes;
    R.snext = (uint32_t)tb_pidx(A, K.z0) * K.pbytes;
    R.qz = (uint32_t)global_z(A, K.z0 - 1) * K.qplane;
    R.qzm = 0;
    const int z1 = K.z1;
    const PrioQ pq(K.z0, z1 - K.z0 + 2);
    for (int p = K.z0 - 1; p <= z1; p += 3) {
        if (A.prio) prio_by_progress(pq.q(p));
        tb_plane<NZ, false, false, true, 0, false, 0, true>(A, K, R, p, I0, I1, I2, T0, T1, T2, lds, tx, f1, f2,
                                                            nullptr);
        if (p + 1 > z1) break;
        tb_plane<NZ, false, false, true, 1, false, 0, true>(A, K, R, p + 1, I1, I2, I0, T1, T2, T0, lds, tx, f1, f2,
                                                            nullptr);
        if (p + 2 > z1) break;
        tb_plane<NZ, false, false, true, 2, false, 0, true>(A, K, R, p + 2, I2, I0, I1, T2, T0, T1, lds, tx, f1, f2,
                                                            nullptr);
    }
    // every wave's write-through stores drained, then one count for the block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(S.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// kid family 3 (phi4_kernel_id_name's bits 0-1): bit 2 NZ, bit 3 LAUX = 16,
// bit 4 the staging kernel
void phi4_run_kernel_id_name(uint64_t k, char *name, size_t cap) {
    if ((k >> 4) & 1)
        snprintf(name, cap, "phi4_tb2_stage_kernel<%s>", ((k >> 2) & 1) ? "true" : "false");
    else
        snprintf(name, cap, "phi4_tb2_run_kernel<%s, %d>", ((k >> 2) & 1) ? "true" : "false",
                 ((k >> 3) & 1) ? 16 : 0);
}

bool phi4_tb2_stage_ok(const Phi4StepArgs &a, int G) {
    return a.Lx == 256 && a.Ly % kTbRows == 0 && !a.periodic && a.nxseg == 1 && a.nyg == a.Ly / kTbRows &&
           a.nzr == a.nzc && a.nunits == a.nyg * a.nzc && a.zlo == 0 && a.zlen == a.nz && a.nz >= 2 &&
           (long long)a.zc * a.nzr >= a.zlen && G >= 1 && G <= a.nz && a.gz >= 2 && a.gate == nullptr &&
           a.flag == nullptr && a.st_md == nullptr && a.snap == nullptr && a.dcoef == nullptr &&
           a.stamps == nullptr && a.tctl == nullptr && a.fold.cin == nullptr && a.clr.md == nullptr &&
           (long long)(a.nz + 2 * a.gz) * a.Lx * a.Ly * 4 < (1ll << 31);
}

hipError_t phi4_tb2_stage_launch(const Phi4StepArgs &a, const Tb2StageArgs &g, hipStream_t s, hipEvent_t e0,
                                 hipEvent_t e1, uint64_t *kid) {
    if (!phi4_tb2_stage_ok(a, g.G) || g.stage == nullptr || g.ctr == nullptr) return hipErrorInvalidValue;
    const bool nz = a.sig != 0.0f;
    const dim3 grid((unsigned)a.nunits), block(kTbWaves * 64);
    if (kid != nullptr) *kid = (uint64_t)3 | (uint64_t)nz << 2 | (uint64_t)1 << 4 | (uint64_t)(grid.x * block.x) << 32;
    Phi4StepArgs q = a;
    static const int prio = getenv("SQ_TB2_PRIO") ? atoi(getenv("SQ_TB2_PRIO")) : 1;
    q.prio = prio;
    Tb2StageArgs gg = g;
    void *args[] = {&q, &gg};
    const void *fn = nz ? (const void *)&phi4_tb2_stage_kernel<true> : (const void *)&phi4_tb2_stage_kernel<false>;
    if (e0 != nullptr || e1 != nullptr) return hipExtLaunchKernel(fn, grid, block, args, 0, s, e0, e1, 0);
    return hipLaunchKernel(fn, grid, block, args, 0, s);
}

static int run_laux() {
    const char *e = getenv("SQ_TB2_RUN_SC1");  // read per launch (tests switch it within a process)
    return (e != nullptr && atoi(e) != 0) ? 16 : 0;
}

static const void *run_fn(bool nz, int laux) {
    if (laux == 16)
        return nz ? (const void *)&phi4_tb2_run_kernel<true, 16> : (const void *)&phi4_tb2_run_kernel<false, 16>;
    return nz ? (const void *)&phi4_tb2_run_kernel<true, 0> : (const void *)&phi4_tb2_run_kernel<false, 0>;
}

bool phi4_tb2_run_ok(const Phi4StepArgs &a, int dev) {
    if (a.Lx != 256 || a.Ly % kTbRows != 0 || !a.periodic || a.nxseg != 1 || a.nyg != a.Ly / kTbRows ||
        a.nzr != a.nzc || a.nunits != a.nyg * a.nzc || a.zlo != 0 || a.zlen != a.nz || a.zc < 2 ||
        a.zlen - (a.nzr - 1) * a.zc < 2 || (long long)a.zc * a.nzr < a.zlen)
        return false;  // every chunk >= 2 planes: the light cone stays in the neighbouring chunks
    if (a.gate != nullptr || a.flag != nullptr || a.st_md != nullptr || a.snap != nullptr || a.dcoef != nullptr ||
        a.stamps != nullptr || a.tctl != nullptr || a.fold.cin != nullptr || a.clr.md != nullptr)
        return false;
    if ((long long)(a.nz + 2 * a.gz) * a.Lx * a.Ly * 4 >= (1ll << 31)) return false;
    // every block resident: blocks per CU from the occupancy query of the
    // instance (both instances alike) x the CUs
    static int per_cu = -1, ncu = -1;
    if (per_cu < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, run_fn(true, 0), kTbWaves * 64, 0) != hipSuccess) n = 0;
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) c = 0;
        per_cu = n;
        ncu = c;
    }
    return (long long)a.nunits <= (long long)per_cu * ncu;
}

hipError_t phi4_tb2_run_launch(const Phi4StepArgs &a, const Tb2RunArgs &r, hipStream_t s, hipEvent_t e0,
                               hipEvent_t e1, uint64_t *kid) {
    if (r.npairs < 1 || r.flags == nullptr || r.err == nullptr) return hipErrorInvalidValue;
    const bool nz = a.sig != 0.0f;
    const int laux = run_laux();
    const dim3 grid((unsigned)a.nunits), block(kTbWaves * 64);
    if (kid != nullptr)
        *kid = (uint64_t)3 | (uint64_t)nz << 2 | (uint64_t)(laux == 16) << 3 | (uint64_t)(grid.x * block.x) << 32;
    Phi4StepArgs q = a;
    const char *pe = getenv("SQ_TB2_RUN_PRIO");  // read per launch (experiments switch it within a process)
    q.prio = pe ? atoi(pe) : 1;
    Tb2RunArgs rr = r;
    void *args[] = {&q, &rr};
    const void *fn = run_fn(nz, laux);
    if (e0 != nullptr || e1 != nullptr) return hipExtLaunchKernel(fn, grid, block, args, 0, s, e0, e1, 0);
    return hipLaunchKernel(fn, grid, block, args, 0, s);
}

}  // namespace sq
