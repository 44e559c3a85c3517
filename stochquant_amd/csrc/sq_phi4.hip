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
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "sq_dpp.h"
#include "sq_internal.h"
#include "sq_rng.h"

namespace sq {

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float from_left_lane(float v) {  // lane i <- lane i-1 (mod 64)
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x13C, 0xF, 0xF, true));
}
__device__ __forceinline__ float from_right_lane(float v) {  // lane i <- lane i+1 (mod 64)
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x134, 0xF, 0xF, true));
}
// Lane i <- lane i-1 and lane 0 <- edge (DPP wave_shr:1 with bound_ctrl off:
// the lane without a source keeps the old value, so no v_cndmask), and
// lane i <- lane i+1, lane 63 <- edge (wave_shl:1).
__device__ __forceinline__ float from_left_lane_or(float v, float edge) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, edge),
                                                                 __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_right_lane_or(float v, float edge) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, edge),
                                                                 __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, false));
}

// Buffer descriptor over ONE plane: the base moves by scalar arithmetic per
// plane and every per-lane offset (row within the plane) is loop-invariant,
// so the z-march does no per-lane address math (guide T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const float *base, int padded,
                                                             size_t plane, uint32_t pbytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)padded * plane), (short)0,
                                             (int)pbytes, 0x00020000);
}
// soff: a wave-uniform byte offset added by the buffer unit (the plane of a
// whole-buffer descriptor, tb2 kernel)
template <int LAUX = 0>
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff = 0) {
    const f32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, LAUX);
    return make_float4(v.x, v.y, v.z, v.w);
}
// Always with soffset 0 (an inline constant), never an SGPR: a 16-byte VMEM
// store reads its data VGPRs after issue, and a VALU write of the first of
// them right behind the store can land first -- on gfx950 the last four lanes
// of every 16 then store the new value (found in round 3: the frame kernels'
// first output component, lanes 12-15 / 28-31 / 44-47 / 60-63 of one row in a
// few launches).  The compiler inserts the wait state for
// this hazard only when soffset is not a register
// (GCNHazardRecognizer::createsVALUHazard), so plane offsets go into the VGPR
// offset; tests/test_isa_hazards.py checks the built code object for the
// pattern.
template <int AUX = 0>
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
    const uint32_t soff = 0;
    const f32x4v w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, r, off, soff, AUX);
}
template <int LAUX = 0>
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff = 0) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, LAUX));
}

__device__ __forceinline__ int padded_index(const Phi4StepArgs &A, int zl) {
    if (A.periodic) {
        if (zl < 0) return A.nz;
        if (zl >= A.nz) return 1;
    }
    return zl + A.gz;
}

// Global z of local plane zl (ghost-zone planes of the first / last slab wrap).
// 32-bit: Lz < 2^31 (create_phi4), so the wrap stays scalar (gfx950 has no
// scalar 64-bit signed compare; the 64-bit form cost 4 VALU per plane).
__device__ __forceinline__ int global_z(const Phi4StepArgs &A, int zl) {
    const int Lz = (int)A.Lzg;
    int zg = (int)A.zg0 + zl;
    if (zg < 0) zg += Lz;
    else if (zg >= Lz) zg -= Lz;
    return zg;
}

// Guard of tau_kernel.cl:119-133 in two instructions: v_min_f32 returns the
// non-NaN operand, so NaN -> +clamp, > clamp -> +clamp; then v_max_f32 gives
// < -clamp -> -clamp.  Same results as the oracle's explicit branches.
template <bool NZ>
__device__ __forceinline__ float site_update(float phi, float xm, float xp, float ym, float yp,
                                             float zm, float zp, float xi, const Phi4StepArgs &A) {
    const float nb = ((xm + xp) + (ym + yp)) + (zm + zp);
    const float lap = __builtin_fmaf(-6.0f, phi, nb);
    const float g = __builtin_fmaf(A.lam6, phi * phi, A.m2);
    const float drift = __builtin_fmaf(-phi, g, lap);
    const float det = __builtin_fmaf(A.h, drift, phi);
    const float v = NZ ? __builtin_fmaf(A.sigq, xi, det) : det;  // NZ = false: C = 0 gradient flow
    return fmaxf(fminf(v, A.clampv), -A.clampv);
}

// The same update for the 4 sites of a float4 with packed f32 arithmetic
// (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 on site pairs): identical
// operations and order per site, so bit-identical results; the x-neighbour
// sums stay scalar (their operands are not register-pair aligned).
typedef float f32x2 __attribute__((ext_vector_type(2)));
// fin: the inputs are known finite (Phi4StepArgs::fin) -- then a finite
// update can only leave [-clampv, clampv] as a finite value or an infinity
// (create_phi4 bounds the drift), never as NaN, so one max3 / max / compare
// decides whether the guard has anything to do and the 8-instruction guard
// runs only in waves where some lane does (bit-identical either way).
// m2v: {m2, m2} (a VOP3P operation reads one scalar operand, and lam6 is the
// one: the tb2 kernel pins the pair in VGPRs once instead of per update).
template <bool NZ>
__device__ __forceinline__ float4 site_update4(float4 c, float lft, float rgt, float4 up, float4 dn,
                                               float4 zm, float4 zp, const f32x4n &xi,
                                               const Phi4StepArgs &A, bool fin, f32x2 m2v,
                                               float *mpre = nullptr) {
    const f32x2 c0 = {c.x, c.y}, c1 = {c.z, c.w};
    // c.x + c.z and c.y + c.w as two single adds: formed as one v_pk_add they
    // share a register pair and take two v_mov to reach x0 / x1
    float s02, s13;
    asm("v_add_f32 %0, %1, %2" : "=v"(s02) : "v"(c.x), "v"(c.z));
    asm("v_add_f32 %0, %1, %2" : "=v"(s13) : "v"(c.y), "v"(c.w));
    const f32x2 x0 = {lft + c.y, s02}, x1 = {s13, c.z + rgt};
    const f32x2 y0 = f32x2{up.x, up.y} + f32x2{dn.x, dn.y}, y1 = f32x2{up.z, up.w} + f32x2{dn.z, dn.w};
    const f32x2 z0 = f32x2{zm.x, zm.y} + f32x2{zp.x, zp.y}, z1 = f32x2{zm.z, zm.w} + f32x2{zp.z, zp.w};
    const f32x2 nb0 = (x0 + y0) + z0, nb1 = (x1 + y1) + z1;
    const f32x2 m6 = {-6.0f, -6.0f}, l6 = {A.lam6, A.lam6}, m2 = m2v, h = {A.h, A.h};
    const f32x2 lap0 = __builtin_elementwise_fma(m6, c0, nb0), lap1 = __builtin_elementwise_fma(m6, c1, nb1);
    const f32x2 g0 = __builtin_elementwise_fma(l6, c0 * c0, m2), g1 = __builtin_elementwise_fma(l6, c1 * c1, m2);
    const f32x2 d0 = __builtin_elementwise_fma(-c0, g0, lap0), d1 = __builtin_elementwise_fma(-c1, g1, lap1);
    f32x2 v0 = __builtin_elementwise_fma(h, d0, c0), v1 = __builtin_elementwise_fma(h, d1, c1);
    if (NZ) {
        const f32x2 sg = {A.sigq, A.sigq};
        v0 = __builtin_elementwise_fma(sg, f32x2{xi.a, xi.b}, v0);
        v1 = __builtin_elementwise_fma(sg, f32x2{xi.c, xi.d}, v1);
    }
    const float cl = A.clampv;
    float4 o = make_float4(v0.x, v0.y, v1.x, v1.y);
    const float m = fmaxf(fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)), fabsf(o.w));  // v_max3 + v_max
    float mo = m;
    if (!fin || !(m < cl)) {
        o = make_float4(fmaxf(fminf(o.x, cl), -cl), fmaxf(fminf(o.y, cl), -cl), fmaxf(fminf(o.z, cl), -cl),
                        fmaxf(fminf(o.w, cl), -cl));
        if (mpre != nullptr) mo = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w)));
    }
    // frames: max |phi'| of the returned float4 -- m itself where the guard had
    // nothing to do (every |phi'| < clamp, finite), else taken after the guard
    // (a NaN that fmaxf dropped from m is +clamp there)
    if (mpre != nullptr) *mpre = mo;
    return o;
}

// Per-lane frame accumulators (frames only, A.flag != nullptr): the guard
// flag of tau_kernel.cl:119-133 and, per step, the record of the stability
// heuristic (tau_kernel.cl:135-143): m = max phi', d = the
// drift increment |phi' - phi - sigma xi| at the sites attaining m (the
// largest one on ties), mw = the wave's running maximum of phi'
// (wave-uniform).  am: the running max |phi'| after the guard (site_update4's
// mpre, or taken from o); the guard flag is am >= clamp (the guard clamps to
// [-clamp, clamp], NaN to +clamp, so some site was clamped iff the maximum
// reached the clamp) and max |phi'| after the guard is min(am, clamp) = am.
// One accumulator: round 2 kept the flag and maximum in two more, and the
// compiler selected between their addresses through 12 bytes of private
// memory per lane.
struct FrameAcc {
    float m, d;
    float mw;
    float am;
};
__device__ __forceinline__ FrameAcc frame_acc() {
    return FrameAcc{-__builtin_inff(), 0.f, -__builtin_inff(), 0.f};
}

// v_max_f32 / v_max3_f32 without the IEEE-mode operand canonicalisation the
// compiler wraps around fmaxf (a quieting v_max_f32 x, x, x per operand it
// cannot prove canonical: 2 of the 4 instructions of a float4's max).  For
// operands that are results of arithmetic, never signalling NaNs; a quiet NaN
// operand still yields the other one, as fmaxf.
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Branch-free: the larger drift increment on ties is computed up front and
// selected (the selects of a conditional fmaxf compiled to exec-masked blocks).
__device__ __forceinline__ void stab_site(FrameAcc &f, float o, float c, float xi, float sig) {
    const float dn = fabsf(__builtin_fmaf(-sig, xi, o - c));
    const float dt = vmax(f.d, dn);
    const bool gt = o > f.m, eq = o == f.m;
    const float d1 = eq ? dt : f.d;
    f.d = gt ? dn : d1;
    f.m = vmax(f.m, o);
}

// The frame bookkeeping of one float4 of outputs o (inputs c, noise xi).
// A site below the wave's running maximum mw can neither set nor tie the
// step's maximum, so the per-site (m, d) update runs only when some lane's
// float4 reaches mw (wave-uniform branch; on iid values a wave meets a new
// maximum in about H(n) of its n planes): the lanes' (m, d) may then miss
// sites below mw, but the wave's maximum key ord(m) << 32 | bits(d), all
// that frame_flush keeps, is exact.  am (guard flag, max |phi'|) takes every site.
// bw (BW, the fused kernels): the block's running maximum of this record in LDS,
// raised by each wave that meets a new maximum of its own; the threshold is
// then the larger of the two, still a value some site of the record attains,
// so the block's key stays exact and a wave takes the per-site path about
// 1 + H(n)/waves times instead of H(n).  Waves read it without
// a barrier: any value read is a valid (monotone, attained) threshold.
// pre: mpre is site_update4's max |phi'| of o (the fused kernels), accumulated
// into am; otherwise taken from o here.
template <bool NZ, bool BW = false>
__device__ __forceinline__ void frame_sites(const Phi4StepArgs &A, FrameAcc &f, const float4 &o, const float4 &c,
                                            const f32x4n &xi, float *bw = nullptr, bool pre = false,
                                            float mpre = 0.f) {
    const float mo = pre ? mpre : fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w)));
    f.am = vmax(f.am, mo);  // mo: never a signalling NaN (arithmetic / the guard's output)
    {  // frame launches always carry the records (the launchers check st_md, st_a)
        // max |o| >= max o: a float4 whose largest magnitude is below the
        // threshold cannot reach it, and mo is already at hand (2 VALU fewer
        // per float4 on the common path than forming max o first)
        if (__ballot(mo >= f.mw) == 0ull) return;
        const float o4 = vmax(vmax3(o.x, o.y, o.z), o.w);  // the guard's output: never NaN
        if (__ballot(o4 >= f.mw) == 0ull) return;  // below the wave's own threshold: no LDS read
        if constexpr (BW) {
            // the block's threshold only when the wave's own one is met; it becomes
            // the wave's (any attained value <= the record's maximum is exact, and
            // the block word only grows), so the next float4s test against it
            // without another LDS read
            f.mw = vmax(f.mw, __hip_atomic_load(bw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        }
        if (!BW || __ballot(o4 >= f.mw) != 0ull) {
            const float s = NZ ? A.sigq : 0.f;
            stab_site(f, o.x, c.x, xi.a, s);
            stab_site(f, o.y, c.y, xi.b, s);
            stab_site(f, o.z, c.z, xi.c, s);
            stab_site(f, o.w, c.w, xi.d, s);
            f.mw = dpp_all_max_f(f.m);
            if (BW && (threadIdx.x & 63) == 0)
                __hip_atomic_fetch_max(bw, f.mw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// Order-preserving float -> uint map (the stability records are u64 maxima of
// (ord(m) << 32) | bits(d): the larger m wins, equal m the larger d).
__device__ __forceinline__ uint32_t ord_f32(float v) {
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Block-wide reduction of the frame accumulators, one atomic per block and
// step record (slot = block % kStabSlots spreads them over kStabSlots words);
// every wave of the block must call it.
__device__ __forceinline__ void frame_flush(const Phi4StepArgs &A, const FrameAcc &f, int rec, uint64_t *sk,
                                            uint32_t *sa) {
    const bool bad = f.am >= A.clampv;
    if (__ballot(bad) != 0ull && (threadIdx.x & 63) == 0) atomicOr(A.flag, 1);
    if (A.st_md == nullptr) return;
    // wave maxima by DPP scans (bits of non-negative floats order as ints)
    uint64_t k = dpp_all_max_u64(((uint64_t)ord_f32(f.m) << 32) | __float_as_uint(f.d));
    uint32_t a = (uint32_t)dpp_all_max_i((int)__float_as_uint(fminf(f.am, A.clampv)));
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        sk[w] = k;
        sa[w] = a;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < nw; ++i) {
            k = sk[i] > k ? sk[i] : k;
            a = sa[i] > a ? sa[i] : a;
        }
        const int slot = rec * kStabSlots + (int)(blockIdx.x % kStabSlots);
        atomicMax(A.st_md + slot, (unsigned long long)k);
        atomicMax(A.st_a + slot, a);
    }
}

// Both step records of a fused launch in one pass (the two-step kernels):
// wave maxima by DPP, combined across the block by LDS atomic maxima (fk / fa,
// cleared at the kernel's start) behind ONE barrier, then one global atomic
// per record.  Two frame_flush calls took four barriers and two serial folds
// at every block's end: 10-20 us of a 20-step 256^3 frame
// (profiles/r03/s2/fdiag/).  Maxima in any order: the same records.
__device__ __forceinline__ void frame_flush2(const Phi4StepArgs &A, const FrameAcc &f1, const FrameAcc &f2,
                                             unsigned long long *fk, uint32_t *fa) {
    const bool bad = f1.am >= A.clampv || f2.am >= A.clampv;
    if (__ballot(bad) != 0ull && (threadIdx.x & 63) == 0) atomicOr(A.flag, 1);
    if (A.st_md == nullptr) return;  // a kernel argument: every thread returns here or none
    // The wave's key: f.mw is the DPP maximum of the lanes' m at their last
    // per-site update (frame_sites), possibly raised since to the block's
    // threshold, so only lanes whose m reaches it can hold the wave's maximum
    // key -- usually one lane -- and only they post it (an exec-masked LDS
    // atomic instead of two 64-bit DPP scans per wave, ~60 VALU).  No lane
    // qualifies when the block's threshold passed the wave's maximum: another
    // wave's lanes hold a key at least as large.  Waves without sites in a
    // record (m = mw = -inf) post nothing.
    if (f1.m >= f1.mw && f1.mw > -__builtin_inff())
        atomicMax(&fk[0], ((uint64_t)ord_f32(f1.m) << 32) | __float_as_uint(f1.d));
    if (f2.m >= f2.mw && f2.mw > -__builtin_inff())
        atomicMax(&fk[1], ((uint64_t)ord_f32(f2.m) << 32) | __float_as_uint(f2.d));
    const uint32_t a1 = (uint32_t)dpp_all_max_i((int)__float_as_uint(fminf(f1.am, A.clampv)));
    const uint32_t a2 = (uint32_t)dpp_all_max_i((int)__float_as_uint(fminf(f2.am, A.clampv)));
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&fa[0], a1);
        atomicMax(&fa[1], a2);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const int slot = (int)threadIdx.x * kStabSlots + (int)(blockIdx.x % kStabSlots);
        atomicMax(A.st_md + slot, fk[threadIdx.x]);
        atomicMax(A.st_a + slot, fa[threadIdx.x]);
    }
}

// Philox4x32-10 of the field-noise counters {q, cy, cz, cw} whose words 1..3
// (stream, step lo, step hi) and key are wave-uniform, R independent q per
// lane, round-major so the chains interleave.  The same function as
// philox4x32_10 (sq_rng.h), with the first three rounds written out so every
// combination of uniform words happens on the scalar unit: round 0's
// M1 * cz product and its xor with cy, k0 (and cw ^ k1), round 1's M0 * n0
// product, round 2's n3 ^ k1 -- VOP3 reads one scalar per instruction on
// gfx950, so a v_bitop3_b32 of two uniform operands otherwise costs a
// v_mov_b32 first.  Rounds 3..9: the three-input xors are one v_bitop3_b32 each.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <int R>
__device__ __forceinline__ void philox_field(u32x4 (&c)[R], uint32_t k0, uint32_t k1) {
    const uint32_t cy = c[0].y, cz = c[0].z, cw = c[0].w;  // uniform already (kernel arguments)
    // round 0
    const uint64_t p1u = (uint64_t)kPhiloxM1 * cz;
    const uint32_t u0 = uni((uint32_t)(p1u >> 32) ^ cy ^ k0), u1 = uni((uint32_t)p1u);
    const uint32_t a0 = cw ^ k1;
    uint32_t n2[R], n3[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c[r].x;
        n2[r] = (uint32_t)(p0 >> 32) ^ a0;
        n3[r] = (uint32_t)p0;
    }
    // round 1
    k0 += kPhiloxW0;
    k1 += kPhiloxW1;
    const uint64_t p0u = (uint64_t)kPhiloxM0 * u0;
    const uint32_t b0 = uni(u1 ^ k0), b2 = uni((uint32_t)(p0u >> 32) ^ k1), u3 = uni((uint32_t)p0u);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t p1 = (uint64_t)kPhiloxM1 * n2[r];
        c[r] = u32x4{(uint32_t)(p1 >> 32) ^ b0, (uint32_t)p1, b2 ^ n3[r], u3};
    }
    // round 2: word 3 is still uniform
    k0 += kPhiloxW0;
    k1 += kPhiloxW1;
    const uint32_t d2 = uni(u3 ^ k1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c[r].x;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * c[r].z;
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c[r].y, k0, 0x96);
        c[r] = u32x4{n0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ d2, (uint32_t)p0};
    }
#pragma unroll
    for (int rnd = 3; rnd < 10; ++rnd) {
        k0 += kPhiloxW0;
        k1 += kPhiloxW1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint64_t p0 = (uint64_t)kPhiloxM0 * c[r].x;
            const uint64_t p1 = (uint64_t)kPhiloxM1 * c[r].z;
            const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c[r].y, k0, 0x96);
            const uint32_t m2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c[r].w, k1, 0x96);
            c[r] = u32x4{n0, (uint32_t)p1, m2, (uint32_t)p0};
        }
    }
}

// Philox4x32-10 on R independent counters, round-major so the R dependency
// chains interleave; the three-input xors are one v_bitop3_b32 each.
template <int R>
__device__ __forceinline__ void philox_rows(u32x4 (&c)[R], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int rnd = 0; rnd < 10; ++rnd) {
        if (rnd) {
            k0 += kPhiloxW0;
            k1 += kPhiloxW1;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint64_t p0 = (uint64_t)kPhiloxM0 * c[r].x;
            const uint64_t p1 = (uint64_t)kPhiloxM1 * c[r].z;
            const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c[r].y, k0, 0x96);
            const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c[r].w, k1, 0x96);
            c[r] = u32x4{n0, (uint32_t)p1, n2, (uint32_t)p0};
        }
    }
}

// A lane holds, per row, V float4 of the wave's x-span: segment v at
// x = x0 + 256 v + 4 lane (each load is still one contiguous 1-KiB wave access).
template <int R, int V>
struct Slot {
    float4 row[R * V];   // index r*V + v
    float4 hm[V], hp[V]; // y-halo rows of the same plane
};

template <int QX, int R, int V>
struct Lane {
    uint32_t voff[R * V];   // byte offset of each float4 inside the plane
    uint32_t vm[V], vp[V];  // halo rows
    uint32_t vl[R], vr[R];  // x-1 of the span's first site / x+1 of its last (MS only)
    uint32_t qoff[R * V];   // Philox quad offset inside the plane
    bool rows_ok;
    int lane;
};

template <int QX, int R, int V>
__device__ __forceinline__ void load_slot(const Phi4StepArgs &A, const Lane<QX, R, V> &L,
                                          Slot<R, V> &s, int zl, bool halo, size_t plane,
                                          uint32_t pbytes) {
    const __amdgpu_buffer_rsrc_t rs = plane_rsrc(A.in, padded_index(A, zl), plane, pbytes);
#pragma unroll
    for (int k = 0; k < R * V; ++k) s.row[k] = bload4(rs, L.voff[k]);
    if (halo) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
            s.hm[v] = bload4(rs, L.vm[v]);
            s.hp[v] = bload4(rs, L.vp[v]);
        }
    }
}

// Update plane z from slots P (z-1), C (z), N (z+1).
// MS: the row spans several wave x-spans (Lx > 256 V): the span's two outer
//     neighbours come from scalar loads by lanes 0 / 63.
// NZ: noise on (C != 0); off, the C = 0 gradient flow skips the RNG.
template <int QX, int R, int V, bool MS, bool NZ, bool PK, int SAUX, bool FR>
__device__ __forceinline__ void plane_compute(const Phi4StepArgs &A, const Lane<QX, R, V> &L,
                                              const Slot<R, V> &P, const Slot<R, V> &C,
                                              const Slot<R, V> &N, int z, size_t plane,
                                              uint32_t pbytes, uint32_t qplane, uint32_t slo, uint32_t shi,
                                              FrameAcc &fa) {
    float el[R], er[R];
    if constexpr (MS) {
        const __amdgpu_buffer_rsrc_t rs = plane_rsrc(A.in, padded_index(A, z), plane, pbytes);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            el[r] = 0.f;
            er[r] = 0.f;
            if (L.lane == 0) el[r] = bload1(rs, L.vl[r]);
            if (L.lane == 63) er[r] = bload1(rs, L.vr[r]);
        }
    }
    // noise for the R*V float4s of plane z: independent of the loads in flight
    f32x4n xi[R * V];
    if constexpr (NZ) {
        u32x4 c[R * V];
        const uint32_t qbase = (uint32_t)global_z(A, z) * qplane;
#pragma unroll
        for (int k = 0; k < R * V; ++k) c[k] = u32x4{qbase + L.qoff[k], kStreamField << 24, slo, shi};
        philox_field<R * V>(c, A.k0, A.k1);
#pragma unroll
        for (int k = 0; k < R * V; ++k) {  // scaled by 1/sqrt(2 ln 2); A.sigq carries the factor
            box_muller_q(c[k].x, c[k].y, xi[k].a, xi[k].b);
            box_muller_q(c[k].z, c[k].w, xi[k].c, xi[k].d);
        }
    } else {
#pragma unroll
        for (int k = 0; k < R * V; ++k) xi[k] = f32x4n{0.f, 0.f, 0.f, 0.f};
    }
    float4 hmv[V], hpv[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        hmv[v] = C.hm[v];
        hpv[v] = C.hp[v];
    }
    const __amdgpu_buffer_rsrc_t ws = plane_rsrc(A.out, A.periodic ? z + 1 : z + A.gz, plane, pbytes);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        // x-neighbours across lanes: rotate every segment's edge element once,
        // then lane 0 / 63 take the value rotated out of the adjacent segment
        float rl[V], rr[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float4 cc = C.row[r * V + v];
            if constexpr (QX == 64) {
                rl[v] = from_left_lane(cc.w);
                rr[v] = from_right_lane(cc.x);
            } else {
                const int seg = L.lane & ~(QX - 1), xq = L.lane & (QX - 1);
                rl[v] = __shfl(cc.w, seg | ((xq + QX - 1) & (QX - 1)), 64);
                rr[v] = __shfl(cc.x, seg | ((xq + 1) & (QX - 1)), 64);
            }
        }
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int k = r * V + v;
            const float4 cc = C.row[k];
            const float4 up = r > 0 ? C.row[r > 0 ? k - V : 0] : hmv[v];
            const float4 dn = r < R - 1 ? C.row[r < R - 1 ? k + V : 0] : hpv[v];
            float lft = rl[v], rgt = rr[v];
            if constexpr (V > 1) {
                if (L.lane == 0) lft = rl[(v + V - 1) % V];
                if (L.lane == 63) rgt = rr[(v + 1) % V];
            }
            if constexpr (MS) {
                if (v == 0 && L.lane == 0) lft = el[r];
                if (v == V - 1 && L.lane == 63) rgt = er[r];
            }
            float4 o;
            if constexpr (PK) {
                o = site_update4<NZ>(cc, lft, rgt, up, dn, P.row[k], N.row[k], xi[k], A, A.fin != 0,
                                     f32x2{A.m2, A.m2});
            } else {
                o.x = site_update<NZ>(cc.x, lft, cc.y, up.x, dn.x, P.row[k].x, N.row[k].x, xi[k].a, A);
                o.y = site_update<NZ>(cc.y, cc.x, cc.z, up.y, dn.y, P.row[k].y, N.row[k].y, xi[k].b, A);
                o.z = site_update<NZ>(cc.z, cc.y, cc.w, up.z, dn.z, P.row[k].z, N.row[k].z, xi[k].c, A);
                o.w = site_update<NZ>(cc.w, cc.z, rgt, up.w, dn.w, P.row[k].w, N.row[k].w, xi[k].d, A);
            }
            // frames only: raw sq_step has no rollback to feed (lanes past Ly
            // compute duplicates of rows 0.., which change no maximum)
            if constexpr (FR) frame_sites<NZ>(A, fa, o, cc, xi[k]);
            if (L.rows_ok) bstore4<SAUX>(ws, L.voff[k], o);
        }
    }
}

// Prefetch distance 1: load plane z+1 into N, then update plane z.
template <int QX, int R, int V, bool MS, bool NZ, bool PK, int SAUX, bool FR>
__device__ __forceinline__ void plane_step(const Phi4StepArgs &A, const Lane<QX, R, V> &L,
                                           const Slot<R, V> &P, const Slot<R, V> &C, Slot<R, V> &N,
                                           int z, int zend, size_t plane, uint32_t pbytes,
                                           uint32_t qplane, uint32_t slo, uint32_t shi, FrameAcc &fa) {
    load_slot<QX, R, V>(A, L, N, z + 1, z + 1 < zend, plane, pbytes);
    plane_compute<QX, R, V, MS, NZ, PK, SAUX, FR>(A, L, P, C, N, z, plane, pbytes, qplane, slo, shi, fa);
}

// One wave's unit of a step: an x-span of 4*QX*V sites by R row sets by a
// z-chunk.
template <int QX, int R, int V, bool MS, bool NZ, int PF, bool FR>
__device__ __forceinline__ void unit_run(const Phi4StepArgs &A, int unit, FrameAcc &fa, uint32_t slo, uint32_t shi) {
    constexpr int RS = 64 / QX;  // row sets per wave
    // x-segments fastest, then y-groups: the waves that share a row's segment
    // edges (MS) and the y-halo rows are consecutive units, i.e. the same or
    // the adjacent block on the same XCD, so those lines are L2 hits
    const int xs = unit % A.nxseg;
    const int rest = unit / A.nxseg;
    const int yg = rest % A.nyg;
    const int zk = rest / A.nyg;
    const int zbeg = A.zlo + zk * A.zstep;
    const int zend = min(zbeg + A.zc, A.zhi);

    const int Lx = A.Lx, Ly = A.Ly;
    const size_t plane = (size_t)Lx * (size_t)Ly;
    const uint32_t pbytes = (uint32_t)(plane * sizeof(float));
    const uint32_t qplane = (uint32_t)(plane >> 2);
    Lane<QX, R, V> L;
    L.lane = threadIdx.x & 63;
    const int xq = L.lane & (QX - 1);
    const int rsid = L.lane / QX;
    const int xspan = xs * (4 * QX * V);     // first site of this wave's x-span
    const int x = xspan + 4 * xq;            // segment 0; segment v adds 4*QX*v
    // lanes whose rows fall past Ly (narrow lattices: a wave covers more rows
    // than Ly has) read row 0 and store nothing; shuffles stay inside their
    // x-segment group, which is idle as a whole.
    const int y0r = yg * (RS * R) + rsid * R;
    L.rows_ok = y0r < Ly;
    const int y0 = L.rows_ok ? y0r : 0;
    const int ym = y0 == 0 ? Ly - 1 : y0 - 1;
    const int yp = (y0 + R == Ly) ? 0 : y0 + R;
    const int xl = (xspan == 0 ? Lx : xspan) - 1;                                 // MS: left of the span
    const int xr = (xspan + 4 * QX * V == Lx) ? 0 : xspan + 4 * QX * V;           // MS: right of the span
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int xv = x + 4 * QX * v;
            L.voff[r * V + v] = (uint32_t)(((y0 + r) * Lx + xv) * 4);
            L.qoff[r * V + v] = (uint32_t)(((y0 + r) * Lx + xv) >> 2);
        }
        L.vl[r] = (uint32_t)(((y0 + r) * Lx + xl) * 4);
        L.vr[r] = (uint32_t)(((y0 + r) * Lx + xr) * 4);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
        L.vm[v] = (uint32_t)((ym * Lx + x + 4 * QX * v) * 4);
        L.vp[v] = (uint32_t)((yp * Lx + x + 4 * QX * v) * 4);
    }

    Slot<R, V> S0, S1, S2;
    load_slot<QX, R, V>(A, L, S0, zbeg - 1, false, plane, pbytes);
    load_slot<QX, R, V>(A, L, S1, zbeg, true, plane, pbytes);
    // three-slot register queue, unrolled so no rotation moves are needed.
    // PF 3: packed-f32 site arithmetic, plain stores; 4: non-temporal output
    // stores, for lattices whose two fields exceed the Infinity Cache (512^3
    // 199.7 -> 186.8 us, 1024^3 1606 -> 1570 us; at 256^3 it costs 21.6 ->
    // 30.0 us, profiles/r01/sw*_ntstore.log); 7: sc0 sc1 (write-through)
    // output stores, which leave the XCD's L2 at once instead of evicting the
    // input rows other waves re-read (guide table "stores of each flavour"),
    // the default for full-row waves.  PF 1: scalar site arithmetic (narrow rows).
    constexpr bool PK = PF >= 3;
    constexpr int SAUX = PF == 4 ? 2 : PF == 7 ? 17 : 0;
    for (int z = zbeg; z < zend; z += 3) {
        plane_step<QX, R, V, MS, NZ, PK, SAUX, FR>(A, L, S0, S1, S2, z, zend, plane, pbytes, qplane, slo, shi, fa);
        if (z + 1 >= zend) break;
        plane_step<QX, R, V, MS, NZ, PK, SAUX, FR>(A, L, S1, S2, S0, z + 1, zend, plane, pbytes, qplane, slo, shi, fa);
        if (z + 2 >= zend) break;
        plane_step<QX, R, V, MS, NZ, PK, SAUX, FR>(A, L, S2, S0, S1, z + 2, zend, plane, pbytes, qplane, slo, shi, fa);
    }
}

// Buffer i of three-buffer frames by a select of scalars: the three are
// separate kernel arguments (a select over an array's elements folds into a
// dynamic index, and that puts the argument block in private memory).
__device__ __forceinline__ uintptr_t pick_buf(const Phi4StepArgs &A, int i) {
    const uintptr_t b0 = reinterpret_cast<uintptr_t>(A.buf0), b1 = reinterpret_cast<uintptr_t>(A.buf1),
                    b2 = reinterpret_cast<uintptr_t>(A.buf2);
    return i == 0 ? b0 : (i == 1 ? b1 : b2);
}

__device__ __forceinline__ float unord_f32_dev(uint32_t o);
__device__ __forceinline__ void frame_decide(FrameCtl &c, float T, float V, int fired, int flag);

// Device frames (FrameFoldArgs, sq_internal.h): the first fused launch of a
// frame takes the previous frame's end -- the work of phi4_frame_end_kernel
// without its launch.  Every block folds the kStabSlots-slot records into LDS
// (u64 / u32 LDS atomic maxima: the same maxima as the end kernel's serial
// fold), one thread applies the stability rule and frame_decide, and the block
// runs with the coefficients and, when the verdict is unstable, the snapshot
// as its input (the frame's rollback: the rejected field is never read
// again, and the snapshot stays the start of the retried frame, so it is not
// stored again).  Block 0 publishes the controller state, the folded records
// and the verdict.  Any launch with clr.md set first zeroes that record set
// (the one the previous launch folded; no block of this launch reads it).
//
// What a frame instance takes from the device instead of its launch
// arguments: a few scalars, so the kernel's argument block is copied once at
// the end (frame_args) -- a copy modified field by field across frame_fold's
// barriers and loops stayed a 360-byte private-memory object (round 4).
struct FrameOv {  // pointers as integers: the struct then stays in registers
    uintptr_t in, out, snap;
    float h, sig, sigq;
};

template <bool FR>
__device__ __forceinline__ void frame_fold(const Phi4StepArgs &A, FrameOv &ov) {
    if constexpr (FR) {
        if (A.clr.md != nullptr) {
            const int gt = (int)(blockIdx.x * blockDim.x + threadIdx.x), gs = (int)(gridDim.x * blockDim.x);
            for (int q = gt; q < A.clr.n; q += gs) {
                A.clr.md[q] = 0ull;
                A.clr.am[q] = 0u;
            }
            if (gt == 0) *A.clr.flag = 0;
        }
        if (A.fold.cin == nullptr) return;
        __shared__ unsigned long long sK[kFoldMaxL];
        __shared__ unsigned int sAm[kFoldMaxL];
        __shared__ float sCoef[3];
        __shared__ int sSt, sBuf[2];
        const int L = A.fold.L;
        for (int j = (int)threadIdx.x; j < L; j += (int)blockDim.x) {
            sK[j] = 0ull;
            sAm[j] = 0u;
        }
        __syncthreads();
        for (int q = (int)threadIdx.x; q < L * kStabSlots; q += (int)blockDim.x) {
            atomicMax(&sK[q / kStabSlots], A.fold.md[q]);
            atomicMax(&sAm[q / kStabSlots], A.fold.am[q]);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            FrameCtl c = *A.fold.cin;
            float T = c.T, V = c.V;
            int fired = -1;
            for (int j = 0; j < L; ++j) {  // stab_rule (sq_api.cpp)
                const float M = unord_f32_dev((uint32_t)(sK[j] >> 32)), D = __uint_as_float((uint32_t)sK[j]);
                const float Aj = __uint_as_float(sAm[j]);
                const bool f = M > T && D > V;
                T = M;
                V = V < Aj ? Aj : V;
                if (f) {
                    fired = j;
                    break;
                }
            }
            frame_decide(c, T, V, fired, *A.fold.flag);
            sCoef[0] = c.coef[0];
            sCoef[1] = c.coef[1];
            sCoef[2] = c.coef[2];
            sSt = c.stable;
            sBuf[0] = c.bs;
            sBuf[1] = c.bw0;
            if (blockIdx.x == 0) {
                *A.fold.cout = c;
                if (A.fold.stable_out) *A.fold.stable_out = c.stable;
                if (A.fold.dtau_out) *A.fold.dtau_out = c.dtau;
            }
        }
        if (blockIdx.x == 0)
            for (int j = (int)threadIdx.x; j < L; j += (int)blockDim.x) {
                A.fold.rec[j] = unord_f32_dev((uint32_t)(sK[j] >> 32));
                A.fold.rec[L + j] = __uint_as_float((uint32_t)sK[j]);
                A.fold.rec[2 * L + j] = __uint_as_float(sAm[j]);
            }
        __syncthreads();
        // every field assigned unconditionally, by selects: stores to different
        // fields on different paths get sunk into one store through a selected
        // address, and the struct then lives in private memory
        const bool tri = A.buf0 != nullptr, st = sSt != 0;
        const uintptr_t snapv = reinterpret_cast<uintptr_t>(A.fold.snap) -
                                sizeof(float) * (size_t)A.gz * (size_t)A.Lx * (size_t)A.Ly;  // padded view
        const uintptr_t in = tri ? pick_buf(A, sBuf[0]) : (st ? ov.in : snapv);
        const uintptr_t out = tri ? pick_buf(A, sBuf[1]) : ov.out;
        const uintptr_t sn = (!tri && !st) ? uintptr_t(0) : ov.snap;
        ov.in = in;
        ov.out = out;
        ov.snap = sn;
        ov.h = sCoef[0];
        ov.sig = sCoef[1];
        ov.sigq = sCoef[2];
    }
}

// The arguments a launch runs with.  Frame instances under device control
// (FR) take {h, sig, sigq} from the frame controller (dcoef: the Δτ adapt of
// tauhost.c:523-541 the previous frame's end may have made), three-buffer
// frames their in / out buffers (tctl), and a frame's first launch the
// previous frame's end (frame_fold).
// Three-buffer frames with the host's guess of a launch's buffers
// (Phi4StepArgs::tspec, SPEC kernels): the launch starts on the guessed in /
// out -- its first plane loads do not wait for the controller's words -- and
// the kernel compares them with the controller's choice once its first loads
// are in flight (TriCheck), starting over on the real buffers when the guess
// was wrong (only after an unstable frame).
struct TriCheck {
    uintptr_t in, out;
    bool on;
};

template <bool FR, bool SPEC = false>
__device__ __forceinline__ Phi4StepArgs frame_args(const Phi4StepArgs &A0, TriCheck *chk = nullptr) {
    if constexpr (FR) {
        FrameOv ov{reinterpret_cast<uintptr_t>(A0.in), reinterpret_cast<uintptr_t>(A0.out),
                   reinterpret_cast<uintptr_t>(A0.snap), A0.h, A0.sig, A0.sigq};
        if (A0.dcoef != nullptr) {
            ov.h = A0.dcoef[0];
            ov.sig = A0.dcoef[1];
            ov.sigq = A0.dcoef[2];
        }
        if (A0.tctl != nullptr) {  // three-buffer device frames: launch tk's buffers
            const int bs = A0.tctl->bs, bw0 = A0.tctl->bw0, bw1 = A0.tctl->bw1;
            const int bi = A0.tk == 0 ? bs : ((A0.tk & 1) ? bw0 : bw1);
            const int bo = A0.tk == 0 ? bw0 : ((A0.tk & 1) ? bw1 : bw0);
            const uintptr_t in = pick_buf(A0, bi), out = pick_buf(A0, bo);
            if (SPEC && A0.tspec != 0) {  // keep the guess (A0.in / out); the kernel checks it
                chk->in = in;
                chk->out = out;
                chk->on = true;
            } else {
                ov.in = in;
                ov.out = out;
            }
        }
        frame_fold<FR>(A0, ov);
        Phi4StepArgs A = A0;
        A.in = reinterpret_cast<const float *>(ov.in);
        A.out = reinterpret_cast<float *>(ov.out);
        A.snap = reinterpret_cast<float *>(ov.snap);
        A.h = ov.h;
        A.sig = ov.sig;
        A.sigq = ov.sigq;
        return A;
    } else {
        return A0;
    }
}

// FR: a frame's launch (guard flag and stability records); the raw sq_step
// path compiles without that bookkeeping.
template <int QX, int R, int V, bool MS, bool NZ, int PF, bool FR>
__global__ __launch_bounds__(256) void phi4_step_kernel(const Phi4StepArgs A0) {
    const Phi4StepArgs A = frame_args<FR>(A0);
    const int nb = gridDim.x, b = blockIdx.x;
    const int lb = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;
    // the unit is wave-uniform: say so, so every descriptor stays scalar (T20)
    const int unit = __builtin_amdgcn_readfirstlane(lb * 4 + (int)(threadIdx.x >> 6));
    FrameAcc fa = frame_acc();
    if (unit < A.nunits) unit_run<QX, R, V, MS, NZ, PF, FR>(A, unit, fa, A.s_lo, A.s_hi);
    if constexpr (FR) {  // every wave of the block, finished or idle, reaches the flush
        __shared__ uint64_t sk[4];
        __shared__ uint32_t sa[4];
        frame_flush(A, fa, 0, sk, sa);
    }
}

// ----------------------------------------------------- two-step fusion ----
// Steps s and s+1 in one pass over the field (temporal blocking), for rows of
// Lx = 256 S sites: a single periodic slab, or the planes [zlo, zhi) of a slab
// whose input is valid on [zlo-2, zhi+2) (deep-halo blocks).  A block owns one
// 256-site x-segment [x0, x0+256) of kTbRows = 8 output rows [y0, y0+8) of a
// z-chunk [z0, z1).  Row wave w = 0..9 holds row y0-1+w of the segment (lane
// l: sites x0+4l..x0+4l+3).  Marching p over [z0-1, z1]:
//   1. every row wave loads input plane p+1 (its row and both y-halo rows),
//      and, when S > 1, plane p's two sites just outside the segment (lane 0
//      x0-1, lane 63 x0+256), and updates its row of plane p by step s ->
//      T(p) (the same site update, noise keyed by step s); T stays in a
//      3-plane register queue and is published in LDS slot p % 3;
//   2. S > 1: the x-halo wave (w = 10) updates the 16 sites (x0-1 | x0+256,
//      y0..y0+7) of plane p by step s from its own 5-point loads and publishes
//      them in LDS -- the x-neighbours of the segment's edge lanes in step s+1;
//   3. barrier;
//   4. row waves 1..8 update their row of plane p-1 by step s+1 from T(p-2),
//      T(p-1), T(p) (registers), the y-neighbour rows of T(p-1) (LDS) and, at
//      the segment edges, the x-halo sites (LDS; S = 1: the DPP rotation wraps
//      the periodic row), and store it with sc0 sc1.
// Rows y0-1, y0+8, planes z0-1, z1 and the x-halo sites of T are recomputed
// by the blocks that own them too: the counter-based noise makes them
// bit-identical, so the result equals two single steps bit for bit.  HBM
// traffic: one read and one write of the field per two steps.  Three LDS
// slots: a slot is rewritten two barriers after its last reader passed the
// barrier before its read.
// Measured and not adopted (profiles/r02/): loads two planes ahead with the
// z-1 neighbour read from a fourth LDS slot (90 VGPRs at S = 1, 109 at S > 1):
// 256^3 21.4 -> 21.8 us per step, 512^3 197 -> 330 us -- the kernel is not
// waiting on its loads.
// Wave priority by march progress (Phi4StepArgs::prio): the two blocks that
// share a CU start together, and the arbiter's age order lets one finish far
// ahead, leaving the other alone on the CU for the rest of the launch (block
// stamps: ends 20..36 us at 256^3, 19-20 us alone).  A block that is behind
// gets the higher priority: 3 in its first quarter of planes, down to 0 in
// its last (4 levels beat 2: 3 then 0 by halves, 512^3 139-140 vs 136-137
// us/step).  q = quarter (0..3), wave-uniform.
// Block stamps (Phi4StepArgs::stamps): [2b, 2b+1] the constant 100 MHz clock
// (s_memrealtime) at the block's start and end, [2 nb + 2b, 2 nb + 2b + 1] the
// shader-clock counter (s_memtime) at the same two points: their ratio is the
// clock the block ran at (the chip's power management moves it; sq_phi4_block_clocks).
__device__ __forceinline__ void block_stamp(const Phi4StepArgs &A, int at) {
    const unsigned long long rt = __builtin_amdgcn_s_memrealtime(), ct = __builtin_amdgcn_s_memtime();
    A.stamps[2 * blockIdx.x + at] = rt;
    A.stamps[2 * gridDim.x + 2 * blockIdx.x + at] = ct;
}
// the end, once every wave is done
__device__ __forceinline__ void block_end_stamp(const Phi4StepArgs &A) {
    if (A.stamps == nullptr) return;
    __syncthreads();
    if (threadIdx.x == 0) block_stamp(A, 1);
}

// The march's quarter boundaries: plane p (p = z0-1 .. z1) is in quarter
// floor(4 (p - z0 + 1) / span) = (p >= t[0]) + (p >= t[1]) + (p >= t[2]),
// t[k] = z0 - 1 + ceil((k+1) span / 4) -- three compares per iteration instead
// of a signed division.
struct PrioQ {
    int t0, t1, t2;
    __device__ __forceinline__ PrioQ(int z0, int span)
        : t0(z0 - 1 + (span + 3) / 4), t1(z0 - 1 + (2 * span + 3) / 4), t2(z0 - 1 + (3 * span + 3) / 4) {}
    __device__ __forceinline__ int q(int p) const { return (p >= t0) + (p >= t1) + (p >= t2); }
};

__device__ __forceinline__ void prio_by_progress(int q) {
    switch (q) {
    case 0: __builtin_amdgcn_s_setprio(3); break;
    case 1: __builtin_amdgcn_s_setprio(2); break;
    case 2: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
    }
}

// A fused launch's block -> (y-band, x-segment, z-chunk).  Blocks are dealt
// XCD-contiguously (consecutive ids round-robin over the 8 XCDs, so the
// y-adjacent blocks sharing halo rows meet in one XCD's L2); a gated launch
// (Phi4StepArgs::gate) appends its thin rim chunks after the n_reg core blocks,
// so they are dispatched last, and maps them without the swizzle.
struct TbBlock {
    int yb, xs, z0, z1;
    bool gated;
};
template <bool WIDE>
__device__ __forceinline__ TbBlock tb_block(const Phi4StepArgs &A, int b, int nb) {
    TbBlock t;
    t.gated = A.gate != nullptr && b >= A.n_reg;
    const int nbr = A.gate != nullptr ? A.n_reg : nb;
    const int lb = t.gated ? b - A.n_reg : ((nbr & 7) == 0 ? (b & 7) * (nbr >> 3) + (b >> 3) : b);
    t.yb = lb % A.nyg;
    const int rest = lb / A.nyg;
    t.xs = WIDE ? rest % A.nxseg : 0;
    const int zk = WIDE ? rest / A.nxseg : rest;
    if (t.gated) {
        const int r0 = zk >= A.ntz ? A.thi0 : A.tlo0;
        t.z0 = r0 + (zk % A.ntz) * A.tzc;
        t.z1 = min(t.z0 + A.tzc, r0 + A.tlen);
    } else {
        const int r0 = A.zlo + (zk / A.nzr) * A.zstep;  // this chunk's range
        t.z0 = r0 + (zk % A.nzr) * A.zc;
        t.z1 = min(t.z0 + A.zc, r0 + A.zlen);
    }
    return t;
}

// A gated block waits for the exchange (its chunk reads ghost planes): one
// thread polls the gate word with acquire loads at agent scope (no stream hop,
// no L2 line kept: the word is fine-grained memory written behind the exchange
// on stream B), the block follows through a barrier, and every wave acquires
// before its first load of the ghost planes.  Bounded: after kGateSpinMax
// polls the block gives up and flags gate_err (the host reports it), so a lost
// exchange ends as an error, not a hung grid.
constexpr unsigned int kGateSpinMax = 1u << 24;  // ~1 s of s_sleep 2
// Returns false when the wait gave up: the block then stores nothing (its
// ghost planes are stale), so a timed-out exchange leaves the chunk's previous
// contents, never values computed from an unfinished exchange.
__device__ __forceinline__ bool tb_gate_wait(const Phi4StepArgs &A) {
    __shared__ int s_gate_ok;
    if (threadIdx.x == 0) {
        unsigned int n = 0;
        int ok = 1;
        while (__hip_atomic_load(A.gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < A.gate_seq) {
            __builtin_amdgcn_s_sleep(2);
            if (++n >= kGateSpinMax) {
                if (A.gate_err) __hip_atomic_fetch_or(A.gate_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
        }
        s_gate_ok = ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return s_gate_ok != 0;
}

constexpr int kTbRows = 8;
constexpr int kTbWaves = kTbRows + 2;  // row waves; S > 1 adds the x-halo wave

// Padded plane of local plane zl: the periodic slab wraps (|overflow| <= 2),
// a slab of a decomposition reads its ghost zone.
__device__ __forceinline__ int tb_pidx(const Phi4StepArgs &A, int zl) {
    if (A.periodic) zl = zl < 0 ? zl + A.nz : (zl >= A.nz ? zl - A.nz : zl);
    return zl + A.gz;
}

// qz: the Philox quad index of the plane's first site (global z * plane / 4)
template <bool NZ>
__device__ __forceinline__ f32x4n tb_noise(const Phi4StepArgs &A, uint32_t qz, uint32_t qoff, uint32_t slo,
                                           uint32_t shi) {
    f32x4n xi;
    if constexpr (NZ) {
        u32x4 c[1];
        c[0] = u32x4{qz + qoff, kStreamField << 24, slo, shi};
        philox_field<1>(c, A.k0, A.k1);
        box_muller_q(c[0].x, c[0].y, xi.a, xi.b);  // scaled by 1/sqrt(2 ln 2); A.sigq carries the factor
        box_muller_q(c[0].z, c[0].w, xi.c, xi.d);
    } else {
        xi = f32x4n{0.f, 0.f, 0.f, 0.f};
    }
    return xi;
}

// One plane of a row wave's inputs: its row and the row's two y-neighbours.
// The x-halo wave keeps the centre values of its sites in row.x, so the two
// roles share one register queue.
struct TbIn {
    float4 row, hm, hp;
};

// Per-block constants of the march.
typedef float f32x4v __attribute__((ext_vector_type(4)));

struct TbCtx {
    size_t plane;
    uint32_t pbytes, qplane;
    __amdgpu_buffer_rsrc_t rin, rout;  // WH: one descriptor over each whole padded buffer
    // byte offsets in a plane and the Philox quad offset.  Row waves: voff
    // their row, vm / vp its y-neighbours, vex the site just outside the
    // segment (lane 0 left, lane 63 right).  x-halo wave lanes (sharing the
    // registers): voff the site, vm / vp its y-neighbours, vex / vx2 its x-1 / x+1.
    uint32_t voff, vm, vp, vex, vx2, qoff;
    uint32_t slo, shi, slo1, shi1;
    uint32_t qwrap;      // Lz_global * plane / 4: where the Philox quad base wraps
    f32x2 m2v;           // {m2, m2}, pinned in VGPRs (site_update4)
    int swrap_at;        // WH, periodic: the plane p at which plane p+1's input wraps to local 0
    int z0, z1, w, lane;
    bool outw;
    int snapw;  // FR: an output row wave of a launch that stores the frame's snapshot
    // STG (sq_phi4_run.hip, phi4_tb2_stage_kernel): the P2P staging slot, whose
    // first stg_g planes take output planes [0, stg_g) and next stg_g planes
    // output planes [stg_hi, stg_hi + stg_g)
    __amdgpu_buffer_rsrc_t rstg;
    int stg_g, stg_hi;
};

// Wave-uniform per-plane scalars carried through the march instead of being
// recomputed from p every plane (the kernel is issue-bound, scalar
// instructions included): the byte offsets of planes p+1 and p in the padded
// input (WH) and the Philox quad bases of planes p (step s) and p-1 (step s+1).
struct TbRun {
    uint32_t snext, scur;
    uint32_t qz, qzm;
};

__device__ __forceinline__ float tb_site(float phi, float xm, float xp, float ym, float yp, float zm, float zp,
                                         float xi, const Phi4StepArgs &A, bool nz) {
    const float nb = ((xm + xp) + (ym + yp)) + (zm + zp);
    const float lap = __builtin_fmaf(-6.0f, phi, nb);
    const float g = __builtin_fmaf(A.lam6, phi * phi, A.m2);
    const float drift = __builtin_fmaf(-phi, g, lap);
    const float det = __builtin_fmaf(A.h, drift, phi);
    const float v = nz ? __builtin_fmaf(A.sigq, xi, det) : det;
    return fmaxf(fminf(v, A.clampv), -A.clampv);
}

// One plane of the march.  Row waves: I0 (p-1), I1 (p), I2 (p+1, loaded
// here); T0 (p-2), T1 (p-1), T2 (p, computed here).  The x-halo wave: the
// centres of its sites at the same planes in row.x.
// J = (p - (z0 - 1)) % 3, the unroll position: plane p's LDS slot (any
// block-wide bijection of the three planes in flight works, and this one is a
// compile-time constant).  WH: the padded buffers fit one 32-bit descriptor
// each, and the plane is the buffer unit's scalar offset (one s_mul per plane
// instead of the 64-bit descriptor base arithmetic).
// P2 (256-site rows; SQ_TB2_SYNC=p2p): no block barrier per plane.
// Each wave publishes the last plane whose step-s row it wrote (prog[w],
// workgroup-scope release) and, before overwriting a slot, waits until its one
// or two row neighbours have published the plane before: they then have both
// written the slot it reads next and finished reading the slot it overwrites
// (three slots, a neighbour at most one plane behind).  A wave waits for two
// waves, not for the block.
__device__ __forceinline__ void tb_wait_nbrs(const int *prog, int w, int need) {
    const int wl = w > 0 ? w - 1 : w + 1, wr = w < kTbWaves - 1 ? w + 1 : w - 1;
    for (;;) {
        const int a = __hip_atomic_load(&prog[wl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int b = __hip_atomic_load(&prog[wr], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(min(a, b)) >= need) break;
        __builtin_amdgcn_s_sleep(1);
    }
}

template <bool NZ, bool WIDE, bool FR, bool WH, int J, bool P2 = false, int LAUX = 0, bool STG = false>
__device__ __forceinline__ void tb_plane(const Phi4StepArgs &A, const TbCtx &K, TbRun &R, int p, const TbIn &I0,
                                         const TbIn &I1, TbIn &I2, const float4 &T0, const float4 &T1, float4 &T2,
                                         float4 (*lds)[kTbWaves][64], float (*tx)[kTbWaves][2], FrameAcc &f1,
                                         FrameAcc &f2, float *bmx, int *prog = nullptr) {
    constexpr int sl = J, sp = (J + 2) % 3;  // slots of planes p and p-1
    __amdgpu_buffer_rsrc_t rs, rc;
    uint32_t ss = 0, sc = 0;
    if constexpr (WH) {
        rs = rc = K.rin;
        ss = R.snext;
        sc = R.scur;
    } else {
        rs = plane_rsrc(A.in, tb_pidx(A, p + 1), K.plane, K.pbytes);
        // S > 1: plane p's values at the segment's outer x-neighbours (lane 0 x0-1,
        // lane 63 x0+256) and at the x-halo sites' in-plane neighbours are loaded
        // in the iteration that uses them, like plane p+1 itself
        rc = plane_rsrc(A.in, tb_pidx(A, p), K.plane, K.pbytes);
    }
    if (!WIDE || K.w < kTbWaves) {
        I2.row = bload4<LAUX>(rs, K.voff, ss);
        I2.hm = bload4<LAUX>(rs, K.vm, ss);
        I2.hp = bload4<LAUX>(rs, K.vp, ss);
        float ex = 0.f;
        if constexpr (WIDE) ex = bload1(rc, K.vex, sc);
        const f32x4n xa = tb_noise<NZ>(A, R.qz, K.qoff, K.slo, K.shi);
        float lft, rgt;
        if constexpr (WIDE) {
            lft = from_left_lane_or(I1.row.w, ex);
            rgt = from_right_lane_or(I1.row.x, ex);
        } else {
            lft = from_left_lane(I1.row.w);
            rgt = from_right_lane(I1.row.x);
        }
        float mp1;
        T2 = site_update4<NZ>(I1.row, lft, rgt, I1.hm, I1.hp, I0.row, I2.row, xa, A, A.fin != 0, K.m2v, &mp1);
        if constexpr (FR) {
            // step s's records over the block's own rows and planes only: the
            // halo rows and chunk-edge planes are recomputed copies of sites
            // another block owns and records (the records are maxima, so the
            // copies never changed them)
            if (K.outw && p >= K.z0 && p < K.z1) frame_sites<NZ, true>(A, f1, T2, I1.row, xa, bmx, true, mp1);
            // the frame's snapshot: each output row's input at its owned planes, once
            if (K.snapw != 0 && p + 1 >= K.z0 && p + 1 < K.z1)
                __builtin_nontemporal_store(
                    (f32x4v){I2.row.x, I2.row.y, I2.row.z, I2.row.w},
                    reinterpret_cast<f32x4v *>(reinterpret_cast<char *>(A.snap) + (size_t)(p + 1) * K.pbytes + K.voff));
        }
        if constexpr (P2) tb_wait_nbrs(prog, K.w, p - 1);
        lds[sl][K.w][K.lane] = T2;
    } else {
        // the x-halo wave: step s at its 16 sites of plane p
        I2.row.x = bload1(rs, K.voff, ss);
        const float xm = bload1(rc, K.vex, sc), xp = bload1(rc, K.vx2, sc), ym = bload1(rc, K.vm, sc),
                    yp = bload1(rc, K.vp, sc);
        const f32x4n n = tb_noise<NZ>(A, R.qz, K.qoff, K.slo, K.shi);
        // lanes 0..7 hold x0-1 (component 3 of its quad), 8..15 x0+256 (component 0)
        const float xi = K.lane >= 8 ? n.a : n.d;
        const float t = tb_site(I1.row.x, xm, xp, ym, yp, I0.row.x, I2.row.x, xi, A, NZ);
        if (K.lane < 16) tx[sl][(K.lane & 7) + 1][K.lane >> 3] = t;
    }
    if constexpr (P2) {
        if (K.lane == 0) __hip_atomic_store(&prog[K.w], p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        __syncthreads();
    }
    if (K.outw && p > K.z0) {
        const f32x4n xb = tb_noise<NZ>(A, R.qzm, K.qoff, K.slo1, K.shi1);
        const float4 up = lds[sp][K.w - 1][K.lane], dn = lds[sp][K.w + 1][K.lane];
        float lft, rgt;
        if constexpr (WIDE) {
            const float2 e = *reinterpret_cast<const float2 *>(&tx[sp][K.w][0]);  // one broadcast LDS read
            lft = from_left_lane_or(T1.w, e.x);
            rgt = from_right_lane_or(T1.x, e.y);
        } else {
            lft = from_left_lane(T1.w);
            rgt = from_right_lane(T1.x);
        }
        // step s+1 reads step s's guarded output: always finite
        float mp2;
        const float4 o = site_update4<NZ>(T1, lft, rgt, up, dn, T0, T2, xb, A, true, K.m2v, &mp2);
        if constexpr (FR) frame_sites<NZ, true>(A, f2, o, T1, xb, bmx + 1, true, mp2);
        if constexpr (WH) {
            // the plane offset in the VGPR offset, soffset 0: see bstore4
            bstore4<17>(K.rout, K.voff + (uint32_t)(p - 1 + A.gz) * K.pbytes, o);
            if constexpr (STG) {  // an edge plane: also into the staging slot (write-through, as the field)
                const int q = p - 1;
                if (q < K.stg_g) bstore4<17>(K.rstg, K.voff + (uint32_t)q * K.pbytes, o);
                if (q >= K.stg_hi) bstore4<17>(K.rstg, K.voff + (uint32_t)(q - K.stg_hi + K.stg_g) * K.pbytes, o);
            }
        } else {
            const __amdgpu_buffer_rsrc_t ws = plane_rsrc(A.out, p - 1 + A.gz, K.plane, K.pbytes);
            bstore4<17>(ws, K.voff, o);
        }
    }
    // advance to plane p+1
    R.qzm = R.qz;
    const uint32_t q = R.qz + K.qplane;
    R.qz = q == K.qwrap ? 0u : q;
    if constexpr (WH) {
        R.scur = R.snext;
        R.snext = p == K.swrap_at ? (uint32_t)A.gz * K.pbytes : R.snext + K.pbytes;
    }
}

// WPE: waves per SIMD the registers are budgeted for (S > 1: 6 = two 11-wave
// blocks per CU at <= 80 VGPRs, spilling 9; 1 = unconstrained, 85 VGPRs).
// 256-wide rows: 65 VGPRs, two 10-wave blocks per CU.  A 64-VGPR budget
// (three blocks per CU) measured slower at every z-chunk
// (profiles/r01/fuse2_sweep.log).
template <bool NZ, bool WIDE, int WPE, bool FR, bool WH, bool P2 = false>
__global__ __launch_bounds__((kTbWaves + (WIDE ? 1 : 0)) * 64)
__attribute__((amdgpu_waves_per_eu(WPE))) void phi4_tb2_kernel(const Phi4StepArgs A0) {
    static_assert(!P2 || !WIDE, "neighbour sync: 256-site rows");
    TriCheck chk{0, 0, false};
    Phi4StepArgs A = frame_args<FR, true>(A0, &chk);
    const int nb = gridDim.x, b = blockIdx.x;
    if (A.stamps != nullptr && threadIdx.x == 0) block_stamp(A, 0);
    // y-bands fastest, then x-segments, then z-chunks, consecutive blocks on
    // one XCD: the blocks sharing halo rows, edge columns and chunk-edge planes
    // meet in that XCD's L2 (tb_block)
    const TbBlock tbk = tb_block<WIDE>(A, b, nb);
    const int yb = tbk.yb, xs = tbk.xs;
    const int Lx = A.Lx, Ly = A.Ly;
    const int x0 = 256 * xs;
    TbCtx K;
    K.w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    K.lane = threadIdx.x & 63;
    K.outw = K.w >= 1 && K.w <= kTbRows;
    K.z0 = tbk.z0;
    const int z1 = tbk.z1;
    K.snapw = __builtin_amdgcn_readfirstlane((FR && A.snap != nullptr && K.outw) ? 1 : 0);
    K.z1 = z1;
    K.plane = (size_t)Lx * (size_t)Ly;
    K.pbytes = (uint32_t)(K.plane * sizeof(float));
    K.qplane = (uint32_t)(K.plane >> 2);
    if constexpr (WH) {
        const int nbytes = (int)((uint32_t)(A.nz + 2 * A.gz) * K.pbytes);  // < 2^31 (phi4_tb2_launch)
        K.rin = __builtin_amdgcn_make_buffer_rsrc((void *)A.in, (short)0, nbytes, 0x00020000);
        K.rout = __builtin_amdgcn_make_buffer_rsrc((void *)A.out, (short)0, nbytes, 0x00020000);
    }
    K.qwrap = (uint32_t)A.Lzg * K.qplane;  // < 2^32 quads (create_phi4)
    K.m2v = f32x2{A.m2, A.m2};
    asm volatile("" : "+v"(K.m2v));  // opaque: kept in VGPRs, not rematerialised from SGPRs per update
    // periodic: plane p+1 = nz is local plane 0 (tb_pidx); p never reaches it otherwise
    K.swrap_at = A.periodic ? A.nz - 2 : INT_MIN;  // slabs: p < 0 in ghost zones, never INT_MIN
    const unsigned long long s0 = ((unsigned long long)A.s_hi << 32) | A.s_lo, s1 = s0 + 1;
    K.slo = (uint32_t)s0;
    K.shi = (uint32_t)(s0 >> 32);
    K.slo1 = (uint32_t)s1;
    K.shi1 = (uint32_t)(s1 >> 32);
    const int xl = (x0 == 0 ? Lx : x0) - 1, xr = x0 + 256 == Lx ? 0 : x0 + 256;  // just outside the segment
    auto wrapy = [Ly](int y) { return y < 0 ? y + Ly : (y >= Ly ? y - Ly : y); };
    if (!WIDE || K.w < kTbWaves) {
        const int y = wrapy(yb * kTbRows - 1 + K.w);
        const int ym = wrapy(y - 1), yp = wrapy(y + 1);
        K.voff = (uint32_t)((y * Lx + x0 + 4 * K.lane) * 4);
        K.vm = (uint32_t)((ym * Lx + x0 + 4 * K.lane) * 4);
        K.vp = (uint32_t)((yp * Lx + x0 + 4 * K.lane) * 4);
        K.vex = (uint32_t)((y * Lx + (K.lane == 63 ? xr : xl)) * 4);
        K.vx2 = 0;
        K.qoff = (uint32_t)((y * Lx + x0 + 4 * K.lane) >> 2);
    } else {  // x-halo wave lanes 0..7: (x0-1, y0+l); 8..15: (x0+256, y0+l-8); the rest repeat lane 0
        const int l = K.lane < 16 ? K.lane : 0;
        const int y = wrapy(yb * kTbRows + (l & 7)), ym = wrapy(y - 1), yp = wrapy(y + 1);
        const int xe = (l >> 3) ? xr : xl;
        const int xem = xe == 0 ? Lx - 1 : xe - 1, xep = xe == Lx - 1 ? 0 : xe + 1;
        K.voff = (uint32_t)((y * Lx + xe) * 4);
        K.vex = (uint32_t)((y * Lx + xem) * 4);
        K.vx2 = (uint32_t)((y * Lx + xep) * 4);
        K.vm = (uint32_t)((ym * Lx + xe) * 4);
        K.vp = (uint32_t)((yp * Lx + xe) * 4);
        K.qoff = (uint32_t)((y * Lx + xe) >> 2);
    }
    __shared__ float4 lds[3][kTbWaves][64];
    __shared__ float tx[WIDE ? 3 : 1][kTbWaves][2];

    if (tbk.gated && !tb_gate_wait(A)) return;  // a rim chunk: its input's ghost planes come with the exchange
    TbIn I0, I1, I2;
    auto prologue = [&]() {
        const __amdgpu_buffer_rsrc_t r0 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 2), K.plane, K.pbytes);
        const __amdgpu_buffer_rsrc_t r1 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 1), K.plane, K.pbytes);
        if (!WIDE || K.w < kTbWaves) {
            I0.row = bload4(r0, K.voff);
            I0.hm = I0.hp = I0.row;
            I1.row = bload4(r1, K.voff);
            I1.hm = bload4(r1, K.vm);
            I1.hp = bload4(r1, K.vp);
        } else {
            I0.row = make_float4(bload1(r0, K.voff), 0.f, 0.f, 0.f);
            I1.row = make_float4(bload1(r1, K.voff), 0.f, 0.f, 0.f);
            I0.hm = I0.hp = I1.hm = I1.hp = I0.row;
        }
    };
    prologue();
    if constexpr (FR) {
        // the host's guess of this launch's buffers against the controller's
        // (wave-uniform: scalar loads of one FrameCtl); wrong only after an
        // unstable frame: start over on the real ones
        if (chk.on && (chk.in != reinterpret_cast<uintptr_t>(A.in) || chk.out != reinterpret_cast<uintptr_t>(A.out))) {
            A.in = reinterpret_cast<const float *>(chk.in);
            A.out = reinterpret_cast<float *>(chk.out);
            if constexpr (WH) {
                const int nbytes = (int)((uint32_t)(A.nz + 2 * A.gz) * K.pbytes);
                K.rin = __builtin_amdgcn_make_buffer_rsrc((void *)A.in, (short)0, nbytes, 0x00020000);
                K.rout = __builtin_amdgcn_make_buffer_rsrc((void *)A.out, (short)0, nbytes, 0x00020000);
            }
            prologue();
        }
    }
    float4 T0 = make_float4(0.f, 0.f, 0.f, 0.f), T1 = T0, T2 = T0;
    FrameAcc f1 = frame_acc(), f2 = frame_acc();  // steps s and s+1
    __shared__ float bmx[2];                        // the block's running maxima of both records (frame_sites)
    __shared__ unsigned long long fk[2];            // frame_flush2's block maxima
    __shared__ uint32_t fa[2];
    if constexpr (FR) {
        if (threadIdx.x < 2) {
            bmx[threadIdx.x] = -__builtin_inff();
            fk[threadIdx.x] = 0ull;
            fa[threadIdx.x] = 0u;
        }
        __syncthreads();
    }
    TbRun R;
    R.scur = (uint32_t)tb_pidx(A, K.z0 - 1) * K.pbytes;
    R.snext = (uint32_t)tb_pidx(A, K.z0) * K.pbytes;
    R.qz = (uint32_t)global_z(A, K.z0 - 1) * K.qplane;
    R.qzm = 0;  // plane z0-2: no step s+1 output there
    __shared__ int prog[P2 ? kTbWaves : 1];  // P2: the last plane each row wave published
    if constexpr (P2) {
        if (threadIdx.x < kTbWaves) prog[threadIdx.x] = K.z0 - 2;
        __syncthreads();
    }
    // three-plane queues unrolled three ways so no rotation moves are emitted
    const PrioQ pq(K.z0, z1 - K.z0 + 2);
    for (int p = K.z0 - 1; p <= z1; p += 3) {
        if (A.prio) prio_by_progress(pq.q(p));
        tb_plane<NZ, WIDE, FR, WH, 0, P2>(A, K, R, p, I0, I1, I2, T0, T1, T2, lds, tx, f1, f2, bmx, prog);
        if (p + 1 > z1) break;
        tb_plane<NZ, WIDE, FR, WH, 1, P2>(A, K, R, p + 1, I1, I2, I0, T1, T2, T0, lds, tx, f1, f2, bmx, prog);
        if (p + 2 > z1) break;
        tb_plane<NZ, WIDE, FR, WH, 2, P2>(A, K, R, p + 2, I2, I0, I1, T2, T0, T1, lds, tx, f1, f2, bmx, prog);
    }
    if constexpr (FR) frame_flush2(A, f1, f2, fk, fa);  // step s's records, then s+1's
    block_end_stamp(A);
}

// ------------------------------------------- pipelined two-step fusion ----
// phi4_tb2_kernel's block and work split (one 256-site x-segment of kTbRows
// output rows of a z-chunk; row wave w holds row y0-1+w; S > 1: the x-halo
// wave w = kTbWaves), with the loads decoupled from their use:
//   * a row wave loads only ITS OWN row of each input plane (waves 0 and
//     kTbWaves-1 also the row beyond, y0-2 / y0+9), one plane iteration
//     before the plane is needed (plane k+2 is issued in iteration k and first
//     read in iteration k+1), so the fetch overlaps a whole iteration of Philox
//     and stencil work instead of the few instructions between a load and its
//     use; in-plane y-neighbours come from an LDS ring of input planes, which
//     replaces the y-halo loads (3 loads per wave and plane -> 1);
//   * one barrier per iteration, at its end: iteration k publishes input plane
//     k+1 (in_lds) and step s of plane k (t_lds) and reads only what iteration
//     k-1 published, so step s+1 of plane k-1 follows step s of plane k with no
//     barrier between them.  Two slots per ring suffice: a slot is rewritten
//     one barrier after the iteration that last read it.
// Iteration k (z0-1 <= k <= z1): A = step s at plane k (T(k)), B = step s+1 at
// plane k-1 (rows y0..y0+7, k > z0), the same site_update4 calls with the same
// operands as phi4_tb2_kernel, so the result is bit-identical to two single
// steps.  Registers: own input rows of planes k-1..k+2 (I[4]) and T(k-2..k)
// (T[4]) by plane index mod 4, so the march is unrolled four ways and nothing
// rotates.
constexpr int kTpRows = kTbWaves + 2;  // in_lds rows: y0-2 .. y0+9
constexpr uint32_t kTpOob = 0x80000000u;  // a buffer offset past every descriptor's range (< 2^31 B): dropped

struct TpRun {
    uint32_t s2, s1;  // WH: byte offsets (in the padded input) of planes k+2 and k+1
    uint32_t qz, qzm; // Philox quad bases of planes k and k-1
};

// Advance the per-plane scalars from k to k+1.
template <bool WH>
__device__ __forceinline__ void tp_advance(const Phi4StepArgs &A, const TbCtx &K, TpRun &R, int k) {
    R.qzm = R.qz;
    const uint32_t q = R.qz + K.qplane;
    R.qz = q == K.qwrap ? 0u : q;
    if constexpr (WH) {
        R.s1 = R.s2;
        R.s2 = k + 3 == K.swrap_at ? (uint32_t)A.gz * K.pbytes : R.s2 + K.pbytes;
    }
}

// One plane iteration of a row wave.
template <bool NZ, bool WIDE, bool FR, bool WH, int J>
__device__ __forceinline__ void tp_row(const Phi4StepArgs &A, const TbCtx &K, TpRun &R, int k, bool xrow,
                                       uint32_t vxr, int xslot, float4 (&I)[4], float4 (&T)[4], float4 (&X)[2],
                                       float (&E)[2], float4 (*in_lds)[kTpRows][64], float4 (*t_lds)[kTbWaves][64],
                                       float (*tx)[kTbWaves][2], FrameAcc &f1, FrameAcc &f2, float *bmx) {
    constexpr int im = J, ic = (J + 1) & 3, ip = (J + 2) & 3, in2 = (J + 3) & 3;  // planes k-1, k, k+1, k+2
    constexpr int tc = J, tm = (J + 3) & 3, tmm = (J + 2) & 3;                    // T(k), T(k-1), T(k-2)
    constexpr int sc = J & 1, sn = (J + 1) & 1;  // ring slots of plane k / T(k) and of plane k+1 / T(k-1)
    const bool more = k < K.z1;                  // planes k+2 (rows) and k+1 (edges) are inputs of the chunk
    __amdgpu_buffer_rsrc_t r2, r1;
    uint32_t o2 = 0, o1 = 0;
    if constexpr (WH) {
        r2 = r1 = K.rin;
        o2 = R.s2;
        o1 = R.s1;
    } else {
        r2 = plane_rsrc(A.in, tb_pidx(A, k + 2), K.plane, K.pbytes);
        r1 = plane_rsrc(A.in, tb_pidx(A, k + 1), K.plane, K.pbytes);
    }
    // 1. prefetch plane k+2 (own row; waves 0 / 9 the row beyond) and, S > 1,
    //    plane k+1's site just outside the segment (lane 0 / 63).  Every
    //    vector-memory op of the march is issued unconditionally, the ones with
    //    nothing to do at an out-of-range offset (the buffer unit drops them), so
    //    every path has the same op sequence and the compiler's vmcnt waits
    //    stay exact: the wait for plane k+1 leaves plane k+2 in flight.
    I[in2] = bload4(r2, more ? K.voff : kTpOob, o2);
    X[sc] = bload4(r2, more ? vxr : kTpOob, o2);
    if constexpr (WIDE) E[sn] = bload1(r1, more ? K.vex : kTpOob, o1);
    // 2. plane k+1 has arrived (issued one iteration ago): publish it for the
    //    y-neighbour reads of iteration k+1, and, frames, snapshot it
    in_lds[sn][K.w + 1][K.lane] = I[ip];
    if (xrow) in_lds[sn][xslot][K.lane] = X[sn];
    if constexpr (FR) {  // each output row's input at its owned planes, once, nontemporal
        const bool sv = K.snapw != 0 && k + 1 >= K.z0 && k + 1 < K.z1;
        bstore4<2>(plane_rsrc(A.snap, k + 1, K.plane, K.pbytes), sv ? K.voff : kTpOob, I[ip]);
    }
    // 3. A: step s at plane k
    const f32x4n xa = tb_noise<NZ>(A, R.qz, K.qoff, K.slo, K.shi);
    const float4 up = in_lds[sc][K.w][K.lane], dn = in_lds[sc][K.w + 2][K.lane];
    float lft, rgt;
    if constexpr (WIDE) {
        lft = from_left_lane_or(I[ic].w, E[sc]);
        rgt = from_right_lane_or(I[ic].x, E[sc]);
    } else {
        lft = from_left_lane(I[ic].w);
        rgt = from_right_lane(I[ic].x);
    }
    float mp1;
    T[tc] = site_update4<NZ>(I[ic], lft, rgt, up, dn, I[im], I[ip], xa, A, A.fin != 0, K.m2v, &mp1);
    if constexpr (FR) {  // own rows and planes only, as phi4_tb2_kernel
        if (K.outw && k >= K.z0 && k < K.z1) frame_sites<NZ, true>(A, f1, T[tc], I[ic], xa, bmx, true, mp1);
    }
    t_lds[sc][K.w][K.lane] = T[tc];
    // 4. B: step s+1 at plane k-1 from T(k-2), T(k-1), T(k) and T(k-1)'s
    //    y-neighbours, published in iteration k-1
    const bool bw = K.outw && k > K.z0;
    float4 o = T[tc];  // stored at an out-of-range offset unless bw
    if (bw) {
        const f32x4n xb = tb_noise<NZ>(A, R.qzm, K.qoff, K.slo1, K.shi1);
        const float4 bu = t_lds[sn][K.w - 1][K.lane], bd = t_lds[sn][K.w + 1][K.lane];
        float bl, br;
        if constexpr (WIDE) {
            const float2 e = *reinterpret_cast<const float2 *>(&tx[sn][K.w][0]);  // one broadcast LDS read
            bl = from_left_lane_or(T[tm].w, e.x);
            br = from_right_lane_or(T[tm].x, e.y);
        } else {
            bl = from_left_lane(T[tm].w);
            br = from_right_lane(T[tm].x);
        }
        float mp2;
        o = site_update4<NZ>(T[tm], bl, br, bu, bd, T[tmm], T[tc], xb, A, true, K.m2v, &mp2);
        if constexpr (FR) frame_sites<NZ, true>(A, f2, o, T[tm], xb, bmx + 1, true, mp2);
    }
    if constexpr (WH) {
        bstore4<17>(K.rout, bw ? K.voff + (uint32_t)(k - 1 + A.gz) * K.pbytes : kTpOob, o);  // soffset 0: bstore4
    } else {
        const __amdgpu_buffer_rsrc_t ws = plane_rsrc(A.out, k - 1 + A.gz, K.plane, K.pbytes);
        bstore4<17>(ws, bw ? K.voff : kTpOob, o);
    }
    __syncthreads();
    tp_advance<WH>(A, K, R, k);
}

// One plane iteration of the x-halo wave (S > 1): step s at its 16 sites of
// plane k from the centres in C[] (planes k-1..k+2 by index mod 4) and plane
// k's in-plane neighbours NB[sc] (xm, xp, ym, yp); plane k+1's are loaded here.
// Its own loop (phi4_tb2p_kernel), so its registers do not add to the row waves'.
template <bool NZ, bool WH, int J>
__device__ __forceinline__ void tp_xhalo(const Phi4StepArgs &A, const TbCtx &K, TpRun &R, int k, float (&C)[4],
                                         float4 (&NB)[2], float (*tx)[kTbWaves][2]) {
    constexpr int im = J, ic = (J + 1) & 3, ip = (J + 2) & 3, in2 = (J + 3) & 3;
    constexpr int sc = J & 1, sn = (J + 1) & 1;
    {
        const bool more = k < K.z1;
        __amdgpu_buffer_rsrc_t r2, r1;
        uint32_t o2 = 0, o1 = 0;
        if constexpr (WH) {
            r2 = r1 = K.rin;
            o2 = R.s2;
            o1 = R.s1;
        } else {
            r2 = plane_rsrc(A.in, tb_pidx(A, k + 2), K.plane, K.pbytes);
            r1 = plane_rsrc(A.in, tb_pidx(A, k + 1), K.plane, K.pbytes);
        }
        C[in2] = bload1(r2, more ? K.voff : kTpOob, o2);
        NB[sn] = make_float4(bload1(r1, more ? K.vex : kTpOob, o1), bload1(r1, more ? K.vx2 : kTpOob, o1),
                             bload1(r1, more ? K.vm : kTpOob, o1), bload1(r1, more ? K.vp : kTpOob, o1));
    }
    const f32x4n n = tb_noise<NZ>(A, R.qz, K.qoff, K.slo, K.shi);
    // lanes 0..7 hold x0-1 (component 3 of its quad), 8..15 x0+256 (component 0)
    const float xi = K.lane >= 8 ? n.a : n.d;
    const float t = tb_site(C[ic], NB[sc].x, NB[sc].y, NB[sc].z, NB[sc].w, C[im], C[ip], xi, A, NZ);
    if (K.lane < 16) tx[sc][(K.lane & 7) + 1][K.lane >> 3] = t;
    __syncthreads();
    tp_advance<WH>(A, K, R, k);
}

template <bool NZ, bool WIDE, int WPE, bool FR, bool WH>
__global__ __launch_bounds__((kTbWaves + (WIDE ? 1 : 0)) * 64)
__attribute__((amdgpu_waves_per_eu(WPE))) void phi4_tb2p_kernel(const Phi4StepArgs A0) {
    const Phi4StepArgs A = frame_args<FR>(A0);
    const int nb = gridDim.x, b = blockIdx.x;
    if (A.stamps != nullptr && threadIdx.x == 0) block_stamp(A, 0);
    const TbBlock tbk = tb_block<WIDE>(A, b, nb);  // as phi4_tb2_kernel
    const int yb = tbk.yb, xs = tbk.xs;
    const int Lx = A.Lx, Ly = A.Ly;
    const int x0 = 256 * xs;
    TbCtx K;
    K.w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    K.lane = threadIdx.x & 63;
    K.outw = K.w >= 1 && K.w <= kTbRows;
    K.snapw = __builtin_amdgcn_readfirstlane((FR && A.snap != nullptr && K.outw) ? 1 : 0);
    K.z0 = tbk.z0;
    K.z1 = tbk.z1;
    K.plane = (size_t)Lx * (size_t)Ly;
    K.pbytes = (uint32_t)(K.plane * sizeof(float));
    K.qplane = (uint32_t)(K.plane >> 2);
    if constexpr (WH) {
        const int nbytes = (int)((uint32_t)(A.nz + 2 * A.gz) * K.pbytes);
        K.rin = __builtin_amdgcn_make_buffer_rsrc((void *)A.in, (short)0, nbytes, 0x00020000);
        K.rout = __builtin_amdgcn_make_buffer_rsrc((void *)A.out, (short)0, nbytes, 0x00020000);
    }
    K.qwrap = (uint32_t)A.Lzg * K.qplane;
    K.m2v = f32x2{A.m2, A.m2};
    asm volatile("" : "+v"(K.m2v));
    // periodic: plane k+3 = nz is local plane 0 again; slabs never wrap
    K.swrap_at = A.periodic ? A.nz : INT_MIN;
    const unsigned long long s0 = ((unsigned long long)A.s_hi << 32) | A.s_lo, s1 = s0 + 1;
    K.slo = (uint32_t)s0;
    K.shi = (uint32_t)(s0 >> 32);
    K.slo1 = (uint32_t)s1;
    K.shi1 = (uint32_t)(s1 >> 32);
    const int xl = (x0 == 0 ? Lx : x0) - 1, xr = x0 + 256 == Lx ? 0 : x0 + 256;
    auto wrapy = [Ly](int y) { return y < 0 ? y + Ly : (y >= Ly ? y - Ly : y); };
    const bool xw = WIDE && K.w == kTbWaves;
    // waves 0 and kTbWaves-1 also carry the rows beyond the band (y0-2, y0+9) into in_lds
    const bool xrow = K.w == 0 || K.w == kTbWaves - 1;
    const int xslot = K.w == 0 ? 0 : kTpRows - 1;
    uint32_t vxr = kTpOob;  // waves 1..8 carry no row beyond the band: their X loads are dropped
    if (!xw) {
        const int y = wrapy(yb * kTbRows - 1 + K.w);
        const int yx = wrapy(K.w == 0 ? y - 1 : y + 1);
        K.voff = (uint32_t)((y * Lx + x0 + 4 * K.lane) * 4);
        if (xrow) vxr = (uint32_t)((yx * Lx + x0 + 4 * K.lane) * 4);
        K.vm = K.vp = 0;
        K.vex = (uint32_t)((y * Lx + (K.lane == 63 ? xr : xl)) * 4);
        K.vx2 = 0;
        K.qoff = (uint32_t)((y * Lx + x0 + 4 * K.lane) >> 2);
    } else {  // x-halo wave lanes 0..7: (x0-1, y0+l); 8..15: (x0+256, y0+l-8); the rest repeat lane 0
        const int l = K.lane < 16 ? K.lane : 0;
        const int y = wrapy(yb * kTbRows + (l & 7)), ym = wrapy(y - 1), yp = wrapy(y + 1);
        const int xe = (l >> 3) ? xr : xl;
        const int xem = xe == 0 ? Lx - 1 : xe - 1, xep = xe == Lx - 1 ? 0 : xe + 1;
        K.voff = (uint32_t)((y * Lx + xe) * 4);
        K.vex = (uint32_t)((y * Lx + xem) * 4);
        K.vx2 = (uint32_t)((y * Lx + xep) * 4);
        K.vm = (uint32_t)((ym * Lx + xe) * 4);
        K.vp = (uint32_t)((yp * Lx + xe) * 4);
        K.qoff = (uint32_t)((y * Lx + xe) >> 2);
    }
    __shared__ float4 in_lds[2][kTpRows][64];
    __shared__ float4 t_lds[2][kTbWaves][64];
    __shared__ float tx[WIDE ? 2 : 1][kTbWaves][2];

    if (tbk.gated && !tb_gate_wait(A)) return;  // a rim chunk: its input's ghost planes come with the exchange
    // prologue: planes z0-2, z0-1, z0 (own rows), the rows beyond of z0-1 and
    // z0, edge sites / x-halo neighbours of plane z0-1; plane z0-1 published
    const __amdgpu_buffer_rsrc_t p0 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 2), K.plane, K.pbytes);
    const __amdgpu_buffer_rsrc_t p1 = plane_rsrc(A.in, tb_pidx(A, K.z0 - 1), K.plane, K.pbytes);
    const __amdgpu_buffer_rsrc_t p2 = plane_rsrc(A.in, tb_pidx(A, K.z0), K.plane, K.pbytes);
    __shared__ float bmx[2];
    __shared__ unsigned long long fk[2];  // frame_flush2's block maxima
    __shared__ uint32_t fa[2];
    if constexpr (FR) {  // published by the prologue's barrier
        if (threadIdx.x < 2) {
            bmx[threadIdx.x] = -__builtin_inff();
            fk[threadIdx.x] = 0ull;
            fa[threadIdx.x] = 0u;
        }
    }
    FrameAcc f1 = frame_acc(), f2 = frame_acc();
    TpRun R;
    R.s1 = (uint32_t)tb_pidx(A, K.z0) * K.pbytes;
    R.s2 = (uint32_t)tb_pidx(A, K.z0 + 1) * K.pbytes;
    R.qz = (uint32_t)global_z(A, K.z0 - 1) * K.qplane;
    R.qzm = 0;
    const int z1 = K.z1;
    // the two roles march in loops of their own (one barrier per iteration in
    // each, the same iteration count), so their registers do not add up
    if (!xw) {
        float4 I[4], T[4], X[2];
        float E[2] = {0.f, 0.f};
        I[0] = bload4(p0, K.voff);
        I[1] = bload4(p1, K.voff);
        I[2] = bload4(p2, K.voff);
        X[0] = bload4(p1, vxr);
        X[1] = bload4(p2, vxr);
        if constexpr (WIDE) E[0] = bload1(p1, K.vex);
        in_lds[0][K.w + 1][K.lane] = I[1];
        if (xrow) in_lds[0][xslot][K.lane] = X[0];
        T[0] = T[1] = T[2] = T[3] = make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
        const PrioQ pq(K.z0, z1 - K.z0 + 2);
        for (int k = K.z0 - 1; k <= z1; k += 4) {
            if (A.prio) prio_by_progress(pq.q(k));
            tp_row<NZ, WIDE, FR, WH, 0>(A, K, R, k, xrow, vxr, xslot, I, T, X, E, in_lds, t_lds, tx, f1, f2, bmx);
            if (k + 1 > z1) break;
            tp_row<NZ, WIDE, FR, WH, 1>(A, K, R, k + 1, xrow, vxr, xslot, I, T, X, E, in_lds, t_lds, tx, f1, f2, bmx);
            if (k + 2 > z1) break;
            tp_row<NZ, WIDE, FR, WH, 2>(A, K, R, k + 2, xrow, vxr, xslot, I, T, X, E, in_lds, t_lds, tx, f1, f2, bmx);
            if (k + 3 > z1) break;
            tp_row<NZ, WIDE, FR, WH, 3>(A, K, R, k + 3, xrow, vxr, xslot, I, T, X, E, in_lds, t_lds, tx, f1, f2, bmx);
        }
    } else {
        float C[4];
        float4 NB[2];
        C[0] = bload1(p0, K.voff);
        C[1] = bload1(p1, K.voff);
        C[2] = bload1(p2, K.voff);
        NB[0] = make_float4(bload1(p1, K.vex), bload1(p1, K.vx2), bload1(p1, K.vm), bload1(p1, K.vp));
        __syncthreads();
        const PrioQ pq(K.z0, z1 - K.z0 + 2);
        for (int k = K.z0 - 1; k <= z1; k += 4) {
            if (A.prio) prio_by_progress(pq.q(k));
            tp_xhalo<NZ, WH, 0>(A, K, R, k, C, NB, tx);
            if (k + 1 > z1) break;
            tp_xhalo<NZ, WH, 1>(A, K, R, k + 1, C, NB, tx);
            if (k + 2 > z1) break;
            tp_xhalo<NZ, WH, 2>(A, K, R, k + 2, C, NB, tx);
            if (k + 3 > z1) break;
            tp_xhalo<NZ, WH, 3>(A, K, R, k + 3, C, NB, tx);
        }
    }
    if constexpr (FR) frame_flush2(A, f1, f2, fk, fa);
    block_end_stamp(A);
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
        *reinterpret_cast<float4 *>(slab + 4 * q) = make_float4(amp * n.a, amp * n.b, amp * n.c, amp * n.d);
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

// ------------------------------------------------ device frame control ----
// After each frame of sq_run_frames (sq_api.cpp phi4_frames_dev), one launch:
// the host loop of phi4_frame (record fold, stab_rule, tauhost.c:523-541's Δτ
// rule) and its rollback, so the next frame is enqueued without a host
// decision.  Every block folds the frame's records into LDS and takes the
// verdict itself (a few KB of L2 reads per block, no grid-wide handoff); block
// 0 writes the controller's next state (cout: the launches of the next frame
// read cout->coef) and the folded records, and clears the other record set,
// which the next frame accumulates into (the previous end launch read it);
// when the verdict is unstable every block copies its share of the snapshot
// back.  The comparisons, the max and the double Δτ arithmetic are the host's,
// operation for operation (bit-identical verdicts, Δτ and coefficients:
// tests/test_gpu_phi4.py::test_run_frames_*).
constexpr int kEndChunk = 512;  // steps folded per LDS pass

__device__ __forceinline__ float unord_f32_dev(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// The host's frame verdict and Δτ controller (sq_api.cpp phi4_frame + adapt,
// tauhost.c:523-529,537-541), operation for operation, on the controller state.
__device__ __forceinline__ void frame_decide(FrameCtl &c, float T, float V, int fired, int flag) {
    const int st = (flag == 0 && fired < 0) ? 1 : 0;
    c.T = T;
    c.V = V;
    c.fired = fired;
    c.flag = flag;
    c.stable = st;
    c.frames += 1;
    if (c.adapt) {
        if (st) {
            if (c.stab_cnt > 10) {
                c.stab_cnt = 0;
                c.dtau /= 0.950;
            }
            c.stab_cnt += 1;
        } else {
            c.dtau *= 0.950;
            c.stab_cnt = 0;
        }
    }
    const float hf = (float)c.dtau;  // phi4_base_args
    c.coef[0] = hf;
    c.coef[1] = (float)(__builtin_sqrt(2.0 * (double)hf) * c.C);
    c.coef[2] = (float)(__builtin_sqrt(2.0 * (double)hf) * c.C * kSqrt2Ln2);
    if (c.tri) {  // the next frame's buffers (FrameCtl): start, then the two others
        const int fin = c.nl_odd ? c.bw0 : c.bw1;
        const int third = 3 - c.bs - fin;
        const int nbs = st ? fin : c.bs, nbw1 = st ? c.bs : fin;
        c.bs = nbs;
        c.bw0 = third;
        c.bw1 = nbw1;
    }
}

__global__ __launch_bounds__(256) void phi4_frame_end_kernel(FrameEndArgs E) {
    __shared__ float sM[kEndChunk], sD[kEndChunk], sA[kEndChunk];
    __shared__ float sT, sV;
    __shared__ int sFired;
    const bool b0 = blockIdx.x == 0;
    if (threadIdx.x == 0) {
        sT = E.cin->T;
        sV = E.cin->V;
        sFired = -1;
    }
    for (int j0 = 0; j0 < E.L; j0 += kEndChunk) {
        const int n = min(kEndChunk, E.L - j0);
        __syncthreads();  // sT / sV / sFired set, the previous chunk's rule done
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
            unsigned long long k = 0;
            unsigned int a = 0;
            const size_t q0 = (size_t)(j0 + j) * kStabSlots;
            for (int i = 0; i < kStabSlots; ++i) {
                const unsigned long long mk = E.md[q0 + i];
                const unsigned int ma = E.am[q0 + i];
                k = k < mk ? mk : k;
                a = a < ma ? ma : a;
            }
            sM[j] = unord_f32_dev((uint32_t)(k >> 32));
            sD[j] = __uint_as_float((uint32_t)k);
            sA[j] = __uint_as_float(a);
            if (b0) {
                E.rec[j0 + j] = sM[j];
                E.rec[E.L + j0 + j] = sD[j];
                E.rec[2 * E.L + j0 + j] = sA[j];
            }
        }
        __syncthreads();
        if (threadIdx.x == 0 && sFired < 0) {  // stab_rule (sq_api.cpp); every chunk still folds (rec)
            float T = sT, V = sV;
            for (int j = 0; j < n; ++j) {
                const bool f = sM[j] > T && sD[j] > V;
                T = sM[j];
                V = V < sA[j] ? sA[j] : V;
                if (f) {
                    sFired = j0 + j;
                    break;
                }
            }
            sT = T;
            sV = V;
        }
    }
    __syncthreads();
    const int st = (*E.flag == 0 && sFired < 0) ? 1 : 0;
    if (b0) {
        if (threadIdx.x == 0) {
            FrameCtl c = *E.cin;
            frame_decide(c, sT, sV, sFired, *E.flag);
            *E.cout = c;
            if (E.stable_out) *E.stable_out = st;
            if (E.dtau_out) *E.dtau_out = c.dtau;
            *E.flag_next = 0;
        }
        for (long long q = threadIdx.x; q < (long long)E.L * kStabSlots; q += blockDim.x) {
            E.md_next[q] = 0;
            E.am_next[q] = 0;
        }
    }
    if (st) return;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < E.n4;
         i += (long long)gridDim.x * blockDim.x)
        E.dst[i] = E.snap[i];
}

// Per-block partials (no atomics: 1024 blocks' double atomics on one address
// serialised at one L2 channel, 57 us per 256^3 call), then one block folds
// them in block order -- the same bits on every call.
__global__ __launch_bounds__(256) void phi4_moments_kernel(const float *p, long long n4, double *part) {
    double s1 = 0, s2 = 0;
    float mx = 0, mp = -__builtin_inff();
    const float4 *q = reinterpret_cast<const float4 *>(p);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
        const float4 v = q[i];
        s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        mp = fmaxf(mp, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    __shared__ double sh1[4], sh2[4];
    __shared__ float shm[4], shp[4];
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    mx = wave_max(mx);
    mp = wave_max(mp);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh1[w] = s1;
        sh2[w] = s2;
        shm[w] = mx;
        shp[w] = mp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t1 = 0, t2 = 0;
        float tm = 0, tp = -__builtin_inff();
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
            t1 += sh1[k];
            t2 += sh2[k];
            tm = fmaxf(tm, shm[k]);
            tp = fmaxf(tp, shp[k]);
        }
        double *q = part + 4 * (size_t)blockIdx.x;
        q[0] = t1;
        q[1] = t2;
        q[2] = (double)tm;
        q[3] = (double)tp;
    }
}

__global__ __launch_bounds__(256) void phi4_moments_final_kernel(const double *part, int nb, double *acc,
                                                                 unsigned int *acc_max) {
    double s1 = 0, s2 = 0, mx = 0, mp = -__builtin_inf();
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const double *q = part + 4 * (size_t)b;
        s1 += q[0];
        s2 += q[1];
        mx = fmax(mx, q[2]);
        mp = fmax(mp, q[3]);
    }
    __shared__ double sh[4][4];
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mx = fmax(mx, __shfl_xor(mx, o, 64));
        mp = fmax(mp, __shfl_xor(mp, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sh[w][0] = s1;
        sh[w][1] = s2;
        sh[w][2] = mx;
        sh[w][3] = mp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t1 = 0, t2 = 0, tm = 0, tp = -__builtin_inf();
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
            t1 += sh[k][0];
            t2 += sh[k][1];
            tm = fmax(tm, sh[k][2]);
            tp = fmax(tp, sh[k][3]);
        }
        acc[0] = t1;
        acc[1] = t2;
        acc_max[0] = __float_as_uint((float)tm);
        acc_max[1] = ord_f32((float)tp);
    }
}

__global__ __launch_bounds__(256) void phi4_slices_kernel(const float *slab, long long plane4,
                                                          double *out) {
    const float4 *q = reinterpret_cast<const float4 *>(slab) + (size_t)blockIdx.x * plane4;
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

#ifndef SQ_PHI4_KERNELS_ONLY  // sq_phi4_run.hip includes the kernels above, not the launchers below
bool phi4_geometry(int Lx, int Ly, Phi4Geom *g) {
    if (Lx <= 0 || Ly <= 0 || (Lx & 3)) return false;
    int qx;
    if (Lx % 256 == 0) qx = 64;
    else if (Lx < 256 && Lx >= 8 && 64 % (Lx / 4) == 0) qx = Lx / 4;
    else return false;
    const int rs = 64 / qx;
    // x-span per wave: two 256-site segments per lane when the row is a
    // multiple of 512 (one wave per 512-site span, no segment-edge loads).
    // Measured (profiles/r01/sweep*): 256-wide rows (256^3 is MALL-resident)
    // want R = 1, zc = 4; 512-wide and wider rows (HBM-bound) want R = 2, zc = 8.
    const int v = (qx == 64 && Lx % 512 == 0) ? 2 : 1;
    // full-row waves use packed-f32 site arithmetic (queue mode 3): bit-identical,
    // 15 % fewer VALU instructions, measured 256^3 22.3 -> 21.3 us, 512^3
    // 196.5 -> 193.4 us (profiles/r01/sweep*_packed.log); and (mode 7) write
    // their output with sc0 sc1 stores, which leave the XCD's L2 at once
    // instead of occupying the lines other waves' halo rows are re-read from:
    // 256^3 21.66 -> 20.98 us per step, 512^3 193.1 -> 190.8 us (faster than
    // the non-temporal stores of mode 4 there), profiles/r01/sweep*_sc1.log
    const int pf = qx == 64 ? 7 : 1;
    const bool narrow = Lx <= 256;
    const int rcand[3] = {narrow ? 1 : 2, narrow ? 2 : 4, narrow ? 4 : 1};
    for (int r : rcand) {  // a full wave tile that divides Ly
        if (Ly % (rs * r) == 0) {
            *g = Phi4Geom{qx, r, rs * r, pf, v};
            return true;
        }
    }
    for (int r : rcand) {  // otherwise a partial last tile (rows past Ly idle)
        if (Ly % r == 0) {
            *g = Phi4Geom{qx, r, rs * r, pf, v};
            return true;
        }
    }
    return false;
}

void phi4_fill_units(Phi4StepArgs &a, const Phi4Geom &g) {
    a.nxseg = a.Lx / (4 * g.qx * g.v);
    a.nyg = (a.Ly + g.wy - 1) / g.wy;
    a.nunits = a.nxseg * a.nyg * a.nzc;
}

template <int QX, int R, int V, bool MS, bool NZ, int PF, bool FR>
static hipError_t launch_fr(const Phi4StepArgs &a, dim3 grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (e0 != nullptr || e1 != nullptr)
        hipExtLaunchKernelGGL((phi4_step_kernel<QX, R, V, MS, NZ, PF, FR>), grid, dim3(256), 0, s, e0, e1, 0, a);
    else
        hipLaunchKernelGGL((phi4_step_kernel<QX, R, V, MS, NZ, PF, FR>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

template <int QX, int R, int V, bool MS, bool NZ, int PF>
static hipError_t launch_pf(const Phi4StepArgs &a, dim3 grid, hipStream_t s, hipEvent_t e0,
                            hipEvent_t e1) {
    if (a.flag != nullptr && (a.st_md == nullptr || a.st_a == nullptr))
        return hipErrorInvalidValue;  // frame launches carry the records (frame_sites)
    return a.flag != nullptr ? launch_fr<QX, R, V, MS, NZ, PF, true>(a, grid, s, e0, e1)
                             : launch_fr<QX, R, V, MS, NZ, PF, false>(a, grid, s, e0, e1);
}

template <int QX, int R, int V, bool MS>
static hipError_t launch_v(const Phi4StepArgs &a, int pf, bool nz, dim3 grid, hipStream_t s,
                           hipEvent_t e0, hipEvent_t e1) {
    if constexpr (QX == 64) {
        if (pf == 3)
            return nz ? launch_pf<QX, R, V, MS, true, 3>(a, grid, s, e0, e1)
                      : launch_pf<QX, R, V, MS, false, 3>(a, grid, s, e0, e1);
        if (pf == 4)
            return nz ? launch_pf<QX, R, V, MS, true, 4>(a, grid, s, e0, e1)
                      : launch_pf<QX, R, V, MS, false, 4>(a, grid, s, e0, e1);
        if (pf == 7)
            return nz ? launch_pf<QX, R, V, MS, true, 7>(a, grid, s, e0, e1)
                      : launch_pf<QX, R, V, MS, false, 7>(a, grid, s, e0, e1);
    }
    return nz ? launch_pf<QX, R, V, MS, true, 1>(a, grid, s, e0, e1)
              : launch_pf<QX, R, V, MS, false, 1>(a, grid, s, e0, e1);
}

template <int QX, int V, bool MS>
static hipError_t launch_r(const Phi4StepArgs &a, const Phi4Geom &g, dim3 grid, hipStream_t s,
                           hipEvent_t e0, hipEvent_t e1) {
    const bool nz = a.sig != 0.0f;
    switch (g.r) {
    case 4: return launch_v<QX, 4, V, MS>(a, g.pf, nz, grid, s, e0, e1);
    case 2: return launch_v<QX, 2, V, MS>(a, g.pf, nz, grid, s, e0, e1);
    default: return launch_v<QX, 1, V, MS>(a, g.pf, nz, grid, s, e0, e1);
    }
}

// Kernel ids (phi4_kernel_id_name): bits 0-1 family (0 phi4_step_kernel, 1
// phi4_tb2_kernel, 2 phi4_tb2p_kernel), 2 NZ, 3 WIDE / MS, 4-7 WPE, 8 FR, 9 WH,
// 10 P2, 11-18 QX, 19-22 R, 23-24 V, 25-28 PF; bits 32-63 the grid in threads.
static uint64_t kid_pack(int fam, bool nz, bool wide, int e, bool fr, bool wh, bool p2, int qx, int r, int v,
                         int pf, unsigned threads) {
    return (uint64_t)fam | (uint64_t)nz << 2 | (uint64_t)wide << 3 | (uint64_t)(e & 15) << 4 | (uint64_t)fr << 8 |
           (uint64_t)wh << 9 | (uint64_t)p2 << 10 | (uint64_t)(qx & 255) << 11 | (uint64_t)(r & 15) << 19 |
           (uint64_t)(v & 3) << 23 | (uint64_t)(pf & 15) << 25 | (uint64_t)threads << 32;
}

void phi4_kernel_id_name(uint64_t k, char *name, size_t cap) {
    const int fam = (int)(k & 3);
    auto b = [&](int bit) { return ((k >> bit) & 1) ? "true" : "false"; };
    const int e = (int)((k >> 4) & 15), qx = (int)((k >> 11) & 255), r = (int)((k >> 19) & 15),
              v = (int)((k >> 23) & 3), pf = (int)((k >> 25) & 15);
    if (fam == 0)
        snprintf(name, cap, "phi4_step_kernel<%d, %d, %d, %s, %s, %d, %s>", qx, r, v, b(3), b(2), pf, b(8));
    else if (fam == 1)
        snprintf(name, cap, "phi4_tb2_kernel<%s, %s, %d, %s, %s, %s>", b(2), b(3), e, b(8), b(9), b(10));
    else
        snprintf(name, cap, "phi4_tb2p_kernel<%s, %s, %d, %s, %s>", b(2), b(3), e, b(8), b(9));
}

hipError_t phi4_step_launch(const Phi4StepArgs &a, const Phi4Geom &g, hipStream_t s, hipEvent_t e0,
                            hipEvent_t e1, uint64_t *kid) {
    if (a.nunits <= 0) return hipSuccess;
    const dim3 grid((unsigned)((a.nunits + 3) / 4));
    const bool ms = a.nxseg > 1;
    if (kid != nullptr) {  // the instance launch_r / launch_v / launch_pf pick below
        const bool q64 = g.qx == 64;
        const int r = g.r == 4 ? 4 : g.r == 2 ? 2 : 1;
        const int pf = q64 && (g.pf == 3 || g.pf == 4 || g.pf == 7) ? g.pf : 1;
        *kid = kid_pack(0, a.sig != 0.0f, q64 && ms, 0, a.flag != nullptr, false, false, g.qx, r,
                        q64 && g.v == 2 ? 2 : 1, pf, grid.x * 256u);
    }
    switch (g.qx) {
    case 64:
        if (g.v == 2) return ms ? launch_r<64, 2, true>(a, g, grid, s, e0, e1) : launch_r<64, 2, false>(a, g, grid, s, e0, e1);
        return ms ? launch_r<64, 1, true>(a, g, grid, s, e0, e1) : launch_r<64, 1, false>(a, g, grid, s, e0, e1);
    case 32: return launch_r<32, 1, false>(a, g, grid, s, e0, e1);
    case 16: return launch_r<16, 1, false>(a, g, grid, s, e0, e1);
    case 8: return launch_r<8, 1, false>(a, g, grid, s, e0, e1);
    case 4: return launch_r<4, 1, false>(a, g, grid, s, e0, e1);
    case 2: return launch_r<2, 1, false>(a, g, grid, s, e0, e1);
    default: return hipErrorInvalidValue;
    }
}

bool phi4_tb2_supported(int Lx, int Ly) { return Lx % 256 == 0 && Ly % kTbRows == 0; }

static bool tb2_sync_p2p() {
    const char *e = getenv("SQ_TB2_SYNC");  // read per launch (tests switch it within a process)
    return e != nullptr && strcmp(e, "p2p") == 0;
}

hipError_t phi4_tb2_launch(const Phi4StepArgs &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1, uint64_t *kid) {
    if (!phi4_tb2_supported(a.Lx, a.Ly) || a.nunits <= 0 || a.nxseg != a.Lx / 256 || a.nyg != a.Ly / kTbRows ||
        a.nzr < 1 || a.nzc % a.nzr != 0 || a.nunits != a.nxseg * a.nyg * a.nzc || a.zlen < 1 ||
        (long long)a.zc * a.nzr < a.zlen)
        return hipErrorInvalidValue;
    const int nr = a.nzc / a.nzr, last_end = a.zlo + (nr - 1) * a.zstep + a.zlen;
    if (nr > 1 && a.zstep < a.zlen) return hipErrorInvalidValue;  // ranges overlap
    if (a.periodic ? (a.nz < 2 || a.zlo != 0 || a.zlen != a.nz || nr != 1)
                   : (a.zlo - 2 < -a.gz || last_end + 2 > a.nz + a.gz))  // input planes outside the buffer
        return hipErrorInvalidValue;
    unsigned grid_n = (unsigned)a.nunits;
    if (a.gate != nullptr) {  // core blocks + the thin gated rim chunks after them
        if (a.n_reg != a.nunits || a.tzc < 1 || a.tlen < 1 || a.ntz != (a.tlen + a.tzc - 1) / a.tzc ||
            a.tlo0 - 2 < -a.gz || a.tlo0 + a.tlen + 2 > a.nz + a.gz || a.thi0 - 2 < -a.gz ||
            a.thi0 + a.tlen + 2 > a.nz + a.gz || a.periodic)
            return hipErrorInvalidValue;
        grid_n += (unsigned)(a.nxseg * a.nyg * 2 * a.ntz);
    }
    const bool wide = a.nxseg > 1;
    const dim3 grid(grid_n), block((kTbWaves + (wide ? 1 : 0)) * 64);
    const bool nz = a.sig != 0.0f;
    static const int wpe = getenv("SQ_TB2_WPE") ? atoi(getenv("SQ_TB2_WPE")) : 6;
    const bool fr = a.flag != nullptr;
    if (fr && (a.st_md == nullptr || a.st_a == nullptr)) return hipErrorInvalidValue;  // frame_sites
    const void *fn;
    // one 32-bit (signed, < 2^31 B) descriptor per padded buffer when it fits
    const bool wh = (long long)(a.nz + 2 * a.gz) * a.Lx * a.Ly * 4 < (1ll << 31);
    // the pipelined kernel (loads one plane iteration ahead) for rows wider than
    // 256 sites, where it is 10 % faster at 512^3 (139-140 vs 155-156 us/step);
    // the round-2 kernel (loads consumed in the iteration that issues them) for
    // 256-site rows, where it is 6 % faster at 256^3 (16.8-17.0 vs 17.8-18.0:
    // profiles/r03/ab).  SQ_TB2_PIPE=0 / 1 pins either.
    const char *pe = getenv("SQ_TB2_PIPE");  // read per launch (tests switch it within a process)
    const bool pipe = pe ? atoi(pe) != 0 : wide;
#define SQ_TB2K(N, W, E, F, H) (pipe ? (const void *)&phi4_tb2p_kernel<N, W, E, F, H> \
                                     : (const void *)&phi4_tb2_kernel<N, W, E, F, H>)
#define SQ_TB2F(N, W, E, F) (wh ? SQ_TB2K(N, W, E, F, true) : SQ_TB2K(N, W, E, F, false))
#define SQ_TB2(N, W, E) (fr ? SQ_TB2F(N, W, E, true) : SQ_TB2F(N, W, E, false))
    if (wide && wpe == 6)
        fn = nz ? SQ_TB2(true, true, 6) : SQ_TB2(false, true, 6);
    else if (wide)
        fn = nz ? SQ_TB2(true, true, 1) : SQ_TB2(false, true, 1);
    else if (fr && !pipe && tb2_sync_p2p())
        fn = nz ? (wh ? (const void *)&phi4_tb2_kernel<true, false, 6, true, true, true>
                      : (const void *)&phi4_tb2_kernel<true, false, 6, true, false, true>)
                : (wh ? (const void *)&phi4_tb2_kernel<false, false, 6, true, true, true>
                      : (const void *)&phi4_tb2_kernel<false, false, 6, true, false, true>);
    else if (fr)  // 78 VGPRs (unconstrained: 81, 88 allocated, 5 waves per SIMD: two 10-wave blocks
                  // fit a CU only when the second one's waves land 2-2-3-3 against the first's
                  // 3-3-2-2; frame launches 53 vs 45 us at 256^3)
        fn = nz ? SQ_TB2F(true, false, 6, true) : SQ_TB2F(false, false, 6, true);
    else if (!pipe && tb2_sync_p2p())  // SQ_TB2_SYNC=p2p: neighbour progress words instead of the barrier
        fn = nz ? (wh ? (const void *)&phi4_tb2_kernel<true, false, 1, false, true, true>
                      : (const void *)&phi4_tb2_kernel<true, false, 1, false, false, true>)
                : (wh ? (const void *)&phi4_tb2_kernel<false, false, 1, false, true, true>
                      : (const void *)&phi4_tb2_kernel<false, false, 1, false, false, true>);
    else
        fn = nz ? SQ_TB2F(true, false, 1, false) : SQ_TB2F(false, false, 1, false);
#undef SQ_TB2
#undef SQ_TB2F
#undef SQ_TB2K
    if (kid != nullptr) {  // the same choice as above, as a kernel id
        const bool p2 = !wide && !pipe && tb2_sync_p2p();
        const int e = wide ? (wpe == 6 ? 6 : 1) : (fr ? 6 : 1);
        *kid = kid_pack(pipe && !p2 ? 2 : 1, nz, wide, e, fr, wh, p2, 0, 0, 0, 0, grid.x * block.x);
    }
    Phi4StepArgs q = a;
    // wave priority by march progress: 256^3 16.3-16.7 vs 17.0 us/step, 512^3
    // 135-137 vs 140-141 (profiles/r03/prio); SQ_TB2_PRIO=0 turns it off
    static const int prio = getenv("SQ_TB2_PRIO") ? atoi(getenv("SQ_TB2_PRIO")) : 1;
    q.prio = prio;
    void *args[] = {&q};
    if (e0 != nullptr || e1 != nullptr) return hipExtLaunchKernel(fn, grid, block, args, 0, s, e0, e1, 0);
    return hipLaunchKernel(fn, grid, block, args, 0, s);
}

hipError_t phi4_init_launch(float *slab, int Lx, int Ly, int nz, long long zg0, uint32_t k0,
                            uint32_t k1, float amp, hipStream_t s) {
    const size_t nq = (size_t)nz * Lx * Ly / 4;
    const unsigned grid = (unsigned)std::min<size_t>((nq + 255) / 256, 8192);
    hipLaunchKernelGGL(phi4_init_kernel, dim3(grid), dim3(256), 0, s, slab, Lx, Ly, nz, zg0, k0, k1,
                       amp);
    return hipGetLastError();
}

hipError_t phi4_frame_end_launch(const FrameEndArgs &e, hipStream_t s) {
    if (e.L < 1 || !e.cin || !e.cout || e.cin == e.cout || !e.md || !e.am || !e.flag || !e.md_next || !e.am_next ||
        !e.flag_next || e.md == e.md_next || !e.rec || (e.n4 > 0 && (!e.dst || !e.snap)))
        return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>((e.n4 + 1023) / 1024, 512));
    FrameEndArgs q = e;
    hipLaunchKernelGGL(phi4_frame_end_kernel, dim3(grid), dim3(256), 0, s, q);
    return hipGetLastError();
}

hipError_t phi4_moments_launch(const float *slab, long long n, double *acc, unsigned int *acc_max, double *part,
                               hipStream_t s) {
    const long long n4 = n / 4;
    const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>((n4 + 255) / 256, kMomBlocks));
    hipLaunchKernelGGL(phi4_moments_kernel, dim3(grid), dim3(256), 0, s, slab, n4, part);
    hipLaunchKernelGGL(phi4_moments_final_kernel, dim3(1), dim3(256), 0, s, (const double *)part, (int)grid, acc,
                       acc_max);
    return hipGetLastError();
}

hipError_t phi4_slices_launch(const float *slab, int Lx, int Ly, int nz, double *out,
                              hipStream_t s) {
    hipLaunchKernelGGL(phi4_slices_kernel, dim3((unsigned)nz), dim3(256), 0, s, slab,
                       (long long)Lx * Ly / 4, out);
    return hipGetLastError();
}

#endif  // SQ_PHI4_KERNELS_ONLY
}  // namespace sq
