// sq_qm1d_gs.hip -- QM1D in the reference's own serial order (SURVEY.md §8f
// row 4): Gauss-Seidel sweep, one shared 48-bit LCG, the stability scan and
// running means exactly as time_dev runs when its work-items execute in id
// order between barriers (oracle/orc_qm1d.c serial).
//
// Launches per frame, all on one stream:
//   gs_lcg_*_kernel  the LCG of tau_kernel.cl:269-284 for every call of a
//                    full launch (rounds 0..loops-1, items 0..N), incl. the
//                    isinf retry; stores the accepted draw's words t1>>16,
//                    t2>>16 and the seed after each call.  The seed update is
//                    affine mod 2^48 except on rare calls, so the serial chain
//                    is a parallel prefix of affine maps (grid-wide) plus an
//                    exact one-block fix-up from the first exception (below).
//   gs_xi_kernel     grid-wide: xi = cos(2*3.1415*v2) * sqrt(-2 log v1) with
//                    the reference's float casts and glibc's own logf / cosf
//                    algorithms (sq_glibcf.h, bit-identical to the host libm
//                    the oracle and the reference use over every argument
//                    random() can pass), so xi is the oracle's bit for bit.
//   gs_omega_kernel  one wave: omega of every step (item N's scalar recurrence).
//   gs_xcl_kernel    grid-wide, potID 3: x_cl and ddPot(x_cl) of every (step,
//                    site), so the serial kernels below do no transcendentals.
//   gs_frame_kernel  two blocks running concurrently:
//     block 0, the sweep (<= 16 waves): the GS field sweep as a skewed
//                    pipeline.  Thread l owns sites [lB, lB+B) and runs step j
//                    in phase p = l + j: the left neighbour's step-j value
//                    comes from thread l-1's previous phase, the right
//                    neighbour's step-(j-1) value from thread l+1's first site
//                    of the same phase (DPP wave shifts inside a wave, LDS
//                    across waves).  Every (step, site) is computed exactly as
//                    the serial order computes it, with the reference's
//                    expression order.  The field of every step goes to hist
//                    (loops x N); completed steps are published to the scan.
//     block 1, the scan: walks the steps as their rows appear and evaluates
//                    the stability scan (tau_kernel.cl:135-143) as prefix
//                    maxima (derivation in DESIGN.md §4.1), finds the first
//                    unstable item (the serial break: items after it never run
//                    that round -- except in round 0, where the stable test has
//                    not started, :168-171) and the running means :144-145.
#include <algorithm>
#include <cstdlib>

#include "sq_dpp.h"
#include "sq_glibcf.h"
#include "sq_internal.h"

namespace sq {

namespace {

constexpr double kEta = .8;  // tau_kernel.cl:19-22
constexpr double kV0 = 2.;
constexpr double kM = 1.;
constexpr double kMax = 1000.;

__device__ __forceinline__ double xcl(double t, double w, int pot) {  // clas(), :184-189,215-226
    if (pot == 3) {
        const double s = 2.0;  // (double)sqrtf((float)(2.*V0/m)) == 2 exactly
        return kEta * (double)sq_glibc_tanhf((float)(s * (t - w) / kEta));  // glibc's tanhf, bit for bit
    }
    return 0.;
}
__device__ __forceinline__ double ddpot(double x, int pot) {  // ddPot(), :190-195,227-236
    if (pot == 3) return (12. * kV0 * x * x / (kEta * kEta) - 4. * kV0) / (kEta * kEta);
    return 2.;
}
__device__ __forceinline__ double absol(double v) { return v <= 0 ? -v : v; }
__device__ __forceinline__ double guard(double v) {  // :119-133
    if (v > kMax) v = kMax;
    if (v < -kMax) v = -kMax;
    if (__builtin_isnan(v)) v = kMax;
    return v;
}

// ---------------------------------------------------------------- LCG ----
// One call of random() for item g from seed s (tau_kernel.cl:269-284):
//   t1 = (A (s+g) + B) mod 2^48,  t2 = (A (t1+g) + B) mod 2^48,
//   s' = s + t2 if s < 2^31 and t2 < 2^31 ("case P"), else t2 - 2^31 (u64,
//   "case Q"); repeat while t1 >> 16 == 0 (the isinf retry: log(0) = -inf).
// In case Q, s' = alpha s + beta(g) (mod 2^48) with alpha = A^2 and
// beta(g) = A^2 g + A B + A g + B - 2^31: affine in s.  Only s mod 2^48 and
// the test s < 2^31 matter to later calls, and a wrapped u64 (t2 < 2^31)
// is >= 2^31 both as u64 and mod 2^48, so the 48-bit residue carries the
// state exactly.  Case P needs s < 2^31 AND t2 < 2^31 (about 2^-34 per call
// after the first) and the retry 2^-32: the chain of a whole launch is a
// composition of affine maps, evaluated by a parallel prefix, with an exact
// serial fix-up at the (practically never taken) exceptions.
constexpr uint64_t kM48 = (1ull << 48) - 1;
constexpr uint64_t kLcgA = 0x5DEECE66DULL, kLcgB = 0xBULL, kTwo31 = 2147483648ull;
constexpr uint64_t kAlpha = (kLcgA * kLcgA) & kM48;

__device__ __forceinline__ uint64_t lcg_beta(uint64_t g) {
    return (kLcgA * kLcgA * g + kLcgA * kLcgB + kLcgA * g + kLcgB - kTwo31) & kM48;
}

struct LcgCall {
    uint64_t t1, t2, s;  // s = the seed after the call (exact u64)
    bool exc;            // the call took case P or a retry (not the affine map)
};

__device__ __forceinline__ LcgCall lcg_case_q(uint64_t s, uint64_t g) {
    LcgCall c;
    c.t1 = ((s + g) * kLcgA + kLcgB) & kM48;
    c.t2 = ((c.t1 + g) * kLcgA + kLcgB) & kM48;
    c.exc = (c.t1 >> 16) == 0 || (s < kTwo31 && c.t2 < kTwo31);
    c.s = c.t2 - kTwo31;
    return c;
}

__device__ __forceinline__ LcgCall lcg_exact(uint64_t s, uint64_t g) {  // the reference's loop, verbatim semantics
    LcgCall c;
    do {
        c.t1 = ((s + g) * kLcgA + kLcgB) & kM48;
        c.t2 = ((c.t1 + g) * kLcgA + kLcgB) & kM48;
        s = (s < kTwo31 && c.t2 < kTwo31) ? s + c.t2 : c.t2 - kTwo31;
    } while ((c.t1 >> 16) == 0);
    c.s = s;
    c.exc = false;
    return c;
}

constexpr int kLcgThreads = 1024;

// The common path is three grid-wide kernels over kLcgChunks contiguous
// chunks of calls: compose each chunk's case-Q map, scan the maps (one
// block), replay each chunk from its start seed (recording the first
// exceptional call).  gs_lcg_kernel (one block) then resumes exactly from
// that call -- it returns at once when there was none.
// scr: maps a[T], b[T], chunk start seeds[T], first exceptional call.

__device__ __forceinline__ void lcg_chunk(long long ncalls, int t, long long &kb, long long &ke) {
    const long long C = (ncalls + kLcgChunks - 1) / kLcgChunks;
    kb = min(ncalls, (long long)t * C);
    ke = min(ncalls, kb + C);
}

__global__ __launch_bounds__(256) void gs_lcg_compose_kernel(int N, long long ncalls, unsigned long long *scr) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t == 0) scr[3 * kLcgChunks] = (unsigned long long)ncalls;
    long long kb, ke;
    lcg_chunk(ncalls, t, kb, ke);
    const uint64_t np1 = (uint64_t)N + 1;
    uint64_t a = 1, b = 0, g = (uint64_t)kb % np1;
    for (long long k = kb; k < ke; ++k) {
        a = (kAlpha * a) & kM48;
        b = (kAlpha * b + lcg_beta(g)) & kM48;
        g = g + 1 == np1 ? 0 : g + 1;
    }
    scr[t] = a;
    scr[kLcgChunks + t] = b;
}

__global__ __launch_bounds__(1024) void gs_lcg_scan_kernel(unsigned long long seed, unsigned long long *scr) {
    constexpr int PER = kLcgChunks / 1024;
    __shared__ uint64_t sa[1024], sb[1024];
    const int t = threadIdx.x;
    uint64_t a = 1, b = 0;
    for (int i = 0; i < PER; ++i) {  // my PER consecutive maps, composed in call order
        const uint64_t am = scr[t * PER + i], bm = scr[kLcgChunks + t * PER + i];
        b = (am * b + bm) & kM48;
        a = (am * a) & kM48;
    }
    sa[t] = a;
    sb[t] = b;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        uint64_t pa = 1, pb = 0;
        if (t >= o) {
            pa = sa[t - o];
            pb = sb[t - o];
        }
        __syncthreads();
        if (t >= o) {
            const uint64_t na = (sa[t] * pa) & kM48, nb = (sa[t] * pb + sb[t]) & kM48;
            sa[t] = na;
            sb[t] = nb;
        }
        __syncthreads();
    }
    // chunk 0 starts from the exact u64 seed; later chunks from its residue image
    uint64_t s = t == 0 ? seed : ((sa[t - 1] * (seed & kM48) + sb[t - 1]) & kM48);
    for (int i = 0; i < PER; ++i) {
        const int m = t * PER + i;
        scr[2 * kLcgChunks + m] = s;
        s = (scr[m] * (s & kM48) + scr[kLcgChunks + m]) & kM48;
    }
}

__global__ __launch_bounds__(256) void gs_lcg_replay_kernel(int N, long long ncalls, uint32_t *w1, uint32_t *w2,
                                                            unsigned long long *seeds,
                                                            unsigned long long *scr) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    long long kb, ke;
    lcg_chunk(ncalls, t, kb, ke);
    const uint64_t np1 = (uint64_t)N + 1;
    uint64_t s = scr[2 * kLcgChunks + t], g = (uint64_t)kb % np1;
    for (long long k = kb; k < ke; ++k) {
        const LcgCall c = lcg_case_q(s, g);
        g = g + 1 == np1 ? 0 : g + 1;
        if (c.exc) {
            atomicMin(&scr[3 * kLcgChunks], (unsigned long long)k);
            break;
        }
        w1[k] = (uint32_t)(c.t1 >> 16);
        w2[k] = (uint32_t)(c.t2 >> 16);
        seeds[k] = c.s;
        s = c.s;
    }
}

// One block from call *kstart on (all calls when kstart is null): the same
// compose / scan / replay in a loop, with the exceptional call done exactly.
__global__ __launch_bounds__(kLcgThreads) void gs_lcg_kernel(unsigned long long seed, int N, long long ncalls,
                                                              uint32_t *w1, uint32_t *w2,
                                                              unsigned long long *seeds,
                                                              const unsigned long long *kstart) {
    __shared__ uint64_t sa[kLcgThreads], sb[kLcgThreads];
    __shared__ long long s_exc;
    const int t = threadIdx.x;
    const uint64_t np1 = (uint64_t)N + 1;
    long long k0 = kstart ? (long long)*kstart : 0;
    if (k0 >= ncalls) return;
    uint64_t s_in = k0 == 0 ? seed : seeds[k0 - 1];  // exact seed before call k0
    while (k0 < ncalls) {
        const long long n = ncalls - k0;
        const long long C = (n + kLcgThreads - 1) / kLcgThreads;
        const long long kb = k0 + t * C, ke = min(ncalls, kb + C);
        // 1. my chunk's composed case-Q map s -> a s + b (mod 2^48)
        uint64_t a = 1, b = 0;
        const uint64_t g0 = kb < ke ? (uint64_t)kb % np1 : 0;
        uint64_t g = g0;
        for (long long k = kb; k < ke; ++k) {
            a = (kAlpha * a) & kM48;
            b = (kAlpha * b + lcg_beta(g)) & kM48;
            g = g + 1 == np1 ? 0 : g + 1;
        }
        sa[t] = a;
        sb[t] = b;
        if (t == 0) s_exc = ncalls;
        __syncthreads();
        // 2. inclusive scan of the maps over threads (Hillis-Steele): after it,
        //    (sa[t], sb[t]) = F_t o ... o F_0
        for (int o = 1; o < kLcgThreads; o <<= 1) {
            uint64_t pa = 1, pb = 0;
            if (t >= o) {
                pa = sa[t - o];
                pb = sb[t - o];
            }
            __syncthreads();
            if (t >= o) {  // mine o earlier: x -> a (pa x + pb) + b
                const uint64_t na = (sa[t] * pa) & kM48, nb = (sa[t] * pb + sb[t]) & kM48;
                sa[t] = na;
                sb[t] = nb;
            }
            __syncthreads();
        }
        // 3. replay my chunk from its start seed (exact for chunks before the
        //    first exception); record the first exceptional call
        uint64_t s = t == 0 ? s_in : ((sa[t - 1] * (s_in & kM48) + sb[t - 1]) & kM48);
        g = g0;
        for (long long k = kb; k < ke; ++k) {
            const LcgCall c = lcg_case_q(s, g);
            g = g + 1 == np1 ? 0 : g + 1;
            if (c.exc) {
                atomicMin(&s_exc, k);
                break;
            }
            w1[k] = (uint32_t)(c.t1 >> 16);
            w2[k] = (uint32_t)(c.t2 >> 16);
            seeds[k] = c.s;
            s = c.s;
        }
        __syncthreads();
        const long long ke0 = s_exc;
        if (ke0 >= ncalls) break;
        // 4. the exceptional call, exactly, then continue after it
        if (t == 0) {
            const uint64_t sprev = ke0 == k0 ? s_in : seeds[ke0 - 1];
            const LcgCall c = lcg_exact(sprev, (uint64_t)ke0 % np1);
            w1[ke0] = (uint32_t)(c.t1 >> 16);
            w2[ke0] = (uint32_t)(c.t2 >> 16);
            seeds[ke0] = c.s;
            sa[0] = c.s;
        }
        __syncthreads();
        s_in = sa[0];
        k0 = ke0 + 1;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void gs_xi_kernel(const uint32_t *w1, const uint32_t *w2, double *xi,
                                                     long long n) {
    const double two32 = 4294967296.0;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const double v1 = (double)w1[k] / two32;
        const double v2 = (double)w2[k] / two32;
        const float lg = sq_glibc_logf((float)v1);
        const float cs = sq_glibc_cosf((float)(2. * 3.1415 * v2));
        const float sq = sqrtf((float)(-2. * (double)lg));
        xi[k] = (double)cs * (double)sq;
    }
}

// -------------------------------------------------------- omega, x_cl ----
// omega of every step: item N's update (:103-110,155-167), a scalar
// recurrence.  64 draws per batch land in lanes; the wave-uniform recurrence
// reads them with readlane, and lane q keeps omega of step jb + q.
__global__ __launch_bounds__(64) void gs_omega_kernel(const Qm1dGsArgs A) {
    const int N = A.N, loops = A.loops, lane = threadIdx.x;
    const double a = A.a;
    double w = A.st->omega_in;
    const double top = (double)(N - 1) * a;
    for (int jb = 0; jb < loops; jb += 64) {
        const int nb = min(64, loops - jb);
        const double dwl = lane < nb ? A.sigw * A.xi[(size_t)(jb + lane) * (N + 1) + N] : 0.;
        const int dlo = __double2loint(dwl), dhi = __double2hiint(dwl);
        double mine = 0.;
        for (int q = 0; q < nb; ++q) {
            if (lane == q) mine = w;
            const double d = __hiloint2double(__builtin_amdgcn_readlane(dhi, q), __builtin_amdgcn_readlane(dlo, q));
            const double nw = w + A.kconst * d;
            if (nw > top) w = 2 * (double)(N - 1) * a - nw;
            else if (nw < 0) w = -nw;
            else w = nw;
        }
        if (lane < nb) A.om[jb + lane] = mine;
    }
    if (lane == 0) A.om[loops] = w;
}

// potID 3: x_cl(i a, omega_j) for i = -1..N and ddPot of it, for every step
// -- the only transcendental work of the sweep and the scan, hoisted off
// their serial chains into one grid-wide pass.
__global__ __launch_bounds__(256) void gs_xcl_kernel(const Qm1dGsArgs A) {
    const int N = A.N, row = N + 2;
    const long long n = (long long)row * A.loops;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (long long)gridDim.x * blockDim.x) {
        const int j = (int)(k / row), i = (int)(k - (long long)j * row) - 1;
        const double x = xcl(i == -1 ? -1. * A.a : (double)i * A.a, A.om[j], 3);
        A.xc[k] = x;
        A.xc[n + k] = ddpot(x, 3);
    }
}

// ---------------------------------------------------- sweep -> scan ----
// The sweep and the scan of a frame run concurrently, as two blocks of one
// launch: the sweep publishes how many steps (rows of hist) are complete,
// the scan waits for the rows it is about to read.  Release/acquire at agent
// scope (the blocks sit on different XCDs, each with its own L2).
constexpr int kPublishEvery = 32;  // default phases between two sweep publications

__device__ __forceinline__ void gs_publish_rows(const Qm1dGsArgs &A, int rows, int W) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this wave's hist stores
    if (W > 1) __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&A.st->rows_ready, rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until `need` rows are complete (avail caches the last value seen).
// False after ~2 s without progress: the frame reports an error instead of
// spinning forever.
__device__ __forceinline__ bool gs_wait_rows(const Qm1dGsArgs &A, int need, int &avail) {
    if (need <= avail) return true;
    int p;
    long long spins = 0;
    while ((p = __hip_atomic_load(&A.st->rows_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < need) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1ll << 25)) return false;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    avail = p;
    return true;
}

// -------------------------------------------------------------- sweep ----
// Pipeline lane g (= thread index; W = blockDim/64 waves) runs step j in
// phase g + j.  Inside a wave the neighbour values move by lane shuffles; the
// two wave-edge values of a phase go through LDS, with one barrier after the
// first site of the phase (right neighbour's step-(j-1) value) and one at its
// end (left neighbour's step-j value).  B <= CH sites per lane, held in
// registers; the noise is prefetched a few phases ahead.
template <int CH>
struct GsChunk {
    double x[CH], d[CH];  // noise, ddPot(x_cl) per site
    double lo, hi;        // x_cl at sites -1 and N (the boundary terms)
};

template <int CH, bool P3>
__device__ __forceinline__ void gs_sweep(const Qm1dGsArgs &A, int B, int nthreads, int publish) {
    __shared__ double s_enew[16], s_eold[16], s_efirst[16];  // wave edges of the current phase
    const int N = A.N, loops = A.loops, pot = A.pot;
    const int g = threadIdx.x, lane = g & 63, wv = g >> 6, W = nthreads >> 6;
    const double h = A.h, a = A.a, a2 = A.a2, sig = A.sig;
    const int nl = (N + B - 1) / B;
    const int i0 = g * B, i1 = min(N, i0 + B);
    const bool owner = g < nl;

    // my sites' field (the serial order's f; only the owner lane reads or writes them)
    double f_[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) f_[q] = (owner && q < B && i0 + q < N) ? A.f0[i0 + q] : 0.;

    double lastnew = 0., lastold = 0.;  // my block's last site after / before my current step
    constexpr bool p3 = P3;  // potID 3 (x_cl terms), else ddPot = 2 and x_cl = 0
    const size_t dd_off = (size_t)(N + 2) * loops;
    // noise (and for potID 3 ddPot(x_cl) and the boundary x_cl) of one chunk
    auto load_chunk = [&](GsChunk<CH> &dst, int j) {
        const bool act = owner && j >= 0 && j < loops;
        const double *xr = A.xi + (size_t)j * (N + 1);
        const double *cr = A.xc + (size_t)j * (N + 2);
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int i = i0 + q;
            dst.x[q] = (act && i < i1) ? xr[i] : 0.;
            dst.d[q] = (p3 && act && i < i1) ? cr[dd_off + i + 1] : 2.;
        }
        dst.lo = (p3 && act && i0 == 0) ? cr[0] : 0.;
        dst.hi = (p3 && act && i1 == N) ? cr[N + 1] : 0.;
    };
    // state carried through one phase
    double prev_new = 0., prev_old = 0., firstval = 0., rfirst = 0.;
    // this lane's sites at step j, noise in cur
    auto run_chunk = [&](int j, const GsChunk<CH> &cur) {
        const bool act = owner && j >= 0 && j < loops;
        const bool last = j == loops - 1;
        // off the serial chain: old values, potential term, noise (same
        // sub-expressions the chain below combines in the reference's order)
        double fi[CH], rr[CH], t2[CH], dw[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int b = q;
            fi[q] = f_[q];
            rr[q] = q + 1 < CH && b < B - 1 ? f_[q + 1] : 0.;  // right neighbour inside the block: old
            t2[q] = cur.d[q] * fi[q] * h;  // ddPot(x_cl) * f * h; ddPot = 2 off potID 3
            dw[q] = sig * cur.x[q];
        }
        const double xlo = cur.lo, xhi = cur.hi;
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int b = q;
            const int i = i0 + b;
            const bool valid = act && i < i1;
            if (b == B - 1) {  // lane g+1's first site, its step j-1 (computed at b = 0 of this phase)
                rfirst = dpp_d<0x130, 0xf, 0xf>(firstval, 0.);  // wave_shl:1
                if (W > 1 && lane == 63 && wv < W - 1) rfirst = s_efirst[wv + 1];
            }
            if (b < B) {
                double v = fi[q];
                if (valid) {
                    const double L = last ? prev_old : prev_new;
                    double sum;
                    if (i == 0) sum = rr[q] + (-kEta) - xlo - 2 * fi[q];  // N >= 2, B >= 2: rr = f[1]
                    else if (i == N - 1) sum = L + kEta - xhi - 2 * fi[q];
                    else sum = (b == B - 1 ? rfirst : rr[q]) + L - 2 * fi[q];
                    v = fi[q] + kM * h * sum / a2 - t2[q] + dw[q];
                    v = guard(v);
                    A.hist[(size_t)j * N + i] = v;
                    if (!last) f_[q] = v;
                }
                prev_old = fi[q];
                prev_new = v;
                if (b == 0) firstval = v;  // = f[i0] after this phase's update (old value if idle)
                if (i == i1 - 1) {
                    lastnew = v;
                    lastold = fi[q];
                }
            }
            if (W > 1 && b == 0) {  // publish the wave's first value for the wave below
                if (lane == 0) s_efirst[wv] = firstval;
                __syncthreads();
            }
        }
    };
    auto begin_phase = [&]() {
        prev_new = dpp_d<0x138, 0xf, 0xf>(lastnew, 0.);  // wave_shr:1: lane g-1's last site, its step j
        prev_old = dpp_d<0x138, 0xf, 0xf>(lastold, 0.);  // (previous phase)
        if (W > 1 && lane == 0 && wv > 0) {
            prev_new = s_enew[wv - 1];
            prev_old = s_eold[wv - 1];
        }
        firstval = rfirst = 0.;
    };
    auto end_phase = [&]() {  // publish the wave's last values for the next phase of the wave above
        if (W > 1) {
            if (lane == 63) {
                s_enew[wv] = lastnew;
                s_eold[wv] = lastold;
            }
            __syncthreads();
        }
    };
    const int nphase = nl - 1 + loops;
    // one chunk per phase (B <= CH): a phase is short, so the noise is
    // prefetched RD phases ahead through a register ring
    constexpr int RD = CH == 2 && !P3 ? 4 : CH == 2 ? 3 : 2;
    GsChunk<CH> ring[RD];
#pragma unroll
    for (int r = 0; r < RD; ++r) load_chunk(ring[r], r - g);
    for (int p = 0; p < nphase; p += RD) {
#pragma unroll
        for (int r = 0; r < RD; ++r) {
            if (p + r >= nphase) break;
            begin_phase();
            run_chunk(p + r - g, ring[r]);
            load_chunk(ring[r], p + r + RD - g);
            end_phase();
            const int q = p + r + 1;  // phases done; step j is complete after phase nl-1+j
            if (q % publish == 0 || q == nphase) gs_publish_rows(A, min(loops, max(0, q - nl + 1)), W);
        }
    }
}

// --------------------------------------------------------------- scan ----

// N <= 64 KB: the lane's KB sites stay in registers (field, running means,
// this step's X, |X|, drift check), the next step's inputs are prefetched, and
// only f / nf go through LDS for the cross-lane reads of nf[E] and f[mid].
// The stability scan of one step as prefix maxima.
template <int KB>
__device__ __forceinline__ void gs_scan_reg(const Qm1dGsArgs &A, double *lds) {
    const int N = A.N, loops = A.loops, pot = A.pot, mid = N / 2;
    double *s_f = lds, *s_n = lds + N;
    const int lane = threadIdx.x;
    const int B = (N + 63) / 64;
    const int i0 = lane * B, i1 = min(N, i0 + B);
    const double a = A.a, sig = A.sig;
    const double NEG = -__builtin_inf();
    double f_[KB], x_[KB], xx_[KB], pr[KB], px[KB], pc[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        const int i = i0 + b;
        const bool in = b < B && i < i1;
        f_[b] = in ? A.f0[i] : 0.;
        x_[b] = in ? A.x0[i] : 0.;
        xx_[b] = in ? A.xx00[i] : 0.;
        if (in) s_f[i] = f_[b];
    }
    const bool p3 = pot == 3;
    auto prefetch = [&](int j) {
        const double *row = A.hist + (size_t)j * N;
        const double *xr = A.xi + (size_t)j * (N + 1);
        const double *cr = A.xc + (size_t)j * (N + 2) + 1;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            const bool in = b < B && i < i1;
            pr[b] = in ? row[i] : 0.;
            px[b] = in ? xr[i] : 0.;
            pc[b] = (p3 && in) ? cr[i] : 0.;
        }
    };
    int avail = 0;
    if (!gs_wait_rows(A, 1, avail)) {
        if (threadIdx.x == 0) A.st->sync_error = 1;
        return;
    }
    prefetch(0);
    __syncthreads();
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int brk_step = -1, brk_item = -1;
    double n[KB];
    for (int j = 0; j < loops; ++j) {
        const double *crow = A.xc + (size_t)j * (N + 2) + 1;  // x_cl of this step (potID 3)
        double X[KB], D[KB], xc[KB];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            n[b] = pr[b];
            xc[b] = pc[b];
            X[b] = n[b] + xc[b];
            D[b] = absol(n[b] - f_[b] - sig * px[b]);  // :139, |nf - f - dw|
            if (b < B && i < i1) s_n[i] = n[b];
        }
        if (j + 1 < loops) {
            if (!gs_wait_rows(A, j + 2, avail)) {
                if (threadIdx.x == 0) A.st->sync_error = 1;
                return;
            }
            prefetch(j + 1);
        }
        // nf[E] before item E runs this step: the previous step's value
        // (the persistent newf buffer at j = 0)
        const double nfE = j == 0 ? A.nfp[E] : s_f[E];
        const double T0 = nfE + (p3 ? crow[E] : 0.);
        double m1 = NEG, ty = NEG, ta = NEG;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            if (b < B && i < i1) {
                if (i < E) m1 = fmax(m1, X[b]);
                ta = fmax(ta, absol(X[b]));
            }
        }
        const bool caseB = dpp_all_max(m1) > T0;  // a leader before E: no reset at item E
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            if (b < B && i < i1 && (caseB || i >= E)) ty = fmax(ty, X[b]);
        }
        double py = dpp_excl_max(ty), pa = dpp_excl_max(ta);
        const double base = caseB ? T0 : NEG;
        int first_bad = 0x7fffffff, last_lead = -1;
        double Vbad = 0.;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            if (b < B && i < i1) {
                const double th = fmax(base, py);
                const bool lead = (caseB || i > E) && X[b] > th;
                const double Vi = fmax(V, pa);  // V seen by item i (max over k < i)
                if (lead) {
                    last_lead = i;
                    if (D[b] > Vi && i < first_bad) {
                        first_bad = i;
                        Vbad = fmax(Vi, absol(X[b]));
                    }
                }
                if (caseB || i >= E) py = fmax(py, X[b]);
                pa = fmax(pa, absol(X[b]));
            }
        }
        const int kb = dpp_all_min_i(first_bad);
        if (kb != 0x7fffffff && j > 0) {  // items after kb see stable != 1 and never run this round
            E = kb;
            V = __shfl(Vbad, kb / B, 64);
            brk_step = j;
            brk_item = kb;
            break;
        }
        const int ll = dpp_all_max_i(last_lead);
        if (ll >= 0) E = ll;
        V = fmax(V, dpp_all_max(ta));
        if (kb != 0x7fffffff) {  // round 0: the stable test only starts at round 1 (:168-171)
            brk_step = 0;
            brk_item = N;
            break;
        }
        __syncthreads();  // s_n of every lane written (f[mid] new)
        const double den = (double)(A.runs + j + 1);
        const double xm = p3 ? crow[mid] : 0.;
        const double fm_old = s_f[mid], fm_new = s_n[mid];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            const double g = f_[b] + xc[b];
            const double fm = (i > mid && j < loops - 1) ? fm_new : fm_old;
            xx_[b] = xx_[b] + (g * (fm + xm) - xx_[b]) / den;
            x_[b] = x_[b] + (g - x_[b]) / den;
        }
        __syncthreads();  // every lane has read s_f[mid] before it is overwritten
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            f_[b] = n[b];
            if (b < B && i < i1) s_f[i] = n[b];
        }
        __syncthreads();
    }
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        const int i = i0 + b;
        if (!(b < B && i < i1)) continue;
        if (brk_step < 0) {
            A.nf[i] = f_[b];
            A.nfp[i] = f_[b];
            A.nx[i] = x_[b];
            A.nxx0[i] = xx_[b];
        } else if (i <= brk_item) {
            A.nfp[i] = n[b];
        } else if (brk_step > 0) {
            A.nfp[i] = f_[b];  // still the previous round's value
        }
    }
    if (lane == 0) {
        A.st->lrgEl = E;
        A.st->lrgVl = V;
        A.st->stable = brk_step < 0 ? 1 : 0;
        A.st->steps_done = brk_step < 0 ? loops : brk_step + 1;
        A.st->omega_out = A.om[loops];
        A.st->consumed = brk_step < 0 ? (long long)loops * (N + 1)
                                      : (long long)brk_step * (N + 1) + brk_item + 1;
    }
}

// --------------------------------------------- scan, several waves ----
// N > 128: W waves (<= 16), KB sites per thread in registers; the wave-level
// DPP scans are joined across waves through LDS (four barriers per step).
// Same semantics and expression order as gs_scan_reg_kernel.
template <int KB>
__device__ __forceinline__ void gs_scan_mw(const Qm1dGsArgs &A, double *lds, int nthreads) {
    __shared__ double s_m1[16], s_ta[16], s_ty[16], s_vbad;
    __shared__ int s_fb[16], s_ll[16];
    const int N = A.N, loops = A.loops, pot = A.pot, mid = N / 2;
    double *s_f = lds, *s_n = lds + N;
    const int g = threadIdx.x, lane = g & 63, wv = g >> 6, W = nthreads >> 6;
    const int B = (N + nthreads - 1) / nthreads;
    const int i0 = g * B, i1 = min(N, i0 + B);
    const double a = A.a, sig = A.sig;
    const double NEG = -__builtin_inf();
    double f_[KB], x_[KB], xx_[KB], pr[KB], px[KB], pc[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        const int i = i0 + b;
        const bool in = b < B && i < i1;
        f_[b] = in ? A.f0[i] : 0.;
        x_[b] = in ? A.x0[i] : 0.;
        xx_[b] = in ? A.xx00[i] : 0.;
        if (in) s_f[i] = f_[b];
    }
    const bool p3 = pot == 3;
    auto prefetch = [&](int j) {
        const double *row = A.hist + (size_t)j * N;
        const double *xr = A.xi + (size_t)j * (N + 1);
        const double *cr = A.xc + (size_t)j * (N + 2) + 1;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            const bool in = b < B && i < i1;
            pr[b] = in ? row[i] : 0.;
            px[b] = in ? xr[i] : 0.;
            pc[b] = (p3 && in) ? cr[i] : 0.;
        }
    };
    int avail = 0;
    if (!gs_wait_rows(A, 1, avail)) {
        if (threadIdx.x == 0) A.st->sync_error = 1;
        return;
    }
    prefetch(0);
    __syncthreads();
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int brk_step = -1, brk_item = -1;
    double n[KB];
    for (int j = 0; j < loops; ++j) {
        const double *crow = A.xc + (size_t)j * (N + 2) + 1;  // x_cl of this step (potID 3)
        double X[KB], D[KB], xc[KB];
        double m1 = NEG, ta = NEG;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            n[b] = pr[b];
            xc[b] = pc[b];
            X[b] = n[b] + xc[b];
            D[b] = absol(n[b] - f_[b] - sig * px[b]);  // :139, |nf - f - dw|
            if (b < B && i < i1) {
                s_n[i] = n[b];
                if (i < E) m1 = fmax(m1, X[b]);
                ta = fmax(ta, absol(X[b]));
            }
        }
        if (j + 1 < loops) {
            if (!gs_wait_rows(A, j + 2, avail)) {
                if (threadIdx.x == 0) A.st->sync_error = 1;
                return;
            }
            prefetch(j + 1);
        }
        const double ta_wex = dpp_excl_max(ta);
        {
            const double m1w = dpp_all_max(m1), taw = dpp_all_max(ta);
            if (lane == 0) {
                s_m1[wv] = m1w;
                s_ta[wv] = taw;
            }
        }
        __syncthreads();  // #1: s_n, wave maxima of X below E and of |X|
        const double nfE = j == 0 ? A.nfp[E] : s_f[E];
        const double T0 = nfE + (p3 ? crow[E] : 0.);
        // lane k reads wave k's partial: one LDS load and a DPP reduction per quantity
        const double M1 = dpp_all_max(lane < W ? s_m1[lane] : NEG);
        const double ta_all = dpp_all_max(lane < W ? s_ta[lane] : NEG);
        const double ta_pre = dpp_all_max(lane < wv ? s_ta[lane] : NEG);
        const bool caseB = M1 > T0;  // a leader before E: no reset at item E
        double ty = NEG;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            if (b < B && i < i1 && (caseB || i >= E)) ty = fmax(ty, X[b]);
        }
        const double ty_wex = dpp_excl_max(ty);
        {
            const double tyw = dpp_all_max(ty);
            if (lane == 0) s_ty[wv] = tyw;
        }
        __syncthreads();  // #2: wave maxima of Y
        const double ty_pre = dpp_all_max(lane < wv ? s_ty[lane] : NEG);
        double py = fmax(ty_pre, ty_wex), pa = fmax(ta_pre, ta_wex);
        const double base = caseB ? T0 : NEG;
        int first_bad = 0x7fffffff, last_lead = -1;
        double Vbad = 0.;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            if (b < B && i < i1) {
                const double th = fmax(base, py);
                const bool lead = (caseB || i > E) && X[b] > th;
                const double Vi = fmax(V, pa);  // V seen by item i (max over k < i)
                if (lead) {
                    last_lead = i;
                    if (D[b] > Vi && i < first_bad) {
                        first_bad = i;
                        Vbad = fmax(Vi, absol(X[b]));
                    }
                }
                if (caseB || i >= E) py = fmax(py, X[b]);
                pa = fmax(pa, absol(X[b]));
            }
        }
        {
            const int fbw = dpp_all_min_i(first_bad), llw = dpp_all_max_i(last_lead);
            if (lane == 0) {
                s_fb[wv] = fbw;
                s_ll[wv] = llw;
            }
        }
        __syncthreads();  // #3: wave first-unstable / last-leader items
        const int kb = dpp_all_min_i(lane < W ? s_fb[lane] : 0x7fffffff);
        const int ll = dpp_all_max_i(lane < W ? s_ll[lane] : -1);
        if (kb != 0x7fffffff && j > 0) {  // items after kb see stable != 1 and never run this round
            if (first_bad == kb) s_vbad = Vbad;
            __syncthreads();
            E = kb;
            V = s_vbad;
            brk_step = j;
            brk_item = kb;
            break;
        }
        if (ll >= 0) E = ll;
        V = fmax(V, ta_all);
        if (kb != 0x7fffffff) {  // round 0: the stable test only starts at round 1 (:168-171)
            brk_step = 0;
            brk_item = N;
            break;
        }
        const double den = (double)(A.runs + j + 1);
        const double xm = p3 ? crow[mid] : 0.;
        const double fm_old = s_f[mid], fm_new = s_n[mid];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            const double gg = f_[b] + xc[b];
            const double fm = (i > mid && j < loops - 1) ? fm_new : fm_old;
            xx_[b] = xx_[b] + (gg * (fm + xm) - xx_[b]) / den;
            x_[b] = x_[b] + (gg - x_[b]) / den;
        }
        __syncthreads();  // #4: every read of s_f (E, mid) done before it is overwritten
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            f_[b] = n[b];
            if (b < B && i < i1) s_f[i] = n[b];
        }
    }
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        const int i = i0 + b;
        if (!(b < B && i < i1)) continue;
        if (brk_step < 0) {
            A.nf[i] = f_[b];
            A.nfp[i] = f_[b];
            A.nx[i] = x_[b];
            A.nxx0[i] = xx_[b];
        } else if (i <= brk_item) {
            A.nfp[i] = n[b];
        } else if (brk_step > 0) {
            A.nfp[i] = f_[b];  // still the previous round's value
        }
    }
    if (g == 0) {
        A.st->lrgEl = E;
        A.st->lrgVl = V;
        A.st->stable = brk_step < 0 ? 1 : 0;
        A.st->steps_done = brk_step < 0 ? loops : brk_step + 1;
        A.st->omega_out = A.om[loops];
        A.st->consumed = brk_step < 0 ? (long long)loops * (N + 1)
                                      : (long long)brk_step * (N + 1) + brk_item + 1;
    }
}

// ------------------------------------------------ scan by candidates ----
// The scan's only step-to-step state is (E, V).  V_j is the running maximum
// of |X| over the previous steps, independent of E; and E after a step is a
// last leader, i.e. the first position of the maximum of X over a suffix of
// that step's row: E_{j+1} is a suffix record of row j (X_i >= X_k for all
// k > i).  Rows have few suffix records (about ln N for a random row, one for
// the rising kink of potID 3), so every step is evaluated in parallel for
// every candidate E (the previous row's suffix records, the state's E at step
// 0), V-free: the candidate's next E and the leaders that are unstable for
// some V -- the leaders with D > max_{k<i}|X_k| at which D is a running
// maximum over those leaders; the first unstable leader for a given V is the
// first of these with D > V.  One wave then walks the steps with a lookup per
// step.  A row with more than kGsSlots candidates, or a candidate with more
// than kGsRec such leaders, is evaluated directly by the walker with its
// actual (E, V) -- the same routine, so the result is the same either way.
constexpr int kGsSlots = 64;   // candidates per step (one per lane of the walker)
constexpr int kGsRec = 4;      // unstable-leader records kept per candidate
constexpr int kPrepBlocks = 32;

struct GsCand {
    int4 a;                // x: candidate E, y: E after the step, z: records (-1: overflow)
    int4 ri;               // record sites
    double2 rdp[kGsRec];   // record (D_i, max_{k<=i} |X_k|)
};

__device__ __forceinline__ GsCand *gs_cand(const Qm1dGsArgs &A, int j) {
    return (GsCand *)A.cand + (size_t)j * kGsSlots;
}
__device__ __forceinline__ int *gs_nslot(const Qm1dGsArgs &A) {
    return (int *)((GsCand *)A.cand + (size_t)A.loops * kGsSlots);
}
__device__ __forceinline__ double *gs_rowmax(const Qm1dGsArgs &A) {
    return (double *)(gs_nslot(A) + ((A.loops + 1) & ~1));
}


struct GsEval {
    int ll;       // last leader of the step (-1: none)
    int nrec;     // unstable-leader records (-1: more than kGsRec)
    int fb;       // first unstable item for the query V (kNone: none)
    int ri[kGsRec];
    double rd[kGsRec], rp[kGsRec];
    double vbad;    // V after a break at fb
    double rowmax;  // max |X| over the row
};
constexpr int kNone = 0x7fffffff;

// Step j of the scan for a given E (one wave; same expressions and order as
// gs_scan_reg per item): leaders, the first unstable item for V = Vq, and the
// V-free records.
__device__ GsEval gs_eval_step(const Qm1dGsArgs &A, int j, int E, double Vq) {
    const int N = A.N, lane = threadIdx.x & 63;
    const double NEG = -__builtin_inf();
    const bool p3 = A.pot == 3;
    const double *nrow = A.hist + (size_t)j * N;
    const double *frow = j > 0 ? A.hist + (size_t)(j - 1) * N : A.f0;
    const double *xr = A.xi + (size_t)j * (N + 1);
    const double *cr = A.xc + (size_t)j * (N + 2) + 1;
    const double nfE = j == 0 ? A.nfp[E] : frow[E];
    const double T0 = nfE + (p3 ? cr[E] : 0.);
    double m1 = NEG;
    for (int c0 = 0; c0 < E; c0 += 64) {
        const int i = c0 + lane;
        if (i < E) m1 = fmax(m1, nrow[i] + (p3 ? cr[i] : 0.));
    }
    const bool caseB = dpp_all_max(m1) > T0;  // a leader before E: no reset at item E
    const double base = caseB ? T0 : NEG;
    GsEval r;
    r.ll = -1;
    r.nrec = 0;
    r.fb = kNone;
    r.vbad = 0.;
#pragma unroll
    for (int q = 0; q < kGsRec; ++q) {
        r.ri[q] = 0;
        r.rd[q] = r.rp[q] = 0.;
    }
    double cpy = NEG, cpa = NEG, cd = NEG;  // carries: max Y, max |X|, max D over the filtered leaders
    for (int c0 = 0; c0 < N; c0 += 64) {
        const int i = c0 + lane;
        const bool in = i < N;
        const double n = in ? nrow[i] : 0., f = in ? frow[i] : 0., xi = in ? xr[i] : 0.;
        const double X = n + ((p3 && in) ? cr[i] : 0.);
        const double AX = in ? absol(X) : NEG;
        const double D = absol(n - f - A.sig * xi);  // :139, |nf - f - dw|
        const double Y = (in && (caseB || i >= E)) ? X : NEG;
        const double py = fmax(cpy, dpp_excl_max(Y));
        const double pa = fmax(cpa, dpp_excl_max(AX));
        const bool lead = in && (caseB || i > E) && X > fmax(base, py);
        const double Vi = fmax(Vq, pa);
        const uint64_t bq = __ballot(lead && D > Vi);
        if (bq != 0ull && r.fb == kNone) {
            const int l = __builtin_ctzll(bq);
            r.fb = c0 + l;
            r.vbad = readlane_d(fmax(Vi, AX), l);
        }
        const bool filt = lead && D > pa;
        const double Dm = filt ? D : NEG;
        const double dpre = fmax(cd, dpp_excl_max(Dm));
        uint64_t br = __ballot(filt && D > dpre);
        const double pinc = fmax(pa, AX);
        while (br != 0ull) {
            const int l = __builtin_ctzll(br);
            br &= br - 1;
            if (r.nrec < 0) break;
            if (r.nrec == kGsRec) {
                r.nrec = -1;
                break;
            }
            const int ii = c0 + l;
            const double dd = readlane_d(D, l), pp = readlane_d(pinc, l);
#pragma unroll
            for (int q = 0; q < kGsRec; ++q) {
                if (q == r.nrec) {
                    r.ri[q] = ii;
                    r.rd[q] = dd;
                    r.rp[q] = pp;
                }
            }
            ++r.nrec;
        }
        const uint64_t bl = __ballot(lead);
        if (bl != 0ull) r.ll = c0 + 63 - __builtin_clzll(bl);
        cpy = fmax(cpy, dpp_all_max(Y));
        cpa = fmax(cpa, dpp_all_max(AX));
        cd = fmax(cd, dpp_all_max(Dm));
    }
    r.rowmax = cpa;
    return r;
}

// The suffix records of row jr (X_i >= X_k for every k > i) into out[];
// their number, or -1 when there are more than kGsSlots.  One wave.
__device__ int gs_suffix_records(const Qm1dGsArgs &A, int jr, int *out) {
    const int N = A.N, lane = threadIdx.x & 63;
    const double NEG = -__builtin_inf();
    const bool p3 = A.pot == 3;
    const double *nrow = A.hist + (size_t)jr * N;
    const double *cr = A.xc + (size_t)jr * (N + 2) + 1;
    double carry = NEG;  // max X right of the current chunk
    int cnt = 0;
    for (int hi = N; hi > 0; hi -= 64) {
        const int i = hi - 1 - lane;  // lanes walk the chunk right to left
        const bool in = i >= 0;
        const double X = in ? nrow[i] + (p3 ? cr[i] : 0.) : NEG;
        const double right = fmax(carry, dpp_excl_max(X));  // max over k > i
        const uint64_t rec = __ballot(in && X >= right);
        const int c = __builtin_popcountll(rec);
        if (cnt + c > kGsSlots) return -1;
        if ((rec >> lane) & 1ull) out[cnt + __builtin_popcountll(rec & ((1ull << lane) - 1ull))] = i;
        cnt += c;
        carry = fmax(carry, dpp_all_max(X));
    }
    return cnt;
}

// Prep block k of K: rows j = k, k+K, ... as the sweep completes them.
__device__ void gs_prep(const Qm1dGsArgs &A, int k, int K, int nthreads) {
    __shared__ int s_cand[kGsSlots];
    __shared__ int s_ns;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, W = nthreads >> 6;
    int avail = 0;
    for (int j = k; j < A.loops; j += K) {
        if (!gs_wait_rows(A, j + 1, avail)) {
            if (threadIdx.x == 0) A.st->sync_error = 1;
            return;
        }
        if (wv == 0) {
            int ns = 1;
            if (j == 0) {
                if (lane == 0) s_cand[0] = A.st->lrgEl;
            } else {
                ns = gs_suffix_records(A, j - 1, s_cand);
            }
            if (lane == 0) {
                s_ns = ns;
                gs_nslot(A)[j] = ns;
            }
        }
        __syncthreads();
        const int ns = s_ns;
        for (int s = wv; s < ns; s += W) {
            const int E = s_cand[s];
            const GsEval r = gs_eval_step(A, j, E, __builtin_inf());
            if (lane == 0) {
                GsCand c;
                c.a = make_int4(E, r.ll >= 0 ? r.ll : E, r.nrec, 0);
                c.ri = make_int4(r.ri[0], r.ri[1], r.ri[2], r.ri[3]);
#pragma unroll
                for (int q = 0; q < kGsRec; ++q) c.rdp[q] = make_double2(r.rd[q], r.rp[q]);
                gs_cand(A, j)[s] = c;
                if (s == 0) gs_rowmax(A)[j] = r.rowmax;
            }
        }
        // row j's candidates are complete: release them to the walker
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();  // (also: s_cand / s_ns are rewritten for the next row)
        if (threadIdx.x == 0) __hip_atomic_store(&A.flags[j], A.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One wave walks the steps as their candidates appear: per step the
// candidate equal to E (a ballot over the lanes, which hold the step's
// candidates), then its records against V.  Rows are taken in batches of
// kWalkBatch: one flag wait, one acquire and one round of loads per batch.
constexpr int kWalkBatch = 8;

__device__ void gs_walk(const Qm1dGsArgs &A) {
    __shared__ GsCand s_wc[kWalkBatch][kGsSlots];  // the batch's candidates, read at the matched slot
    const int N = A.N, loops = A.loops, lane = threadIdx.x & 63;
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int brk_step = -1, brk_item = -1;
    bool done = false;
    for (int j0 = 0; j0 < loops && !done; j0 += kWalkBatch) {
        const int nb = min(kWalkBatch, loops - j0);
        // wait for the batch's rows (lane q watches row j0 + q)
        long long spins = 0;
        while (true) {
            const bool ok = lane >= nb ||
                            __hip_atomic_load(&A.flags[j0 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == A.tag;
            if (__ballot(!ok) == 0ull) break;
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1ll << 25)) {
                if (lane == 0) A.st->sync_error = 1;
                return;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        int ns[kWalkBatch], ce[kWalkBatch];
        double rm[kWalkBatch];
#pragma unroll
        for (int q = 0; q < kWalkBatch; ++q) {
            const int j = min(j0 + q, loops - 1);
            ns[q] = gs_nslot(A)[j];
            rm[q] = gs_rowmax(A)[j];
            const GsCand c = gs_cand(A, j)[lane];
            ce[q] = c.a.x;
            s_wc[q][lane] = c;
        }
        __builtin_amdgcn_wave_barrier();  // (one wave: LDS writes precede the reads below)
#pragma unroll
        for (int q = 0; q < kWalkBatch; ++q) {
            const int j = j0 + q;
            if (q >= nb || done) break;
            const uint64_t m = ns[q] > 0 ? __ballot(lane < ns[q] && ce[q] == E) : 0ull;
            int fb = kNone, en = E;
            double vbad = 0., rmax = 0.;
            bool direct = m == 0ull;
            if (!direct) {
                const GsCand &c = s_wc[q][__builtin_ctzll(m)];
                en = c.a.y;
                const int nrec = c.a.z;
                rmax = rm[q];
                if (nrec < 0) {
                    direct = true;
                } else {
                    const int rr[kGsRec] = {c.ri.x, c.ri.y, c.ri.z, c.ri.w};
#pragma unroll
                    for (int q2 = 0; q2 < kGsRec; ++q2) {
                        if (q2 < nrec && fb == kNone && c.rdp[q2].x > V) {
                            fb = rr[q2];
                            vbad = fmax(V, c.rdp[q2].y);
                        }
                    }
                }
            }
            if (direct) {  // the step itself, with the actual E and V
                const GsEval r = gs_eval_step(A, j, E, V);
                fb = r.fb;
                vbad = r.vbad;
                en = r.ll >= 0 ? r.ll : E;
                rmax = r.rowmax;
            }
            if (fb != kNone && j > 0) {  // items after fb see stable != 1 and never run this round
                E = fb;
                V = vbad;
                brk_step = j;
                brk_item = fb;
                done = true;
            } else {
                E = en;
                V = fmax(V, rmax);
                if (fb != kNone) {  // round 0: the stable test only starts at round 1 (:168-171)
                    brk_step = 0;
                    brk_item = N;
                    done = true;
                }
            }
        }
    }
    // the persistent newf buffer (never rolled back, tauhost.c): the last
    // step's field, or at a break the break step's field up to the breaking
    // item and the previous step's after it
    for (int i = lane; i < N; i += 64) {
        if (brk_step < 0) A.nfp[i] = A.hist[(size_t)(loops - 1) * N + i];
        else if (i <= brk_item) A.nfp[i] = A.hist[(size_t)brk_step * N + i];
        else if (brk_step > 0) A.nfp[i] = A.hist[(size_t)(brk_step - 1) * N + i];
    }
    if (lane == 0) {
        A.st->lrgEl = E;
        A.st->lrgVl = V;
        A.st->stable = brk_step < 0 ? 1 : 0;
        A.st->steps_done = brk_step < 0 ? loops : brk_step + 1;
        A.st->omega_out = A.om[loops];
        A.st->consumed = brk_step < 0 ? (long long)loops * (N + 1) : (long long)brk_step * (N + 1) + brk_item + 1;
        A.st->brk_step = brk_step;
        A.st->brk_item = brk_item;
    }
}

// The running means of :144-145 for sites [i0, i0 + 256), over every step
// as the sweep completes it (the same recurrences and operand order as the
// scan kernels).  Written to the frame's new x / xx0 / f, which the host
// adopts only if the frame is stable.
constexpr int kMeansBatch = 8;
__device__ void gs_means(const Qm1dGsArgs &A, int i0) {
    const int N = A.N, loops = A.loops, mid = N / 2;
    const int i = i0 + (int)threadIdx.x;
    const bool in = i < N;
    const int ic = in ? i : N - 1;
    const bool p3 = A.pot == 3;
    double x = A.x0[ic], xx = A.xx00[ic], f = A.f0[ic], fmo = A.f0[mid];
    int avail = 0;
    for (int j0 = 0; j0 < loops; j0 += kMeansBatch) {
        const int nb = min(kMeansBatch, loops - j0);
        if (!gs_wait_rows(A, j0 + nb, avail)) {
            if (threadIdx.x == 0) A.st->sync_error = 1;
            return;
        }
        double cn[kMeansBatch], cm[kMeansBatch], cc[kMeansBatch], ccm[kMeansBatch];
#pragma unroll
        for (int q = 0; q < kMeansBatch; ++q) {
            const int j = min(j0 + q, loops - 1);
            cn[q] = A.hist[(size_t)j * N + ic];
            cm[q] = A.hist[(size_t)j * N + mid];
            cc[q] = p3 ? A.xc[(size_t)j * (N + 2) + 1 + ic] : 0.;
            ccm[q] = p3 ? A.xc[(size_t)j * (N + 2) + 1 + mid] : 0.;
        }
#pragma unroll
        for (int q = 0; q < kMeansBatch; ++q) {
            const int j = j0 + q;
            if (q >= nb) break;
            const double den = (double)(A.runs + j + 1);
            const double g = f + cc[q];
            const double fm = (i > mid && j < loops - 1) ? cm[q] : fmo;
            xx = xx + (g * (fm + ccm[q]) - xx) / den;
            x = x + (g - x) / den;
            f = cn[q];
            fmo = cm[q];
        }
    }
    if (in) {
        A.nf[i] = f;
        A.nx[i] = x;
        A.nxx0[i] = xx;
    }
}

// One frame: the sweep (block 0, XCD 0), candidate prep, running means and
// the walk, all concurrently.  Blocks b with b % 8 == 0 (XCD 0, round-robin
// dispatch) other than 0 stay idle so that the other roles' acquires do not
// invalidate the sweep's L2.
__host__ __device__ constexpr int gs_role_blocks(int need) {  // grid size giving `need` non-XCD-0 blocks
    return 1 + need + (need + 6) / 7;
}

template <int CH, bool P3>
__global__ __launch_bounds__(1024) void gs_frame_cand_kernel(const Qm1dGsArgs A, int B, int sweep_threads,
                                                             int publish, int nprep, int nmeans) {
    const int b = (int)blockIdx.x;
    if (b == 0) {
        if ((int)threadIdx.x < sweep_threads) gs_sweep<CH, P3>(A, B, sweep_threads, publish);
        return;
    }
    if ((b & 7) == 0 || threadIdx.x >= 256) return;
    const int k = b - 1 - (b >> 3);  // index among the non-XCD-0 blocks
    if (k < nprep) gs_prep(A, k, nprep, 256);
    else if (k < nprep + nmeans) gs_means(A, (k - nprep) * 256);
    else if (k == nprep + nmeans && threadIdx.x < 64) gs_walk(A);
}

// One frame's sweep (block 0) and scan (block 1), concurrently.  Waves past
// a block's own thread count exit at once.  SC: scan variant (0: one wave,
// 2 sites per lane; 1: one wave, 4; 2: multi-wave).
template <int CH, bool P3, int SC>
__global__ __launch_bounds__(SC == 2 ? 1024 : 256) void gs_frame_kernel(const Qm1dGsArgs A, int B, int sweep_threads,
                                                                        int scan_threads, int publish) {
    extern __shared__ double lds[];
    if (blockIdx.x == 0) {
        if ((int)threadIdx.x < sweep_threads) gs_sweep<CH, P3>(A, B, sweep_threads, publish);
    } else if ((int)threadIdx.x < scan_threads) {
        if constexpr (SC == 0) gs_scan_reg<2>(A, lds);
        else if constexpr (SC == 1) gs_scan_reg<4>(A, lds);
        else gs_scan_mw<4>(A, lds, scan_threads);
    }
}

}  // namespace

int qm1d_gs_block(int N) {  // sites per pipeline lane: 2 while <= 1024 lanes (16 waves) suffice
    if (N < 2 || N > kQm1dGsMaxN) return 0;
    return std::max(2, (N + 1023) / 1024);
}

hipError_t qm1d_gs_lcg_launch(unsigned long long seed, int N, long long ncalls, uint32_t *w1,
                              uint32_t *w2, unsigned long long *seeds, double *xi,
                              unsigned long long *scr, hipStream_t s) {
    if (scr == nullptr) {  // one block, all calls
        hipLaunchKernelGGL(gs_lcg_kernel, dim3(1), dim3(kLcgThreads), 0, s, seed, N, ncalls, w1, w2, seeds,
                           (const unsigned long long *)nullptr);
    } else {
        constexpr int blocks = kLcgChunks / 256;
        hipLaunchKernelGGL(gs_lcg_compose_kernel, dim3(blocks), dim3(256), 0, s, N, ncalls, scr);
        hipLaunchKernelGGL(gs_lcg_scan_kernel, dim3(1), dim3(1024), 0, s, seed, scr);
        hipLaunchKernelGGL(gs_lcg_replay_kernel, dim3(blocks), dim3(256), 0, s, N, ncalls, w1, w2, seeds, scr);
        hipLaunchKernelGGL(gs_lcg_kernel, dim3(1), dim3(kLcgThreads), 0, s, seed, N, ncalls, w1, w2, seeds,
                           (const unsigned long long *)(scr + 3 * kLcgChunks));
    }
    const int blocks = (int)std::min<long long>(2048, (ncalls + 255) / 256);
    hipLaunchKernelGGL(gs_xi_kernel, dim3(blocks), dim3(256), 0, s, w1, w2, xi, ncalls);
    return hipGetLastError();
}

size_t qm1d_gs_cand_bytes(int loops) {
    return sizeof(GsCand) * kGsSlots * (size_t)loops + sizeof(int) * (size_t)((loops + 1) & ~1) +
           sizeof(double) * (size_t)loops;  // + the per-row flags, allocated apart
}

hipError_t qm1d_gs_frame_launch(const Qm1dGsArgs &a, hipStream_t s) {
    const int B = qm1d_gs_block(a.N);
    if (B == 0) return hipErrorInvalidValue;
    const size_t lds1 = sizeof(double) * (size_t)a.N;
    hipLaunchKernelGGL(gs_omega_kernel, dim3(1), dim3(64), 0, s, a);
    if (a.pot == 3) {
        const long long n = (long long)(a.N + 2) * a.loops;
        const int blocks = (int)std::min<long long>(2048, (n + 255) / 256);
        hipLaunchKernelGGL(gs_xcl_kernel, dim3(blocks), dim3(256), 0, s, a);
    }
    // the dynamic-LDS limit is a per-device function attribute: set it once per device
    static bool attr_set[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    bool &attr = attr_set[dev];
    if (!attr) {
        hipError_t e;
        for (const void *k : {(const void *)gs_frame_kernel<2, false, 0>, (const void *)gs_frame_kernel<2, true, 0>,
                              (const void *)gs_frame_kernel<2, false, 1>, (const void *)gs_frame_kernel<2, true, 1>,
                              (const void *)gs_frame_kernel<2, false, 2>, (const void *)gs_frame_kernel<2, true, 2>,
                              (const void *)gs_frame_kernel<4, false, 2>, (const void *)gs_frame_kernel<4, true, 2>})
            if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)(2 * sizeof(double) * kQm1dGsMaxN))) != hipSuccess)
                return e;
        attr = true;
    }
    const int nl = (a.N + B - 1) / B;
    const int sweep_threads = 64 * ((nl + 63) / 64);  // one pipeline lane per thread, <= 1024
    // scan: one wave up to 256 sites (measured faster than two waves with barriers),
    // else 2 sites per thread up to 2048 sites (16 waves), up to 4 beyond
    const int scan_threads = a.N <= 256 ? 64 : 64 * std::min(16, (a.N + 127) / 128);
    static const int publish = [] {
        const char *e = getenv("SQ_GS_PUBLISH");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : kPublishEvery;
    }();
    static const bool seq_scan = [] {
        const char *e = getenv("SQ_GS_SCAN");
        return e != nullptr && e[0] == 's';
    }();
    if (!seq_scan) {  // sweep + candidate prep, then the walk and the outputs
        const int nprep = kPrepBlocks, nmeans = (a.N + 255) / 256;
        const dim3 g2(gs_role_blocks(nprep + nmeans + 1)), b2(std::max(sweep_threads, 256));
#define SQ_GS_CAND(CH, P3) \
    hipLaunchKernelGGL((gs_frame_cand_kernel<CH, P3>), g2, b2, 0, s, a, B, sweep_threads, publish, nprep, nmeans)
        if (B <= 2 && a.pot == 3) SQ_GS_CAND(2, true);
        else if (B <= 2) SQ_GS_CAND(2, false);
        else if (a.pot == 3) SQ_GS_CAND(4, true);
        else SQ_GS_CAND(4, false);
#undef SQ_GS_CAND
        return hipGetLastError();
    }
    const dim3 grid(2), block(std::max(sweep_threads, scan_threads));
    const size_t lds2 = 2 * lds1;
    const bool p3 = a.pot == 3;
#define SQ_GS_FRAME(CH, SC)                                                                                     \
    hipLaunchKernelGGL((p3 ? gs_frame_kernel<CH, true, SC> : gs_frame_kernel<CH, false, SC>), grid, block, lds2, \
                       s, a, B, sweep_threads, scan_threads, publish)
    if (a.N <= 128) SQ_GS_FRAME(2, 0);
    else if (a.N <= 256) SQ_GS_FRAME(2, 1);
    else if (B <= 2) SQ_GS_FRAME(2, 2);
    else SQ_GS_FRAME(4, 2);
#undef SQ_GS_FRAME
    return hipGetLastError();
}

}  // namespace sq
