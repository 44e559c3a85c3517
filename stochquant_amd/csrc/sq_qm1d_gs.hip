// sq_qm1d_gs.hip -- QM1D in the reference's own serial order (SURVEY.md §8f
// row 4): Gauss-Seidel sweep, one shared 48-bit LCG, the stability scan and
// running means exactly as time_dev runs when its work-items execute in id
// order between barriers (oracle/orc_qm1d.c serial).
//
// Four launches per frame, all on one stream:
//   gs_lcg_kernel    one block: the LCG of tau_kernel.cl:269-284 for every
//                    call of a full launch (rounds 0..loops-1, items 0..N),
//                    incl. the isinf retry; stores the accepted draw's words
//                    t1>>16, t2>>16 and the seed after each call.  The seed
//                    update is affine mod 2^48 except on rare calls, so the
//                    serial chain is a parallel prefix of affine maps plus an
//                    exact serial fix-up at the exceptions (see below).
//   gs_xi_kernel     grid-wide: xi = cos(2*3.1415*v2) * sqrt(-2 log v1) with
//                    the reference's float casts (correctly rounded float
//                    log/cos via fp64; glibc's logf/cosf round differently in
//                    ~1% of arguments, so xi is within 1 ulp of the oracle's,
//                    and bit-exact when the stream is injected).
//   gs_sweep_kernel  one wave: the GS field sweep as a skewed pipeline.  Lane l
//                    owns sites [lB, lB+B) and runs step j in phase p = l + j:
//                    the left neighbour's step-j value comes from lane l-1's
//                    previous phase, the right neighbour's step-(j-1) value
//                    from lane l+1's first site of the same phase.  Every
//                    (step, site) is computed exactly as the serial order
//                    computes it, with the reference's expression order.  The
//                    field of every step goes to hist (loops x N).
//   gs_scan_kernel   one wave: walks the steps in order and evaluates the
//                    stability scan (tau_kernel.cl:135-143) as prefix maxima
//                    (derivation in DESIGN.md §QM1D serial mode), finds the
//                    first unstable item (the serial break: items after it
//                    never run that round -- except in round 0, where the
//                    stable test has not started, :168-171) and the running
//                    means :144-145.
#include <algorithm>

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
        return kEta * (double)tanhf((float)(s * (t - w) / kEta));
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

__global__ __launch_bounds__(kLcgThreads) void gs_lcg_kernel(unsigned long long seed, int N, long long ncalls,
                                                              uint32_t *w1, uint32_t *w2,
                                                              unsigned long long *seeds) {
    __shared__ uint64_t sa[kLcgThreads], sb[kLcgThreads];
    __shared__ long long s_exc;
    const int t = threadIdx.x;
    const uint64_t np1 = (uint64_t)N + 1;
    long long k0 = 0;
    uint64_t s_in = seed;  // exact seed before call k0
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
        const float lg = (float)log((double)(float)v1);
        const float cs = (float)cos((double)(float)(2. * 3.1415 * v2));
        const float sq = sqrtf((float)(-2. * (double)lg));
        xi[k] = (double)cs * (double)sq;
    }
}

// -------------------------------------------------------------- sweep ----
// Lane l's step j happens in phase l + j.  CH sites per chunk; the chunk's
// noise is loaded one chunk ahead (the next phase's first chunk while the
// last chunk of this phase computes).
template <int CH>
__global__ __launch_bounds__(64) void gs_sweep_kernel(const Qm1dGsArgs A, int B, int om_lds) {
    extern __shared__ double s_f[];  // the field, updated in place (the serial order's f)
    double *s_om = s_f + A.N;        // om_lds: omega of every step, read once per phase
    const int N = A.N, loops = A.loops, pot = A.pot;
    const int lane = threadIdx.x;
    const double h = A.h, a = A.a, a2 = A.a2, sig = A.sig;
    const int nl = (N + B - 1) / B;
    const int i0 = lane * B, i1 = min(N, i0 + B);
    const bool owner = lane < nl;

    for (int i = lane; i < N; i += 64) s_f[i] = A.f0[i];
    {  // omega of every step: item N's update, :103-110,155-167.  64 draws
       // per batch land in lanes; the (wave-uniform) recurrence reads them
       // with readlane, and lane q keeps omega of step jb + q.
        double w = A.st->omega_in;
        const double top = (double)(N - 1) * a;
        for (int jb = 0; jb < loops; jb += 64) {
            const int nb = min(64, loops - jb);
            const double dwl = lane < nb ? A.sigw * A.xi[(size_t)(jb + lane) * (N + 1) + N] : 0.;
            double mine = 0.;
            for (int q = 0; q < nb; ++q) {
                if (lane == q) mine = w;
                const double nw = w + A.kconst * __shfl(dwl, q, 64);
                if (nw > top) w = 2 * (double)(N - 1) * a - nw;
                else if (nw < 0) w = -nw;
                else w = nw;
            }
            if (lane < nb) {
                A.om[jb + lane] = mine;
                if (om_lds) s_om[jb + lane] = mine;
            }
        }
        if (lane == 0) A.om[loops] = w;
    }
    __syncthreads();

    double lastnew = 0., lastold = 0.;  // my block's last site after / before my current step
    const int nchunk = (B + CH - 1) / CH;
    auto load_chunk = [&](double (&dst)[CH], int j, int c) {
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int i = i0 + c * CH + q;
            dst[q] = (owner && j >= 0 && j < loops && i < i1) ? A.xi[(size_t)j * (N + 1) + i] : 0.;
        }
    };
    // state carried between the chunks of one phase
    double prev_new = 0., prev_old = 0., firstval = 0., rfirst = 0.;
    // sites c*CH .. c*CH+CH-1 of this lane's block at step j, noise in cur
    auto run_chunk = [&](int j, int c, const double (&cur)[CH]) {
        const bool act = owner && j >= 0 && j < loops;
        const bool last = j == loops - 1;
        const double w = act ? (om_lds ? s_om[j] : A.om[j]) : 0.;
        // off the serial chain: old values, potential term, noise (same
        // sub-expressions the chain below combines in the reference's order)
        double fi[CH], rr[CH], t2[CH], dw[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int b = c * CH + q;
            const int i = i0 + b;
            fi[q] = (b < B && i < N) ? s_f[i] : 0.;
            rr[q] = (b < B - 1 && i + 1 < N) ? s_f[i + 1] : 0.;  // right neighbour inside the block: old
            t2[q] = ddpot(xcl((double)i * a, w, pot), pot) * fi[q] * h;
            dw[q] = sig * cur[q];
        }
        const double xlo = xcl(-1. * a, w, pot), xhi = xcl((double)N * a, w, pot);
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int b = c * CH + q;
            const int i = i0 + b;
            const bool valid = act && i < i1;
            if (b == B - 1) rfirst = __shfl_down(firstval, 1, 64);  // lane l+1's first site, its step j-1
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
                    if (!last) s_f[i] = v;
                }
                prev_old = fi[q];
                prev_new = v;
                if (b == 0) firstval = v;  // = s_f[i0] after this phase's update (old value if idle)
                if (i == i1 - 1) {
                    lastnew = v;
                    lastold = fi[q];
                }
            }
        }
    };
    auto begin_phase = [&]() {
        prev_new = __shfl_up(lastnew, 1, 64);  // lane l-1's last site, its step j (previous phase)
        prev_old = __shfl_up(lastold, 1, 64);
        firstval = rfirst = 0.;
    };
    const int nphase = nl - 1 + loops;
    if (nchunk == 1) {
        // one chunk per phase: a phase is short, so the noise is prefetched
        // four phases ahead through a four-slot register ring
        double r0[CH], r1[CH], r2[CH], r3[CH];
        load_chunk(r0, 0 - lane, 0);
        load_chunk(r1, 1 - lane, 0);
        load_chunk(r2, 2 - lane, 0);
        load_chunk(r3, 3 - lane, 0);
        auto phase = [&](int p, double (&slot)[CH]) {
            begin_phase();
            run_chunk(p - lane, 0, slot);
            load_chunk(slot, p + 4 - lane, 0);
        };
        for (int p = 0; p < nphase; p += 4) {
            phase(p, r0);
            if (p + 1 >= nphase) break;
            phase(p + 1, r1);
            if (p + 2 >= nphase) break;
            phase(p + 2, r2);
            if (p + 3 >= nphase) break;
            phase(p + 3, r3);
        }
    } else {
        // several chunks per phase: the next chunk is prefetched while this one computes
        double cur[CH], nxt[CH];
        load_chunk(cur, -lane, 0);
        for (int p = 0; p < nphase; ++p) {
            const int j = p - lane;
            begin_phase();
            for (int c = 0; c < nchunk; ++c) {
                if (c + 1 < nchunk) load_chunk(nxt, j, c + 1);
                else load_chunk(nxt, j + 1, 0);
                run_chunk(j, c, cur);
#pragma unroll
                for (int q = 0; q < CH; ++q) cur[q] = nxt[q];
            }
        }
    }
}

// --------------------------------------------------------------- scan ----
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_excl_max(double v, int lane) {  // max over lanes < lane
    double incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(incl, o, 64);
        if (lane >= o) incl = fmax(incl, u);
    }
    const double ex = __shfl_up(incl, 1, 64);
    return lane == 0 ? -__builtin_inf() : ex;
}

// LDS: f (previous step's field, the serial order's "old f"), n (this step),
// d = |n - f - dw|, x, xx0 -- 5N doubles.
__global__ __launch_bounds__(64) void gs_scan_kernel(const Qm1dGsArgs A) {
    extern __shared__ double lds[];
    const int N = A.N, loops = A.loops, pot = A.pot, mid = N / 2;
    double *s_f = lds, *s_n = lds + N, *s_x = lds + 2 * N, *s_xx0 = lds + 3 * N, *s_d = lds + 4 * N;
    const int lane = threadIdx.x;
    const int B = (N + 63) / 64;
    const int i0 = lane * B, i1 = min(N, i0 + B);
    const double a = A.a, sig = A.sig;
    const double NEG = -__builtin_inf();
    for (int i = lane; i < N; i += 64) {
        s_f[i] = A.f0[i];
        s_x[i] = A.x0[i];
        s_xx0[i] = A.xx00[i];
    }
    __syncthreads();
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int brk_step = -1, brk_item = -1;
    double w_next = A.om[0];
    // B <= KP sites per lane: the next step's history row and noise are loaded
    // into registers while this step is scanned (the loads' latency is then
    // off the per-step critical path)
    constexpr int KP = 16;
    double pr[KP], px[KP];
    auto prefetch = [&](int j) {
        const double *row = A.hist + (size_t)j * N;
        const double *xr = A.xi + (size_t)j * (N + 1);
#pragma unroll
        for (int b = 0; b < KP; ++b) {
            const int i = i0 + b;
            pr[b] = i < i1 ? row[i] : 0.;
            px[b] = i < i1 ? xr[i] : 0.;
        }
    };
    if (B <= KP) prefetch(0);
    for (int j = 0; j < loops; ++j) {
        const double w = w_next;
        if (j + 1 < loops) w_next = A.om[j + 1];  // in flight during this step
        const double *row = A.hist + (size_t)j * N;
        const double *xr = A.xi + (size_t)j * (N + 1);
        // nf[E] as the serial order sees it before item E runs this step:
        // the previous step's value (the persistent newf buffer at j = 0)
        const double nfE = j == 0 ? A.nfp[E] : s_f[E];
        const double T0 = nfE + xcl((double)E * a, w, pot);
        // this step's global inputs, staged once
        if (B <= KP) {
#pragma unroll
            for (int b = 0; b < KP; ++b) {
                const int i = i0 + b;
                if (i < i1) {
                    s_n[i] = pr[b];
                    s_d[i] = absol(pr[b] - s_f[i] - sig * px[b]);  // :139, |nf - f - dw|
                }
            }
            if (j + 1 < loops) prefetch(j + 1);
        } else {
#pragma unroll 4
            for (int i = i0; i < i1; ++i) {
                const double v = row[i];
                s_n[i] = v;
                s_d[i] = absol(v - s_f[i] - sig * xr[i]);  // :139, |nf - f - dw|
            }
        }
        double m1 = NEG;
        for (int i = i0; i < min(i1, E); ++i) m1 = fmax(m1, s_n[i] + xcl((double)i * a, w, pot));
        __syncthreads();
        const bool caseB = wave_max(m1) > T0;  // a leader before E: no reset at item E
        // lane totals of Y (X, masked below E in case A) and |X|
        double ty = NEG, ta = NEG;
        for (int i = i0; i < i1; ++i) {
            const double X = s_n[i] + xcl((double)i * a, w, pot);
            if (caseB || i >= E) ty = fmax(ty, X);
            ta = fmax(ta, absol(X));
        }
        double py = wave_excl_max(ty, lane), pa = wave_excl_max(ta, lane);
        const double base = caseB ? T0 : NEG;
        int first_bad = 0x7fffffff, last_lead = -1;
        double Vbad = 0.;
        for (int i = i0; i < i1; ++i) {
            const double X = s_n[i] + xcl((double)i * a, w, pot);
            const double th = fmax(base, py);
            const bool lead = (caseB || i > E) && X > th;
            const double Vi = fmax(V, pa);  // V seen by item i (max over k < i)
            if (lead) {
                last_lead = i;
                if (s_d[i] > Vi && i < first_bad) {
                    first_bad = i;
                    Vbad = fmax(Vi, absol(X));
                }
            }
            if (caseB || i >= E) py = fmax(py, X);
            pa = fmax(pa, absol(X));
        }
        const int kb = wave_min_i(first_bad);
        if (kb != 0x7fffffff && j > 0) {  // items after kb see stable != 1 and never run this round
            E = kb;
            V = __shfl(Vbad, kb / B, 64);
            brk_step = j;
            brk_item = kb;
            break;
        }
        const int ll = wave_max_i(last_lead);
        if (ll >= 0) E = ll;
        V = fmax(V, wave_max(ta));
        if (kb != 0x7fffffff) {  // round 0: the stable test only starts at round 1 (:168-171), all items ran
            brk_step = 0;
            brk_item = N;
            break;
        }
        // running means, :144-145 (f[i] old; f[mid] already updated for i > mid
        // except in the last step, which commits nothing)
        const double den = (double)(A.runs + j + 1);
        const double xm = xcl((double)mid * a, w, pot);
        const double fm_old = s_f[mid], fm_new = s_n[mid];
        for (int i = i0; i < i1; ++i) {
            const double g = s_f[i] + xcl((double)i * a, w, pot);
            const double fm = (i > mid && j < loops - 1) ? fm_new : fm_old;
            s_xx0[i] = s_xx0[i] + (g * (fm + xm) - s_xx0[i]) / den;
            s_x[i] = s_x[i] + (g - s_x[i]) / den;
        }
        __syncthreads();
        for (int i = i0; i < i1; ++i) s_f[i] = s_n[i];
        __syncthreads();
    }
    // persistent newf (never rolled back by the host): the last value each item wrote
    if (brk_step < 0) {
        for (int i = i0; i < i1; ++i) {
            A.nf[i] = s_f[i];
            A.nfp[i] = s_f[i];
            A.nx[i] = s_x[i];
            A.nxx0[i] = s_xx0[i];
        }
    } else {
        for (int i = i0; i < i1; ++i)
            if (i <= brk_item) A.nfp[i] = s_n[i];
            else if (brk_step > 0) A.nfp[i] = s_f[i];  // still the previous round's value
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

// ------------------------------------------------- scan, register path ----
// Wave-wide max-scans by DPP (row_shr 1/2/4/8, row_bcast 15/31: the gfx9
// inclusive-scan sequence), no LDS round trips; 64-bit values move as two
// 32-bit DPP halves.  Out-of-range lanes read the identity (bound_ctrl off).
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_d(double v, double id) {
    const int lo = __builtin_amdgcn_update_dpp((int)__double2loint(id), (int)__double2loint(v), CTRL, RM, BM, false);
    const int hi = __builtin_amdgcn_update_dpp((int)__double2hiint(id), (int)__double2hiint(v), CTRL, RM, BM, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_i(int v, int id) {
    return __builtin_amdgcn_update_dpp(id, v, CTRL, RM, BM, false);
}
__device__ __forceinline__ double dpp_incl_max(double v) {
    const double id = -__builtin_inf();
    v = fmax(v, dpp_d<0x111, 0xf, 0xf>(v, id));
    v = fmax(v, dpp_d<0x112, 0xf, 0xf>(v, id));
    v = fmax(v, dpp_d<0x114, 0xf, 0xf>(v, id));
    v = fmax(v, dpp_d<0x118, 0xf, 0xf>(v, id));
    v = fmax(v, dpp_d<0x142, 0xa, 0xf>(v, id));
    v = fmax(v, dpp_d<0x143, 0xc, 0xf>(v, id));
    return v;
}
__device__ __forceinline__ double dpp_excl_max(double v) {  // max over lanes < this lane
    return dpp_d<0x138, 0xf, 0xf>(dpp_incl_max(v), -__builtin_inf());  // wave_shr:1
}
__device__ __forceinline__ double dpp_all_max(double v) {
    const double s = dpp_incl_max(v);
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(s), 63),
                            __builtin_amdgcn_readlane(__double2loint(s), 63));
}
__device__ __forceinline__ int dpp_all_max_i(int v) {
    const int id = (int)0x80000000;
    v = max(v, dpp_i<0x111, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x112, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x114, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x118, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x142, 0xa, 0xf>(v, id));
    v = max(v, dpp_i<0x143, 0xc, 0xf>(v, id));
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int dpp_all_min_i(int v) { return -dpp_all_max_i(-v); }

// N <= 64 KB: the lane's KB sites stay in registers (field, running means,
// this step's X, |X|, drift check), the next step's inputs are prefetched, and
// only f / nf go through LDS for the cross-lane reads of nf[E] and f[mid].
// Same semantics and expression order as gs_scan_kernel.
template <int KB>
__global__ __launch_bounds__(64) void gs_scan_reg_kernel(const Qm1dGsArgs A) {
    extern __shared__ double lds[];
    const int N = A.N, loops = A.loops, pot = A.pot, mid = N / 2;
    double *s_f = lds, *s_n = lds + N;
    const int lane = threadIdx.x;
    const int B = (N + 63) / 64;
    const int i0 = lane * B, i1 = min(N, i0 + B);
    const double a = A.a, sig = A.sig;
    const double NEG = -__builtin_inf();
    double f_[KB], x_[KB], xx_[KB], pr[KB], px[KB];
#pragma unroll
    for (int b = 0; b < KB; ++b) {
        const int i = i0 + b;
        const bool in = b < B && i < i1;
        f_[b] = in ? A.f0[i] : 0.;
        x_[b] = in ? A.x0[i] : 0.;
        xx_[b] = in ? A.xx00[i] : 0.;
        if (in) s_f[i] = f_[b];
    }
    auto prefetch = [&](int j) {
        const double *row = A.hist + (size_t)j * N;
        const double *xr = A.xi + (size_t)j * (N + 1);
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            const bool in = b < B && i < i1;
            pr[b] = in ? row[i] : 0.;
            px[b] = in ? xr[i] : 0.;
        }
    };
    prefetch(0);
    __syncthreads();
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int brk_step = -1, brk_item = -1;
    double w_next = A.om[0];
    double n[KB];
    for (int j = 0; j < loops; ++j) {
        const double w = w_next;
        if (j + 1 < loops) w_next = A.om[j + 1];
        double X[KB], D[KB], xc[KB];
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            const int i = i0 + b;
            n[b] = pr[b];
            xc[b] = xcl((double)i * a, w, pot);
            X[b] = n[b] + xc[b];
            D[b] = absol(n[b] - f_[b] - sig * px[b]);  // :139, |nf - f - dw|
            if (b < B && i < i1) s_n[i] = n[b];
        }
        if (j + 1 < loops) prefetch(j + 1);
        // nf[E] before item E runs this step: the previous step's value
        // (the persistent newf buffer at j = 0)
        const double nfE = j == 0 ? A.nfp[E] : s_f[E];
        const double T0 = nfE + xcl((double)E * a, w, pot);
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
        const double xm = xcl((double)mid * a, w, pot);
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

}  // namespace

constexpr int kSweepLdsMax = 96 * 1024;

int qm1d_gs_block(int N) {
    if (N < 2 || N > kQm1dGsMaxN) return 0;
    return N <= 128 ? 2 : (N + 63) / 64;
}

hipError_t qm1d_gs_lcg_launch(unsigned long long seed, int N, long long ncalls, uint32_t *w1,
                              uint32_t *w2, unsigned long long *seeds, double *xi, hipStream_t s) {
    hipLaunchKernelGGL(gs_lcg_kernel, dim3(1), dim3(kLcgThreads), 0, s, seed, N, ncalls, w1, w2, seeds);
    const int blocks = (int)std::min<long long>(2048, (ncalls + 255) / 256);
    hipLaunchKernelGGL(gs_xi_kernel, dim3(blocks), dim3(256), 0, s, w1, w2, xi, ncalls);
    return hipGetLastError();
}

hipError_t qm1d_gs_frame_launch(const Qm1dGsArgs &a, hipStream_t s) {
    const int B = qm1d_gs_block(a.N);
    if (B == 0) return hipErrorInvalidValue;
    const size_t lds1 = sizeof(double) * (size_t)a.N, lds5 = 5 * lds1;
    // the dynamic-LDS limit is a per-device function attribute: set it once per device
    static bool attr_set[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    bool &attr = attr_set[dev];
    if (!attr) {
        hipError_t e;
        if ((e = hipFuncSetAttribute((const void *)gs_scan_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(5 * sizeof(double) * kQm1dGsMaxN))) != hipSuccess)
            return e;
        for (const void *k : {(const void *)gs_sweep_kernel<2>, (const void *)gs_sweep_kernel<8>})
            if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kSweepLdsMax)) != hipSuccess)
                return e;
        attr = true;
    }
    // omega of all steps next to the field in LDS when it fits (one LDS read per phase
    // instead of a global load on the pipeline's critical path)
    const size_t lds_om = sizeof(double) * ((size_t)a.N + a.loops + 1);
    const int om_lds = lds_om <= (size_t)kSweepLdsMax ? 1 : 0;
    const size_t lds_sw = om_lds ? lds_om : lds1;
    if (B <= 2) hipLaunchKernelGGL(gs_sweep_kernel<2>, dim3(1), dim3(64), lds_sw, s, a, B, om_lds);
    else hipLaunchKernelGGL(gs_sweep_kernel<8>, dim3(1), dim3(64), lds_sw, s, a, B, om_lds);
    const int B3 = (a.N + 63) / 64;
    const size_t lds2 = 2 * lds1;
    if (B3 <= 2) hipLaunchKernelGGL(gs_scan_reg_kernel<2>, dim3(1), dim3(64), lds2, s, a);
    else if (B3 <= 4) hipLaunchKernelGGL(gs_scan_reg_kernel<4>, dim3(1), dim3(64), lds2, s, a);
    else if (B3 <= 8) hipLaunchKernelGGL(gs_scan_reg_kernel<8>, dim3(1), dim3(64), lds2, s, a);
    else if (B3 <= 16) hipLaunchKernelGGL(gs_scan_reg_kernel<16>, dim3(1), dim3(64), lds2, s, a);
    else hipLaunchKernelGGL(gs_scan_kernel, dim3(1), dim3(64), lds5, s, a);
    return hipGetLastError();
}

}  // namespace sq
