// sq_qm1d.hip -- the reference model (tau_kernel.cl:25-175) on gfx950, fp64.
//
// One frame = `loops` Euler-Maruyama steps of the fluctuation chain f (N sites,
// Dirichlet ghosts) plus the collective coordinate omega, in ONE launch of ONE
// workgroup (the reference also relies on a single work-group: its barrier at
// tau_kernel.cl:168 is the only step-to-step sync).  What differs by design:
//   * Jacobi ordering: every site reads the old field (the reference's order
//     is whatever its runtime serialises);
//   * noise from Philox4x32-10 per (site, step) instead of one shared LCG
//     that every work-item races on (tau_kernel.cl:269-284);
//   * the stability scan (tau_kernel.cl:135-143, racy shared lrgEl/lrgVl)
//     becomes an order-independent block prefix-max scan with the serial
//     scan's meaning (oracle/orc_qm1d.c, orc_qm1d_frame);
//   * omega is computed redundantly by every thread from its own counter-based
//     normal, so no broadcast is needed.
// Thread t owns K consecutive sites in registers; neighbour edges, f[mid] and
// scan partials go through LDS.  Expressions keep the reference's order and
// the file is built with -ffp-contract=off, so for potID 0 the deterministic
// part is bit-identical to the oracle.
#include <hip/hip_cooperative_groups.h>

#include <algorithm>
#include <cstdlib>

#include "sq_dpp.h"
#include "sq_glibcf.h"
#include "sq_internal.h"
#include "sq_rng.h"

namespace sq {

namespace {

constexpr double kEta = .8;  // tau_kernel.cl:19-22
constexpr double kV0 = 2.;
constexpr double kM = 1.;
constexpr int kMaxThreads = 1024;

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
// potID 3: the float tanhf inside clas() (x_cl = kEta * (double) of it)
__device__ __forceinline__ float xcl_tanh(double t, double w) {
    const double s = 2.0;  // (double)sqrtf((float)(2.*V0/m)) == 2 exactly
    return sq_glibc_tanhf((float)(s * (t - w) / kEta));
}

// a / b for a divisor b shared by many quotients (a2 for the frame, the step's
// den), bit-identical to the compiler's fp64 division.  That expansion is
//   r = rcp(b'); two Newton steps R = fma(r1, fma(-b', r1, 1), r1) with
//   r1 = fma(r, fma(-b', r, 1), r); m = a' R; q = fixup(fmas(fma(-b', m, a'), R, m))
// where b', a' are v_div_scale's operands: b and a themselves, with vcc clear,
// unless an exponent is extreme.  With b in [2^-60, 2^60] (UDiv::ok) and
// 2^-960 < |a| < 2^700 nothing is scaled, div_fmas is a plain fma and
// div_fixup returns its (finite, normal) input, so R is computed once per
// divisor and a quotient is a multiply and two fmas instead of 10 instructions
// with a quarter-rate v_rcp_f64.  Any other a (0, -0, inf, NaN, tiny or huge)
// takes the full division (udiv_step).
struct UDiv {
    double b, r;
    bool ok;  // b in [2^-60, 2^60]: otherwise every quotient takes the full division
};
__device__ __forceinline__ UDiv udiv_prep(double b) {
    const double r0 = __builtin_amdgcn_rcp(b);
    const double r1 = __builtin_fma(r0, __builtin_fma(-b, r0, 1.0), r0);
    return UDiv{b, __builtin_fma(r1, __builtin_fma(-b, r1, 1.0), r1), b >= 0x1p-60 && b <= 0x1p+60};
}
__device__ __forceinline__ bool udiv_range(double a) {  // false for 0, NaN, inf, tiny, huge
    const double x = __builtin_fabs(a);
    return x > 0x1p-960 && x < 0x1p+700;
}
__device__ __forceinline__ double udiv_fast(double a, const UDiv &d) {
    const double m = a * d.r;
    return __builtin_fma(__builtin_fma(-d.b, m, a), d.r, m);
}
// The quotients of one step: the fast form unless some lane of the wave has a
// numerator outside its range (one wave-uniform branch per step, not one per
// quotient: per-quotient branches cost more than the division they skip).
template <int M, bool FAST>
__device__ __forceinline__ void udiv_step(const double (&n)[M], const UDiv &d, double (&q)[M], bool bad) {
    if (!FAST || __ballot(bad || !d.ok) != 0ull) {
        asm volatile("");  // a real branch: an fdiv is one IR instruction, cheap enough to speculate
#pragma unroll
        for (int k = 0; k < M; ++k) q[k] = n[k] / d.b;
    } else {
#pragma unroll
        for (int k = 0; k < M; ++k) q[k] = udiv_fast(n[k], d);
    }
}

__device__ __forceinline__ double wave_incl_max(double v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(v, o, 64);
        if (lane >= o) v = fmax(v, u);
    }
    return v;
}

template <int K>
__device__ __forceinline__ double pick(const double (&v)[K], int k) {  // v[k], k wave-uniform
    double r = v[0];
#pragma unroll
    for (int q = 1; q < K; ++q)
        if (q == k) r = v[q];
    return r;
}

// One frame, N <= 4,096: thread g (= 64 wave + lane) owns sites [gK, gK+K)
// in registers; W = blockDim/64 <= 16 waves (MW) or one wave.  The
// field-independent work -- omega's recurrence, the site normals, potID 3's
// x_cl and ddPot -- comes precomputed from qm1d_prep_launch's tables (read one
// step ahead), so a step is only the chain's own arithmetic.  Per step:
//   1. site updates from the old field (left/right neighbours by DPP wave
//      shifts; across waves through LDS), running means, guard, X', drift
//      check;
//   2. the scan's maxima: lane max of X' (first index) and |X'|, DPP
//      prefix maxima inside the wave, one LDS slot per wave across waves;
//      the step's last leader is the first index of the maximum X' when that
//      exceeds X'(E) (leaders are strict running-maximum records), V' =
//      max(V, max |X'|), a site is an unstable leader iff X' exceeds every X'
//      before it and X'(E) while its drift check exceeds V and every |X'|
//      before it (oracle/orc_qm1d.c orc_qm1d_frame, tau_kernel.cl:135-143).
// One wave needs no barrier at all (readlane / ballot); W waves use two per
// step, with the LDS slots double-buffered by step parity.  The maxima are
// v_max_f64 as is (dpp_vmax_d): every operand is a result of arithmetic or
// the carried state, never a signalling NaN, so fmax's quieting is dead weight.
template <int K>
struct StepTab {  // one step's table values of a lane's K sites
    float xi[K], t[K];
    double dd[K];
    float tl, tr, tm;  // x_cl tanhf at -a, N a and mid a (potID 3)
};

template <int K>
__device__ __forceinline__ void load_tab(const Qm1dArgs &A, int j, int i0, int mid, bool p3, StepTab<K> &T) {
    const int N = A.N, nq4 = (N + 3) & ~3;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = min(i0 + k, N - 1);
        T.xi[k] = A.xi[(size_t)j * nq4 + i];
        if (p3) {
            T.t[k] = A.tcl[(size_t)j * (N + 2) + i + 1];
            T.dd[k] = A.dd[(size_t)j * N + i];
        }
    }
    if (p3) {
        const float *r = A.tcl + (size_t)j * (N + 2);
        T.tl = r[0];
        T.tr = r[N + 1];
        T.tm = r[mid + 1];
    }
}

template <int K, bool MW, bool P3>
__global__ __launch_bounds__(MW ? 1024 : 64) void qm1d_frame_wave(const Qm1dArgs A) {
    constexpr int kW = 16;
    __shared__ double s_first[2][kW], s_last[2][kW], s_mx[2][kW], s_ma[2][kW];
    __shared__ int s_arg[2][kW], s_un[2][kW];
    __shared__ double s_fmid[2], s_xe[2];

    const int N = A.N, mid = N / 2;
    constexpr bool p3 = P3;  // potID 3 (the launcher picks the instance by A.pot)
    // the shared-divisor division pays at 4 sites per lane (N = 1000: 3.12 -> 2.71 ms
    // per 1000-step frame, N = 3072: 1.20 -> 0.95); with fewer sites the step's
    // uniform branch costs more than it saves (N = 100: 1.18 -> 1.24)
    constexpr bool kFastDiv = K >= 4;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int W = MW ? (int)(blockDim.x >> 6) : 1;
    const int i0 = (int)threadIdx.x * K;
    const double h = A.h;
    const UDiv da2 = udiv_prep(A.a2);
    const double ninf = -__builtin_inf();

    double f[K], x[K], xx0[K], Xn[K], dchk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = i0 + k;
        f[k] = i < N ? A.f[i] : 0.;
        x[k] = i < N ? A.x[i] : 0.;
        xx0[k] = i < N ? A.xx0[i] : 0.;
    }
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int stable = 1, steps = 0;

    // neighbours and f[mid] of the frame-start field
    double fL = dpp_from_left(f[K - 1], 0.), fR = dpp_from_right(f[0], 0.), fmid;
    if constexpr (MW) {
        if (lane == 0) s_first[1][wv] = f[0];
        if (lane == 63) s_last[1][wv] = f[K - 1];
        if (mid / K == (int)threadIdx.x) s_fmid[1] = pick(f, mid % K);
        __syncthreads();
        if (lane == 0 && wv > 0) fL = s_last[1][wv - 1];
        if (lane == 63 && wv + 1 < W) fR = s_first[1][wv + 1];
        fmid = s_fmid[1];
    } else {
        fmid = readlane_d(pick(f, mid % K), mid / K);
    }
    StepTab<K> cur, nxt;
    load_tab<K>(A, 0, i0, mid, p3, cur);

    // one step; true when it ends the frame.  Unrolled two ways below so the
    // tables alternate between cur and nxt without copies.
    auto step = [&](const int j, const StepTab<K> &cur, StepTab<K> &nxt) -> bool {
        const int p = j & 1;
        if (j + 1 < A.loops) load_tab<K>(A, j + 1, i0, mid, p3, nxt);  // one step ahead
        // ---- 1. site updates ----
        const double Xm = fmid + (p3 ? kEta * (double)cur.tm : 0.);
        const UDiv dden = udiv_prep((double)(A.runs + j + 1));
        // numerators first, then every quotient of the step (udiv_step)
        double nA[K], qA[K];
        double nM2[2 * K], qM2[2 * K];  // the running means': xx0's K numerators, then x's
        bool bad = false;
        {
            double prev_old = fL;  // old f[i-1]
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = i0 + k;
                const double fi = f[k];
                const double xc = p3 ? kEta * (double)cur.t[k] : 0.;  // clas(), :184-189
                const double fr = (k + 1 < K) ? f[k + 1] : fR;
                if (i == 0)
                    nA[k] = kM * h * (fr + (-kEta) - (p3 ? kEta * (double)cur.tl : 0.) - 2 * fi);
                else if (i == N - 1)
                    nA[k] = kM * h * (prev_old + kEta - (p3 ? kEta * (double)cur.tr : 0.) - 2 * fi);
                else
                    nA[k] = kM * h * (fr + prev_old - 2 * fi);
                // running means from the OLD field, :144-145
                const double Xi = fi + xc;
                nM2[k] = Xi * Xm - xx0[k];
                nM2[K + k] = Xi - x[k];
                if (i < N) bad = bad || !(udiv_range(nA[k]) && udiv_range(nM2[k]) && udiv_range(nM2[K + k]));
                prev_old = fi;
            }
        }
        udiv_step<K, kFastDiv>(nA, da2, qA, bad);
        udiv_step<2 * K, kFastDiv>(nM2, dden, qM2, bad);
        double lmaxX = ninf, lmaxA = ninf;
        int larg = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = i0 + k;
            Xn[k] = ninf;
            dchk[k] = 0.;
            if (i < N) {
                const double fi = f[k];
                const double xc = p3 ? kEta * (double)cur.t[k] : 0.;  // clas(), :184-189
                const double dp = p3 ? cur.dd[k] : 2.;                // ddPot(), :190-195
                const double dw = A.sig * (double)cur.xi[k];
                double v = fi + qA[k] - dp * fi * h + dw;
                if (v > 1000) v = 1000;  // guard, :119-133
                if (v < -1000) v = -1000;
                if (v != v) v = 1000;
                dchk[k] = absol(v - fi - dw);
                const double X = v + xc;
                Xn[k] = X;
                if (X > lmaxX) {
                    lmaxX = X;
                    larg = i;
                }
                lmaxA = dpp_vmax_d(lmaxA, absol(X));
                xx0[k] = xx0[k] + qM2[k];
                x[k] = x[k] + qM2[K + k];
                f[k] = v;
            }
        }
        // ---- 2. scan maxima ----
        const double wmx = dpp_all_max(lmaxX), wma = dpp_all_max(lmaxA);
        const unsigned long long hit = __ballot(lmaxX == wmx);
        const int warg = __builtin_amdgcn_readlane(larg, (int)__builtin_ctzll(hit));
        double XE, pX, pA, gX, totA;
        int garg;
        if constexpr (MW) {
            if (lane == 0) {
                s_mx[p][wv] = wmx;
                s_ma[p][wv] = wma;
                s_arg[p][wv] = warg;
                s_first[p][wv] = f[0];
            }
            if (lane == 63) s_last[p][wv] = f[K - 1];
            if (E / K == (int)threadIdx.x) s_xe[p] = pick(Xn, E % K);
            if (mid / K == (int)threadIdx.x) s_fmid[p] = pick(f, mid % K);
            __syncthreads();
            XE = s_xe[p];
            pX = XE;
            pA = V;
            gX = ninf;
            garg = 0;
            totA = V;
            for (int w = 0; w < W; ++w) {
                const double mx = s_mx[p][w], ma = s_ma[p][w];
                if (w < wv) {
                    pX = dpp_vmax_d(pX, mx);
                    pA = dpp_vmax_d(pA, ma);
                }
                totA = dpp_vmax_d(totA, ma);
                if (mx > gX) {
                    gX = mx;
                    garg = s_arg[p][w];
                }
            }
        } else {
            XE = readlane_d(pick(Xn, E % K), E / K);
            pX = XE;
            pA = V;
            gX = wmx;
            garg = warg;
            totA = dpp_vmax_d(V, wma);
        }
        double runX = dpp_vmax_d(pX, dpp_excl_max(lmaxX)), runA = dpp_vmax_d(pA, dpp_excl_max(lmaxA));
        int unst = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (Xn[k] > runX) {
                runX = Xn[k];
                if (dchk[k] > runA) unst = 1;
            }
            runA = dpp_vmax_d(runA, absol(Xn[k]));
        }
        int any = __ballot(unst) != 0ull;
        // neighbours of the new field for the next step
        fL = dpp_from_left(f[K - 1], 0.);
        fR = dpp_from_right(f[0], 0.);
        if constexpr (MW) {
            if (lane == 0) s_un[p][wv] = any;
            if (lane == 0 && wv > 0) fL = s_last[p][wv - 1];
            if (lane == 63 && wv + 1 < W) fR = s_first[p][wv + 1];
            fmid = s_fmid[p];
            __syncthreads();
            any = 0;
            for (int w = 0; w < W; ++w) any |= s_un[p][w];
        } else {
            fmid = readlane_d(pick(f, mid % K), mid / K);
        }
        if (gX > XE) E = garg;
        V = totA;
        steps = j + 1;
        if (any) {
            stable = 0;
            return true;
        }
        return false;
    };
    for (int j = 0; j < A.loops; j += 2) {
        if (step(j, cur, nxt)) break;
        if (j + 1 >= A.loops || step(j + 1, nxt, cur)) break;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = i0 + k;
        if (i < N) {
            A.nf[i] = f[k];
            A.nx[i] = x[k];
            A.nxx0[i] = xx0[k];
        }
    }
    if (threadIdx.x == 0) {
        A.st->omega_out = A.om[steps];  // the collective coordinate after the last step run
        A.st->lrgEl = E;
        A.st->lrgVl = V;
        A.st->stable = stable;
        A.st->steps_done = steps;
    }
}

// omega at the start of every step of a frame, om[0..loops] (item N's scalar
// recurrence, tau_kernel.cl:103-110,155-167), one wave: the normals of 64
// steps at once, one step per lane, the recurrence by readlane.
__global__ __launch_bounds__(64) void qm1d_omega_kernel(const Qm1dArgs A) {
    const int lane = threadIdx.x;
    const int N = A.N;
    double om = A.st->omega_in;
    if (lane == 0) A.om[0] = om;
    const double top = (double)(N - 1) * A.a;
    for (int j0 = 0; j0 < A.loops; j0 += 64) {
        const unsigned long long sl = A.tick + (unsigned long long)(j0 + lane);
        const float w = normals4(0ull, kStreamOmega, (uint32_t)sl, (uint32_t)(sl >> 32), A.k0, A.k1).a;
        const double d = A.kconst * (A.sigw * (double)w);
        const int n = min(64, A.loops - j0);
        for (int q = 0; q < n; ++q) {
            const double nwo = om + readlane_d(d, q);
            if (nwo > top) om = 2 * (double)(N - 1) * A.a - nwo;
            else if (nwo < 0) om = -nwo;
            else om = nwo;
            if (lane == 0) A.om[j0 + q + 1] = om;
        }
    }
}

// The site normals of every step (4 per Philox call, quad q of step j) and,
// potID 3, x_cl's tanhf at i = -1..N and ddPot at i = 0..N-1 for omega om[j].
__global__ __launch_bounds__(256) void qm1d_tables_kernel(const Qm1dArgs A) {
    const int N = A.N, nq = (N + 3) >> 2, nq4 = nq * 4;
    const long long total = (long long)A.loops * nq;
    for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (long long)gridDim.x * blockDim.x) {
        const int j = (int)(g / nq), q = (int)(g % nq);
        const unsigned long long step = A.tick + (unsigned long long)j;
        const f32x4n n = normals4((unsigned long long)q, kStreamField, (uint32_t)step, (uint32_t)(step >> 32), A.k0,
                                  A.k1);
        float *xo = A.xi + (size_t)j * nq4 + 4 * q;
        xo[0] = n.a;
        xo[1] = n.b;
        xo[2] = n.c;
        xo[3] = n.d;
        if (A.pot == 3) {
            const double w = A.om[j];
            float *to = A.tcl + (size_t)j * (N + 2);
            double *dout = A.dd + (size_t)j * N;
            for (int i = 4 * q; i < min(4 * q + 4, N); ++i) {
                const float t = xcl_tanh((double)i * A.a, w);
                to[i + 1] = t;
                dout[i] = ddpot(kEta * (double)t, 3);
            }
            if (q == 0) {
                to[0] = xcl_tanh(-1. * A.a, w);
                to[N + 1] = xcl_tanh((double)N * A.a, w);
            }
        }
    }
}

// The same frame for N > 4096 (config C1's 32,768-site chain): one work-group,
// K sites per thread held in global memory (L2-resident at these sizes)
// instead of registers.  Every thread reads and writes only its own sites;
// neighbour edges and f[mid] still go through LDS, so no cross-thread global
// visibility is needed.  f ping-pongs between nf and the scratch fs (the
// frame-start f stays untouched: it is the rollback snapshot); X' and the
// drift check of each site are parked in scratch for the scan walk.
template <int K>
__global__ __launch_bounds__(kMaxThreads) void qm1d_frame_kernel_glob(const Qm1dArgs A) {
    __shared__ double s_first[kMaxThreads], s_last[kMaxThreads];
    __shared__ double s_wmaxX[kMaxThreads / 64], s_wmaxA[kMaxThreads / 64];
    __shared__ double s_fmid, s_R;
    __shared__ int s_leader[2];

    const int N = A.N, pot = A.pot, mid = N / 2;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = blockDim.x >> 6;
    const int i0 = t * K;
    const int own = max(0, min(K, N - i0));
    const double h = A.h, a = A.a, a2 = A.a2;
    for (int k = 0; k < own; ++k) {
        A.nx[i0 + k] = A.x[i0 + k];
        A.nxx0[i0 + k] = A.xx0[i0 + k];
    }
    double om = A.st->omega_in;
    int E = A.st->lrgEl;
    double V = A.st->lrgVl;
    int stable = 1, steps = 0;
    const double *fin = A.f;
    double *fout = A.nf;

    for (int j = 0; j < A.loops; ++j) {
        const unsigned long long step = A.tick + (unsigned long long)j;
        const uint32_t slo = (uint32_t)step, shi = (uint32_t)(step >> 32);
        s_first[t] = own ? fin[i0] : 0.;
        s_last[t] = own ? fin[i0 + own - 1] : 0.;
        if (mid >= i0 && mid < i0 + own) s_fmid = fin[mid];
        if (t == 0) s_leader[j & 1] = -1;
        __syncthreads();
        const double fL = t > 0 ? s_last[t - 1] : 0.;
        const double fR = (t + 1 < (int)blockDim.x) ? s_first[t + 1] : 0.;
        const double Xm = s_fmid + xcl((double)mid * a, om, pot);
        const double den = (double)(A.runs + j + 1);
        double prev_old = fL;
        double lmaxX = -INFINITY, lmaxA = -INFINITY;
        f32x4n nq{0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < own; ++k) {
            const int i = i0 + k;
            if ((k & 3) == 0)
                nq = normals4((unsigned long long)(i >> 2), kStreamField, slo, shi, A.k0, A.k1);
            const float xi = (k & 3) == 0 ? nq.a : (k & 3) == 1 ? nq.b : (k & 3) == 2 ? nq.c : nq.d;
            const double fi = fin[i];
            const double fr = (k + 1 < own) ? fin[i + 1] : fR;
            const double xc = xcl((double)i * a, om, pot);
            const double dw = A.sig * (double)xi;
            double v;
            if (i == 0)
                v = fi + kM * h * (fr + (-kEta) - xcl(-1. * a, om, pot) - 2 * fi) / a2 -
                    ddpot(xc, pot) * fi * h + dw;
            else if (i == N - 1)
                v = fi + kM * h * (prev_old + kEta - xcl((double)N * a, om, pot) - 2 * fi) / a2 -
                    ddpot(xc, pot) * fi * h + dw;
            else
                v = fi + kM * h * (fr + prev_old - 2 * fi) / a2 - ddpot(xc, pot) * fi * h + dw;
            if (v > 1000) v = 1000;
            if (v < -1000) v = -1000;
            if (v != v) v = 1000;
            const double X = v + xc;
            A.xs[i] = X;
            A.ds[i] = absol(v - fi - dw);
            lmaxX = fmax(lmaxX, X);
            lmaxA = fmax(lmaxA, absol(X));
            const double Xi = fi + xc;
            A.nxx0[i] = A.nxx0[i] + (Xi * Xm - A.nxx0[i]) / den;
            A.nx[i] = A.nx[i] + (Xi - A.nx[i]) / den;
            prev_old = fi;
            fout[i] = v;
        }
        if (E >= i0 && E < i0 + own) s_R = A.xs[E];
        const double ix = wave_incl_max(lmaxX, lane);
        const double ia = wave_incl_max(lmaxA, lane);
        double ex = __shfl_up(ix, 1, 64), ea = __shfl_up(ia, 1, 64);
        if (lane == 0) {
            ex = -INFINITY;
            ea = -INFINITY;
        }
        if (lane == 63) {
            s_wmaxX[wv] = ix;
            s_wmaxA[wv] = ia;
        }
        __syncthreads();
        double runX = s_R, runA = V, totA = V;
        for (int w = 0; w < nw; ++w) {
            const double wx = s_wmaxX[w], wa = s_wmaxA[w];
            if (w < wv) {
                runX = fmax(runX, wx);
                runA = fmax(runA, wa);
            }
            totA = fmax(totA, wa);
        }
        runX = fmax(runX, ex);
        runA = fmax(runA, ea);
        int unst = 0, leader = -1;
        for (int k = 0; k < own; ++k) {
            const int i = i0 + k;
            const double X = A.xs[i];
            if (X > runX) {
                runX = X;
                leader = i;
                if (A.ds[i] > runA) unst = 1;
            }
            runA = fmax(runA, absol(X));
        }
        if (leader >= 0) atomicMax(&s_leader[j & 1], leader);
        const int any_unst = __syncthreads_or(unst);
        const int Lw = s_leader[j & 1];
        if (Lw >= 0) E = Lw;
        V = totA;
        const f32x4n nwn = normals4(0ull, kStreamOmega, slo, shi, A.k0, A.k1);
        const double nwo = om + A.kconst * (A.sigw * (double)nwn.a);
        if (nwo > (double)(N - 1) * a) om = 2 * (double)(N - 1) * a - nwo;
        else if (nwo < 0) om = -nwo;
        else om = nwo;
        steps = j + 1;
        fin = fout;
        fout = (fout == A.nf) ? A.fs : A.nf;
        if (any_unst) {
            stable = 0;
            break;
        }
    }
    if (fin != A.nf)
        for (int k = 0; k < own; ++k) A.nf[i0 + k] = fin[i0 + k];
    if (t == 0) {
        A.st->omega_out = om;
        A.st->lrgEl = E;
        A.st->lrgVl = V;
        A.st->stable = stable;
        A.st->steps_done = steps;
    }
}

// The same frame for N > 4096 on the whole chip (config C1's 32,768-site
// chain; qm1d_frame_kernel_glob runs it on one CU): G = ceil(N / (256 K))
// co-resident blocks of 256 threads, thread g owning sites [Kg, Kg+K) in
// registers -- the field, the drift checks and the running means never leave
// them (K = the fewest sites with G <= 128: 1 at N = 32,768).  ONE grid
// barrier per step, between
//   1. site updates from the old field (the two neighbour sites and f[mid]
//      loaded right after the previous barrier, written by their owners
//      before it), running means, guard, X', drift check; stored for other
//      threads only: the thread's edge sites, f[mid], X' at the sites the
//      next scan can need (by parity), the per-block maxima of X' and |X'|;
//   2. the outcome of the previous step's scan (its leader and instability:
//      step-tagged atomic-max words its scan wrote before this barrier, so no
//      slot needs resetting) -- an unstable previous step ends the frame here,
//      this step's updates discarded as the one-CU kernel never makes them --
//      then this step's ordered scan: every block forms the exclusive prefix
//      over the blocks before it (G values) and the in-block prefix by wave
//      scans, and walks its sites in order exactly as qm1d_frame_kernel_glob
//      (a site is a leader when X' exceeds X'(E) and every X' before it,
//      unstable when its drift check also exceeds V and every |X'| before it),
//      then omega's step, computed redundantly by every thread.
// Everything phase 2 of step j reads was written in phase 1 of step j (by
// parity, so phase 1 of step j+1 in a faster block does not overwrite it) or
// before the previous barrier.  Bit-identical to the one-CU kernel (same
// expressions, the same order of every max; tests/test_gpu_qm1d.py::
// test_grid_frame_equals_one_cu_frame, and the oracle tests at N > 4096).
// Scratch: xs / ds (N + kGridAux doubles each) hold X' of even / odd steps,
// xs[N..] the block maxima, ds[N..] the tagged words (leader by parity,
// instability), the counter and the per-block flags of the barrier.
constexpr int kGridT = 256;

// Grid barrier of a grid whose blocks are all co-resident: thread 0 of
// each block releases its block's writes, counts the block in and spins until
// every block of barrier `n` (1-based) has; the counter was zeroed ahead of the
// launch.  A vector atomic and a relaxed load, no scalar-memory writes.
// Bounded: the plain launch leaves co-residency to the host's occupancy check
// (qm1d_frame_launch), so a block that is never scheduled -- or never arrives
// -- must not hang the process.  After `polls` polls (or once another block has
// given up, err != 0) the block raises *err and the barrier returns false: the
// caller's block leaves the kernel, every other block then gives up in turn,
// and the host reports the frame as failed (Qm1dState::sync_error).
constexpr unsigned int kGridSpinMax = 1u << 22;  // ~2-4 s of polls; a barrier normally waits a few us
__device__ __forceinline__ bool grid_barrier(unsigned int *ctr, unsigned int n, int *err, unsigned int polls,
                                             bool skip) {
    __shared__ int s_ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!skip) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int target = n * gridDim.x;
        int ok = 1;
        for (unsigned int k = 0; __hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target; ++k) {
            if (k >= polls ||
                ((k & 1023u) == 1023u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// The same barrier without a shared counter (SQ_QM1D_BAR=3): every block
// publishes its arrival in its own flag word (64 B apart) -- lane 0, behind the
// block's stores, a release fence and a relaxed store -- and wave 0 polls all
// G flags in parallel with relaxed loads (lane l the blocks l, l+64, ...)
// until every one has reached barrier n, then one acquire fence for the CU.
// The counter barrier's atomic adds queue on one address (≈0.35 us per block
// and step: C1 per-step time grows by that much per block, SQ_QM1D_GK
// 8 / 4 / 2 = 16 / 32 / 64 blocks, profiles/r03/qm1d_grid/), and it polls with
// acquire loads (an L1 invalidate per poll); flags cost one store per block.
// Bounded like grid_barrier.
template <bool FENCED = true>
__device__ __forceinline__ bool grid_barrier_flags(unsigned int *flags, unsigned int n, int *err,
                                                   unsigned int polls, bool skip) {
    __shared__ int s_ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have left
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = (int)threadIdx.x, G = (int)gridDim.x;
        if (lane == 0 && !skip) {
            if (FENCED) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the block's writes, past the XCD's L2
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flags + 16 * blockIdx.x, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int ok = 1;
        for (unsigned int k = 0;; ++k) {
            bool mine = true;
            for (int q = lane; q < G; q += 64)
                mine = mine && __hip_atomic_load(flags + 16 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n;
            if (__all(mine)) break;
            if (k >= polls ||
                ((k & 1023u) == 1023u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (FENCED && ok) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's L1: the other blocks' writes
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// SC1 (SQ_QM1D_BAR=4): the values one block hands to another -- edge sites,
// f[mid], X' at the candidate leaders, the block maxima -- stored with sc1
// stores (write-through) and read with sc1 loads (past the reader's L1), so
// the flag barrier needs no release (L2 write-back) and no acquire (L1
// invalidate): MI355X_MICROARCH.md's "Valid forms", one lane signalling for
// its workgroup, 8-B sc1 stores and loads, hipMalloc memory.
typedef __attribute__((address_space(1))) double gdouble;
template <bool SC1>
__device__ __forceinline__ double ld_x(const double *p) {
    if constexpr (SC1)
        return __hip_atomic_load((const gdouble *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool SC1>
__device__ __forceinline__ void st_x(double *p, double v) {
    if constexpr (SC1) __hip_atomic_store((gdouble *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

template <int kGridK, bool SC1>
__global__ __launch_bounds__(kGridT) void qm1d_frame_grid(const Qm1dArgs A) {
    cooperative_groups::grid_group grid = cooperative_groups::this_grid();
    unsigned int *bar = reinterpret_cast<unsigned int *>(A.ds + A.N) + 4;  // zeroed before the launch
    __shared__ double s_wX[2][kGridT / 64], s_wA[2][kGridT / 64];
    const int N = A.N, pot = A.pot, mid = N / 2, G = (int)gridDim.x, b = (int)blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int gt = b * kGridT + t;
    const int i0 = gt * kGridK;
    const int own = max(0, min(kGridK, N - i0));
    const double h = A.h, a = A.a, a2 = A.a2;
    double *Xb[2] = {A.xs, A.ds};
    double *bm = A.xs + N;  // [parity][X | A][G]
    // The leader word comes in two copies by step parity: scan j writes tag j+1
    // into lead[(j+1)&1] and step j+1 reads it back; the next write to that copy
    // is scan j+2's, behind barrier j+3, which no block passes before every
    // block has read it.  (One shared word let a block that left barrier j+2
    // early overwrite tag j+1 with j+2 before a slower block had read it.)  The
    // copies: ds[N] bytes 0 and 24 (the barrier counter sits at byte 16).
    // (the copy of parity q is lw + 3 q: an address by arithmetic, not an array
    // of two pointers indexed by the step, which would live in private memory)
    unsigned long long *lw = reinterpret_cast<unsigned long long *>(A.ds + N), *unst = lw + 1;
    if (gt == 0) {  // write-through: the other blocks' atomics (and, SC1, loads) must see the zeros
        __hip_atomic_store(lw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lw + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(unst, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    double nx[kGridK], nxx0[kGridK], D[kGridK];
#pragma unroll
    for (int k = 0; k < kGridK; ++k) {
        nx[k] = k < own ? A.x[i0 + k] : 0.;
        nxx0[k] = k < own ? A.xx0[i0 + k] : 0.;
        D[k] = 0.;
    }
    double om = A.st->omega_in;
    int E = A.st->lrgEl;
    double V = A.st->lrgVl, totA = 0.;
    int stable = 1, steps = 0;
    double *fout = A.nf;
    // The field of the previous step: this thread's own sites stay in
    // registers; its two neighbour sites and f[mid] -- written by other
    // threads and blocks -- are loaded right after each barrier, so the loads
    // overlap the scan instead of opening the next step's site updates.
    double fc[kGridK];
#pragma unroll
    for (int k = 0; k < kGridK; ++k) fc[k] = k < own ? A.f[i0 + k] : 0.;
    double fL = (own > 0 && i0 > 0) ? A.f[i0 - 1] : 0.;
    double fR = (own > 0 && i0 + own < N) ? A.f[i0 + own] : 0.;
    double fmid = A.f[mid];
    int myLead = -1;  // this thread's last leader in the previous step's scan (-1: none)
    auto stamp = [&](int j, int ph) {  // diagnostics only (A.dbg, SQ_QM1D_STAMPS)
        if (A.dbg != nullptr && t == 0 && j < 64 && b < kQm1dStampBlocks) A.dbg[((size_t)b * 64 + j) * 5 + ph] = __builtin_amdgcn_s_memrealtime();
    };
    for (int j = 0; j <= A.loops; ++j) {
        const int par = j & 1;
        double X[kGridK], vn[kGridK];
        double ix = -INFINITY, ia = -INFINITY;
        stamp(j, 0);
        if (j < A.loops) {
            // 1. site updates of step j
            const unsigned long long step = A.tick + (unsigned long long)j;
            const uint32_t slo = (uint32_t)step, shi = (uint32_t)(step >> 32);
            const double Xm = fmid + xcl((double)mid * a, om, pot);
            const double den = (double)(A.runs + j + 1);
            double lmaxX = -INFINITY, lmaxA = -INFINITY;
            if (own > 0) {
                f32x4n nq = normals4((unsigned long long)(i0 >> 2), kStreamField, slo, shi, A.k0, A.k1);
#pragma unroll
                for (int k = 0; k < kGridK; ++k) {
                    if (k >= own) break;
                    const int i = i0 + k;
                    const int c = i & 3;  // component of site i's quad (K = 2: i0 may be 2 mod 4)
                    if (c == 0 && k > 0)
                        nq = normals4((unsigned long long)(i >> 2), kStreamField, slo, shi, A.k0, A.k1);
                    const float xi = c == 0 ? nq.a : c == 1 ? nq.b : c == 2 ? nq.c : nq.d;
                    const double fi = fc[k];
                    const double fr = (k + 1 < own) ? fc[k + 1] : fR;
                    const double prev_old = k == 0 ? fL : fc[k - 1];
                    const double xc = xcl((double)i * a, om, pot);
                    const double dw = A.sig * (double)xi;
                    double v;
                    if (i == 0)
                        v = fi + kM * h * (fr + (-kEta) - xcl(-1. * a, om, pot) - 2 * fi) / a2 -
                            ddpot(xc, pot) * fi * h + dw;
                    else if (i == N - 1)
                        v = fi + kM * h * (prev_old + kEta - xcl((double)N * a, om, pot) - 2 * fi) / a2 -
                            ddpot(xc, pot) * fi * h + dw;
                    else
                        v = fi + kM * h * (fr + prev_old - 2 * fi) / a2 - ddpot(xc, pot) * fi * h + dw;
                    if (v > 1000) v = 1000;
                    if (v < -1000) v = -1000;
                    if (v != v) v = 1000;
                    X[k] = v + xc;
                    D[k] = absol(v - fi - dw);
                    lmaxX = fmax(lmaxX, X[k]);
                    lmaxA = fmax(lmaxA, absol(X[k]));
                    const double Xi = fi + xc;
                    nxx0[k] = nxx0[k] + (Xi * Xm - nxx0[k]) / den;
                    nx[k] = nx[k] + (Xi - nx[k]) / den;
                    vn[k] = v;
                    // only what another thread reads: the thread's edge sites and
                    // f[mid] (the next step's neighbours / running means), and X'
                    // at the two sites the scan can need it at -- the current
                    // leader E and this thread's last leader of the previous
                    // scan (the new E is the largest such index, or E itself)
                    if (k == 0 || k == own - 1 || i == mid) st_x<SC1>(fout + i, v);
                    if (i == E || i == myLead) st_x<SC1>(Xb[par] + i, X[k]);
                }
            }
            // wave prefix maxima by DPP row scans (max is exact: the same values
            // as any other order)
            ix = dpp_incl_max(lmaxX);
            ia = dpp_incl_max(lmaxA);
            if (lane == 63) {
                s_wX[par][wv] = ix;
                s_wA[par][wv] = ia;
            }
            __syncthreads();
            if (t == 0) {
                double bx = -INFINITY, ba = -INFINITY;
                for (int w = 0; w < kGridT / 64; ++w) {
                    bx = fmax(bx, s_wX[par][w]);
                    ba = fmax(ba, s_wA[par][w]);
                }
                st_x<SC1>(bm + (2 * par) * G + b, bx);
                st_x<SC1>(bm + (2 * par + 1) * G + b, ba);
            }
        }
        stamp(j, 1);
        const unsigned int polls = A.bar_polls ? A.bar_polls : kGridSpinMax;
        if (SC1 || A.gbar == 3) {
            if (!grid_barrier_flags<!SC1>(bar + 16, (unsigned int)(j + 1), &A.st->sync_error, polls,
                                          j == 0 && b == A.bar_skip))
                return;  // a barrier gave up: the frame is void (the host reports it)
        } else {
            if (A.gbar) {
                if (!grid_barrier(bar, (unsigned int)(j + 1), &A.st->sync_error, polls, j == 0 && b == A.bar_skip))
                    return;
            } else {
                grid.sync();
            }
            // acquire only: every block's writes before the barrier were released by
            // its thread 0 (after the block's __syncthreads) -- a full __threadfence
            // here made every wave write back the L2 again each step
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        stamp(j, 2);
        // every load the rest of the step needs that does not depend on the
        // previous scan's outcome, issued together: the next step's neighbour
        // sites and f[mid] (this step's output), and the block maxima (lane q:
        // blocks q, q + 64, ...; exclusive prefix over the blocks before this
        // one, and the total of |X'|)
        double nL = 0., nR = 0., nmid = 0., pX = -INFINITY, pA = -INFINITY, tA = -INFINITY;
        if (j < A.loops) {
            nL = (own > 0 && i0 > 0) ? ld_x<SC1>(fout + i0 - 1) : 0.;
            nR = (own > 0 && i0 + own < N) ? ld_x<SC1>(fout + i0 + own) : 0.;
            nmid = ld_x<SC1>(fout + mid);
            for (int q = lane; q < G; q += 64) {
                const double qx = ld_x<SC1>(bm + (2 * par) * G + q), qa = ld_x<SC1>(bm + (2 * par + 1) * G + q);
                if (q < b) {
                    pX = fmax(pX, qx);
                    pA = fmax(pA, qa);
                }
                tA = fmax(tA, qa);
            }
        }
        // 2a. the outcome of step j-1's scan
        if (j > 0) {
            const unsigned long long tag = (unsigned long long)j;
            const unsigned long long lv = __hip_atomic_load(lw + 3 * (j & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((lv >> 32) == tag) E = (int)(lv & 0xffffffffull) - 1;
            V = totA;
            steps = j;
            if (__hip_atomic_load(unst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag) {
                stable = 0;
                break;
            }
        }
        if (j == A.loops) break;
        stamp(j, 3);
        // 2b. step j's ordered scan
        double runX = (E >= 0 && E < N) ? ld_x<SC1>(Xb[par] + E) : -INFINITY, runA = V;
        runX = fmax(runX, dpp_all_max(pX));
        runA = fmax(runA, dpp_all_max(pA));
        totA = fmax(V, dpp_all_max(tA));
        for (int w = 0; w < wv; ++w) {
            runX = fmax(runX, s_wX[par][w]);
            runA = fmax(runA, s_wA[par][w]);
        }
        runX = fmax(runX, dpp_from_left(ix, -INFINITY));  // lanes before this one (lane 0: none)
        runA = fmax(runA, dpp_from_left(ia, -INFINITY));
        int un = 0, leader = -1;
#pragma unroll
        for (int k = 0; k < kGridK; ++k) {
            if (k >= own) break;
            if (X[k] > runX) {
                runX = X[k];
                leader = i0 + k;
                if (D[k] > runA) un = 1;
            }
            runA = fmax(runA, absol(X[k]));
        }
        const unsigned long long tag1 = (unsigned long long)(j + 1);
        if (leader >= 0) atomicMax(lw + 3 * ((j + 1) & 1), (tag1 << 32) | (unsigned long long)(leader + 1));
        if (un) atomicMax(unst, tag1);
        myLead = leader;
        stamp(j, 4);
        // omega's step j
        const unsigned long long step = A.tick + (unsigned long long)j;
        const f32x4n nwn = normals4(0ull, kStreamOmega, (uint32_t)step, (uint32_t)(step >> 32), A.k0, A.k1);
        const double nwo = om + A.kconst * (A.sigw * (double)nwn.a);
        if (nwo > (double)(N - 1) * a) om = 2 * (double)(N - 1) * a - nwo;
        else if (nwo < 0) om = -nwo;
        else om = nwo;
        // step j becomes the previous step
#pragma unroll
        for (int k = 0; k < kGridK; ++k) fc[k] = vn[k];
        fL = nL;
        fR = nR;
        fmid = nmid;
        fout = (fout == A.nf) ? A.fs : A.nf;
    }
    // unstable after step s: the break came before iteration s+1's swap, so fc
    // is step s's output, as in the one-CU kernel (the host discards it)
#pragma unroll
    for (int k = 0; k < kGridK; ++k) {
        if (k >= own) break;
        A.nf[i0 + k] = fc[k];
        A.nx[i0 + k] = nx[k];
        A.nxx0[i0 + k] = nxx0[k];
    }
    if (gt == 0) {
        A.st->omega_out = om;
        A.st->lrgEl = E;
        A.st->lrgVl = V;
        A.st->stable = stable;
        A.st->steps_done = steps;
    }
}

}  // namespace

int qm1d_sites_per_thread(int N) {
    if (N < 2 || N > kQm1dMaxN) return 0;
    for (int k : {1, 2, 4, 8, 16, 32, 64})
        if ((N + k - 1) / k <= kMaxThreads) return k;
    return 0;
}

// Register kernel shape for N <= 4,096: one wave with K <= 2 sites per lane
// up to N = 128, one site per lane up to 256, then W = ceil(N/256) <= 16
// waves with K = 4 (16 waves are 4 per SIMD, <= 128 VGPRs each: K = 8 would
// spill).
static bool qm1d_wave_shape(int N, int &K, int &W) {
    if (N < 2 || N > kQm1dRegMaxN) return false;
    static const int kforce = [] {  // tuning override: sites per lane (1, 2, 4)
        const char *e = getenv("SQ_QM1D_K");
        return e ? atoi(e) : 0;
    }();
    if (kforce == 1 || kforce == 2 || kforce == 4) {
        K = kforce;
        W = (N + 64 * K - 1) / (64 * K);
        if (W <= 16) return true;
    }
    // measured (profiles/r01/bench_qm1d_wave.log): a lone wave costs about
    // 1.0 us + 0.47 us per site per lane per step, a multi-wave block ~0.75 us
    // more for its two barriers
    if (N <= 128) W = 1;
    else if (N <= 256) W = (N + 63) / 64;
    else W = std::min(16, (N + 255) / 256);
    for (K = 1; 64 * W * K < N; K *= 2) {}
    return K <= 4;
}

template <int K, bool P3>
static void launch_wave_p(const Qm1dArgs &a, int W, hipStream_t s) {
    if (W == 1) hipLaunchKernelGGL((qm1d_frame_wave<K, false, P3>), dim3(1), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((qm1d_frame_wave<K, true, P3>), dim3(1), dim3(64 * W), 0, s, a);
}
template <int K>
static void launch_wave(const Qm1dArgs &a, int W, hipStream_t s) {
    if (a.pot == 3) launch_wave_p<K, true>(a, W, s);
    else launch_wave_p<K, false>(a, W, s);
}

hipError_t qm1d_prep_launch(const Qm1dArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(qm1d_omega_kernel, dim3(1), dim3(64), 0, s, a);
    const long long total = (long long)a.loops * ((a.N + 3) / 4);
    const unsigned grid = (unsigned)std::max(1ll, std::min(2048ll, (total + 255) / 256));
    hipLaunchKernelGGL(qm1d_tables_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t qm1d_frame_launch(const Qm1dArgs &a, hipStream_t s) {
    int K = 0, W = 0;
    if (qm1d_wave_shape(a.N, K, W)) {
        switch (K) {
        case 1: launch_wave<1>(a, W, s); break;
        case 2: launch_wave<2>(a, W, s); break;
        default: launch_wave<4>(a, W, s); break;
        }
        return hipGetLastError();
    }
    // N > 4096: the cooperative grid kernel (SQ_QM1D_GRID=0: the one-CU kernel)
    const char *ge = getenv("SQ_QM1D_GRID");  // read per frame (tests switch it within a process)
    const bool grid = ge ? atoi(ge) != 0 : true;
    if (grid && a.N <= kQm1dMaxN) {
        const char *gk = getenv("SQ_QM1D_GK");
        // sites per thread: the fewest that keep G <= 128 blocks (N = 32,768: 1 site,
        // 128 blocks, 4.92 ms per 1000-step frame; 2 sites 5.03; 4 sites 5.77; 8
        // sites 8.0 -- profiles/r05/c11, c12); SQ_QM1D_GK pins it
        int kk = 1;
        while (kk < 32 && (a.N + kGridT * kk - 1) / (kGridT * kk) > 128) kk *= 2;
        if (gk) kk = atoi(gk);
        if (kk != 1 && kk != 2 && kk != 4 && kk != 8 && kk != 16 && kk != 32) kk = 8;  // the instances built
        const int G = (a.N + kGridT * kk - 1) / (kGridT * kk);
        if (4 * G > kQm1dGridAux) return hipErrorInvalidValue;  // xs[N..]: the block maxima by parity
        Qm1dArgs q = a;
        // the barrier (SQ_QM1D_BAR): 4 (default) per-block flags with sc1 hand-offs
        // and no fences; 3 per-block flags with release / acquire fences; 1 one
        // counter with fences (round 3's, 10.8 ms per C1 frame vs 11.7 with 0,
        // cooperative groups' grid.sync: profiles/r03/qm1d_grid/)
        const char *gb = getenv("SQ_QM1D_BAR");
        q.gbar = gb ? atoi(gb) : 4;
        // tests: a block that never arrives (SQ_QM1D_BAR_SKIP=b) and a shorter poll budget
        const char *bs = getenv("SQ_QM1D_BAR_SKIP"), *bp = getenv("SQ_QM1D_BAR_POLLS");
        q.bar_skip = bs ? atoi(bs) : -1;
        q.bar_polls = bp ? (unsigned int)strtoul(bp, nullptr, 10) : 0u;
        if (q.gbar) {  // the counter barrier's word: ds[N] + 16 bytes (between the tagged words); the
                       // flag barrier's G words 64 B apart after it (ds[N] + 80 bytes: < kQm1dGridAux doubles)
            if (80 + 64 * (size_t)G > sizeof(double) * kQm1dGridAux) return hipErrorInvalidValue;
            hipError_t e = hipMemsetAsync(reinterpret_cast<unsigned int *>(q.ds + q.N) + 4, 0, 64 + 64 * (size_t)G, s);
            if (e != hipSuccess) return e;
        }
        void *args[] = {&q};
        const bool sc1 = q.gbar == 4;
#define SQ_GRIDK(K) (sc1 ? (const void *)qm1d_frame_grid<K, true> : (const void *)qm1d_frame_grid<K, false>)
        const void *fn = kk == 1 ? SQ_GRIDK(1) : kk == 2 ? SQ_GRIDK(2) : kk == 8 ? SQ_GRIDK(8)
                         : kk == 16 ? SQ_GRIDK(16) : kk == 32 ? SQ_GRIDK(32) : SQ_GRIDK(4);
#undef SQ_GRIDK
        if (q.gbar) {
            // the counter barrier needs every block resident, not the
            // cooperative-launch machinery (GWS, its own queue); a plain launch
            // of G <= the chip's resident capacity (G = 128 at N = 32,768) keeps
            // the frame on the context's stream like every other kernel, and
            // profilers that mishandle cooperative dispatches at exit see none
            int dev = 0, cus = 0, per_cu = 0;
            hipError_t e = hipGetDevice(&dev);
            if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kGridT, 0);
            if (e != hipSuccess) return e;
            if (G > cus * per_cu) return hipErrorCooperativeLaunchTooLarge;
            return hipLaunchKernel(fn, dim3(G), dim3(kGridT), args, 0, s);
        }
        return hipLaunchCooperativeKernel(fn, dim3(G), dim3(kGridT), args, 0, s);
    }
    K = qm1d_sites_per_thread(a.N);
    if (K == 0) return hipErrorInvalidValue;
    int threads = (a.N + K - 1) / K;
    threads = ((threads + 63) / 64) * 64;
    switch (K) {
    case 8: hipLaunchKernelGGL(qm1d_frame_kernel_glob<8>, dim3(1), dim3(threads), 0, s, a); break;
    case 16: hipLaunchKernelGGL(qm1d_frame_kernel_glob<16>, dim3(1), dim3(threads), 0, s, a); break;
    case 32: hipLaunchKernelGGL(qm1d_frame_kernel_glob<32>, dim3(1), dim3(threads), 0, s, a); break;
    default: hipLaunchKernelGGL(qm1d_frame_kernel_glob<64>, dim3(1), dim3(threads), 0, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace sq
