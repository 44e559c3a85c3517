/*
 * orc_qm1d.c -- oracle restatements of the reference's 1-D QM Langevin path
 * (TEST INFRASTRUCTURE ONLY, see sq_oracle.h).
 *
 * Reference: /root/reference/tau_kernel.cl (time_dev + helpers) and
 * /root/reference/tauhost.c (host frame loop).  Every expression keeps the
 * reference's evaluation order and its fp32 casts so that the serial
 * restatement is bit-exact with the reference under a serialising runtime.
 * Build with -ffp-contract=off (see Makefile): contraction would change bits.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "sq_oracle.h"

/* tau_kernel.cl:19-22 */
static const double ETA = .8;
static const double V0 = 2.;
static const double M = 1.;

/* clas(): tau_kernel.cl:215-226 -> doubleWellSol :184-189 / harmOscSol :201-205 */
double orc_xcl(double t, double w, int pot)
{
    if (pot == 3) {
        const double s = (double)sqrtf((float)(2. * V0 / M));
        return ETA * (double)tanhf((float)(s * (t - w) / ETA));
    }
    return 0.;
}

/* ddPot(): tau_kernel.cl:227-236 -> doubleWellPot :190-195 / harmOscPot :206-209 */
double orc_ddpot(double x, int pot)
{
    if (pot == 3) return (12. * V0 * x * x / (ETA * ETA) - 4. * V0) / (ETA * ETA);
    return 2.;
}

/* intConst(): tau_kernel.cl:237-246 -> doubleWellConst :196-200 (all float) */
double orc_intconst(int pot)
{
    if (pot == 3)
        return (double)(sqrtf((float)3.) * powf((float)2., (float)(-5. / 4.)) *
                        powf((float)V0, (float)(-1. / 4.)) / sqrtf((float)ETA));
    return 0.;
}

/* boundary(): tau_kernel.cl:247-256 */
static double ghost(int rl) { return rl == 1 ? ETA : -ETA; }

/* absol(): tau_kernel.cl:259-267 */
static double absol(double v) { return v <= 0 ? -v : v; }

static double a2_of(double a) { float fa = (float)a; return (double)(fa * fa); } /* pown((float)a,2) */

/* ------------------------------------------------------------------------ */
/* 1. Serial restatement: time_dev body for one work-item at step j          */
/* ------------------------------------------------------------------------ */
typedef struct { double dw, newomega; } item_locals;

static void serial_item_step(orc_serial_dev *d, int i, int j, item_locals *L)
{
    const int N = d->N, pot = d->pot, loops = d->loops;
    const double h = d->dtau, a = d->a, c = d->c, mm = M;
    const double max = 1000;
    const int mid = N / 2;
    double *f = d->f, *nf = d->nf, *x = d->x, *nx = d->nx, *xx0 = d->xx0, *nxx0 = d->nxx0;
    const double om = d->omega;                                   /* :65 */
    const double a2 = a2_of(a);
    if (i == 0) {                                                 /* :68-85, bc = 1 */
        L->dw = c * (double)sqrtf((float)(2. * h / a)) * orc_ref_random(&d->seed, i);
        nf[i] = f[0] + mm * h * (f[1] + ghost(-1) - orc_xcl(-1. * a, om, pot) - 2 * f[0]) / a2
              - orc_ddpot(orc_xcl((double)i * a, om, pot), pot) * f[0] * h + L->dw;
    }
    if (i == N - 1) {                                             /* :86-102 */
        L->dw = c * (double)sqrtf((float)(2. * h / a)) * orc_ref_random(&d->seed, i);
        nf[i] = f[N - 1] + mm * h * (f[N - 2] + ghost(1) - orc_xcl((double)N * a, om, pot) - 2 * f[N - 1]) / a2
              - orc_ddpot(orc_xcl((double)i * a, om, pot), pot) * f[N - 1] * h + L->dw;
    }
    if (i == N) {                                                 /* :103-110 */
        L->dw = c * (double)sqrtf((float)(2. * h)) * orc_ref_random(&d->seed, i);
        L->newomega = om + orc_intconst(pot) * L->dw;
    }
    if (i < N - 1 && i > 0) {                                     /* :111-117 */
        L->dw = c * (double)sqrtf((float)(2. * h / a)) * orc_ref_random(&d->seed, i);
        nf[i] = f[i] + mm * h * (f[i + 1] + f[i - 1] - 2 * f[i]) / a2
              - orc_ddpot(orc_xcl((double)i * a, om, pot), pot) * f[i] * h + L->dw;
    }
    if (i < N) {
        if (nf[i] > max) nf[i] = max;                             /* :119-133 */
        if (nf[i] < -max) nf[i] = -max;
        if ((isinf((float)nf[i]) ? 1 : 0) == 1 || (isnan((float)nf[i]) ? 1 : 0) == 1) nf[i] = max;
        const int E = d->lrgEl;                                   /* :135-143 */
        if (nf[i] + orc_xcl((double)i * a, om, pot) > nf[E] + orc_xcl((double)E * a, om, pot)) {
            d->lrgEl = i;
            if (absol(nf[i] - f[i] - L->dw) > d->lrgVl) d->stable = 0;
        }
        if (absol(nf[i] + orc_xcl((double)i * a, om, pot)) > d->lrgVl)
            d->lrgVl = absol(nf[i] + orc_xcl((double)i * a, om, pot));
        const double den = (double)(d->runs + j + 1);             /* :144-145 */
        nxx0[i] = xx0[i] + ((f[i] + orc_xcl((double)i * a, om, pot)) *
                            (f[mid] + orc_xcl((double)mid * a, om, pot)) - xx0[i]) / den;
        nx[i] = x[i] + ((f[i] + orc_xcl((double)i * a, om, pot)) - x[i]) / den;
        if (j < loops - 1) { f[i] = nf[i]; xx0[i] = nxx0[i]; x[i] = nx[i]; }   /* :147-151 */
    } else {                                                      /* :155-167 */
        if (L->newomega > (double)(N - 1) * a)
            d->omega = 2 * (double)(N - 1) * a - L->newomega;
        else if (L->newomega < 0)
            d->omega = -L->newomega;
        else
            d->omega = L->newomega;
    }
}

/* One launch with global size N+1 executed as one work-group whose items run
 * to each barrier in id order (the fiber-serialised semantics of SURVEY.md
 * Appendix A/B): in round r every live item first tests `*stable` (after the
 * barrier of step r-1, :168-171) and then runs step r. */
void orc_serial_launch(orc_serial_dev *d)
{
    const int n_items = d->N + 1;
    char *alive = (char *)malloc((size_t)n_items);
    item_locals *L = (item_locals *)calloc((size_t)n_items, sizeof(item_locals));
    memset(alive, 1, (size_t)n_items);
    for (int r = 0; r <= d->loops; ++r) {
        for (int i = 0; i < n_items; ++i) {
            if (!alive[i]) continue;
            if (r > 0 && d->stable != 1) { alive[i] = 0; continue; }
            if (r == d->loops) { alive[i] = 0; continue; }
            serial_item_step(d, i, r, &L[i]);
        }
    }
    free(alive);
    free(L);
}

/* ------------------------------------------------------------------------ */
/* 2. Jacobi restatement (the HIP kernel's semantics)                        */
/* ------------------------------------------------------------------------ */
/* Per step j of a frame, with om = omega at the step's start, all sites read
 * the OLD field (f_{i-1}, f_{i+1}, f_mid) and the noise
 *   dw_i = c*sqrtf(2h/a) * xi(seed, stream 0, quad i>>2, comp i&3, tick),
 *   dw_w = c*sqrtf(2h)   * xi(seed, stream 1, quad 0,    comp 0,   tick).
 * Stability (order-independent statement of :135-143, all new values known):
 *   X'_i = f'_i + x_cl(i a);  R = X'_{E_prev};  V_prev carried.
 *   i is a leader  <=>  X'_i > max(R, max_{k<i} X'_k)
 *   unstable       <=>  some leader i has |f'_i - f_i - dw_i| > max(V_prev, max_{k<i}|X'_k|)
 *   E_new = last leader (else E_prev);  V_new = max(V_prev, max_k |X'_k|).
 * Running means use the old field exactly as :144-145.                      */
void orc_qm1d_frame(orc_qm1d *s)
{
    const int N = s->N, pot = s->pot, mid = N / 2;
    const double h = s->dtau, a = s->a, c = s->c, a2 = a2_of(a);
    const double sig = c * (double)sqrtf((float)(2. * h / a));
    const double sigw = c * (double)sqrtf((float)(2. * h));
    const double K = orc_intconst(pot);
    double *f = (double *)malloc(sizeof(double) * N), *x = (double *)malloc(sizeof(double) * N);
    double *xx0 = (double *)malloc(sizeof(double) * N), *fn = (double *)malloc(sizeof(double) * N);
    double *dw = (double *)malloc(sizeof(double) * N);
    memcpy(f, s->f, sizeof(double) * N);
    memcpy(x, s->x, sizeof(double) * N);
    memcpy(xx0, s->xx0, sizeof(double) * N);
    double om = s->omega;
    s->stable = 1;
    s->steps_done = 0;
    for (int j = 0; j < s->loops; ++j) {
        const uint64_t step = s->tick + (uint64_t)j;
        for (int i = 0; i < N; ++i) {
            float nz[4];
            orc_normals4(s->seed, 0, (uint64_t)(i >> 2), step, nz);
            dw[i] = sig * (double)nz[i & 3];
            const double L = i == 0 ? ghost(-1) - orc_xcl(-1. * a, om, pot) : f[i - 1];
            const double R = i == N - 1 ? ghost(1) - orc_xcl((double)N * a, om, pot) : f[i + 1];
            double v;
            if (i == 0)
                v = f[0] + M * h * (f[1] + ghost(-1) - orc_xcl(-1. * a, om, pot) - 2 * f[0]) / a2
                  - orc_ddpot(orc_xcl((double)i * a, om, pot), pot) * f[0] * h + dw[i];
            else if (i == N - 1)
                v = f[N - 1] + M * h * (f[N - 2] + ghost(1) - orc_xcl((double)N * a, om, pot) - 2 * f[N - 1]) / a2
                  - orc_ddpot(orc_xcl((double)i * a, om, pot), pot) * f[N - 1] * h + dw[i];
            else
                v = f[i] + M * h * (R + L - 2 * f[i]) / a2
                  - orc_ddpot(orc_xcl((double)i * a, om, pot), pot) * f[i] * h + dw[i];
            if (v > 1000) v = 1000;
            if (v < -1000) v = -1000;
            if (isnan(v)) v = 1000;
            fn[i] = v;
        }
        /* stability scan */
        double run_max = fn[s->lrgEl] + orc_xcl((double)s->lrgEl * a, om, pot);
        double V = s->lrgVl;
        int unstable = 0;
        for (int i = 0; i < N; ++i) {
            const double X = fn[i] + orc_xcl((double)i * a, om, pot);
            if (X > run_max) {
                run_max = X;
                s->lrgEl = i;
                if (absol(fn[i] - f[i] - dw[i]) > V) unstable = 1;
            }
            if (absol(X) > V) V = absol(X);
        }
        s->lrgVl = V;
        /* running means (old field), :144-145 */
        const double den = (double)(s->runs + j + 1);
        const double Xm = f[mid] + orc_xcl((double)mid * a, om, pot);
        for (int i = 0; i < N; ++i) {
            const double Xi = f[i] + orc_xcl((double)i * a, om, pot);
            xx0[i] = xx0[i] + (Xi * Xm - xx0[i]) / den;
            x[i] = x[i] + (Xi - x[i]) / den;
        }
        /* collective coordinate, :103-110,155-167 */
        float nw[4];
        orc_normals4(s->seed, 1, 0, step, nw);
        const double nwo = om + K * (sigw * (double)nw[0]);
        if (nwo > (double)(N - 1) * a) om = 2 * (double)(N - 1) * a - nwo;
        else if (nwo < 0) om = -nwo;
        else om = nwo;
        memcpy(f, fn, sizeof(double) * N);
        s->steps_done = j + 1;
        if (unstable) { s->stable = 0; break; }
    }
    memcpy(s->nf, f, sizeof(double) * N);
    memcpy(s->nx, x, sizeof(double) * N);
    memcpy(s->nxx0, xx0, sizeof(double) * N);
    s->nomega = om;
    free(f); free(x); free(xx0); free(fn); free(dw);
}
