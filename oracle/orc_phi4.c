/*
 * orc_phi4.c -- oracle for the north-star 3-D extension (TEST INFRASTRUCTURE
 * ONLY, see sq_oracle.h; also bench.py's cpu_baseline, kind "port").
 *
 * The reference's per-site update (tau_kernel.cl:111-117: old value + Δτ ×
 * (lattice Laplacian − V'') + noise, then the ±max / NaN guard :119-133)
 * generalised to a periodic 3-D fp32 lattice with the full non-linear force
 * of V(φ) = ½ m² φ² + (λ/4!) φ⁴ (SURVEY.md §8a "Build-side hot-path unit"):
 *
 *   nb   = ((φ[x-1] + φ[x+1]) + (φ[y-1] + φ[y+1])) + (φ[z-1] + φ[z+1])
 *   lap  = fma(-6, φ, nb)
 *   g    = fma(λ/6, φ·φ, m²)
 *   drift= fma(-φ, g, lap)
 *   φ'   = fma(σ, ξ, fma(Δτ, drift, φ)),     σ = C·sqrt(2Δτ) (C = 1 physical)
 *   φ'   = NaN ? max : clamp(φ', -max, max)
 *
 * The evaluation order is the product's (fp32, explicit fma).  ξ is the
 * double-evaluated normal by default, or (orc_set_bm_tables) the device's own
 * Box-Muller factors, with which the result is the GPU's bit for bit.  Site index s = (z·Ly + y)·Lx + x (global),
 * noise quad s>>2, component s&3, stream 0.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "sq_oracle.h"
#ifdef _OPENMP
#include <omp.h>
#endif

float orc_phi4_sigma(float h, double C) { return (float)(sqrt(2.0 * (double)h) * C); }
/* sigma * sqrt(2 ln 2): the amplitude of the kernels' box_muller_q pairs
 * (sq_api.cpp phi4_base_args, kSqrt2Ln2 = 1.1774100225154747). */
float orc_phi4_sigq(float h, double C) { return (float)(sqrt(2.0 * (double)h) * C * 1.1774100225154747); }
float orc_phi4_lam6(float lam) { return (float)((double)lam / 6.0); }

/* Order-preserving float -> uint32 map (larger float, larger code). */
static uint32_t ord_f32(float v)
{
    uint32_t u;
    memcpy(&u, &v, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

/* The stability record of one site: key = ord(phi') << 32 |
 * bits(|phi' - phi - sigma xi|), so the maximum key over a step is its maximum
 * phi' with the largest drift increment among the sites attaining it. */
static void stab_site(uint64_t *key, float *amax, float o, float c, float xi, float sig)
{
    const float dn = fabsf(fmaf(-sig, xi, o - c));
    uint32_t db;
    memcpy(&db, &dn, 4);
    const uint64_t k = ((uint64_t)ord_f32(o) << 32) | db;
    if (k > *key) *key = k;
    if (fabsf(o) > *amax) *amax = fabsf(o);
}

/* One plane of the update: c = plane z, zm/zp = planes z-1, z+1 (already
 * resolved by the caller: periodic wrap or ghost planes), zg = global z.
 * key / amax (nullable): the step's stability record, accumulated. */
static void phi4_plane(const orc_phi4 *p, const float *cz, const float *czmp, const float *czpp,
                       float *oz, uint64_t zg, uint64_t step, uint64_t *key, float *amax)
{
    const int Lx = p->Lx, Ly = p->Ly;
    const float h = p->h, m2 = p->m2, lam6 = orc_phi4_lam6(p->lam);
    /* device-transcendental mode: the kernels' exact noise (q pairs, sigq) */
    const int dev = orc_bm_tables_on();
    const float sig = dev ? orc_phi4_sigq(h, p->C) : orc_phi4_sigma(h, p->C), mx = p->clampv;
    for (int y = 0; y < Ly; ++y) {
        const int ym = (y + Ly - 1) % Ly, yp = (y + 1) % Ly;
        const float *c = cz + (size_t)y * Lx;
        const float *cym = cz + (size_t)ym * Lx;
        const float *cyp = cz + (size_t)yp * Lx;
        const float *czm = czmp + (size_t)y * Lx;
        const float *czp = czpp + (size_t)y * Lx;
        float *o = oz + (size_t)y * Lx;
        const uint64_t row0 = (zg * (uint64_t)Ly + (uint64_t)y) * (uint64_t)Lx;
        for (int x0 = 0; x0 < Lx; x0 += 4) {
            float xi[4];
            if (dev)
                orc_normals4_q(p->seed, 0, (row0 + (uint64_t)x0) >> 2, step, xi);
            else
                orc_normals4(p->seed, 0, (row0 + (uint64_t)x0) >> 2, step, xi);
            for (int k = 0; k < 4; ++k) {
                const int x = x0 + k;
                const int xm = (x + Lx - 1) % Lx, xp = (x + 1) % Lx;
                const float phi = c[x];
                const float nb = ((c[xm] + c[xp]) + (cym[x] + cyp[x])) + (czm[x] + czp[x]);
                const float lap = fmaf(-6.0f, phi, nb);
                const float g = fmaf(lam6, phi * phi, m2);
                const float drift = fmaf(-phi, g, lap);
                float v = fmaf(sig, xi[k], fmaf(h, drift, phi));
                v = isnan(v) ? mx : (v > mx ? mx : (v < -mx ? -mx : v));
                o[x] = v;
                if (key) stab_site(key, amax, v, phi, xi[k], sig);
            }
        }
    }
}

void orc_phi4_step(const orc_phi4 *p, const float *in, float *out, uint64_t step, int nthreads)
{
    const int Lz = p->Lz;
    const size_t plane = (size_t)p->Lx * p->Ly;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int z = 0; z < Lz; ++z) {
        const int zm = (z + Lz - 1) % Lz, zp = (z + 1) % Lz;
        phi4_plane(p, in + (size_t)z * plane, in + (size_t)zm * plane, in + (size_t)zp * plane,
                   out + (size_t)z * plane, (uint64_t)z, step, NULL, NULL);
    }
}

void orc_phi4_step_stab(const orc_phi4 *p, const float *in, float *out, uint64_t step, float rec[3])
{
    const int Lz = p->Lz;
    const size_t plane = (size_t)p->Lx * p->Ly;
    uint64_t key = 0;
    float amax = 0.f;
    for (int z = 0; z < Lz; ++z) {
        const int zm = (z + Lz - 1) % Lz, zp = (z + 1) % Lz;
        phi4_plane(p, in + (size_t)z * plane, in + (size_t)zm * plane, in + (size_t)zp * plane,
                   out + (size_t)z * plane, (uint64_t)z, step, &key, &amax);
    }
    const uint32_t o = (uint32_t)(key >> 32), db = (uint32_t)key;
    const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    memcpy(&rec[0], &u, 4);
    memcpy(&rec[1], &db, 4);
    rec[2] = amax;
}

int orc_phi4_stab_rule(float *T, float *V, const float *M, const float *D, const float *A, int n)
{
    for (int j = 0; j < n; ++j) {
        const int fired = M[j] > *T && D[j] > *V;
        *T = M[j];
        if (A[j] > *V) *V = A[j];
        if (fired) return j;
    }
    return -1;
}

/* Slab form used by the decomposition tests: `in` holds nz+2 planes (ghost,
 * slab, ghost), `out` the nz updated planes; z0 = global z of slab plane 0. */
void orc_phi4_step_slab(const orc_phi4 *p, const float *in, float *out, int nz, uint64_t z0,
                        uint64_t step)
{
    const size_t plane = (size_t)p->Lx * p->Ly;
    for (int z = 0; z < nz; ++z)
        phi4_plane(p, in + (size_t)(z + 1) * plane, in + (size_t)z * plane, in + (size_t)(z + 2) * plane,
                   out + (size_t)z * plane, z0 + (uint64_t)z, step, NULL, NULL);
}

void orc_phi4_step_range(const orc_phi4 *p, const float *in, float *out, int nz, int gpad, int lo, int hi,
                         uint64_t z0, uint64_t step)
{
    const size_t plane = (size_t)p->Lx * p->Ly;
    const int64_t Lz = p->Lz;
    (void)nz;
    for (int zl = lo; zl < hi; ++zl) {
        const int64_t zg = (((int64_t)z0 + zl) % Lz + Lz) % Lz;
        const size_t c = (size_t)(zl + gpad);
        phi4_plane(p, in + c * plane, in + (c - 1) * plane, in + (c + 1) * plane, out + c * plane,
                   (uint64_t)zg, step, NULL, NULL);
    }
}

void orc_phi4_init(const orc_phi4 *p, float amp, float *out)
{
    const size_t n = (size_t)p->Lx * p->Ly * p->Lz;
    for (size_t s = 0; s < n; s += 4) {
        float xi[4];
        orc_normals4(p->seed, 2, (uint64_t)(s >> 2), 0, xi);
        for (int k = 0; k < 4 && s + k < n; ++k) out[s + k] = amp * xi[k];
    }
}
