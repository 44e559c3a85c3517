/*
 * sq_oracle.h -- CPU restatement of SebTanz/StochQuant's Langevin path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker (or the timed CPU baseline),
 * never as the thing measured or shipped.
 *
 * Three restatements live here:
 *
 *  1. "serial" QM1D  -- the reference's exact semantics under a serialising
 *     OpenCL runtime (work-items 0..N in id order between barriers, one shared
 *     48-bit LCG), restating tau_kernel.cl:25-175 + :184-284 and the host
 *     frame loop tauhost.c:29-581.  Pinned against the only reference outputs
 *     that exist (recorded during the survey from the
 *     reference's unmodified sources); see tests/golden/README.md.
 *
 *  2. "jacobi" QM1D  -- the same update with Jacobi ordering, counter-based
 *     Philox4x32-10 noise and an order-independent statement of the stability
 *     scan.  This is the semantics the HIP kernel implements; parity of the GPU
 *     against the reference is therefore: (i) bitwise for the deterministic
 *     part (C = 0, potID 0), (ii) a stated fp tolerance otherwise, (iii)
 *     statistical observables.  The reference's own trajectory is defined only
 *     under one serialisation, so bitwise GPU-vs-reference
 *     trajectory parity is impossible by construction.
 *
 *  3. "phi4" 3-D     -- the north-star extension: fp32 φ⁴ Jacobi Langevin step
 *     on a periodic Lx×Ly×Lz lattice, same Philox noise.  Also the CPU baseline
 *     of bench.py (OpenMP over host cores, kind "port").
 */
#ifndef SQ_ORACLE_H
#define SQ_ORACLE_H
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- RNG ---------------- */
/* Philox4x32-10 (Salmon et al., SC'11, "Random123"), published algorithm. */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* Four standard normals for (seed, stream, quad, step); layout in DESIGN.md §RNG. */
void orc_normals4(uint64_t seed, uint32_t stream, uint64_t quad, uint64_t step, float out[4]);
/* Device-transcendental mode: tab = the 4 x 2^23 Box-Muller factors of
 * sq_selftest_bm_tables (NULL: back to the double-evaluated normals).  While
 * set, orc_normals4 is the device's normals4 bit for bit and the phi^4 steps
 * draw the kernels' box_muller_q pairs scaled by sigq (orc_phi4_sigq). */
void orc_set_bm_tables(const float *tab);
int orc_bm_tables_on(void);
void orc_normals4_q(uint64_t seed, uint32_t stream, uint64_t quad, uint64_t step, float out[4]);
/* The reference's shared-seed LCG + Box-Muller, tau_kernel.cl:269-284. */
double orc_ref_random(uint64_t *seed, int gid);
/* All draws of one full launch in call order (k = round*(N+1) + item), the
 * accepted draws' 32-bit words t1>>16 / t2>>16, and the seed after each call. */
void orc_ref_noise_stream(uint64_t seed, int N, int loops, double *xi, uint32_t *w1, uint32_t *w2,
                          uint64_t *seeds);

/* The host libm's float logf / cosf / tanhf (glibc: what the reference's
 * random() and clas() evaluate, tau_kernel.cl:222,276-277), element-wise:
 * fn 0 logf, 1 cosf, 2 tanhf.  The device restatement is checked against it. */
void orc_libm_f32(int fn, const float *x, float *y, long long n);

/* ---------------- physics helpers (tau_kernel.cl:184-267) ---------------- */
double orc_xcl(double t, double w, int pot);
double orc_ddpot(double x, int pot);
double orc_intconst(int pot);

/* ---------------- serial (reference-order) QM1D ---------------- */
typedef struct {
    int N, pot, loops;
    double a, c;
    double *f, *x, *xx0, *nf, *nx, *nxx0; /* "device" buffers, length N */
    double omega;
    uint64_t seed;   /* rand1 */
    int stable;
    double dtau;     /* dt_mem_obj */
    int lrgEl;
    double lrgVl;
    int runs;        /* nr_mem_obj */
} orc_serial_dev;

/* One clEnqueueNDRangeKernel of time_dev with global size N+1 (single WG). */
void orc_serial_launch(orc_serial_dev *d);

/* The whole of tauhost.c main() (argv[1..13]) with the serial kernel in place
 * of OpenCL.  stdout lines go to `out`; returns the process exit code. */
int orc_tauhost_main(int argc, const char **argv, FILE *out);

/* ---------------- Jacobi QM1D (the GPU's semantics) ---------------- */
typedef struct {
    int N, pot, loops;
    double a, c, dtau;
    uint64_t seed;
    uint64_t tick;   /* attempted-step counter = Philox step index */
    int runs;
    double *f, *x, *xx0;        /* in: frame-start state */
    double *nf, *nx, *nxx0;     /* out: state after the frame */
    double omega, nomega;
    int lrgEl; double lrgVl;    /* carried across frames, not rolled back */
    int stable;
    int steps_done;
} orc_qm1d;

void orc_qm1d_frame(orc_qm1d *s);

/* ---------------- φ⁴ 3-D (fp32) ---------------- */
typedef struct {
    int Lx, Ly, Lz;
    float h, m2, lam, clampv;
    uint64_t seed;
    double C;        /* noise amplitude: sigma = (float)(sqrt(2h) * C) */
} orc_phi4;

/* One Jacobi Langevin step in -> out at noise step index `step`.
 * nthreads <= 0: OpenMP default. */
void orc_phi4_step(const orc_phi4 *p, const float *in, float *out, uint64_t step, int nthreads);
/* Slab with explicit ghost planes: in = nz+2 planes, out = nz planes. */
void orc_phi4_step_slab(const orc_phi4 *p, const float *in, float *out, int nz, uint64_t z0, uint64_t step);
/* Deep-halo form (the slab path's shrinking ranges): `in` and `out` are padded
 * slabs of nz + 2*gpad planes (local plane zl at padded index zl + gpad); the
 * planes [lo, hi) of `out` are updated from `in` (which must be valid on
 * [lo-1, hi+1)), every other plane of `out` is left alone.  Global z of local
 * plane zl = (z0 + zl) mod Lz (ghost-zone planes wrap). */
void orc_phi4_step_range(const orc_phi4 *p, const float *in, float *out, int nz, int gpad, int lo, int hi,
                         uint64_t z0, uint64_t step);
/* One step with the stability record of DESIGN.md §7 (the 3-D restatement of
 * tau_kernel.cl:135-143): rec = {M = max phi', D = max over the sites
 * attaining M of |phi' - phi - sigma xi| (fp32, fmaf(-sigma, xi, phi' - phi)),
 * A = max |phi'|}.  Single-threaded. */
void orc_phi4_step_stab(const orc_phi4 *p, const float *in, float *out, uint64_t step, float rec[3]);
/* The frame rule over n step records: returns the first step with M > T and
 * D > V (-1: none); T <- M_j and V <- max(V, A_j) through that step. */
int orc_phi4_stab_rule(float *T, float *V, const float *M, const float *D, const float *A, int n);
/* Derived float parameters exactly as the product computes them. */
float orc_phi4_sigma(float h, double C);
float orc_phi4_lam6(float lam);
/* Initial field: phi = amp * normal(seed, stream 2, quad, step 0). */
void orc_phi4_init(const orc_phi4 *p, float amp, float *out);

#ifdef __cplusplus
}
#endif
#endif
