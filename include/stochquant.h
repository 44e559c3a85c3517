/*
 * stochquant.h -- C ABI of libstochquant.so, the MI355X-native (gfx950) drop-in
 * for SebTanz/StochQuant's Langevin path.
 *
 * The reference has no library API: its host program tauhost.c drives one
 * OpenCL kernel inline from main() (clCreateBuffer / clEnqueueWriteBuffer /
 * clEnqueueNDRangeKernel / clEnqueueReadBuffer, tauhost.c:255-560) and its
 * Python driver talks to that program over argv + stdout (taumain.py:132).
 * Each entry point below names the reference code it replaces.  All functions
 * are extern "C", take plain pointers and sizes, never throw, and return 0 on
 * success or a negative SQ_E* code; sq_last_error() gives the message
 * (thread-local).  A context is not thread-safe; the library owns all device
 * memory, HIP streams and RCCL communicators; host arrays are only copied
 * in/out and never retained.
 */
#ifndef STOCHQUANT_H
#define STOCHQUANT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SQ_ABI_VERSION 6

/* status codes */
#define SQ_OK 0
#define SQ_E_ARG -1      /* invalid argument / unsupported shape */
#define SQ_E_HIP -2      /* HIP runtime error */
#define SQ_E_COMM -3     /* RCCL / halo-exchange error */
#define SQ_E_STATE -4    /* call not valid for this context's model/state */
#define SQ_E_NODEV -5    /* no HIP device */

/* models */
#define SQ_MODEL_QM1D 0  /* the reference's 1-D chain + collective coordinate (tau_kernel.cl:25-175), fp64 */
#define SQ_MODEL_PHI4 1  /* 3-D phi^4 lattice, fp32 (north-star extension) */

/* QM1D sweep order (sq_qm1d_set_ordering) */
#define SQ_ORDER_JACOBI 0   /* default: Jacobi sweep, counter-based Philox noise, one launch per frame */
#define SQ_ORDER_SERIAL 1   /* the reference's serial order: Gauss-Seidel sweep, shared 48-bit LCG
                               (tau_kernel.cl:25-175,269-284 with items run in id order) */

/* halo transport for slab decomposition (SQ_MODEL_PHI4 only) */
#define SQ_COMM_NONE 0      /* one slab, periodic z handled in-kernel */
#define SQ_COMM_LOOPBACK 1  /* nslabs slabs on this device, halos by D2D copies */
#define SQ_COMM_RCCL 2      /* one slab per process, halos by ncclSend/ncclRecv over xGMI */
#define SQ_COMM_P2P 3       /* one slab per process, halos pulled from the neighbours' memory through
                               IPC peer pointers (copy engines, no CUs), cross-process ordering by
                               stream-ordered flag writes/waits; frame collectives through peer
                               memory too (no RCCL); bootstrap: sq_p2p_handle / sq_p2p_connect */

typedef struct sq_params {
    int struct_size;            /* = sizeof(sq_params) */
    int model;                  /* SQ_MODEL_* */
    long long dims[3];          /* QM1D: {N,1,1} (argv[1]); PHI4: global {Lx, Ly, Lz} */
    double deltat;              /* QM1D lattice spacing Δt (argv[2]); PHI4: unused (a = 1) */
    double deltatau;            /* Langevin step Δτ (argv[3]) */
    int pot;                    /* QM1D potID 0 = harmonic, 3 = double well (argv[5]) */
    double C;                   /* noise amplitude (argv[6]) */
    int loops;                  /* Langevin steps per frame (argv[10]) */
    unsigned long long seed;    /* Philox key (tauhost.c:185 seeds from rand()) */
    double m2, lambda;          /* PHI4: V = m2/2 phi^2 + lambda/24 phi^4 */
    double clamp;               /* guard: |v| > clamp -> +-clamp, NaN -> clamp (tau_kernel.cl:119-133); 1000 */
    int device;                 /* HIP device ordinal (argv[7] was an OpenCL platform index) */
    int adapt_dtau;             /* 1: reference Δτ controller in sq_run_frame (tauhost.c:523-541) */
    int comm;                   /* SQ_COMM_* */
    int nranks, rank;           /* SQ_COMM_RCCL / SQ_COMM_P2P: processes, this process' rank */
    int nslabs;                 /* SQ_COMM_LOOPBACK: slabs on this device */
    unsigned char comm_id[128]; /* SQ_COMM_RCCL: ncclUniqueId from sq_comm_unique_id on rank 0 */
} sq_params;

typedef struct sq_perf_t {
    long long steps;            /* Langevin steps executed since the last sq_perf_reset */
    long long site_updates;     /* local sites x steps (ghost-zone recomputation not counted) */
    double step_kernel_ms;      /* sum of hipEvent-timed durations of the step kernels (profiling on) */
    long long step_kernel_launches; /* steps covered by step_kernel_ms (profiling on) */
    double frame_ms;            /* wall time inside sq_run_frame / sq_step (host clock) */
    double halo_bytes;          /* bytes sent by halo exchange */
    long long kernel_launches;  /* step-kernel launches issued (any profiling mode): steps / this =
                                   steps per launch (2 for two-step fused launches; a slab block of
                                   G steps issues its core, rim, pairs and edge launches) */
    long long fused_steps;      /* steps executed inside two-step fused launches */
} sq_perf_t;

/* One operation of a deep-halo block (PHI4 slab decompositions),
 * in an issue order that is also a valid sequential order; each op runs on
 * stream A (interior, stream = 0) or stream B (exchange and rims, stream = 1).
 * See sq_phi4_block_plan. */
#define SQ_OP_EXCHANGE 0       /* after the previous block's SQ_OP_EDGES_DONE, send the ghost-depth edge
                                  planes of the latest field to both z-neighbours, receive their ghosts */
#define SQ_OP_STEP 1           /* step `step` on planes [lo, hi) (and [lo2, hi2) when lo2 < hi2) */
#define SQ_OP_PAIR 2           /* steps `step`, `step`+1 in one launch; output [lo, hi), reads [lo-2, hi+2)
                                  of the field the previous launch group wrote */
#define SQ_OP_WAIT_EXCHANGE 3  /* waits for this block's exchange (and, loopback, the neighbours') */
#define SQ_OP_EDGES_DONE 4     /* the planes the next exchange sends are final (event) */
#define SQ_OP_WAIT_STAGED 5    /* waits until the exchange has copied its edge planes aside (an EXCHANGE
                                  op with lo = 1 sends from that staged copy) */
#define SQ_OP_SIGNAL 6         /* records event slot `lo` on the op's stream */
#define SQ_OP_WAIT 7           /* the op's stream waits for event slot `lo` */
typedef struct sq_block_op {
    int kind;                  /* SQ_OP_* */
    int step;                  /* block-relative index of the (first) step computed */
    int lo, hi, lo2, hi2;      /* local plane ranges; negative = lower ghost zone, >= nz = upper */
    int stream;                /* 0: stream A (interior), 1: stream B (exchange, rims) */
} sq_block_op;

typedef struct sq_ctx sq_ctx;

/* Defaults: QM1D, reference constants (clamp 1000, adapt_dtau 1, comm none). */
void sq_params_init(sq_params *p);
const char *sq_last_error(void);
int sq_abi_version(void);

/* Replaces the OpenCL context/queue/buffer/program/kernel set-up,
 * tauhost.c:196-453 (clGetPlatformIDs ... clSetKernelArg). */
int sq_create(const sq_params *p, sq_ctx **out);
/* Replaces the clRelease* tail, tauhost.c:587-612. */
int sq_destroy(sq_ctx *ctx);

/* QM1D state upload: replaces the initial clEnqueueWriteBuffer calls
 * tauhost.c:319-377 and the per-frame re-upload :550-554.  f, x, xx0 have N
 * doubles; runs is the running-mean count (nr_mem_obj). */
int sq_upload(sq_ctx *ctx, const double *f, const double *x, const double *xx0, double omega, long runs);
/* QM1D state download: replaces clEnqueueReadBuffer of newf/newx/newxx0/omega,
 * tauhost.c:508-515.  Any pointer may be NULL. */
int sq_download(sq_ctx *ctx, double *f, double *x, double *xx0, double *omega, long *runs);
/* QM1D carried stability-scan state (lrgEl/lrgVl, tauhost.c:65-66,350-354)
 * and the Philox step counter; for tests and checkpoint/resume. */
int sq_qm1d_get_scan(sq_ctx *ctx, int *lrgEl, double *lrgVl, unsigned long long *tick);
int sq_qm1d_set_scan(sq_ctx *ctx, int lrgEl, double lrgVl, unsigned long long tick);

/* QM1D sweep order.  SQ_ORDER_SERIAL reproduces the
 * serial semantics of time_dev: Gauss-Seidel order,
 * the last step of a frame Jacobi, the racy stability scan as the in-order
 * scan, the break after the first unstable item, newf / lrgEl / lrgVl / the
 * seed never rolled back.  2 <= N <= 4096.  Its noise is the reference's
 * random() (tau_kernel.cl:269-284) on the shared seed rand1 (tauhost.c:185):
 * sq_qm1d_set_lcg_seed sets it, each frame advances it by the calls it made
 * (sq_qm1d_noise_consumed).  sq_qm1d_inject_noise replaces the next frame's
 * draws with a caller-supplied stream in call order (k = round*(N+1) + item,
 * n >= (N+1)*loops); the seed is then left alone. */
int sq_qm1d_set_ordering(sq_ctx *ctx, int ordering);
int sq_qm1d_set_lcg_seed(sq_ctx *ctx, unsigned long long seed);
int sq_qm1d_get_lcg_seed(sq_ctx *ctx, unsigned long long *seed);
int sq_qm1d_inject_noise(sq_ctx *ctx, const double *xi, size_t n);
int sq_qm1d_noise_consumed(sq_ctx *ctx, unsigned long long *n);

/* One frame = `loops` Langevin steps (one clEnqueueNDRangeKernel + clFinish,
 * tauhost.c:481-483) with the stability read-back :504-505, adoption of the
 * new state on success :506-532, rollback to the frame-start snapshot on
 * failure :533-554 (kept on device, no host round trip), and, if
 * adapt_dtau, the reference Δτ controller :523-541. */
int sq_run_frame(sq_ctx *ctx, int *stable);
/* nframes frames back to back, as nframes sq_run_frame calls (same field,
 * verdicts, Δτ sequence, stability state and last-frame records, bit for
 * bit): stable[f] is frame f's verdict, dtau[f] (nullable) the Δτ after it
 * (what the next frame runs at).  PHI4, one slab without an exchange: the
 * verdict, rollback and Δτ controller run on the device between frames (no
 * host round trip; one read-back per call).  Replaces a caller's loop over
 * tauhost.c:479-560 when no per-frame observable is needed in between. */
int sq_run_frames(sq_ctx *ctx, int nframes, int *stable, double *dtau);

/* PHI4: raw Langevin steps without frame control (the bench's hot path). */
int sq_step(sq_ctx *ctx, int nsteps);
/* PHI4 field I/O of this process' slab(s): nz_local*Ly*Lx floats, z slowest.
 * In multi-rank contexts (SQ_COMM_RCCL / SQ_COMM_P2P, nranks > 1) sq_upload_field,
 * sq_init_field and sq_load_field are collective like sq_step: every rank calls
 * them before its next step call, which agrees across the ranks on whether the
 * field (and so every rank's ghost planes) is known to be guarded. */
int sq_upload_field(sq_ctx *ctx, const float *phi, size_t count);
int sq_download_field(sq_ctx *ctx, float *phi, size_t count);
/* PHI4: phi = amp * Philox normal(seed, stream 2, site), generated on device. */
int sq_init_field(sq_ctx *ctx, float amp);
/* PHI4: phi = amp * (h - 2^23) / 2^23, h = the top 24 bits of splitmix64(i ^ key)
 * for global site index i = (z Ly + y) Lx + x: a field any host reproduces
 * bit for bit without the device's RNG (bench.py's oracle_check starts the
 * noise-off parity protocol from it).  Collective like sq_init_field. */
int sq_init_field_hash(sq_ctx *ctx, double amp, unsigned long long key);
/* PHI4 local slab geometry: nz_local and the global z of its first plane. */
int sq_slab(sq_ctx *ctx, long long *nz_local, long long *z0);
/* PHI4 register tile of the step kernel: out = {lanes per x segment, rows
 * per lane, z planes per wave, float4 segments per lane per row}. */
int sq_phi4_tile(sq_ctx *ctx, int out[4]);
/* PHI4: the step kernel's template instance, as rocprofv3 names it, plus its
 * z-chunk, e.g. "phi4_step_kernel<64, 1, 1, false, true, 3> zc=4". */
int sq_phi4_kernel(sq_ctx *ctx, char *name, size_t cap);
/* PHI4 slab decompositions: the ghost-zone depth G in use (= steps per halo
 * exchange; multi-rank RCCL contexts pick it by timed trial blocks during the
 * first sq_step / sq_run_frame calls) and the depth allocated; 0, 0 for a
 * single periodic slab. */
int sq_phi4_ghost(sq_ctx *ctx, int *active, int *allocated);
/* The rest of a slab decomposition's block schedule: core pairs ahead of
 * each exchange, rims on the exchange stream (1) or the interior stream (0),
 * and whether the timed trials chose them (1) or they are the defaults /
 * SQ_CORE_PAIRS / SQ_RIMS_B (0).  Single periodic slab: 0, 0, 0. */
int sq_phi4_schedule(sq_ctx *ctx, int *core_pairs, int *rims_b, int *tuned);
/* Whether the block's last pair computes the slab's edge planes first, so the
 * next exchange starts before the middle (1), or runs whole (0).  Default: 1,
 * except 0 for one rank's RCCL self-exchange; the timed trials of multi-rank
 * contexts try both; SQ_EDGE_FIRST=0|1 pins it.  Single periodic slab: 0. */
int sq_phi4_edge_first(sq_ctx *ctx, int *edge_first);
/* Where a deep-halo block's exchange runs: in_order 1 = in order on the
 * interior stream between the block's last pair and the next block's first
 * (no core / rim split, no cross-stream event), 0 = on the exchange stream,
 * overlapped with the core pairs.  Default: 1 for one rank's RCCL or P2P
 * self-exchange, 0 for ranks on a link, where the timed trials also try 1;
 * SQ_XCHG_ON_A=0|1 pins it.  kstaged (P2P): the block's last pair also
 * writes the next exchange's staging slot (no staging copy); default: with
 * in_order, SQ_P2P_KSTAGE=0|1 pins it.  Single slab / loopback: 0, 0. */
int sq_phi4_exchange_stream(sq_ctx *ctx, int *in_order, int *kstaged);
/* The launch schedule of one deep-halo block (pure host logic, no device
 * needed; the product's phi4_block executes exactly this list): a slab of nz
 * planes with a ghost zone of `ghost` planes (the exchange depth G) running
 * g <= G steps; fuse2 != 0 runs the steps as two-step pairs, the first
 * core_pairs of them on the ghost-free core ahead of the exchange (0: no
 * core/rim split, the first launch waits for the exchange), their rims on the
 * exchange stream when rims_b != 0; edge_first != 0 computes the last step's
 * edge planes first.  Writes *nops ops (at most cap).  sq_phi4_pick_ghost returns the index of the fastest candidate of the
 * rank-max-reduced per-step times ms[n] (the ghost-depth trial, identical on
 * every rank once the times are reduced). */
int sq_phi4_block_plan(int nz, int ghost, int g, int fuse2, int edge_first, int core_pairs, int rims_b,
                       sq_block_op *ops, int cap, int *nops);
int sq_phi4_pick_ghost(const double *ms, int n);
/* PHI4 frame stability (the heuristic of tau_kernel.cl:135-143 restated for
 * the 3-D lattice).  Every frame records per step j the maximum
 * M_j of phi', the drift increment D_j = |phi' - phi - sigma xi| at the sites
 * attaining it (the largest on ties) and A_j = max |phi'|, reduced over all
 * slabs and ranks (RCCL max); the frame is unstable -- rolled back like a
 * clamp / NaN hit -- at the first step with M_j > T and D_j > V, where T is
 * the previous step's maximum and V the running max |phi| of the steps before
 * (carried across frames and never rolled back, as lrgEl / lrgVl; initialised
 * from the field at the first frame).  sq_phi4_stability returns {T, V}, the
 * step at which the last frame fired (-1: none) and that frame's records
 * (n <= loops); sq_phi4_set_stability sets T and V. */
int sq_phi4_stability(sq_ctx *ctx, double state[2], int *fired_step, float *M, float *D, float *A, int n);
int sq_phi4_set_stability(sq_ctx *ctx, double T, double V);
/* PHI4 observables over this process' slab: out[0] = sum phi, out[1] = sum
 * phi^2, out[2] = max |phi| (double accumulation on device). */
int sq_moments(sq_ctx *ctx, double out[3]);

/* The context's parameters (deltatau = the current, possibly adapted, Δτ). */
int sq_get_params(sq_ctx *ctx, sq_params *out);

/* PHI4 binary checkpoint of this process' slab: <path>
 * is a NumPy .npy float32 array of shape (nz, Ly, Lx); <path>.json holds the
 * lattice dims, z0, the Philox step counter, Δτ and the seed.  Replaces the
 * reference's text end/start file (tauhost.c:91-173,562-581) for 3-D fields.
 * sq_load_field with restore_counters != 0 also restores step and Δτ, and the
 * frame state carried across frames (the stability heuristic's T, V and the Δτ
 * controller's stable-frame count; files without it restart that state). */
int sq_save_field(sq_ctx *ctx, const char *path);
int sq_load_field(sq_ctx *ctx, const char *path, int restore_counters);

/* Δτ (dt_mem_obj, tauhost.c:346,526,540). */
int sq_set_dtau(sq_ctx *ctx, double dtau);
int sq_get_dtau(sq_ctx *ctx, double *dtau);
int sq_get_step(sq_ctx *ctx, unsigned long long *step);
int sq_set_step(sq_ctx *ctx, unsigned long long step);

/* Correlator of the reference's observables: QM1D out[i] = xx0[i] -
 * x[i]*x[mid] (host xavg, tauhost.c:519-521), n <= N.  PHI4: zero-momentum
 * time-slice correlator over z, out[t] = <S(z) S(z+t)>/V, n <= Lz, where
 * S(z) = sum_{x,y} phi over the whole lattice (slab contexts: one RCCL sum
 * all-reduce of the slice sums; collective, every rank must call it). */
int sq_correlator(sq_ctx *ctx, double *out, int n);

/* Profiling of the step kernels on their stream: mode 1 = every launch timed
 * by hipExtLaunchKernel start/stop events (dispatch timestamps, no extra
 * packets); mode 2 = one event pair around each sq_step call (region average,
 * includes inter-kernel gaps); 0 = off.  Read with sq_perf. */
int sq_set_profiling(sq_ctx *ctx, int mode);
int sq_perf(sq_ctx *ctx, sq_perf_t *out);
int sq_perf_reset(sq_ctx *ctx);
/* Joins the context's streams and reports asynchronous errors.  A slab
 * exchange whose gated rim chunks timed out (SQ_E_COMM) is sticky: the
 * field's rim planes are stale, so sq_sync, sq_download_field, sq_step and
 * the frame calls keep failing with it until sq_upload_field / sq_load_field
 * / sq_init_field(_hash) replaces the field. */
int sq_sync(sq_ctx *ctx);
/* PHI4: the step kernel launched most often since the last sq_perf_reset, as
 * its template instance (e.g. "phi4_tb2_kernel<true, false, 1, false, true,
 * false>", the name rocprofv3 prints inside "void sq::(anonymous
 * namespace)::...(sq::Phi4StepArgs)"), its grid in threads and its launch
 * count (0 and "" when nothing ran).  Ties a profiler record to the launch. */
int sq_phi4_launch_info(sq_ctx *ctx, char *name, size_t cap, long long *grid_threads, long long *launches);
/* Identity of the compiled code: "phi4:<16 hex> lib:<16 hex>", the first a
 * hash of the φ⁴ kernels' code object, the second of every object linked. */
const char *sq_build_id(void);
/* Noise amplitude C (argv[6], sigma = C sqrt(2 Δτ), tau_kernel.cl:112) of an
 * open context; C = 0 runs the deterministic drift-only update (bench.py's
 * oracle_check).  Not collective: every rank sets the same C.  SQ_E_ARG for
 * |C| > 1e12, and (PHI4) when the new C breaks the creation-time bound of the
 * guard's fast path at the current Δτ. */
int sq_set_noise(sq_ctx *ctx, double C);
/* PHI4, one slab without an exchange, fused launches: run the next two steps
 * (one fused launch, as sq_step(ctx, 2)) with per-block stamps of the
 * constant 100 MHz clock: out[2b], out[2b+1] = start / end of block b
 * (cap >= blocks of the launch); *nblocks = blocks.  A measurement hook for
 * the launch's ramp, tail and busy fraction (bench.py roofline). */
int sq_phi4_block_stamps(sq_ctx *ctx, unsigned long long *out, int cap, int *nblocks);
/* The same launch's shader-clock counter (s_memtime) at each block's start and
 * end, out[2b], out[2b+1]: with sq_phi4_block_stamps, the clock the launch ran
 * at under the chip's power management (bench.py clock_MHz_measured). */
int sq_phi4_block_clocks(sq_ctx *ctx, unsigned long long *out, int cap, int *nblocks);

/* RCCL bootstrap: rank 0 creates the id, the caller distributes it (e.g. via
 * torch.distributed) into sq_params.comm_id of every rank. */
int sq_comm_unique_id(unsigned char out[128]);

/* SQ_COMM_P2P bootstrap: every rank exports one handle blob (IPC handles of
 * its staging buffer, mailbox and collective slots, plus its rank and the
 * lattice it was created for); the caller all-gathers the blobs in rank order
 * (e.g. torch.distributed.all_gather_object) and passes all of them to
 * sq_p2p_connect, which validates and maps them.  Steps, frames and the
 * correlator of a P2P context fail with SQ_E_STATE until connected.  Every
 * rank must run the same sequence of steps (the exchanges pair up by count). */
#define SQ_P2P_HANDLE_BYTES 512
int sq_p2p_handle(sq_ctx *ctx, unsigned char out[SQ_P2P_HANDLE_BYTES]);
int sq_p2p_connect(sq_ctx *ctx, const unsigned char *handles, int nranks); /* nranks * SQ_P2P_HANDLE_BYTES */

/* Device queries / self-tests used by tests and bench (no reference analogue). */
int sq_device_count(int *n);
int sq_selftest_normals(int device, unsigned long long seed, unsigned int stream,
                        unsigned long long quad0, unsigned long long step, float *out, size_t nquads);
int sq_selftest_dpp(int device, float *out64x2);
/* DPP cross-wave stress: mode 0 every wave rotates (wave_ror/rol:1), 1 even waves
 * run the records' row_shr/row_bcast wave-max scan while odd waves rotate, 2 every
 * wave does both, 3 as 1 without row_bcast; errs64[lane] = wrong rotated values. */
int sq_selftest_dpp_mix(int device, int mode, int blocks, int iters, unsigned int *errs64);
int sq_selftest_philox(int device, const unsigned int ctr[4], const unsigned int key[2], unsigned int out[4]);
int sq_copy_bandwidth(int device, size_t bytes, int iters, double *gbps);
/* The serial order's draws of one full launch from `seed` on the device:
 * words t1>>16, t2>>16, the seed after each call, xi ((N+1)*loops each).
 * generator 1 = the grid-wide generator the frames use, 0 = the one-block
 * generator it falls back to from the first exceptional call. */
int sq_selftest_lcg(int device, unsigned long long seed, int N, int loops, unsigned int *w1,
                    unsigned int *w2, unsigned long long *seeds, double *xi, int generator);
/* y[i] = f(x[i]) on the device with the serial order's float transcendentals
 * (glibc's algorithms, csrc/sq_glibcf.h): fn 0 logf, 1 cosf, 2 tanhf. */
int sq_selftest_libm(int device, int fn, const float *x, float *y, long long n);
/* The device's Box-Muller factors for every 23-bit argument m (4 x 2^23 floats,
 * csrc/sq_rng.h): out[m] = sqrt(-2 ln u), out[2^23 + m] = sqrt(-log2 u),
 * out[2*2^23 + m] = cos(t), out[3*2^23 + m] = sin(t), u = 2 - [1.m], t = [1.m]
 * revolutions.  A device normal is one fp32 product of two entries. */
int sq_selftest_bm_tables(int device, float *out);

#ifdef __cplusplus
}
#endif
#endif /* STOCHQUANT_H */
