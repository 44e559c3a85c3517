// sq_internal.h -- kernel argument blocks and launchers shared between the
// kernel translation units and the C-ABI layer (sq_api.cpp).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace sq {

// Sets the thread-local message returned by sq_last_error(); returns code.
int set_error(int code, const std::string &msg);

}  // namespace sq

struct sq_ctx;

namespace sq {

// Frame-control state a phi^4 checkpoint carries besides the field and the
// counters (sq_io.cpp): the stability heuristic's carried T and V and whether
// they were set, and the dtau controller's stable-frame count
// (tauhost.c:523-541).  Not part of the C ABI.
struct FrameState {
    float T, V;
    int init;
    int stab_cnt;
};
int frame_state_get(const sq_ctx *c, FrameState *fs);
int frame_state_set(sq_ctx *c, const FrameState &fs);

// ---------------------------------------------------------------- PHI4 ----
// One slab lives in a padded buffer of (nz + 2*gz) planes of Lx*Ly floats, z
// slowest: padded plane gz + zl holds local plane zl, for zl in [-gz, nz+gz).
// The gz planes on each side are the ghost zone (deep halo) of the
// neighbouring slabs.  With periodic != 0 the slab is the whole lattice in z
// (gz = 1, ghosts unused) and the kernel wraps z itself.
struct FrameCtl;
// Device frames (sq_run_frames): the first fused launch of frame f+1 takes
// frame f's end itself -- every block folds frame f's records, applies the
// stability rule and the Δτ controller to *cin (block 0 writes *cout, the
// folded records, the verdict and Δτ), runs with the new coefficients, and
// reads frame f's start snapshot instead of the field when the verdict is
// unstable (the rollback without a copy); cin == nullptr: none.  The launch
// after it clears the consumed record set (RecClear).  DESIGN.md §7.
struct FrameFoldArgs {
    const FrameCtl *cin;
    FrameCtl *cout;
    const unsigned long long *md;
    const unsigned int *am;
    const int *flag;
    float *rec;
    int *stable_out;
    double *dtau_out;
    const float *snap;  // frame f's start (interior planes, nz of them)
    int L;
};
struct RecClear {  // zero n words of md and am and the flag (md == nullptr: none)
    unsigned long long *md;
    unsigned int *am;
    int *flag;
    int n;
};
constexpr int kFoldMaxL = 64;  // frames of at most this many steps fold (LDS: 12 B per step)

struct Phi4StepArgs {
    const float *in;
    float *out;
    int Lx, Ly, nz, gz;            // gz: ghost planes allocated on either side (local plane 0 is padded plane gz)
    int zlo, zhi, zstep, zc, nzc;  // chunk k updates planes [zlo + k*zstep, +zc) clipped to zhi
    int nzr, zlen;                 // two-step kernel: chunks per range and range length; chunk k covers
                                   // [r0 + (k % nzr)*zc, +zc) clipped to r0 + zlen, r0 = zlo + (k / nzr)*zstep
    int periodic;
    int nxseg, nyg, nunits;
    long long zg0;            // global z of local plane 0
    long long Lzg;            // global Lz (the noise index of ghost-zone planes wraps)
    float h, m2, lam6, sig, clampv;
    float sigq;               // sig * sqrt(2 ln 2): the amplitude of the kernels' box_muller_q normals
    int fin;                  // the input field is known finite (every plane has been through the
                              // guard): the guard then runs only where |phi'| >= clampv
    uint32_t k0, k1, s_lo, s_hi;
    int *flag;                // guard flag: set to 1 when a site was clamped / NaN (nullable: frames only)
    // stability records of this launch's step(s) (nullable; frames only): for
    // step k of the launch, kStabSlots words each at st_md + k*kStabSlots
    // (u64 max of ord(max phi') << 32 | bits(drift increment there)) and
    // st_a + k*kStabSlots (u32 max of bits(max |phi'|)); DESIGN.md §7
    unsigned long long *st_md;
    unsigned int *st_a;
    // frames (nullable): the frame's first fused launch also stores its input's
    // interior planes here -- the rollback snapshot, without a copy kernel
    float *snap;
    // frames under device control (nullable): {h, sig, sigq} of the frame, read
    // by the frame instances at launch start (FrameCtl::coef; the controller
    // kernel of the previous frame may have changed Δτ)
    const float *dcoef;
    int prio;  // fused kernels: wave priority by march progress (prio_by_progress)
    // fused kernels (nullable): per block b, the constant 100 MHz clock
    // (s_memrealtime) at its start and end, stamps[2b], stamps[2b+1]
    unsigned long long *stamps;
    FrameFoldArgs fold;  // frame instances of the fused kernels only
    RecClear clr;
    // three-buffer device frames (frame instances): in / out are buf0..buf2 picked
    // by the frame's launch index tk from *tctl (FrameCtl::bs / bw0 / bw1);
    // tctl == nullptr: in / out as given
    float *buf0, *buf1, *buf2;  // (named fields: a dynamic index would put the argument block in private memory)
    const FrameCtl *tctl;
    int tk;
    // tctl != nullptr and tspec: in / out hold the host's guess of launch tk's
    // buffers (every earlier frame of the batch stable); kernels that can
    // (phi4_tb2_kernel) start on it and check it against *tctl, others ignore it
    int tspec;
    // slab paths, gated launch (gate != nullptr; fused kernels): the first n_reg
    // blocks are the usual chunks of the core range; the blocks after them are
    // thin chunks (tzc planes, ntz per range) of the two rim ranges [tlo0, +tlen)
    // and [thi0, +tlen), which read ghost planes: each first waits until
    // *gate >= gate_seq -- stream B writes it behind the exchange -- so the
    // core and the rims run in one launch without a stream hop
    const unsigned int *gate;
    unsigned int gate_seq;
    int n_reg, tzc, tlen, tlo0, thi0, ntz;
    int *gate_err;  // bit 0 set when a wait gave up (kGateSpinMax); bit 1: a P2P hand-shake gave up
};
constexpr int kStabSlots = 32;

// Device-resident frame controller (sq_run_frames): the
// stability rule's carried state, the Δτ controller (tauhost.c:523-541) and the
// step coefficients the next frame's launches read, so frames run back to back
// without a host decision between them.
struct FrameCtl {
    double dtau;     // the next frame's Δτ
    double C;        // noise amplitude (sigma = C sqrt(2 Δτ))
    float coef[4];   // {h, sig, sigq, 0} of the next frame, computed from dtau as phi4_base_args does
    float T, V;      // stability rule: last step's max phi', running max |phi'| (never rolled back)
    int stab_cnt;    // stable frames since the last Δτ change
    int adapt;       // Δτ controller on
    int stable;      // the last frame's verdict (1 stable)
    int fired;       // its firing step, -1 none
    int flag;        // its guard flag
    int frames;      // frames decided since the context's controller was (re)loaded
    // three-buffer device frames (tri != 0; Phi4StepArgs::buf0..buf2): the frame
    // starts from buffer bs, which no launch of the frame writes -- it IS the
    // rollback snapshot -- and its launches alternate bs -> bw0 -> bw1 -> bw0
    // ...; the frame's result is in bw0 when it has an odd number of launches
    // (nl_odd), else bw1.  frame_decide rotates them: stable -> the next frame
    // starts from the result, unstable -> from bs again.
    int tri, bs, bw0, bw1, nl_odd;
};
// One launch after a frame (phi4_frame_end_kernel): folds the frame's
// kStabSlots-slot records (md, am, flag), writes the per-step maxima to rec
// (M[L] | D[L] | A[L]), applies the stability rule and the Δτ controller to
// *cin and writes the result to *cout (cout->coef: the next frame's
// coefficients), clears the other record set (md_next, am_next, flag_next)
// for the next frame, writes the verdict to *stable_out and the new Δτ to
// *dtau_out when non-null, and, unstable, copies snap back to dst (n4 float4).
struct FrameEndArgs {
    const FrameCtl *cin;
    FrameCtl *cout;
    const unsigned long long *md;
    const unsigned int *am;
    const int *flag;
    unsigned long long *md_next;
    unsigned int *am_next;
    int *flag_next;
    int L;
    float *rec;
    int *stable_out;
    double *dtau_out;
    float4 *dst;
    const float4 *snap;
    long long n4;
};
hipError_t phi4_frame_end_launch(const FrameEndArgs &e, hipStream_t s);
constexpr double kSqrt2Ln2 = 1.1774100225154747;  // sqrt(2 ln 2): box_muller_q's missing factor (sq_rng.h)

struct Phi4Geom {
    int qx;   // lanes per x segment (4 sites each)
    int r;    // rows per lane
    int wy;   // rows per wave unit
    int pf;   // store / arithmetic mode: 1 scalar site arithmetic (narrow rows); 3 packed-f32 site
              // arithmetic (qx == 64); 4 as 3 with non-temporal output stores (default above 2 GiB
              // of fields per device); 7 as 3 with sc0 sc1 output stores (default for full-row waves)
    int v;    // float4 segments per lane per row (x-span of a wave = 4*qx*v sites): 1 or 2
};

// Two steps per launch (steps s and s+1, s = a.s_hi:a.s_lo) on one or more
// equal ranges of planes: range r = [zlo + r*zstep, + zlen) (a single periodic
// slab: [0, nz)); a.zc = output planes per block, a.nzr chunks per range,
// a.nzc = all chunks, a.nxseg = Lx / 256, a.nyg = Ly / 8 y-bands, a.nunits =
// blocks; the input must be valid two planes beyond every range.
// Bit-identical to two step launches.
bool phi4_tb2_supported(int Lx, int Ly);
hipError_t phi4_tb2_launch(const Phi4StepArgs &a, hipStream_t s, hipEvent_t start = nullptr,
                           hipEvent_t stop = nullptr, uint64_t *kid = nullptr);

// Several two-step pairs in ONE resident launch (sq_phi4_run.hip): pair t reads
// a.in (t even) or a.out (t odd) and writes the other, steps s + 2t and s + 2t + 1;
// a block starts pair t + 1 once its 3 x 3 neighbourhood of blocks (y-bands x
// z-chunks, periodic) has finished pair t.  flags: one word per block, the epoch
// base + t + 1 after pair t (base: the context's running count, so nothing is
// cleared between launches); err: bit 2 set when a wait gave up (kRunSpinMax),
// which ends every block's waits.  Single periodic slab of 256-site rows, no
// frames, every block resident (phi4_tb2_run_ok).
struct Tb2RunArgs {
    unsigned int *flags;
    int *err;
    unsigned int base;
    int npairs;
    // diagnostics (nullable, SQ_DIAG_RUN_STAMPS): per pair t and block b, the
    // constant 100 MHz clock at [2 (t nb + b)] the pair's start (its wait done)
    // and [+1] its end (stores drained); then per block its hardware slot
    // (XCC_ID << 16 | HW_ID) at [2 npairs nb + b]
    unsigned long long *stamps;
};
bool phi4_tb2_run_ok(const Phi4StepArgs &a, int dev);
hipError_t phi4_tb2_run_launch(const Phi4StepArgs &a, const Tb2RunArgs &r, hipStream_t s, hipEvent_t start = nullptr,
                               hipEvent_t stop = nullptr, uint64_t *kid = nullptr);
void phi4_run_kernel_id_name(uint64_t kid, char *name, size_t cap);

// The last pair of a P2P deep-halo block with its edge planes also stored into
// the next exchange's staging slot (sq_phi4_run.hip): phi4_tb2_kernel's
// launch (one range, 256-site rows, no frame records) whose output planes
// [0, G) and [nz - G, nz) are also written, write-through, to stage[0, G)
// and stage[G, 2G) planes; every block then adds 1 to *ctr behind its drained
// stores, so the exchange stream's hand-shake waits for the count
// (p2p_handshake_launch's pre) instead of a cross-stream event and a copy.
struct Tb2StageArgs {
    float *stage;
    int G;
    unsigned int *ctr;
};
bool phi4_tb2_stage_ok(const Phi4StepArgs &a, int G);
hipError_t phi4_tb2_stage_launch(const Phi4StepArgs &a, const Tb2StageArgs &g, hipStream_t s,
                                 hipEvent_t start = nullptr, hipEvent_t stop = nullptr, uint64_t *kid = nullptr);

// Kernel identity of a launch (kid out-parameters of the launchers): the
// template instance the launcher picked, packed with the grid in threads (high
// 32 bits), so a caller can name the dominant kernel exactly as rocprofv3 does
// (sq_phi4_launch_info; bench.py ties its committed PMC record to it).
void phi4_kernel_id_name(uint64_t kid, char *name, size_t cap);  // family 3: phi4_run_kernel_id_name
inline unsigned phi4_kernel_id_grid(uint64_t kid) { return (unsigned)(kid >> 32); }

// Picks the register tile for (Lx, Ly); returns false if unsupported.
bool phi4_geometry(int Lx, int Ly, Phi4Geom *g);
// Fills the work decomposition of a launch that updates `nzc` chunks.
void phi4_fill_units(Phi4StepArgs &a, const Phi4Geom &g);
// start/stop non-null: timed through hipExtLaunchKernel (timestamps of the
// dispatch itself, no extra marker packets on the stream).
hipError_t phi4_step_launch(const Phi4StepArgs &a, const Phi4Geom &g, hipStream_t s,
                            hipEvent_t start = nullptr, hipEvent_t stop = nullptr, uint64_t *kid = nullptr);
// slab = local plane 0 (past the ghost zone)
// phi = amp * (top 24 bits of splitmix64(global index ^ key) - 2^23) / 2^23
// (sq_fields.hip; the host restatement is stochquant_amd/verify.py hash_field)
hipError_t phi4_init_hash_launch(float *slab, int Lx, int Ly, int nz, long long zg0, unsigned long long key,
                                 double amp, hipStream_t s);
hipError_t phi4_init_launch(float *slab, int Lx, int Ly, int nz, long long zg0, uint32_t k0,
                            uint32_t k1, float amp, hipStream_t s);
// Moments of a slab: acc = {sum phi, sum phi^2}, acc_max = {bits(max |phi|),
// ord(max phi)} (order-preserving bits, sq_phi4.hip ord_f32), written, not
// accumulated; part: kMomBlocks * 4 doubles of scratch.  Deterministic:
// per-block partials folded in block order by a second one-block kernel.
constexpr int kMomBlocks = 1024;
hipError_t phi4_moments_launch(const float *slab, long long n, double *acc, unsigned int *acc_max, double *part,
                               hipStream_t s);
// Slice sums S(z) = sum_{x,y} phi(x,y,z) for z in [0,nz): out[z] (double); slab = local plane 0.
hipError_t phi4_slices_launch(const float *slab, int Lx, int Ly, int nz, double *out,
                              hipStream_t s);

// Peer-pointer transport (sq_p2p.hip): out[i] = fold over q < nranks of
// slot q's element i, slot q at slots + q * cap bytes, in rank order.
enum class P2pRed { kMaxU32, kMaxI32, kMaxU64, kMaxF64, kSumF64 };
// P2P exchange e's hand-shake as one launch of one wave (sq_p2p.hip): write e
// into both neighbours' mailbox words, then wait for both of ours to reach e;
// after `polls` polls it gives up and sets bit 1 of *err.  pre (nullable):
// first wait until *pre has reached pre_n (phi4_tb2_stage_launch's count)
hipError_t p2p_handshake_launch(unsigned int *up_from_dn, unsigned int *dn_from_up, const unsigned int *from_dn,
                                const unsigned int *from_up, unsigned int e, unsigned int polls, int *err,
                                hipStream_t s, const unsigned int *pre = nullptr, unsigned int pre_n = 0);
// d0[0..n) = s0[0..n) and d1[0..n) = s1[0..n) in one launch (sq_p2p.hip)
hipError_t p2p_copy2_launch(float *d0, const float *s0, float *d1, const float *s1, size_t n, hipStream_t s);
hipError_t p2p_fold_launch(const unsigned char *slots, int nranks, size_t cap, void *out, size_t n, P2pRed red,
                           hipStream_t s);

// ---------------------------------------------------------------- QM1D ----
struct Qm1dState {    // device-resident frame scalars
    double omega_in;  // ω at frame start
    double omega_out; // ω after the frame
    double lrgVl;     // carried running max |X| (tauhost.c:66, never rolled back)
    int lrgEl;        // carried leader index (tauhost.c:65)
    int stable;       // 1 stable, 0 unstable
    int steps_done;
    int sync_error;   // qm1d_frame_grid: a grid barrier gave up waiting (kGridSpinMax polls); the frame is void
};

struct Qm1dArgs {
    const double *f, *x, *xx0;  // frame-start state (N)
    double *nf, *nx, *nxx0;     // state after the frame (N)
    double *fs, *xs, *ds;       // N > kQm1dRegMaxN only: f ping-pong, X' and drift-check scratch (N each)
    // N <= kQm1dRegMaxN: the field-independent work of the frame, precomputed
    // grid-wide (qm1d_prep_launch) so the per-step chain keeps only the field
    // arithmetic: om[j] = omega at the start of step j (loops + 1), xi[j*nq4 + i]
    // the site normals (nq4 = N rounded up to 4), and for potID 3
    // tcl[j*(N+2) + i+1] = the float tanhf of x_cl(i a; om[j]) for i = -1..N and
    // dd[j*N + i] = ddPot(x_cl(i a; om[j]))
    double *om;
    float *xi, *tcl;
    double *dd;
    Qm1dState *st;
    int N, pot, loops, runs;
    double a, a2, h, sig, sigw, kconst;
    uint32_t k0, k1;
    unsigned long long tick;    // Philox step index of the frame's first step
    int gbar;                   // qm1d_frame_grid: 1 = its own counter barrier (else cooperative groups)
    unsigned int bar_polls;     // ... the barrier's poll budget (0: kGridSpinMax)
    int bar_skip;               // ... (tests, SQ_QM1D_BAR_SKIP) this block never arrives at barrier 1; -1 none
    unsigned long long *dbg;    // ... (diagnostics, SQ_QM1D_STAMPS) per block and step < 64, five 100 MHz clock
                                //     stamps: step start, stores done, past the barrier, past the previous scan's
                                //     outcome, scan done (nullable)
};

int qm1d_sites_per_thread(int N);  // 0 if N unsupported (global-memory variant: N > kQm1dRegMaxN)
constexpr int kQm1dMaxN = 1024 * 64;
constexpr int kQm1dRegMaxN = 4096;  // register-resident frame kernel up to here; beyond, f ping-pong + scan scratch
constexpr int kQm1dGridAux = 2048;
// SQ_QM1D_STAMPS diagnostics: the stamp buffer's blocks (the grid kernel's default G
// is at most this; SQ_QM1D_GK can force more); blocks past it record nothing
constexpr int kQm1dStampBlocks = kQm1dMaxN / 512;
// device bytes the precomputed frame tables may take (loops x N x 4-16 B); a
// frame longer than this at its N is refused rather than allocated
constexpr size_t kQm1dTableCap = size_t(16) << 30;  // N > kQm1dRegMaxN: xs and ds hold N + this many doubles (qm1d_frame_grid)
hipError_t qm1d_frame_launch(const Qm1dArgs &a, hipStream_t s);
// The precomputed tables of a register-kernel frame (N <= kQm1dRegMaxN), on the
// same stream ahead of qm1d_frame_launch; a.om / a.xi (/ a.tcl, a.dd) sized as above.
hipError_t qm1d_prep_launch(const Qm1dArgs &a, hipStream_t s);

// QM1D in the reference's serial order (sq_qm1d_gs.hip)
struct Qm1dGsState {
    double omega_in, omega_out, lrgVl;
    int lrgEl, stable, steps_done;
    int rows_ready;      // steps the sweep has completed (sweep -> scan handshake; 0 at upload)
    long long consumed;  // random() calls the launch made (the shared seed advances by these)
    int sync_error;      // the scan timed out waiting for the sweep
    int brk_step, brk_item;  // the serial break (-1: stable frame)
    int pad;
};

struct Qm1dGsArgs {
    const double *f0, *x0, *xx00;  // frame-start state (N)
    double *nf, *nx, *nxx0;        // state after a stable frame (N)
    double *nfp;                   // the persistent newf buffer (never rolled back, tauhost.c)
    const double *xi;              // (N+1)*loops draws in call order
    double *om;                    // omega at the start of each step (loops+1)
    double *xc;                    // potID 3: x_cl(i a, om[j]) at [j (N+2) + i + 1], i = -1..N,
                                   // then ddPot of it at the same index + (N+2) loops
    void *cand;                    // per-step scan candidates (qm1d_gs_cand_bytes)
    int *flags;                    // per-step "candidates ready" flags (== tag)
    int tag;                       // this frame's flag value (never 0)
    double *hist;                  // field after each step (loops*N)
    Qm1dGsState *st;
    int N, pot, loops, runs;
    double a, a2, h, sig, sigw, kconst;
};

constexpr int kQm1dGsMaxN = 4096;  // <= 4 sites per thread of a 1024-thread block; 2N doubles of LDS
int qm1d_gs_block(int N);  // sites per lane of the sweep pipeline, 0 if N unsupported
// The LCG stream of a launch: w1/w2/seeds/xi per call.  scr (kLcgScratch
// words, or null for the one-block generator) holds the grid-wide
// generator's chunk maps and start seeds.
constexpr int kLcgChunks = 16384;
constexpr size_t kLcgScratch = 3 * (size_t)kLcgChunks + 1;
hipError_t qm1d_gs_lcg_launch(unsigned long long seed, int N, long long ncalls, uint32_t *w1,
                              uint32_t *w2, unsigned long long *seeds, double *xi,
                              unsigned long long *scr, hipStream_t s);
size_t qm1d_gs_cand_bytes(int loops);
hipError_t qm1d_gs_frame_launch(const Qm1dGsArgs &a, hipStream_t s);

// -------------------------------------------------------------- selftest --
hipError_t selftest_normals_launch(float *out, size_t nquads, unsigned long long quad0,
                                   uint32_t stream, unsigned long long step, uint32_t k0,
                                   uint32_t k1, hipStream_t s);
hipError_t selftest_dpp_launch(float *out, hipStream_t s);
hipError_t selftest_dpp_mix_launch(int mode, int blocks, int iters, unsigned *errs, float *sink, hipStream_t s);
hipError_t selftest_philox_launch(const uint32_t *ck, uint32_t *out, hipStream_t s);
hipError_t selftest_libm_launch(int fn, const float *x, float *y, long long n, hipStream_t s);
hipError_t selftest_bm_tables_launch(float *t, hipStream_t s);
hipError_t copy_launch(const float4 *in, float4 *out, size_t n4, bool nt, hipStream_t s);

}  // namespace sq
