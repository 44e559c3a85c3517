// sq_api.cpp -- C ABI of libstochquant.so (include/stochquant.h).
//
// Replaces the OpenCL host plumbing of tauhost.c (buffers, kernel args, the
// per-frame launch / read-back / rollback / re-upload, tauhost.c:196-560) with
// a library that owns device memory, HIP streams and RCCL communicators:
//   * QM1D: frame-start state and frame result live in two device buffer sets;
//     a stable frame flips the set, an unstable one simply keeps the old set
//     (rollback without the reference's 3N+1-double host round trip).
//   * PHI4: a slab per process (RCCL) or several slabs per device (loopback),
//     each a padded ping-pong pair; per step the interior planes update on
//     stream A while the halo exchange and the two boundary planes run on
//     stream B, joined by events.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/stochquant.h"
#include "sq_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define SQ_HIP(expr)                                                                             \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail(SQ_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));           \
    } while (0)

#define SQ_NCCL(expr)                                                                            \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess)                                                                   \
            return fail(SQ_E_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_));        \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct Slab {
    float *buf[2] = {nullptr, nullptr};  // padded ping-pong
    float *snap = nullptr;               // frame-start snapshot (interior planes) = snap_pad + gpad planes
    float *snap_pad = nullptr;           // its allocation, padded like buf[]: three-buffer device frames
                                         // rotate the three (phi4_frames_dev)
    int nz = 0;
    long long z0 = 0;
    hipStream_t sA = nullptr, sB = nullptr;
    hipEvent_t evC = nullptr;                 // C: the block's halo exchange done
    hipEvent_t evE = nullptr;                 // E: the block's output edge planes (what the next exchange sends) done
    float *stage = nullptr;                   // 2 G planes (x stage_slots): the staged copy of the edge planes an exchange sends
    hipEvent_t evS = nullptr;                 // S: the staged copy is complete (the field's edges may change)
    std::vector<hipEvent_t> evk;              // the block plan's SIGNAL / WAIT slots (kPlanSlots)
};

struct EvPair {
    hipEvent_t a, b;
};

// SQ_COMM_P2P: the words of a rank's mailbox its neighbours
// and peers write with stream-ordered flag writes; every value is a sequence
// number that only grows, so a wait is ">= this exchange / collective".
constexpr int kMbStagedFromDn = 0;  // the lower neighbour's staged edge planes of exchange e are complete
constexpr int kMbStagedFromUp = 1;  // ... the upper neighbour's
constexpr int kMbAckFromDn = 2;     // the lower neighbour has finished reading our staged copies (teardown)
constexpr int kMbAckFromUp = 3;     // ... the upper neighbour
constexpr int kMbColl = 16;         // + q: rank q's contribution to collective k is in our slot q
// staged copies per slab: P2P double-buffers them by exchange parity
inline size_t stage_slots(int comm) { return comm == SQ_COMM_P2P ? 2 : 1; }
// polls of the P2P hand-shake wave before it gives up (s_sleep 2 between: ~1-2 s)
constexpr unsigned int kHandshakePolls = 1u << 24;
constexpr int kMbWords = 1024;
constexpr int kP2pMaxRanks = kMbWords - kMbColl;
constexpr unsigned int kP2pMagic = 0x53513250u;  // "SQ2P"
// RCCL halo communicator: blocks per send/recv kernel (ncclConfig_t.maxCTAs)
constexpr int kRcclMaxCtas = 0;

struct Peer {  // a rank's buffers as this process addresses them
    float *stage = nullptr;
    unsigned int *mbox = nullptr;
    unsigned char *coll = nullptr;
    bool mapped = false;  // opened through IPC (closed by sq_destroy)
};

struct P2pBlob {  // sq_p2p_handle's output
    unsigned int magic, version;
    int rank, nranks, Lx, Ly, gpad, loops, gz, gauto;  // gz / gauto: active ghost depth, timed pick
    // the block schedule: pinned settings and which of them the timed pick may
    // change (the pick's candidate list and every exchange depend on them)
    int ef_auto, k_auto, edge_first, core_pairs, rims_b;
    int a_auto, on_a, kstage;  // the exchange's stream and the staged last pair (SQ_XCHG_ON_A, SQ_P2P_KSTAGE)
    long long Lz, coll_cap;
    unsigned long long seed;
    hipIpcMemHandle_t stage, mbox, coll;
};
static_assert(sizeof(P2pBlob) <= SQ_P2P_HANDLE_BYTES, "P2P handle blob");

// Inverse of the kernels' order-preserving float -> uint map (sq_phi4.hip ord_f32).
float unord_f32(unsigned int o) {
    const unsigned int u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
    float f;
    memcpy(&f, &u, sizeof f);
    return f;
}

double host_intconst(int pot) {  // tau_kernel.cl:196-200,237-246 (float arithmetic)
    if (pot == 3)
        return (double)(sqrtf((float)3.) * powf((float)2., (float)(-5. / 4.)) *
                        powf((float)2., (float)(-1. / 4.)) / sqrtf((float).8));
    return 0.;
}

}  // namespace

int sq::set_error(int code, const std::string &msg) { return fail(code, msg); }

struct sq_ctx {
    sq_params p{};
    int dev = 0;
    double dtau = 0;
    int stab_cnt = 0;
    unsigned long long step = 0;  // Philox step counter (attempted steps)
    // QM1D
    int N = 0;
    double *qf[2] = {nullptr, nullptr}, *qx[2] = {nullptr, nullptr}, *qxx0[2] = {nullptr, nullptr};
    int qcur = 0;
    sq::Qm1dState *qst = nullptr;
    double *qscr[3] = {nullptr, nullptr, nullptr};  // N > kQm1dRegMaxN: fs, xs, ds of Qm1dArgs
    // N <= kQm1dRegMaxN, Jacobi frames: the precomputed tables of Qm1dArgs (om, xi, tcl, dd)
    double *qom = nullptr, *qdd = nullptr;
    float *qxi = nullptr, *qtcl = nullptr;
    double omega = 0;
    long runs = 0;
    int lrgEl = 0;
    double lrgVl = 0;
    hipStream_t qstream = nullptr;
    // QM1D serial order (SQ_ORDER_SERIAL): LCG state and per-frame buffers
    int order = SQ_ORDER_JACOBI;
    unsigned long long lcg_seed = 0;  // rand1 (tauhost.c:185), advanced by the calls each frame makes
    bool inject_pending = false;       // g_xi holds a caller-supplied stream for the next frame
    unsigned long long consumed = 0;   // random() calls of the last serial frame
    long long g_calls = 0, g_hist = 0, g_loops = 0; // capacities
    double *g_xc = nullptr;  // potID 3: x_cl and ddPot(x_cl) of every (step, site), 2 (N+2) loops
    void *g_cand = nullptr;  // serial scan candidates per step
    int *g_flags = nullptr;  // per-step "candidates ready" flags, compared with gs_tag
    int gs_tag = 0;
    double *g_xi = nullptr, *g_om = nullptr, *g_hist_buf = nullptr, *g_nfp = nullptr;
    uint32_t *g_w1 = nullptr, *g_w2 = nullptr;
    unsigned long long *g_seeds = nullptr;
    unsigned long long *g_lcg_scr = nullptr;  // grid-wide LCG generator scratch (sq::kLcgScratch words)
    sq::Qm1dGsState *g_st = nullptr;
    // PHI4
    int Lx = 0, Ly = 0;
    long long Lz = 0;
    sq::Phi4Geom geom{};
    int zc = 8;
    int gz = 1;    // active ghost-zone depth (planes) of slab decompositions = steps per halo exchange
    int gpad = 1;  // allocated ghost planes on either side of each slab (gz <= gpad)
    bool g_auto = false, g_tuned = false;  // ghost depth chosen by timed trial blocks (phi4_autotune)
    bool k_auto = true;                    // ... and the core pairs (unless SQ_CORE_PAIRS pins them)
    double *dtune = nullptr;
    std::vector<Slab> slabs;
    int cur = 0;
    int *flag = nullptr;
    bool in_frame = false;  // phi4_frame: the step kernels raise the guard flag
    float *snap_next = nullptr;  // phi4_frame: the next fused launch writes its input here (Phi4StepArgs::snap)
    unsigned long long *stamps_next = nullptr;  // sq_phi4_block_stamps: the next fused launch's block stamps
    unsigned long long *dstamps = nullptr;
    int stamps_cap = 0, stamps_blocks = 0;
    bool field_finite = true;  // every plane of the current field has been through the guard (or
                               // came from sq_init_field); false after a caller's upload / load
    bool fin_sync = false;     // multi-rank: field_finite changed locally; the next step call
                               // agrees on it across ranks first (ghost planes come from neighbours)
    bool edge_first = true; // deep-halo blocks: last step's edge planes first (SQ_EDGE_FIRST=0|1 pins it)
    bool diag_no_xwait = false;  // SQ_DIAG_NO_XWAIT: timing diagnostics only (results wrong)
    bool diag_no_ewait = false;  // SQ_DIAG_NO_EWAIT: no EDGES_DONE event at all (timing only, results wrong)
    bool p2p_kernel_handshake = true;  // P2P: the hand-shake as one wave (SQ_P2P_STREAMOPS=1: stream flag ops)
    bool ef_auto = true;    // the timed pick also tries the other edge_first (unless SQ_EDGE_FIRST pins it)
    int core_pairs = 1;     // deep-halo blocks: fused pairs of the core run ahead of the exchange (0: none)
    bool rims_b = false;    // ... and their rims run on the exchange stream (block_plan)
                            // (SQ_CORE_PAIRS pins; multi-rank runs time 1, 2, 4 on the real link)
    double *dacc = nullptr;
    double *dpart = nullptr;       // moments: per-block partials (sq::kMomBlocks x 4)
    double *dslice = nullptr;      // correlator: slice sums of the global lattice (Lz), allocated once
    unsigned int *dmax = nullptr;  // [0] max |phi| bits, [1] ordered max phi
    // stability heuristic of phi4 frames (tau_kernel.cl:135-143):
    // per-step device records of the current frame, kStabSlots words per step
    unsigned long long *st_md = nullptr;
    unsigned int *st_a = nullptr;
    // phi^4 frames: st_md | st_a | flag in ONE device block (one memset, one
    // read-back per frame) and its pinned host mirror
    void *frame_rec = nullptr;  // two record sets of frame_bytes (device frames alternate them)
    void *frame_cur = nullptr;  // the active set (st_md, st_a, flag point into it)
    int rec_set = 0;
    void *frame_host = nullptr;
    size_t frame_bytes = 0;
    bool frame_rec_zero = true;  // frame_rec is (or is queued to be) all zero: the next frame skips its memset
    unsigned long long frame_step0 = 0;  // Philox step of the frame's first step
    bool stab_init = false;              // T, V set from the field at the first frame
    float stab_T = 0, stab_V = 0;        // carried across frames, never rolled back (as lrgEl / lrgVl)
    int stab_fired = -1;                 // step of the last frame at which the rule fired, -1 none
    std::vector<float> rec_M, rec_D, rec_A;  // the last frame's per-step records
    // device frame control (phi4_frames_dev): controller state and its pinned
    // mirror, the last frame's folded records (M | D | A, loops floats each) and
    // per-frame verdicts / Δτ of a batch (fr_cap entries, device and pinned)
    sq::FrameCtl *ctl = nullptr, *ctl_host = nullptr;  // ctl: two states (frame f reads ctl[f&1], writes the other)
    float *rec_dev = nullptr;
    int *fr_stable = nullptr, *fr_stable_h = nullptr;
    double *fr_dtau = nullptr, *fr_dtau_h = nullptr;
    int fr_cap = 0;
    bool dev_frames = false;  // the current frame's launches read {h, sig, sigq} from ctl_cur->coef
    sq::FrameFoldArgs fold_next{};  // the next fused launch takes the previous frame's end (phi4_frames_dev)
    sq::RecClear clr_next{};        // ... and the launch after it clears that frame's record set
    bool clr_armed = false;
    // three-buffer device frames (phi4_frames_dev): buffers of the batch, the
    // frame's launch index, the controller state the launches read
    bool tri = false;
    float *tri_bufs[3] = {nullptr, nullptr, nullptr};
    int frame_tk = 0;
    // the host's guess of the current frame's buffer roles (FrameCtl::bs / bw0 /
    // bw1 if every earlier frame of the batch was stable); SQ_FRAME_SPEC=0: off
    int spec_bs = 0, spec_bw0 = 1, spec_bw1 = 2;
    bool tri_spec = true;
    bool clr_first = false;         // ... armed by the next launch even without a fold (a batch's frame 0)
    sq::FrameCtl *ctl_cur = nullptr;
    int tbz = 0;                    // two-step fused launches: > 0 on; planes per block when pinned
    bool tbz_pin = false;           // SQ_FUSE2_Z pinned the planes per block
    int tb_minz = 4;                // fewest planes per block of a fused launch (SQ_TB2_MINZ, an experiment)
    int tb_blocks = 512;            // otherwise: blocks per launch aimed at (two per CU)
    // slab paths: the fused launches that run beside an exchange (the core
    // pairs, the middle pair after EDGES_DONE) aim at fewer blocks: the
    // exchange's kernels hold a few CUs, and a full one-round grid then leaves
    // its last blocks for a second round (core pair 43-45 us vs 33)
    int tb_blocks_xchg = 416;
    bool beside_xchg = false;       // the launch being issued runs beside an exchange
    // EDGES_DONE as the stop event of the pair before it (SQ_EDGES_STOPEV=1):
    // hipExtLaunchKernel binds the event to the dispatch itself instead of a
    // marker packet behind it on stream A (each marker leaves a 5-7 us bubble)
    bool edges_stopev = false;
    hipEvent_t stop_next = nullptr;  // the next fused launch's stop event
    bool stop_used = false;          // ... which EDGES_DONE then need not record
    // gated pair 0 (SQ_SLAB_GATE=1; default off, slower: DESIGN.md §8.0): K = 1 blocks run the core pair and
    // the rim pair as ONE launch whose thin rim chunks wait in-kernel for the
    // exchange (Phi4StepArgs::gate), no WAIT_EXCHANGE hop and no small rim grid
    bool slab_gate = false;
    unsigned int *gate_word = nullptr;  // fine-grained: stream B writes ++gate_seq behind each exchange
    unsigned int gate_seq = 0;
    int *gate_err = nullptr;
    // sticky: a gated rim chunk timed out, so the field's rim planes are stale;
    // every call that would use the field fails until a new field is uploaded
    // or initialised (gate_check / gate_reset)
    bool gate_failed = false;
    // single slab (SQ_TB2_RUN=1): a call's pairs as ONE resident launch
    // (sq_phi4_run.hip); run_flags: one epoch word per block, run_base the
    // epoch every block has reached (gate_err bit 2: a march wait gave up)
    // P2P, SQ_P2P_KSTAGE=1: the last pair of a deep-halo block writes the next
    // exchange's staging slot itself and counts its blocks into kstage_ctr
    // (phi4_tb2_stage_kernel); the exchange's hand-shake waits for kstage_n
    // instead of the EDGES_DONE event plus a staging copy.  kstage_pending:
    // the slot holds the current field's edges (dropped when anything else
    // writes the field); evE_stale: EDGES_DONE was not recorded behind that
    // pair, so an exchange of the old form records it first
    // P2P, SQ_XCHG_ON_A=1: the exchange (staging, hand-shake, pull) runs on the
    // interior stream in order, between a block's last pair and the next
    // block's first (no core / rim split, no cross-stream event or spin)
    bool xchg_on_a = false;
    bool a_auto = true;   // multi-rank timed pick also tries it (unless SQ_XCHG_ON_A pins it)
    int kstage_env = -1;  // SQ_P2P_KSTAGE if set; else kstage follows xchg_on_a
    unsigned int *kstage_ctr = nullptr;
    unsigned int kstage_n = 0;
    bool kstage_pending = false, kstage_next = false, kstage_issued = false, evE_stale = false;
    float *kstage_slot = nullptr;
    bool tb_run = false;
    unsigned int *run_flags = nullptr;
    int run_nflags = 0;
    unsigned int run_base = 0;
    struct {
        bool on;
        int tlo0, thi0, tlen;
    } gate_next{false, 0, 0, 0};
    long long ev_extra_steps = 0;   // profiling mode 1: steps beyond the first in timed launches
    ncclComm_t comm = nullptr;
    // SQ_COMM_P2P: mailbox, collective slots (2 parities x nranks x coll_cap
    // bytes) and every rank's buffers as mapped here (own ones at [rank])
    unsigned int *mbox = nullptr;
    unsigned char *coll = nullptr;
    size_t coll_cap = 0;
    std::vector<Peer> peers;
    bool p2p_ready = false;
    unsigned int xchg_seq = 0, coll_seq = 0;  // exchanges / collectives issued so far
    // profiling: 0 off, 1 per launch (hipExtLaunchKernel dispatch timestamps),
    // 2 one event pair around every sq_step call on the step-kernel stream
    int profiling = 0;
    std::vector<EvPair> evpool;
    size_t ev_used = 0;
    long long region_steps = 0;
    sq_perf_t perf{};
    // step-kernel launches since the last sq_perf_reset by kernel id (template
    // instance + grid, sq::phi4_kernel_id_name): sq_phi4_launch_info names the
    // dominant one, which bench.py matches against its committed PMC record
    std::map<uint64_t, long long> kstat;
};

namespace {

bool is_phi4(const sq_ctx *c) { return c->p.model == SQ_MODEL_PHI4; }

// one slab per process, ranks of a job (RCCL or peer pointers)
bool per_rank(int comm) { return comm == SQ_COMM_RCCL || comm == SQ_COMM_P2P; }

// RCCL communicators are created non-blocking (ncclConfig_t.blocking = 0) so
// that no call can hang the host: a call that returns ncclInProgress (the
// init, a group end launching in the background) is polled with
// ncclCommGetAsyncError up to a deadline (SQ_COMM_TIMEOUT_S, default 300 s);
// past it the communicator is aborted (ncclCommAbort) and the call fails
// with SQ_E_COMM instead of waiting forever on a peer that never comes.
double comm_timeout_s() {
    const char *e = getenv("SQ_COMM_TIMEOUT_S");
    const double v = e ? atof(e) : 300.0;
    return v > 0 ? v : 300.0;
}

int nccl_settle(sq_ctx *c, ncclResult_t r, const char *what);

#define SQ_NCCLW(c, expr)                                                                        \
    do {                                                                                         \
        int rc_ = nccl_settle((c), (expr), #expr);                                               \
        if (rc_ != SQ_OK) return rc_;                                                            \
    } while (0)

hipError_t wait_seq(hipStream_t s, unsigned int *word, unsigned int seq) {
    return hipStreamWaitValue32(s, word, seq, hipStreamWaitValueGte, 0xFFFFFFFFu);
}

// Collective over peer memory: our contribution into slot `rank` of every
// rank's gather buffer (parity seq & 1), a flag to each, wait for every rank's
// flag, then fold our buffer's slots in rank order (sq_p2p.hip).  Round k + 2
// reuses round k's slots: a rank issues it only after every rank's flag of
// round k + 1, which each rank writes after its fold of round k.
int p2p_allreduce(sq_ctx *c, void *d, size_t n, sq::P2pRed red, hipStream_t st) {
    const int P = c->p.nranks, r = c->p.rank;
    if (!c->p2p_ready) return fail(SQ_E_STATE, "SQ_COMM_P2P context not connected (sq_p2p_connect)");
    const size_t esz = (red == sq::P2pRed::kMaxU32 || red == sq::P2pRed::kMaxI32) ? 4 : 8;
    if (n * esz > c->coll_cap) return fail(SQ_E_ARG, "collective larger than the P2P slot");
    const unsigned int seq = ++c->coll_seq;
    const size_t base = (size_t)(seq & 1u) * (size_t)P * c->coll_cap;
    for (int q = 0; q < P; ++q)
        SQ_HIP(hipMemcpyAsync(c->peers[q].coll + base + (size_t)r * c->coll_cap, d, n * esz, hipMemcpyDeviceToDevice, st));
    for (int q = 0; q < P; ++q) SQ_HIP(hipStreamWriteValue32(st, c->peers[q].mbox + kMbColl + r, seq, 0));
    for (int q = 0; q < P; ++q) SQ_HIP(wait_seq(st, c->mbox + kMbColl + q, seq));
    SQ_HIP(sq::p2p_fold_launch(c->coll + base, P, c->coll_cap, d, n, red, st));
    return SQ_OK;
}

// All-reduce of n elements at d across the ranks of a one-slab-per-process
// context (no-op for one rank and for single-process contexts).
int rank_allreduce(sq_ctx *c, void *d, size_t n, sq::P2pRed red, hipStream_t st) {
    if (c->p.nranks <= 1 || !per_rank(c->p.comm)) return SQ_OK;
    if (c->p.comm == SQ_COMM_P2P) return p2p_allreduce(c, d, n, red, st);
    if (!c->comm) return fail(SQ_E_STATE, "no RCCL communicator");
    ncclDataType_t t = ncclFloat64;
    ncclRedOp_t op = ncclMax;
    switch (red) {
    case sq::P2pRed::kMaxU32: t = ncclUint32; break;
    case sq::P2pRed::kMaxI32: t = ncclInt32; break;
    case sq::P2pRed::kMaxU64: t = ncclUint64; break;
    case sq::P2pRed::kMaxF64: t = ncclFloat64; break;
    case sq::P2pRed::kSumF64: t = ncclFloat64; op = ncclSum; break;
    }
    SQ_NCCLW(c, ncclAllReduce(d, d, n, t, op, c->comm, st));
    return SQ_OK;
}

int nccl_settle(sq_ctx *c, ncclResult_t r, const char *what) {
    if (r == ncclInProgress && c->comm != nullptr) {
        const auto t0 = std::chrono::steady_clock::now();
        const double lim = comm_timeout_s();
        long spins = 0;
        for (;;) {
            ncclResult_t st = ncclSuccess;
            const ncclResult_t q = ncclCommGetAsyncError(c->comm, &st);
            if (q != ncclSuccess) {
                r = q;
                break;
            }
            if (st != ncclInProgress) {
                r = st;
                break;
            }
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > lim) {
                (void)ncclCommAbort(c->comm);
                c->comm = nullptr;
                return fail(SQ_E_COMM, std::string(what) + ": no completion within " + std::to_string((int)lim) +
                                           " s (SQ_COMM_TIMEOUT_S); communicator aborted");
            }
            if (++spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(50));
            else std::this_thread::yield();
        }
    }
    if (r != ncclSuccess) return fail(SQ_E_COMM, std::string(what) + ": " + ncclGetErrorString(r));
    return SQ_OK;
}

int flush_events(sq_ctx *c) {
    for (size_t i = 0; i < c->ev_used; ++i) {
        SQ_HIP(hipEventSynchronize(c->evpool[i].b));
        float ms = 0;
        SQ_HIP(hipEventElapsedTime(&ms, c->evpool[i].a, c->evpool[i].b));
        c->perf.step_kernel_ms += ms;
        c->perf.step_kernel_launches += 1;
    }
    c->perf.step_kernel_launches += c->ev_extra_steps;
    c->ev_extra_steps = 0;
    if (c->region_steps > 0) {  // region mode: one pair per sq_step call covering its steps
        c->perf.step_kernel_launches += c->region_steps - (long long)c->ev_used;
        c->region_steps = 0;
    }
    c->ev_used = 0;
    return SQ_OK;
}

int ev_take(sq_ctx *c, EvPair **out) {
    *out = nullptr;
    if (c->ev_used == c->evpool.size()) {
        if (c->evpool.size() >= 8192) {
            int rc = flush_events(c);
            if (rc) return rc;
        } else {
            EvPair e;
            SQ_HIP(hipEventCreate(&e.a));
            SQ_HIP(hipEventCreate(&e.b));
            c->evpool.push_back(e);
        }
    }
    *out = &c->evpool[c->ev_used++];
    return SQ_OK;
}

// Marker-event pair around one launch (QM1D frames; per-launch mode only).
int ev_begin(sq_ctx *c, hipStream_t s, EvPair **out) {
    *out = nullptr;
    if (c->profiling != 1) return SQ_OK;
    int rc = ev_take(c, out);
    if (rc) return rc;
    SQ_HIP(hipEventRecord((*out)->a, s));
    return SQ_OK;
}

size_t plane_floats(const sq_ctx *c) { return (size_t)c->Lx * (size_t)c->Ly; }

// Local plane 0 of buffer k (the ghost zone is the c->gpad planes on either side).
float *plane0(const sq_ctx *c, const Slab &s, int k) { return s.buf[k] + (size_t)c->gpad * plane_floats(c); }

sq::Phi4StepArgs phi4_base_args(sq_ctx *c, const Slab &s, int in_buf) {
    sq::Phi4StepArgs a{};
    a.in = s.buf[in_buf];
    a.out = s.buf[in_buf ^ 1];
    a.Lx = c->Lx;
    a.Ly = c->Ly;
    a.nz = s.nz;
    a.gz = c->gpad;
    a.zg0 = s.z0;
    a.Lzg = c->Lz;
    const float h = (float)c->dtau;
    a.h = h;
    a.m2 = (float)c->p.m2;
    a.lam6 = (float)((double)(float)c->p.lambda / 6.0);
    a.sig = (float)(sqrt(2.0 * (double)h) * c->p.C);  // sigma = C*sqrt(2 dtau) (tau_kernel.cl:112, a = 1)
    a.sigq = (float)(sqrt(2.0 * (double)h) * c->p.C * sq::kSqrt2Ln2);  // for the kernels' box_muller_q normals
    a.fin = c->field_finite ? 1 : 0;
    a.clampv = (float)c->p.clamp;
    a.k0 = (uint32_t)c->p.seed;
    a.k1 = (uint32_t)(c->p.seed >> 32);
    a.s_lo = (uint32_t)c->step;
    a.s_hi = (uint32_t)(c->step >> 32);
    a.flag = c->in_frame ? c->flag : nullptr;  // the guard flag only feeds a frame's rollback
    a.st_md = nullptr;
    a.st_a = nullptr;
    a.dcoef = (c->in_frame && c->dev_frames) ? c->ctl_cur->coef : nullptr;
    if (c->in_frame && c->st_md != nullptr) {
        const size_t k = (size_t)(c->step - c->frame_step0) * sq::kStabSlots;
        a.st_md = c->st_md + k;
        a.st_a = c->st_a + k;
    }
    if (c->tri && c->in_frame) {  // the kernel picks in / out from the controller (FrameCtl::bs/bw0/bw1)
        a.buf0 = c->tri_bufs[0];
        a.buf1 = c->tri_bufs[1];
        a.buf2 = c->tri_bufs[2];
        a.tctl = c->ctl_cur;
        a.tk = c->frame_tk++;
        // the guess: the roles every earlier frame of the batch being stable
        // gives (phi4_frames_dev keeps them); kernels that can start on it
        // check it against the controller once their first loads are out
        const int bi = a.tk == 0 ? c->spec_bs : ((a.tk & 1) ? c->spec_bw0 : c->spec_bw1);
        const int bo = a.tk == 0 ? c->spec_bw0 : ((a.tk & 1) ? c->spec_bw1 : c->spec_bw0);
        a.in = c->tri_bufs[bi];
        a.out = c->tri_bufs[bo];
        a.tspec = c->tri_spec ? 1 : 0;
    }
    return a;
}

// Update local planes of the given chunks: chunk k = [zlo + k*zstep, +zc) clipped to zhi.
int phi4_launch_range(sq_ctx *c, const Slab &s, int in_buf, hipStream_t st, int zlo, int zhi,
                      int zstep, int zc, int nzc, int periodic, bool timed) {
    if (nzc <= 0 || zhi <= zlo) return SQ_OK;
    sq::Phi4StepArgs a = phi4_base_args(c, s, in_buf);
    a.zlo = zlo;
    a.zhi = zhi;
    a.zstep = zstep;
    a.zc = zc;
    a.nzc = nzc;
    a.periodic = periodic;
    sq::phi4_fill_units(a, c->geom);
    EvPair *e = nullptr;
    if (timed && c->profiling == 1) {
        int rc = ev_take(c, &e);
        if (rc) return rc;
    }
    uint64_t kid = 0;
    SQ_HIP(sq::phi4_step_launch(a, c->geom, st, e ? e->a : nullptr, e ? e->b : nullptr, &kid));
    c->perf.kernel_launches += 1;
    c->kstat[kid] += 1;
    return SQ_OK;
}

// Planes [lo, hi) in chunks of c->zc.
int phi4_launch_span(sq_ctx *c, const Slab &s, int in_buf, hipStream_t st, int lo, int hi, bool timed) {
    if (hi <= lo) return SQ_OK;
    return phi4_launch_range(c, s, in_buf, st, lo, hi, c->zc, c->zc, (hi - lo + c->zc - 1) / c->zc, 0, timed);
}

void count_step(sq_ctx *c) {
    c->step += 1;
    c->perf.steps += 1;
    for (auto &s : c->slabs) c->perf.site_updates += (long long)s.nz * (long long)plane_floats(c);
}

constexpr int kRunUnsupported = -1000;  // phi4_tb2_range: a resident march does not apply (internal)

// Steps s and s+1 in one launch (sq_phi4.hip, phi4_tb2_kernel) on the planes
// [lo, hi) of slab s and, when lo2 < hi2, also [lo2, hi2) (a range of the same
// length): reads buffer in_buf, writes in_buf ^ 1.
int phi4_tb2_range(sq_ctx *c, const Slab &s, int in_buf, hipStream_t st, int lo, int hi, int lo2, int hi2,
                   int periodic, bool timed, int run_pairs = 0) {
    if (hi <= lo) return SQ_OK;
    const int nr = lo2 < hi2 ? 2 : 1, len = hi - lo;
    if (nr == 2 && hi2 - lo2 != len) return fail(SQ_E_STATE, "two-step launch: ranges of different lengths");
    sq::Phi4StepArgs a = phi4_base_args(c, s, in_buf);
    a.snap = c->snap_next;  // only a one-stream frame's first launch (phi4_frame)
    c->snap_next = nullptr;
    a.stamps = c->stamps_next;  // sq_phi4_block_stamps
    c->stamps_next = nullptr;
    // device frames: a folding first launch (it computes its own coefficients,
    // so it must not read the ones its block 0 writes) arms the clear of the
    // folded record set for the launch after it
    if (c->clr_armed) {
        a.clr = c->clr_next;
        c->clr_armed = false;
    }
    if (c->fold_next.cin != nullptr) {
        a.fold = c->fold_next;
        a.dcoef = nullptr;
        a.tctl = nullptr;  // it derives its buffers itself (frame_fold)
        c->fold_next = sq::FrameFoldArgs{};
        c->clr_armed = true;
    } else if (c->clr_first) {  // a batch's first frame clears the set its second frame uses
        c->clr_armed = true;
    }
    c->clr_first = false;
    // planes per block: pinned, or as many as make one round of tb_blocks
    // blocks (a ragged second round costs more than the deeper chunks), but
    // not fewer than 4 (a chunk recomputes 2 planes of the first step)
    const int nyg = c->Ly / 8, nxseg = c->Lx / 256;
    // (the slabs of a loopback decomposition run concurrently on their own streams)
    const int target = c->beside_xchg ? c->tb_blocks_xchg : c->tb_blocks;
    const int nzc_t = std::max(1, target / (nyg * nxseg * (int)c->slabs.size() * nr));
    const int zb = c->tbz_pin ? c->tbz : std::min(len, std::max(c->tb_minz, (len + nzc_t - 1) / nzc_t));
    a.zlo = lo;
    a.zhi = nr == 2 ? hi2 : hi;
    a.zstep = nr == 2 ? lo2 - lo : 0;
    a.zc = zb;
    a.zlen = len;
    a.nzr = (len + zb - 1) / zb;
    a.nzc = nr * a.nzr;
    a.periodic = periodic;
    a.nxseg = nxseg;
    a.nyg = nyg;
    a.nunits = a.nxseg * a.nyg * a.nzc;
    if (c->gate_next.on) {  // the rim ranges as thin gated chunks of this launch
        a.gate = c->gate_word;
        a.gate_seq = c->gate_seq;
        a.gate_err = c->gate_err;
        a.n_reg = a.nunits;
        a.tzc = 4;
        a.tlen = c->gate_next.tlen;
        a.tlo0 = c->gate_next.tlo0;
        a.thi0 = c->gate_next.thi0;
        a.ntz = (a.tlen + a.tzc - 1) / a.tzc;
        c->gate_next.on = false;
    }
    if (run_pairs > 0) {  // one resident launch of run_pairs pairs (the caller left no frame / stamp / stop state)
        const int pairs = run_pairs;
        if (c->profiling == 1 || c->run_flags == nullptr || c->gate_err == nullptr || !sq::phi4_tb2_run_ok(a, c->dev))
            return kRunUnsupported;  // nothing consumed: the caller falls back to one launch per pair
        sq::Tb2RunArgs r{c->run_flags, c->gate_err, c->run_base, pairs, nullptr};
        // diagnostics: SQ_DIAG_RUN_STAMPS=<file> appends each launch's per-pair
        // block stamps (Tb2RunArgs::stamps) as {npairs, nblocks, words...} u64
        const char *dpath = getenv("SQ_DIAG_RUN_STAMPS");
        const size_t nst = 2 * (size_t)pairs * a.nunits + a.nunits;
        if (dpath) SQ_HIP(hipMalloc(&r.stamps, nst * sizeof(unsigned long long)));
        uint64_t kid = 0;
        SQ_HIP(sq::phi4_tb2_run_launch(a, r, st, nullptr, nullptr, &kid));
        if (dpath) {
            std::vector<unsigned long long> h(nst + 2);
            h[0] = (unsigned long long)pairs;
            h[1] = (unsigned long long)a.nunits;
            SQ_HIP(hipStreamSynchronize(st));
            SQ_HIP(hipMemcpy(h.data() + 2, r.stamps, nst * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            SQ_HIP(hipFree(r.stamps));
            if (FILE *f = fopen(dpath, "ab")) {
                fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
                fclose(f);
            }
        }
        c->run_base += (unsigned int)pairs;
        c->perf.kernel_launches += 1;
        c->kstat[kid] += 1;
        c->perf.fused_steps += 2 * pairs;
        return SQ_OK;
    }
    EvPair *e = nullptr;
    if (timed && c->profiling == 1) {
        int rc = ev_take(c, &e);
        if (rc) return rc;
        c->ev_extra_steps += 1;
    }
    if (a.stamps != nullptr) {  // every block of the grid stamps (a gated launch adds its rim chunks)
        const int grid_n = a.nunits + (a.gate != nullptr ? a.nxseg * a.nyg * 2 * a.ntz : 0);
        if (grid_n > c->stamps_cap) return fail(SQ_E_STATE, "block stamps: more blocks than stamp slots");
        c->stamps_blocks = grid_n;
    }
    hipEvent_t stop = c->stop_next;
    c->stop_next = nullptr;
    uint64_t kid = 0;
    if (c->kstage_next && stop == nullptr && sq::phi4_tb2_stage_ok(a, c->gz)) {
        const sq::Tb2StageArgs g{c->kstage_slot, c->gz, c->kstage_ctr};
        SQ_HIP(sq::phi4_tb2_stage_launch(a, g, st, e ? e->a : nullptr, e ? e->b : nullptr, &kid));
        c->kstage_n += (unsigned int)a.nunits;
        c->kstage_issued = true;
    } else if (e == nullptr && stop != nullptr) {
        SQ_HIP(sq::phi4_tb2_launch(a, st, nullptr, stop, &kid));
        c->stop_used = true;
    } else {
        SQ_HIP(sq::phi4_tb2_launch(a, st, e ? e->a : nullptr, e ? e->b : nullptr, &kid));
    }
    c->perf.kernel_launches += 1;
    c->kstat[kid] += 1;
    c->perf.fused_steps += 2;
    return SQ_OK;
}

// Single slab covering the lattice: steps s and s+1 in one launch; the
// output lands in the other buffer.
int phi4_tb2_pair(sq_ctx *c) {
    Slab &s = c->slabs[0];
    int rc = phi4_tb2_range(c, s, c->cur, s.sA, 0, s.nz, 0, 0, 1, true);
    if (rc) return rc;
    c->cur ^= 1;
    count_step(c);
    count_step(c);
    return SQ_OK;
}

// Single slab, SQ_TB2_RUN=1: `pairs` pairs as one resident launch
// (sq_phi4_run.hip); the output lands in buffer cur ^ (pairs & 1).
int phi4_tb2_run_pairs(sq_ctx *c, int pairs) {
    Slab &s = c->slabs[0];
    int rc = phi4_tb2_range(c, s, c->cur, s.sA, 0, s.nz, 0, 0, 1, true, pairs);
    if (rc) return rc;
    c->cur ^= pairs & 1;
    for (int i = 0; i < 2 * pairs; ++i) count_step(c);
    return SQ_OK;
}

// Single slab covering the lattice: one launch per step, z wraps in-kernel.
int phi4_periodic_step(sq_ctx *c) {
    Slab &s = c->slabs[0];
    const int nzc = (s.nz + c->zc - 1) / c->zc;
    int rc = phi4_launch_range(c, s, c->cur, s.sA, 0, s.nz, c->zc, c->zc, nzc, 1, true);
    if (rc) return rc;
    c->cur ^= 1;
    count_step(c);
    return SQ_OK;
}

// The schedule of a deep-halo block of g <= G steps on a slab of nz planes
// with a ghost zone of G planes.  Each op names its stream:
// A (interior) or B (exchange, and the rims when rims_b).
//   EXCHANGE     stream B, after the previous block's EDGES_DONE: G edge planes
//                of the block's input field to both z-neighbours, their ghosts in.
//   Step k updates the shrinking extended range [-(g-1-k), nz+g-1-k),
//   recomputing ghost-zone sites.  With fuse2 (two steps per launch) and g >= 3
//   every step runs in pairs, and the first K pairs (kc = core pairs) are split:
//     PAIR 2j core  stream A, step 2j+1 on [2j+2, nz-2j-2), j < K: reads no ghost
//                   (step s is valid without ghosts on [s+1, nz-s-1)), so the
//                   core pairs overlap the exchange;
//     PAIR 2j rim   step 2j+1 on [-(g-2-2j), 2j+2) u [nz-2j-2, nz+g-2-2j) (two
//                   ranges, one launch), either on stream A after WAIT_EXCHANGE
//                   (short exchanges: no cross-stream hop before the next pair),
//                   or, rims_b, on stream B right behind the exchange, rim j > 0
//                   after core j-1 (SIGNAL A / WAIT B on slot j-1), stream A
//                   continuing once they are in (SIGNAL B / WAIT A on kRimSlot):
//                   long exchanges then overlap the cores with the rims too;
//     K = 0: no split -- stream A waits for the exchange and the first pair
//                   covers the whole range (an exchange shorter than the
//                   previous block's last middle pair is then hidden for free);
//     PAIR s        stream A, the remaining pairs on step s+1's whole range;
//     the last pair (or single step) computes its edge planes [0, G) u
//     [nz-G, nz) first and marks EDGES_DONE, so the NEXT block's exchange
//     overlaps this step's middle as well as the next cores (when the core
//     pairs reach the last step, EDGES_DONE follows the rims);
//   without fuse2 (or g < 3) step 0 is a single-step core [1, nz-1) and rim
//   [-(g-1), 1) u [nz-1, nz+g-1) (K = 0: one span), the later steps single
//   launches on A.
// Ghost-zone sites are recomputed redundantly; the counter-based noise makes
// them bit-identical to their owner's, so the result equals the monolithic run.
// Buffers: a launch group (the ops of one first step) reads the buffer of the
// step before it and writes the other (phi4_block counts the groups); a core
// pair running ahead of the rims only writes [2j+2, nz-2j-2), which no earlier
// rim pair reads ([.., 2i+4) u [nz-2i-4, ..) for i < j).
constexpr int kPlanSlots = 16;            // events per slab the plan's SIGNAL / WAIT ops name
constexpr int kRimSlot = kPlanSlots - 1;  // the rims of the block are done
constexpr int kA = 0, kB = 1;

std::vector<sq_block_op> block_plan(int nz, int G, int g, bool fuse2, bool edge_first, int kc, bool rims_b) {
    std::vector<sq_block_op> ops;
    auto add = [&](int kind, int step, int lo, int hi, int lo2, int hi2, int stream) {
        ops.push_back(sq_block_op{kind, step, lo, hi, lo2, hi2, stream});
    };
    const int rs = rims_b ? kB : kA;  // the rims' stream
    auto rims_done = [&]() {
        if (!rims_b) return;
        add(SQ_OP_SIGNAL, 0, kRimSlot, 0, 0, 0, kB);
        add(SQ_OP_WAIT, 0, kRimSlot, 0, 0, 0, kA);
    };
    const bool split_edges = edge_first && nz > 2 * G;
    add(SQ_OP_EXCHANGE, 0, 0, 0, 0, 0, kB);
    int st;
    bool edges = false;
    if (kc <= 0) {  // no core/rim split
        add(SQ_OP_WAIT_EXCHANGE, 0, 0, 0, 0, 0, kA);
        st = 0;
    } else if (fuse2 && g >= 3) {
        // core pairs: at least one, at most the pairs of the block, and only
        // while the core is not empty
        int K = std::max(1, std::min(std::min(kc, g / 2), kRimSlot));
        while (K > 1 && nz <= 4 * K) --K;
        // core pair 1 writes step 3 into the buffer the exchange sends its edge
        // planes from: with K >= 2 the exchange sends a staged copy of them, and
        // core pair 1 waits only for that copy
        if (K >= 2) ops[0].lo = 1;
        int nc = 0;
        for (int j = 0; j < K && nz > 4 * j + 4; ++j, ++nc) {
            if (j == 1) add(SQ_OP_WAIT_STAGED, 0, 0, 0, 0, 0, kA);
            add(SQ_OP_PAIR, 2 * j, 2 * j + 2, nz - 2 * j - 2, 0, 0, kA);
            if (rims_b && j + 1 < K) add(SQ_OP_SIGNAL, 2 * j, j, 0, 0, 0, kA);
        }
        add(SQ_OP_WAIT_EXCHANGE, 0, 0, 0, 0, 0, rs);
        for (int j = 0; j < K; ++j) {
            if (rims_b && j > 0 && j - 1 < nc) add(SQ_OP_WAIT, 2 * j, j - 1, 0, 0, 0, kB);
            const int lo_a = -(g - 2 - 2 * j), hi_a = 2 * j + 2, lo_b = nz - 2 * j - 2, hi_b = nz + g - 2 - 2 * j;
            if (hi_a >= lo_b)  // rims meet (no core): one span
                add(SQ_OP_PAIR, 2 * j, lo_a, hi_b, 0, 0, rs);
            else
                add(SQ_OP_PAIR, 2 * j, lo_a, hi_a, lo_b, hi_b, rs);
        }
        rims_done();
        st = 2 * K;
    } else {
        if (nz - 1 > 1) add(SQ_OP_STEP, 0, 1, nz - 1, 0, 0, kA);
        add(SQ_OP_WAIT_EXCHANGE, 0, 0, 0, 0, 0, rs);
        const int lo_a = -(g - 1), hi_a = 1, lo_b = nz - 1, hi_b = nz + g - 1;
        if (hi_a >= lo_b)  // rims meet (nz <= 2): one span
            add(SQ_OP_STEP, 0, lo_a, hi_b, 0, 0, rs);
        else
            add(SQ_OP_STEP, 0, lo_a, hi_a, lo_b, hi_b, rs);
        rims_done();
        st = 1;
    }
    while (st < g) {
        const bool pair = fuse2 && st + 1 <= g - 1;
        const int last = pair ? st + 1 : st;  // the step this op group completes
        const int kind = pair ? SQ_OP_PAIR : SQ_OP_STEP;
        if (last == g - 1 && split_edges) {
            add(kind, st, 0, G, nz - G, nz, kA);
            add(SQ_OP_EDGES_DONE, st, 0, 0, 0, 0, kA);
            add(kind, st, G, nz - G, 0, 0, kA);
            edges = true;
        } else {
            const int e = g - 1 - last;  // ghost planes the completed step still updates on either side
            add(kind, st, -e, nz + e, 0, 0, kA);
        }
        st = last + 1;
    }
    if (!edges) add(SQ_OP_EDGES_DONE, g - 1, 0, 0, 0, 0, kA);
    return ops;
}

// The index of a plan's [PAIR core (A), WAIT_EXCHANGE (A), PAIR rim (A, two
// equal ranges)] of one step -- the K = 1, rims-on-A block start -- or -1.
int gate_pattern(const std::vector<sq_block_op> &ops) {
    for (size_t i = 0; i + 2 < ops.size(); ++i) {
        const sq_block_op &a = ops[i], &w = ops[i + 1], &r = ops[i + 2];
        if (a.kind == SQ_OP_PAIR && a.stream == kA && a.lo2 >= a.hi2 && w.kind == SQ_OP_WAIT_EXCHANGE &&
            w.stream == kA && r.kind == SQ_OP_PAIR && r.stream == kA && r.step == a.step && r.lo2 < r.hi2 &&
            r.hi - r.lo == r.hi2 - r.lo2)
            return (int)i;
        if (a.kind == SQ_OP_WAIT_EXCHANGE) return -1;  // the pattern is the block's start or absent
    }
    return -1;
}

// P2P: does the block's last pair write the next exchange's staging slot
// (SQ_P2P_KSTAGE pins it; by default with the exchange on stream A, whose
// stream order replaces the count wait on stream B)
bool kstage_on(const sq_ctx *c) { return c->kstage_env >= 0 ? c->kstage_env != 0 : c->xchg_on_a; }

// Deep-halo block of g <= gz steps on every slab: executes block_plan.
int phi4_block(sq_ctx *c, int g) {
    const size_t plane = plane_floats(c);
    const int ns = (int)c->slabs.size(), G = c->gz;
    const size_t gbytes = (size_t)G * plane * sizeof(float);
    const int cur = c->cur;
    const unsigned long long step0 = c->step;
    std::vector<std::vector<sq_block_op>> plans;
    for (const Slab &s : c->slabs) plans.push_back(block_plan(s.nz, G, g, c->tbz > 0, c->edge_first, c->core_pairs, c->rims_b));
    // 1. exchange (stream B), for every slab before any slab waits for one;
    //    staged (EXCHANGE op lo = 1): the edge planes are copied aside first and
    //    sent from the copy, so the block's core pairs may overwrite them early
    std::vector<const float *> src_lo(ns), src_hi(ns);
    for (int i = 0; i < ns; ++i) {
        Slab &s = c->slabs[i];
        const float *p0 = plane0(c, s, cur);
        src_lo[i] = p0;
        src_hi[i] = p0 + (size_t)(s.nz - G) * plane;
    }
    // P2P with the staging slot already written by the previous block's last
    // pair (kstage): no EDGES_DONE wait and no staging copy on stream B, the
    // hand-shake waits for that pair's block count instead
    // SQ_XCHG_ON_A: the whole exchange on stream A, in order (no events)
    const bool on_a = c->xchg_on_a && ns == 1 &&
                      ((c->p.comm == SQ_COMM_P2P && c->p2p_kernel_handshake) || c->p.comm == SQ_COMM_RCCL);
    // the staged slot is used on stream A (stream order) or, when pinned
    // (SQ_P2P_KSTAGE=1), on stream B behind a wait for the pair's block count
    const bool kst = c->p.comm == SQ_COMM_P2P && c->kstage_pending && ns == 1 && c->p2p_kernel_handshake &&
                     (on_a || c->kstage_env == 1);
    c->kstage_pending = false;
    for (int i = 0; i < ns; ++i) {
        Slab &s = c->slabs[i];
        if (kst || on_a) continue;
        if (c->evE_stale) {  // the last pair before is complete in stream-A order: record it now
            SQ_HIP(hipEventRecord(s.evE, s.sA));
            c->evE_stale = false;
        }
        if (!c->diag_no_ewait) SQ_HIP(hipStreamWaitEvent(s.sB, s.evE, 0));
        if (c->p.comm == SQ_COMM_LOOPBACK) {  // we write the neighbours' ghosts: wait for them too
            SQ_HIP(hipStreamWaitEvent(s.sB, c->slabs[(i + ns - 1) % ns].evE, 0));
            SQ_HIP(hipStreamWaitEvent(s.sB, c->slabs[(i + 1) % ns].evE, 0));
        }
    }
    const bool p2p = c->p.comm == SQ_COMM_P2P;
    if (p2p && !c->p2p_ready) return fail(SQ_E_STATE, "SQ_COMM_P2P context not connected (sq_p2p_connect)");
    // P2P: this exchange's staged slot (two, by parity).  Reusing slot e & 1 at
    // exchange e needs both neighbours to have pulled our exchange e - 2; each
    // wrote its staged flag of exchange e - 1 behind that pull (stream order on
    // its exchange stream), and our exchange e - 1 waited for both flags before
    // anything of exchange e is issued behind it -- no acknowledgement words
    // and no waits on them per exchange (sq_destroy still drains with them).
    const size_t slot_stride = 2 * (size_t)c->gpad * plane;
    const size_t slot = p2p ? (size_t)((c->xchg_seq + 1) & 1u) * slot_stride : 0;
    for (int i = 0; i < ns; ++i) {
        Slab &s = c->slabs[i];
        const bool staged_wait = plans[i][0].lo == 1;  // core pair 1 waits for the copy (WAIT_STAGED)
        if (kst) continue;                              // the slot is written already
        if (!staged_wait && !p2p) continue;            // P2P: the neighbours always read the staged copy
        if (!s.stage) return fail(SQ_E_STATE, "staged exchange without a staging buffer");
        float *stg = s.stage + slot;
        // both ranges in one two-range copy launch (a 2-D hipMemcpy ran as a
        // rect-copy kernel of 23 us against 2 x 6 for two linear copies,
        // profiles/r06/c6/tr_p2p)
        SQ_HIP(sq::p2p_copy2_launch(stg, src_lo[i], stg + (size_t)G * plane, src_hi[i], (size_t)G * plane,
                                    on_a ? s.sA : s.sB));
        if (staged_wait && !on_a) SQ_HIP(hipEventRecord(s.evS, s.sB));
        src_lo[i] = stg;
        src_hi[i] = stg + (size_t)G * plane;
    }
    if (c->p.comm == SQ_COMM_LOOPBACK) {
        for (int i = 0; i < ns; ++i) {
            Slab &s = c->slabs[i];
            Slab &dn = c->slabs[(i + ns - 1) % ns];
            Slab &up = c->slabs[(i + 1) % ns];
            // my bottom G planes -> lower neighbour's upper ghosts [nz_dn, nz_dn+G)
            SQ_HIP(hipMemcpyAsync(plane0(c, dn, cur) + (size_t)dn.nz * plane, src_lo[i], gbytes,
                                  hipMemcpyDeviceToDevice, s.sB));
            // my top G planes -> upper neighbour's lower ghosts [-G, 0)
            SQ_HIP(hipMemcpyAsync(plane0(c, up, cur) - (size_t)G * plane, src_hi[i], gbytes,
                                  hipMemcpyDeviceToDevice, s.sB));
            SQ_HIP(hipEventRecord(s.evC, s.sB));
            c->perf.halo_bytes += 2.0 * (double)gbytes;
        }
    } else if (p2p) {
        // peer pointers: tell both neighbours our staged copy is complete, pull
        // theirs into our ghosts (lower ghosts <- the lower neighbour's top G
        // planes, upper ghosts <- the upper neighbour's bottom G planes), tell
        // them we are done reading.  Flag writes run after everything before
        // them on the stream; P = 2 (both neighbours one peer) and P = 1 (our
        // own copy) need no special case.
        Slab &s = c->slabs[0];
        float *p0 = plane0(c, s, cur);
        const int P = c->p.nranks, r = c->p.rank;
        const int up = (r + 1) % P, dn = (r + P - 1) % P;
        const unsigned int e = ++c->xchg_seq;
        const size_t n = (size_t)G * plane;
        hipStream_t xs = on_a ? s.sA : s.sB;
        if (c->p2p_kernel_handshake) {
            // one wave: "staged e" to both neighbours, then wait for both of theirs
            // (kstage on stream B: first for the last pair's block count; on
            // stream A that pair is complete in stream order)
            SQ_HIP(sq::p2p_handshake_launch(c->peers[up].mbox + kMbStagedFromDn, c->peers[dn].mbox + kMbStagedFromUp,
                                            c->mbox + kMbStagedFromDn, c->mbox + kMbStagedFromUp, e,
                                            kHandshakePolls, c->gate_err, xs,
                                            (kst && !on_a) ? c->kstage_ctr : nullptr, c->kstage_n));
        } else {  // stream-ordered flag writes and waits (SQ_P2P_STREAMOPS=1)
            SQ_HIP(hipStreamWriteValue32(s.sB, c->peers[up].mbox + kMbStagedFromDn, e, 0));
            SQ_HIP(hipStreamWriteValue32(s.sB, c->peers[dn].mbox + kMbStagedFromUp, e, 0));
            SQ_HIP(wait_seq(s.sB, c->mbox + kMbStagedFromDn, e));
            SQ_HIP(wait_seq(s.sB, c->mbox + kMbStagedFromUp, e));
        }
        // both neighbours' staged copies, pulled by one launch
        SQ_HIP(sq::p2p_copy2_launch(p0 - n, c->peers[dn].stage + slot + n, p0 + (size_t)s.nz * plane,
                                    c->peers[up].stage + slot, n, xs));
        if (!on_a) SQ_HIP(hipEventRecord(s.evC, s.sB));
        c->perf.halo_bytes += 2.0 * (double)gbytes;
    } else {  // RCCL: one slab per process; this send/recv order pairs correctly for P = 2 too
        Slab &s = c->slabs[0];
        float *p0 = plane0(c, s, cur);
        const int P = c->p.nranks, r = c->p.rank;
        const int up = (r + 1) % P, dn = (r + P - 1) % P;
        const size_t n = (size_t)G * plane;
        hipStream_t xs = on_a ? s.sA : s.sB;
        SQ_NCCLW(c, ncclGroupStart());
        SQ_NCCLW(c, ncclSend(src_hi[0], n, ncclFloat32, up, c->comm, xs));
        SQ_NCCLW(c, ncclSend(src_lo[0], n, ncclFloat32, dn, c->comm, xs));
        SQ_NCCLW(c, ncclRecv(p0 - n, n, ncclFloat32, dn, c->comm, xs));
        SQ_NCCLW(c, ncclRecv(p0 + (size_t)s.nz * plane, n, ncclFloat32, up, c->comm, xs));
        SQ_NCCLW(c, ncclGroupEnd());
        if (!on_a) SQ_HIP(hipEventRecord(s.evC, s.sB));
        c->perf.halo_bytes += 2.0 * (double)gbytes;
    }
    // gated pair 0: the exchange's completion as a device word the rim chunks poll
    const bool gated = c->slab_gate && c->gate_word != nullptr && ns == 1 && per_rank(c->p.comm) &&
                       gate_pattern(plans[0]) >= 0;
    if (gated) SQ_HIP(hipStreamWriteValue32(c->slabs[0].sB, c->gate_word, ++c->gate_seq, 0));
    // 2. the rest of the schedule, slab by slab (each slab has its own streams;
    //    slabs of a loopback decomposition may differ in nz, hence in schedule)
    int out_buf = cur;
    for (int i = 0; i < ns; ++i) {
        Slab &s = c->slabs[i];
        const std::vector<sq_block_op> &ops = plans[i];
        // launch groups: the ops of one first step read the buffer written by
        // the group before (every group flips the parity once)
        std::vector<int> starts;
        for (const sq_block_op &op : ops)
            if (op.kind == SQ_OP_STEP || op.kind == SQ_OP_PAIR) starts.push_back(op.step);
        std::sort(starts.begin(), starts.end());
        starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
        std::vector<char> timed(starts.size(), 0);
        // stream-A launches issued while an exchange may run: from the block's
        // exchange to its WAIT_EXCHANGE (the core pairs), and after EDGES_DONE
        // (the middle pair, beside the next block's exchange)
        bool xchg_live = true;
        for (size_t oi = 0; oi < ops.size(); ++oi) {
            const sq_block_op &op = ops[oi];
            int rc = SQ_OK;
            hipStream_t st = op.stream == kB ? s.sB : s.sA;
            c->beside_xchg = xchg_live && op.stream != kB && c->p.comm != SQ_COMM_NONE;
            // gated pair 0: [PAIR core (A), WAIT_EXCHANGE (A), PAIR rim (A, two ranges)] of the
            // same step as one launch whose rim chunks wait in-kernel for the exchange
            if (gated && (int)oi == gate_pattern(ops)) {
                const sq_block_op &rim = ops[oi + 2];
                const size_t gi = (size_t)(std::lower_bound(starts.begin(), starts.end(), op.step) - starts.begin());
                const int in = cur ^ (int)(gi & 1);
                const bool first = !timed[gi];
                timed[gi] = 1;
                c->step = step0 + (unsigned long long)op.step;
                c->gate_next = {true, rim.lo, rim.lo2, rim.hi - rim.lo};
                rc = phi4_tb2_range(c, s, in, st, op.lo, op.hi, 0, 0, 0, first);
                c->gate_next.on = false;
                if (rc) return rc;
                xchg_live = false;
                oi += 2;
                continue;
            }
            if (op.kind == SQ_OP_STEP || op.kind == SQ_OP_PAIR) {
                const size_t gi = (size_t)(std::lower_bound(starts.begin(), starts.end(), op.step) - starts.begin());
                const int in = cur ^ (int)(gi & 1);
                const bool first = !timed[gi];  // it carries the group's timing
                timed[gi] = 1;
                c->step = step0 + (unsigned long long)op.step;
                c->stop_used = false;
                if (c->edges_stopev && op.kind == SQ_OP_PAIR && oi + 1 < ops.size() &&
                    ops[oi + 1].kind == SQ_OP_EDGES_DONE && ops[oi + 1].stream == op.stream)
                    c->stop_next = s.evE;  // phi4_tb2_range binds it to the launch (stop_used)
                // P2P kstage: the block's last pair (the whole slab, right before
                // EDGES_DONE) also writes the next exchange's staging slot
                c->kstage_issued = false;
                c->kstage_next = p2p && kstage_on(c) && ns == 1 && c->p2p_kernel_handshake && !c->in_frame &&
                                 s.stage != nullptr && op.kind == SQ_OP_PAIR && op.stream == kA && op.lo == 0 &&
                                 op.hi == s.nz && op.lo2 >= op.hi2 && oi + 1 < ops.size() &&
                                 ops[oi + 1].kind == SQ_OP_EDGES_DONE && ops[oi + 1].stream == kA;
                if (c->kstage_next) c->kstage_slot = s.stage + (size_t)((c->xchg_seq + 1) & 1u) * slot_stride;
                if (op.kind == SQ_OP_PAIR)
                    rc = phi4_tb2_range(c, s, in, st, op.lo, op.hi, op.lo2, op.hi2, 0, first);
                else if (op.lo2 < op.hi2)  // two equal ranges in one launch: two chunks zstep apart
                    rc = phi4_launch_range(c, s, in, st, op.lo, op.hi2, op.lo2 - op.lo, op.hi - op.lo, 2, 0, first);
                else
                    rc = phi4_launch_span(c, s, in, st, op.lo, op.hi, first);
                c->kstage_next = false;
                c->stop_next = nullptr;  // an empty range launched nothing: EDGES_DONE records
            } else if (op.kind == SQ_OP_WAIT_EXCHANGE) {
                if (op.stream != kB) xchg_live = false;
                // (SQ_DIAG_NO_XWAIT=1, timing diagnostics only: no wait, the rims race the exchange)
                if (op.stream != kB && !c->diag_no_xwait && !on_a) SQ_HIP(hipStreamWaitEvent(st, s.evC, 0));
                if (c->p.comm == SQ_COMM_LOOPBACK) {
                    SQ_HIP(hipStreamWaitEvent(st, c->slabs[(i + ns - 1) % ns].evC, 0));
                    SQ_HIP(hipStreamWaitEvent(st, c->slabs[(i + 1) % ns].evC, 0));
                }
            } else if (op.kind == SQ_OP_WAIT_STAGED) {
                if (!kst) SQ_HIP(hipStreamWaitEvent(st, s.evS, 0));  // kstage: no copy reads the field
            } else if (op.kind == SQ_OP_EDGES_DONE) {
                xchg_live = true;
                if (c->kstage_issued) {  // the next exchange waits for the pair's block count instead
                    c->kstage_pending = true;
                    c->evE_stale = true;
                    c->kstage_issued = false;
                } else if (on_a) {  // the next exchange follows on stream A in order
                    c->evE_stale = true;
                } else if (!c->stop_used && !c->diag_no_ewait) {
                    SQ_HIP(hipEventRecord(s.evE, st));  // else bound to the pair before
                    c->evE_stale = false;
                }
                c->stop_used = false;
            } else if (op.kind == SQ_OP_SIGNAL || op.kind == SQ_OP_WAIT) {
                if (op.lo < 0 || op.lo >= kPlanSlots) return fail(SQ_E_STATE, "block op event slot out of range");
                if (op.kind == SQ_OP_SIGNAL)
                    SQ_HIP(hipEventRecord(s.evk[op.lo], st));
                else
                    SQ_HIP(hipStreamWaitEvent(st, s.evk[op.lo], 0));
            } else if (op.kind != SQ_OP_EXCHANGE) {  // the exchange was issued above for every slab
                return fail(SQ_E_STATE, "unknown block op");
            }
            if (rc) return rc;
        }
        out_buf = cur ^ (int)(starts.size() & 1);
        c->beside_xchg = false;
    }
    c->step = step0;
    for (int k = 0; k < g; ++k) count_step(c);
    c->cur = out_buf;
    return SQ_OK;
}

int phi4_join(sq_ctx *c);

// Gated rim chunks that gave up waiting for their exchange (tb_gate_wait) store
// nothing, so the field is corrupt from then on: the error is sticky on the
// context.  read_device: the caller has joined the streams, read the device
// word (otherwise only the sticky flag, no synchronisation).
int gate_check(sq_ctx *c, bool read_device) {
    if (!c->gate_failed && read_device && c->gate_err) {
        int e = 0;
        SQ_HIP(hipMemcpy(&e, c->gate_err, sizeof e, hipMemcpyDeviceToHost));
        if (e) c->gate_failed = true;
    }
    if (c->gate_failed)
        return fail(SQ_E_COMM, "slab exchange: gated rim chunks timed out waiting for the exchange, a P2P "
                               "hand-shake gave up waiting for a neighbour, or a resident march's block gave up "
                               "waiting for its neighbours (planes are stale; the field is corrupt until it is "
                               "uploaded or initialised again)");
    return SQ_OK;
}

// a new field replaces every plane: the timed-out chunks no longer matter
// (a resident march's epochs start over too: a timed-out launch left them uneven)
int gate_reset(sq_ctx *c) {
    if (c->gate_err) SQ_HIP(hipMemset(c->gate_err, 0, sizeof(int)));
    if (c->run_flags) SQ_HIP(hipMemset(c->run_flags, 0, (size_t)c->run_nflags * sizeof(unsigned int)));
    c->kstage_pending = false;  // the staged edges are the old field's
    c->run_base = 0;
    c->gate_failed = false;
    return SQ_OK;
}

// Ghost depth by measurement (slab paths): G in {4, 8, 16} (<= the allocated
// depth), each timed over two blocks after one warm-up block on the interior
// stream; across ranks the per-candidate times are max-reduced (RCCL or peer
// memory) so every rank picks the same G (exchange sizes must match).  With
// fused pairs the deepest zone is also tried without a core/rim split (K = 0)
// and with K = 2, 4 core pairs, rims on A or on the exchange stream.  The
// trial steps are ordinary steps: the field is the same for any schedule
// (DESIGN.md §8).
int phi4_autotune(sq_ctx *c, int &n) {
    struct Cand {
        int g, k;
        bool rb, ef, a;
    };
    std::vector<Cand> cand;
    const bool ef = c->edge_first, a0 = c->xchg_on_a;
    for (int g : {4, 8, 16})
        if (g <= c->gpad) cand.push_back({g, c->core_pairs, c->rims_b, ef, a0});
    if (cand.empty()) cand.push_back({c->gpad, c->core_pairs, c->rims_b, ef, a0});
    const int gd = cand.back().g;
    if (c->tbz > 0 && c->k_auto && !a0) {
        cand.push_back({gd, 0, false, ef, false});
        for (bool rb : {false, true})
            for (int k : {2, 4})
                if (k <= gd / 2) cand.push_back({gd, k, rb, ef, false});
    }
    // the exchange in order on stream A (no overlap, no cross-stream hop):
    // cheaper when the transfer is short, so timed like the rest
    if (c->a_auto && !a0) cand.push_back({gd, 0, false, ef, true});
    // the edges-first split of the block's last pair buys the next exchange a
    // longer window at the price of a split launch and an event bubble: worth
    // it when the exchange is long (a real link), not on one GPU (19.3 vs 19.9
    // us/step at 256^3, profiles/r03/s2/slab_ef/), so both are timed
    if (c->ef_auto) cand.push_back({gd, c->core_pairs, c->rims_b, !ef, a0});
    if (cand.size() > 16) cand.resize(16);  // dtune holds 16 times
    int need = 0;
    for (const Cand &k : cand) need += 3 * k.g;
    if (n < need) return SQ_OK;  // too few steps requested: try again on a later call
    hipEvent_t t0, t1;
    SQ_HIP(hipEventCreate(&t0));
    SQ_HIP(hipEventCreate(&t1));
    std::vector<double> ms(cand.size());
    for (size_t k = 0; k < cand.size(); ++k) {
        const int g = cand[k].g;
        c->gz = g;
        c->core_pairs = cand[k].k;
        c->rims_b = cand[k].rb;
        c->edge_first = cand[k].ef;
        c->xchg_on_a = cand[k].a;
        int rc = phi4_block(c, g);
        if (!rc) rc = phi4_join(c);
        if (rc) return rc;
        SQ_HIP(hipEventRecord(t0, c->slabs[0].sA));
        for (int b = 0; b < 2 && !rc; ++b) rc = phi4_block(c, g);
        if (rc) return rc;
        SQ_HIP(hipEventRecord(t1, c->slabs[0].sA));
        SQ_HIP(hipEventSynchronize(t1));
        rc = phi4_join(c);
        if (rc) return rc;
        float e = 0;
        SQ_HIP(hipEventElapsedTime(&e, t0, t1));
        ms[k] = (double)e / (2.0 * g);
        n -= 3 * g;
    }
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    if (per_rank(c->p.comm) && c->p.nranks > 1) {
        hipStream_t st = c->slabs[0].sA;
        SQ_HIP(hipMemcpyAsync(c->dtune, ms.data(), sizeof(double) * ms.size(), hipMemcpyHostToDevice, st));
        int rc = rank_allreduce(c, c->dtune, ms.size(), sq::P2pRed::kMaxF64, st);
        if (rc) return rc;
        SQ_HIP(hipMemcpyAsync(ms.data(), c->dtune, sizeof(double) * ms.size(), hipMemcpyDeviceToHost, st));
        SQ_HIP(hipStreamSynchronize(st));
    }
    const Cand best = cand[(size_t)sq_phi4_pick_ghost(ms.data(), (int)ms.size())];
    c->gz = best.g;
    c->core_pairs = best.k;
    c->rims_b = best.rb;
    c->edge_first = best.ef;
    c->xchg_on_a = best.a;
    c->g_tuned = true;
    return SQ_OK;
}

int phi4_steps_impl(sq_ctx *c, int n);

// Multi-rank: one rank's unguarded upload makes the others' ghost planes
// unguarded too, so after a local change of field_finite the ranks agree on it
// (max-reduce of "not finite") before the next step call or frame uses it.
int fin_agree(sq_ctx *c) {
    if (!c->fin_sync) return SQ_OK;
    c->fin_sync = false;
    if (!per_rank(c->p.comm) || c->p.nranks <= 1) return SQ_OK;
    hipStream_t st = c->slabs[0].sA;
    double v = c->field_finite ? 0.0 : 1.0;
    SQ_HIP(hipMemcpyAsync(c->dtune, &v, sizeof v, hipMemcpyHostToDevice, st));
    int rc = rank_allreduce(c, c->dtune, 1, sq::P2pRed::kMaxF64, st);
    if (rc) return rc;
    SQ_HIP(hipMemcpyAsync(&v, c->dtune, sizeof v, hipMemcpyDeviceToHost, st));
    SQ_HIP(hipStreamSynchronize(st));
    c->field_finite = v == 0.0;
    return SQ_OK;
}

// Every launch of the call reads c->field_finite as its `fin`; once one step
// has run, every plane (ghost zones included: they are exchanged copies) has
// been through the guard.
int phi4_steps(sq_ctx *c, int n) {
    const int rc = phi4_steps_impl(c, n);
    if (rc == SQ_OK && n > 0) c->field_finite = true;
    return rc;
}

int phi4_steps_impl(sq_ctx *c, int n) {
    if (c->p.comm == SQ_COMM_NONE) {
        if (c->tb_run && c->tbz > 0 && n >= 4 && !c->in_frame && c->snap_next == nullptr &&
            c->stamps_next == nullptr && c->stop_next == nullptr && c->fold_next.cin == nullptr && !c->clr_armed &&
            !c->clr_first) {
            int rc = gate_check(c, false);  // no march on a field a timed-out launch left corrupt
            if (rc) return rc;
            // SQ_TB2_RUN_MAXP (experiments): at most this many pairs per launch
            const char *mp = getenv("SQ_TB2_RUN_MAXP");
            const int maxp = mp ? std::max(1, atoi(mp)) : INT_MAX;
            while (n >= 2) {
                const int np = std::min(n / 2, maxp);
                rc = phi4_tb2_run_pairs(c, np);
                if (rc == kRunUnsupported) {
                    c->tb_run = false;  // this context's shape: one launch per pair from now on
                    break;
                }
                if (rc) return rc;
                n -= 2 * np;
            }
        }
        for (; c->tbz > 0 && n >= 2; n -= 2) {
            int rc = phi4_tb2_pair(c);
            if (rc) return rc;
        }
        for (int i = 0; i < n; ++i) {
            int rc = phi4_periodic_step(c);
            if (rc) return rc;
        }
        return SQ_OK;
    }
    if (c->p.comm == SQ_COMM_P2P && !c->p2p_ready)
        return fail(SQ_E_STATE, "SQ_COMM_P2P context not connected (sq_p2p_connect)");
    {
        int rc = fin_agree(c);
        if (rc) return rc;
    }
    if (c->g_auto && !c->g_tuned) {
        int rc = phi4_autotune(c, n);
        if (rc) return rc;
    }
    // balanced blocks: the fewest blocks of <= gz steps, of near-equal length
    // (even where fused pairs can use it), so a call of n steps pays
    // ceil(n / gz) exchanges and the least redundant ghost-zone work: 20 steps
    // at gz = 16 run as 10 + 10, not 16 + 4
    while (n > 0) {
        const int nb = (n + c->gz - 1) / c->gz;
        int g = (n + nb - 1) / nb;
        if (c->tbz > 0 && (g & 1) && g < c->gz) ++g;
        g = std::min(g, n);
        int rc = phi4_block(c, g);
        if (rc) return rc;
        n -= g;
    }
    return SQ_OK;
}

int phi4_join(sq_ctx *c) {
    for (auto &s : c->slabs) {
        SQ_HIP(hipStreamSynchronize(s.sA));
        SQ_HIP(hipStreamSynchronize(s.sB));
    }
    return SQ_OK;
}

// Before an observable's kernels on stream A: one slab without an exchange
// puts every step on stream A, so stream order suffices; otherwise join.
int observe_join(sq_ctx *c) {
    if (c->slabs.size() == 1 && c->p.comm == SQ_COMM_NONE) return SQ_OK;
    return phi4_join(c);
}

// Point st_md / st_a / flag at record set k of frame_rec (st_md | st_a | flag).
void use_rec_set(sq_ctx *c, int k) {
    const size_t nrec = (size_t)sq::kStabSlots * (size_t)std::max(c->p.loops, 0);
    char *b = static_cast<char *>(c->frame_rec) + (size_t)k * c->frame_bytes;
    c->rec_set = k;
    c->frame_cur = b;
    c->st_md = nrec > 0 ? reinterpret_cast<unsigned long long *>(b) : nullptr;
    c->st_a = nrec > 0 ? reinterpret_cast<unsigned int *>(b + nrec * sizeof(unsigned long long)) : nullptr;
    c->flag = reinterpret_cast<int *>(b + nrec * (sizeof(unsigned long long) + sizeof(unsigned int)));
}

int create_phi4(sq_ctx *c) {
    const sq_params &p = c->p;
    if (p.dims[0] <= 0 || p.dims[1] <= 0 || p.dims[2] <= 0 || p.dims[0] > (1 << 20) ||
        p.dims[1] > (1 << 20))
        return fail(SQ_E_ARG, "PHI4 dims must be positive");
    c->Lx = (int)p.dims[0];
    c->Ly = (int)p.dims[1];
    c->Lz = p.dims[2];
    if (!sq::phi4_geometry(c->Lx, c->Ly, &c->geom))
        return fail(SQ_E_ARG, "PHI4 needs Lx in {8,16,32,64,128,256} or a multiple of 256, and Ly a "
                              "multiple of the wave's row count");
    // Philox counter word 0 holds the global site quad (sites/4): < 2^32 quads,
    // i.e. up to 1.7e10 sites (68 GB of fp32 field, a quarter of one MI355X).
    if ((long long)c->Lx * c->Ly * c->Lz / 4 >= (1ll << 32))
        return fail(SQ_E_ARG, "lattice exceeds 2^34 sites (Philox counter layout)");
    if ((long long)c->Lx * c->Ly * 4 >= (1ll << 31))
        return fail(SQ_E_ARG, "plane exceeds 2 GiB (32-bit buffer offsets)");
    if (c->Lz >= (1ll << 31)) return fail(SQ_E_ARG, "Lz must be < 2^31 (32-bit plane indices)");
    {   // the guard's fast path (Phi4StepArgs::fin) needs every update of a field
        // inside [-clamp, clamp] to be finite or +-inf, never NaN: bound the drift
        const double cl = p.clamp, h = p.deltatau;
        const double drift = 12.0 * cl + std::fabs(p.m2) * cl + std::fabs(p.lambda) / 6.0 * cl * cl * cl;
        // (float)clamp squared finite too: with lambda = 0, clamp^2 = inf would make
        // fma(lam/6, phi^2, m2) = 0 * inf = NaN at |phi| = clamp
        const float clf = (float)cl;
        if (!std::isfinite(cl) || !(cl > 0) || !std::isfinite(p.m2) || !std::isfinite(p.lambda) ||
            !std::isfinite(p.C) || !std::isfinite(clf * clf) ||
            !(h * drift + cl + 16.0 * sqrt(2.0 * h) * std::fabs(p.C) < 1e30))
            return fail(SQ_E_ARG, "PHI4 parameters must be finite with clamp^2 finite in fp32 and "
                                  "dtau * drift(clamp) < 1e30");
    }
    if (const char *e = getenv("SQ_ROWS")) {  // tuning override of the rows per lane
        const int r = atoi(e), rs = 64 / c->geom.qx;
        if ((r == 1 || r == 2 || r == 4) && c->Ly % r == 0)
            c->geom = sq::Phi4Geom{c->geom.qx, r, rs * r, c->geom.pf, c->geom.v};
    }
    if (const char *e = getenv("SQ_VSEG"))  // tuning override: float4 segments per lane
        if (atoi(e) == 1 || (atoi(e) == 2 && c->geom.qx == 64 && c->Lx % 512 == 0)) c->geom.v = atoi(e);
    {   // very large per-device fields: non-temporal output stores (mode 4) beat the
        // sc0 sc1 stores of mode 7 at 1024^3 (1575 vs 1598 us per step), not at
        // 512^3 (193.5 vs 190.8 us), profiles/r01/sweep*_sc1.log
        const long long nz_dev = per_rank(p.comm) ? (c->Lz + p.nranks - 1) / std::max(1, p.nranks) : c->Lz;
        const double field_bytes = 4.0 * c->Lx * c->Ly * (double)nz_dev;  // this device's share
        if (c->geom.pf == 7 && 2.0 * field_bytes > 2.0 * (1 << 30)) c->geom.pf = 4;
    }
    if (const char *e = getenv("SQ_PREFETCH")) {  // tuning override of the store / arithmetic mode
        const int m = atoi(e);
        c->geom.pf = (m == 3 || m == 4 || m == 7) && c->geom.qx == 64 ? m : 1;
    }
    int nslab = 1;
    long long zfirst = 0;
    std::vector<long long> zs;
    if (p.comm == SQ_COMM_NONE) {
        zs = {0, c->Lz};
    } else if (p.comm == SQ_COMM_LOOPBACK) {
        nslab = p.nslabs;
        if (nslab < 1 || nslab > c->Lz) return fail(SQ_E_ARG, "nslabs must be in [1, Lz]");
        for (int i = 0; i <= nslab; ++i) zs.push_back(c->Lz * i / nslab);
    } else if (per_rank(p.comm)) {
        if (p.nranks < 1 || p.rank < 0 || p.rank >= p.nranks || p.nranks > c->Lz)
            return fail(SQ_E_ARG, "bad rank/nranks for the slab decomposition");
        if (p.comm == SQ_COMM_P2P && p.nranks > kP2pMaxRanks) return fail(SQ_E_ARG, "SQ_COMM_P2P: too many ranks");
        zfirst = c->Lz * p.rank / p.nranks;
        zs = {zfirst, c->Lz * (p.rank + 1) / p.nranks};
    } else {
        return fail(SQ_E_ARG, "unknown comm");
    }
    // ghost-zone depth: one exchange of gz planes per gz steps;
    // bounded by the thinnest slab so a ghost zone never spans two neighbours
    if (p.comm != SQ_COMM_NONE) {
        long long nz_min = c->Lz;
        for (int i = 0; i < nslab; ++i) nz_min = std::min(nz_min, zs[i + 1] - zs[i]);
        if (per_rank(p.comm)) nz_min = c->Lz / p.nranks;  // identical on every rank
        // measured (profiles/r01/ghost_sweep.log, 256^3 slab, RCCL): 51.8 / 37.0 /
        // 30.4 / 26.9 / 25.6 us per step at G = 1 / 2 / 4 / 8 / 16: a fixed
        // ~28 us per exchange amortised over G steps against (G-1)/nz of
        // redundant ghost-zone planes.  G = nz/16 keeps the redundancy <= ~6 %.
        int g = (int)std::min(16ll, std::max(1ll, nz_min / 16));
        // multi-rank RCCL runs measure G in {4, 8, 16} on the real link (the
        // fixed cost and bandwidth of an xGMI exchange are not those of the
        // one-GPU self-exchange these defaults were measured on); SQ_GHOST
        // pins G, SQ_GHOST_AUTO=1 forces the trials on any slab path
        c->g_auto = per_rank(p.comm) && p.nranks > 1 && nz_min >= 64;
        if (const char *e = getenv("SQ_GHOST_AUTO")) c->g_auto = atoi(e) != 0;
        if (c->g_auto) g = (int)std::min(16ll, nz_min / 2);
        if (const char *e = getenv("SQ_GHOST")) {
            g = std::max(1, atoi(e));
            c->g_auto = false;
        }
        c->gz = (int)std::max(1ll, std::min((long long)g, nz_min));
        c->gpad = c->gz;
        SQ_HIP(hipMalloc(&c->dtune, 16 * sizeof(double)));
    }
    const size_t plane = plane_floats(c);
    for (int i = 0; i < nslab; ++i) {
        c->slabs.emplace_back();  // owned by the context from here on: sq_destroy frees a partial set-up
        Slab &s = c->slabs.back();
        s.z0 = zs[i];
        s.nz = (int)(zs[i + 1] - zs[i]);
        if (s.nz < 1) return fail(SQ_E_ARG, "empty slab");
        const size_t bytes = (size_t)(s.nz + 2 * c->gpad) * plane * sizeof(float);
        for (int k = 0; k < 2; ++k) {
            SQ_HIP(hipMalloc(&s.buf[k], bytes));
            SQ_HIP(hipMemset(s.buf[k], 0, bytes));
        }
        SQ_HIP(hipStreamCreateWithFlags(&s.sA, hipStreamNonBlocking));
        // halo stream at the highest priority: its RCCL and boundary-plane
        // kernels must not queue behind the interior kernel's waves
        // (SQ_XCHG_PRIO=0: the default priority, an experiment)
        int prio_lo = 0, prio_hi = 0;
        SQ_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        const char *xp = getenv("SQ_XCHG_PRIO");
        SQ_HIP(hipStreamCreateWithPriority(&s.sB, hipStreamNonBlocking, (xp && atoi(xp) == 0) ? prio_lo : prio_hi));
        SQ_HIP(hipEventCreateWithFlags(&s.evC, hipEventDisableTiming));
        SQ_HIP(hipEventCreateWithFlags(&s.evE, hipEventDisableTiming));
        SQ_HIP(hipEventCreateWithFlags(&s.evS, hipEventDisableTiming));
        s.evk.assign(kPlanSlots, nullptr);
        for (hipEvent_t &e : s.evk) SQ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        // the staged copy of the 2 G edge planes; P2P keeps two, by exchange parity
        // (phi4_block: a neighbour's staged flag of exchange e-1 then implies it
        // has read our copy of exchange e-2, so no per-exchange acknowledgement)
        if (p.comm != SQ_COMM_NONE)
            SQ_HIP(hipMalloc(&s.stage, stage_slots(p.comm) * 2 * (size_t)c->gpad * plane * sizeof(float)));
        SQ_HIP(hipEventRecord(s.evC, s.sB));
        SQ_HIP(hipEventRecord(s.evE, s.sA));
    }
    {
        const size_t nrec = (size_t)sq::kStabSlots * (size_t)std::max(p.loops, 0);
        c->frame_bytes = nrec * (sizeof(unsigned long long) + sizeof(unsigned int)) + 2 * sizeof(int);
        SQ_HIP(hipMalloc(&c->frame_rec, 2 * c->frame_bytes));
        SQ_HIP(hipMemset(c->frame_rec, 0, 2 * c->frame_bytes));
        SQ_HIP(hipHostMalloc(&c->frame_host, c->frame_bytes, hipHostMallocDefault));
        use_rec_set(c, 0);
    }
    SQ_HIP(hipMalloc(&c->dacc, 2 * sizeof(double)));
    SQ_HIP(hipMalloc(&c->dpart, 4 * sizeof(double) * sq::kMomBlocks));
    SQ_HIP(hipMalloc(&c->dmax, 2 * sizeof(unsigned int)));
    if (p.comm == SQ_COMM_RCCL) {
        ncclUniqueId id;
        static_assert(sizeof(id.internal) <= 128, "ncclUniqueId size");
        memcpy(id.internal, p.comm_id, sizeof(id.internal));
        // non-blocking (bounded bring-up, nccl_settle) with the halo kernels'
        // CU footprint capped: the exchange's send/recv kernel shares the CUs
        // with the core pair it overlaps, so it gets
        // SQ_RCCL_MAX_CTAS blocks (default kRcclMaxCtas; 0 = RCCL's choice)
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        const char *nb = getenv("SQ_RCCL_BLOCKING");
        cfg.blocking = (nb && atoi(nb) != 0) ? 1 : 0;
        const char *mc = getenv("SQ_RCCL_MAX_CTAS");
        const int max_ctas = mc ? atoi(mc) : kRcclMaxCtas;
        if (max_ctas > 0) {
            cfg.maxCTAs = max_ctas;
            cfg.minCTAs = 1;
        }
        ncclResult_t r = ncclCommInitRankConfig(&c->comm, p.nranks, id, p.rank, &cfg);
        if (r != ncclSuccess && r != ncclInProgress) {
            c->comm = nullptr;
            return fail(SQ_E_COMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
        }
        int rc = nccl_settle(c, r, "ncclCommInitRankConfig");
        if (rc) return rc;
    }
    if (per_rank(p.comm)) {  // the gated pair 0's word (fine-grained: written by stream B, polled by kernels)
        SQ_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&c->gate_word), 64, hipDeviceMallocFinegrained));
        SQ_HIP(hipMemset(c->gate_word, 0, 64));
        SQ_HIP(hipMalloc(&c->gate_err, sizeof(int)));
        SQ_HIP(hipMemset(c->gate_err, 0, sizeof(int)));
        const char *e = getenv("SQ_SLAB_GATE");
        c->slab_gate = e ? atoi(e) != 0 : false;  // off: its spinning rim blocks hold the CU slots the exchange needs
    }
    if (p.comm == SQ_COMM_P2P) {
        // the last pair's block count (phi4_tb2_stage_kernel; monotonic, never reset)
        SQ_HIP(hipMalloc(&c->kstage_ctr, 64));
        SQ_HIP(hipMemset(c->kstage_ctr, 0, 64));
        const char *ks = getenv("SQ_P2P_KSTAGE");
        if (ks) c->kstage_env = atoi(ks) != 0 ? 1 : 0;
    }
    if (p.comm == SQ_COMM_P2P || p.comm == SQ_COMM_RCCL) {
        // one rank's self-exchange moves no bytes over a link: in order on the
        // interior stream it costs less than the two cross-stream hops that
        // overlap it (RCCL 1.117 vs 1.148, P2P with the staged last pair 1.078
        // vs 1.142 x the single slab, profiles/r06/c25); ranks on a link get
        // it as one more candidate of the timed pick (phi4_autotune)
        if (const char *xa = getenv("SQ_XCHG_ON_A")) {
            c->xchg_on_a = atoi(xa) != 0;
            c->a_auto = false;
        }
    }
    if (p.comm == SQ_COMM_P2P) {  // mailbox and collective slots; peers mapped by sq_p2p_connect
        // fine-grained device memory: the words are written by the peers'
        // command processors (hipStreamWriteValue32) and copy engines from
        // other devices over xGMI and polled here by hipStreamWaitValue32 /
        // read by the fold kernel -- in coarse-grained memory a reader may keep
        // serving a stale cached line (round 3 recorded such a hang on a flag)
        SQ_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&c->mbox), kMbWords * sizeof(unsigned int),
                                     hipDeviceMallocFinegrained));
        SQ_HIP(hipMemset(c->mbox, 0, kMbWords * sizeof(unsigned int)));
        const size_t need = std::max({(size_t)8 * (size_t)c->Lz, (size_t)8 * sq::kStabSlots * (size_t)std::max(1, p.loops),
                                      (size_t)256});
        c->coll_cap = (need + 255) / 256 * 256;
        SQ_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&c->coll), 2 * (size_t)p.nranks * c->coll_cap,
                                     hipDeviceMallocFinegrained));
        c->peers.assign(p.nranks, Peer{});
        c->peers[p.rank] = Peer{c->slabs[0].stage, c->mbox, c->coll, false};
        c->p2p_ready = p.nranks == 1;  // one rank: its own buffers, nothing to map
    }
    // z chunk per wave: long enough to amortise the chunk-edge planes, short
    // enough to give >= ~8 waves per CU.
    const long long rows = (long long)(c->Lx / (4 * c->geom.qx * c->geom.v)) * (c->Ly / c->geom.wy);
    const int nz_max = c->slabs[0].nz;
    // measured optima (profiles/r01/sweep*): zc = 4 for one-segment rows (256^3),
    // zc = 8 when rows span several 256-site segments (512^3); big lattices
    // lengthen the chunk while >= 32 waves per SIMD remain, which cuts the
    // chunk-edge plane re-reads (1024^3: zc 32, 1760 -> 1711 us,
    // profiles/r01/sweep1024_zc.log)
    int zc = c->Lx > 256 ? 8 : 4;
    while (zc > 1 && rows * ((nz_max + zc - 1) / zc) < 2048) zc /= 2;
    while (zc < 32 && rows * ((nz_max + 2 * zc - 1) / (2 * zc)) >= 32768) zc *= 2;
    if (const char *e = getenv("SQ_ZCHUNK")) zc = std::max(1, atoi(e));
    // edges-first by default except for one rank's self-exchange, which is short
    // enough to fit beside the next core pair: RCCL (off 19.2-19.4 vs 19.9
    // us/step, round 3) and, since round 6's shorter P2P chain, P2P (off 1.180
    // vs 1.201 x the single slab, profiles/r06/c7/slab_ab.log); the timed pick
    // of multi-rank contexts tries both
    c->edge_first = !((c->p.comm == SQ_COMM_RCCL || c->p.comm == SQ_COMM_P2P) && c->p.nranks == 1);
    if (const char *e = getenv("SQ_EDGE_FIRST")) {
        c->edge_first = atoi(e) != 0;
        c->ef_auto = false;
    }
    if (const char *e = getenv("SQ_CORE_PAIRS")) {
        c->core_pairs = std::max(0, atoi(e));
        c->k_auto = false;
    }
    if (const char *e = getenv("SQ_RIMS_B")) {
        c->rims_b = atoi(e) != 0;
        c->k_auto = false;
    }
    // one rank's self-exchange: in order on stream A unless pinned otherwise
    // (SQ_XCHG_ON_A, or a pinned core / rim split)
    if ((p.comm == SQ_COMM_P2P || p.comm == SQ_COMM_RCCL) && p.nranks == 1 && c->a_auto && c->k_auto)
        c->xchg_on_a = true;
    if (c->xchg_on_a) {  // the exchange runs between two pairs on stream A: nothing to split around it
        c->core_pairs = 0;
        c->rims_b = false;
        c->k_auto = false;
    }
    c->zc = zc;
    // Two steps per launch on 256-wide lattices (SQ_FUSE2=0: off; SQ_FUSE2_Z:
    // pin the output planes per block), single slab and deep-halo slabs alike.
    // 256^3: 19.5 vs 22.0 us per step on the same box; one round of two
    // blocks per CU (z = 16 at 256^3) measured best of z = 8/11/12/16/22/32
    // (profiles/r01/fuse2_sweep.log), so every launch picks the depth that
    // makes one such round.
    // Loopback decompositions (several slabs on one GPU, a rehearsal mode)
    // keep one step per launch unless SQ_FUSE2=1: there the concurrent slab
    // launches ran slower fused (29.1 vs 25.4 us per step, 2 slabs of 128
    // planes), while one RCCL slab of 256 planes gains (24.2 vs 26.0,
    // profiles/r01/fuse2_slabs.log).
    // Rows of several 256-site segments fuse through the x-halo wave: measured
    // (profiles/r02/sweep_tb2_*.log, us per step, fused vs one step per launch)
    // 512^3 153 vs 200 (with the guard's fast path; 197 before it), 1024 x
    // 1024 x 128 194 vs 225, 1024^3 1537 vs 1678.
    const char *fe = getenv("SQ_FUSE2");
    const bool fuse = fe ? atoi(fe) != 0 : p.comm != SQ_COMM_LOOPBACK;
    if (fuse && sq::phi4_tb2_supported(c->Lx, c->Ly) && (p.comm != SQ_COMM_NONE || c->slabs[0].nz >= 2)) {
        c->tbz = 16;
        if (const char *z = getenv("SQ_TB2_MINZ")) c->tb_minz = std::max(1, atoi(z));
        if (const char *z = getenv("SQ_FUSE2_Z")) {
            c->tbz = std::max(1, atoi(z));
            c->tbz_pin = true;
        }
        int ncu = 0;
        SQ_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->dev));
        // two blocks per CU (256-wide rows: 65 VGPRs, 10 waves; wider rows: 11 waves at <= 80)
        c->tb_blocks = 2 * std::max(1, ncu);
        if (const char *e = getenv("SQ_TB2_BLOCKS_PER_CU")) c->tb_blocks = std::max(1, atoi(e)) * std::max(1, ncu);
        // 96 slots left to the exchange's kernels: RCCL self-exchange, 256^3, G = 16
        // (profiles/r04/slab/): 512 blocks 19.36 / 19.54 us/step, 480 19.49 / 19.47,
        // 448 19.02 / 19.32, 416 18.89 / 19.24; SQ_XCHG_BLOCKS pins the target
        c->tb_blocks_xchg = std::max(1, c->tb_blocks - 96);
        if (const char *e = getenv("SQ_XCHG_BLOCKS")) c->tb_blocks_xchg = std::max(1, atoi(e));
        if (const char *e = getenv("SQ_EDGES_STOPEV")) c->edges_stopev = atoi(e) != 0;
        if (const char *e = getenv("SQ_DIAG_NO_XWAIT")) c->diag_no_xwait = atoi(e) != 0;
        if (const char *e = getenv("SQ_DIAG_NO_EWAIT")) c->diag_no_ewait = atoi(e) != 0;
        if (const char *e = getenv("SQ_P2P_STREAMOPS")) c->p2p_kernel_handshake = atoi(e) == 0;
        const char *rn = getenv("SQ_TB2_RUN");
        if (rn && atoi(rn) != 0 && p.comm == SQ_COMM_NONE && c->slabs.size() == 1) {
            // one epoch word per block: at most Ly / 8 y-bands x nz / 2 chunks (>= 2 planes each)
            c->run_nflags = (c->Ly / 8) * std::max(1, c->slabs[0].nz / 2);
            SQ_HIP(hipMalloc(&c->run_flags, (size_t)c->run_nflags * sizeof(unsigned int)));
            SQ_HIP(hipMemset(c->run_flags, 0, (size_t)c->run_nflags * sizeof(unsigned int)));
            if (c->gate_err == nullptr) {
                SQ_HIP(hipMalloc(&c->gate_err, sizeof(int)));
                SQ_HIP(hipMemset(c->gate_err, 0, sizeof(int)));
            }
            c->tb_run = true;
        }
    }
    SQ_HIP(hipDeviceSynchronize());  // the set-up memsets ran on the null stream
    return SQ_OK;
}

int create_qm1d(sq_ctx *c) {
    const sq_params &p = c->p;
    if (p.dims[0] < 2 || p.dims[0] > (1 << 30)) return fail(SQ_E_ARG, "QM1D needs N >= 2");
    c->N = (int)p.dims[0];
    if (sq::qm1d_sites_per_thread(c->N) == 0)
        return fail(SQ_E_ARG, "QM1D supports 2 <= N <= 65536 (one work-group per frame)");
    if (p.pot != 0 && p.pot != 3) return fail(SQ_E_ARG, "potID must be 0 or 3 (tau_kernel.cl:215-246)");
    if (!(p.deltat > 0)) return fail(SQ_E_ARG, "deltat must be > 0");
    if (p.loops < 1) return fail(SQ_E_ARG, "loops must be >= 1");
    const size_t bytes = sizeof(double) * (size_t)c->N;
    for (int k = 0; k < 2; ++k) {
        SQ_HIP(hipMalloc(&c->qf[k], bytes));
        SQ_HIP(hipMalloc(&c->qx[k], bytes));
        SQ_HIP(hipMalloc(&c->qxx0[k], bytes));
        SQ_HIP(hipMemset(c->qf[k], 0, bytes));
        SQ_HIP(hipMemset(c->qx[k], 0, bytes));
        SQ_HIP(hipMemset(c->qxx0[k], 0, bytes));
    }
    if (c->N > sq::kQm1dRegMaxN)  // global-memory variant: f ping-pong + scan scratch
        for (int k = 0; k < 3; ++k)  // xs, ds: + the grid kernel's block maxima and scan words
            SQ_HIP(hipMalloc(&c->qscr[k], k == 0 ? bytes : bytes + sizeof(double) * sq::kQm1dGridAux));
    SQ_HIP(hipMalloc(&c->qst, sizeof(sq::Qm1dState)));
    SQ_HIP(hipStreamCreateWithFlags(&c->qstream, hipStreamNonBlocking));
    SQ_HIP(hipDeviceSynchronize());  // the set-up memsets ran on the null stream
    return SQ_OK;
}

// Capacity of the serial-order buffers for one full launch.
int gs_reserve(sq_ctx *c) {
    const long long calls = (long long)(c->N + 1) * c->p.loops;
    const long long hist = (long long)c->N * c->p.loops;
    if (calls > c->g_calls) {
        (void)hipFree(c->g_xi);
        (void)hipFree(c->g_w1);
        (void)hipFree(c->g_w2);
        (void)hipFree(c->g_seeds);
        c->g_xi = nullptr;
        c->g_w1 = c->g_w2 = nullptr;
        c->g_seeds = nullptr;
        c->g_calls = 0;
        SQ_HIP(hipMalloc(&c->g_xi, sizeof(double) * calls));
        SQ_HIP(hipMalloc(&c->g_w1, sizeof(uint32_t) * calls));
        SQ_HIP(hipMalloc(&c->g_w2, sizeof(uint32_t) * calls));
        SQ_HIP(hipMalloc(&c->g_seeds, sizeof(unsigned long long) * calls));
        c->g_calls = calls;
    }
    if (c->g_lcg_scr == nullptr) SQ_HIP(hipMalloc(&c->g_lcg_scr, sizeof(unsigned long long) * sq::kLcgScratch));
    if (hist > c->g_hist) {
        (void)hipFree(c->g_hist_buf);
        c->g_hist_buf = nullptr;
        c->g_hist = 0;
        SQ_HIP(hipMalloc(&c->g_hist_buf, sizeof(double) * hist));
        c->g_hist = hist;
    }
    if (c->p.loops > c->g_loops) {
        (void)hipFree(c->g_om);
        (void)hipFree(c->g_xc);
        (void)hipFree(c->g_cand);
        (void)hipFree(c->g_flags);
        c->g_om = c->g_xc = nullptr;
        c->g_cand = nullptr;
        c->g_flags = nullptr;
        c->g_loops = 0;
        SQ_HIP(hipMalloc(&c->g_om, sizeof(double) * (c->p.loops + 1)));
        SQ_HIP(hipMalloc(&c->g_xc, sizeof(double) * 2 * (c->N + 2) * (size_t)c->p.loops));
        SQ_HIP(hipMalloc(&c->g_cand, sq::qm1d_gs_cand_bytes(c->p.loops)));
        SQ_HIP(hipMalloc(&c->g_flags, sizeof(int) * (size_t)c->p.loops));
        SQ_HIP(hipMemset(c->g_flags, 0, sizeof(int) * (size_t)c->p.loops));
        c->gs_tag = 0;
        c->g_loops = c->p.loops;
    }
    if (!c->g_st) SQ_HIP(hipMalloc(&c->g_st, sizeof(sq::Qm1dGsState)));
    return SQ_OK;
}

// One launch of time_dev in the reference's serial order (sq_qm1d_gs.hip);
// host bookkeeping as qm1d_frame, plus the shared seed: it advances by the
// calls the launch made, whether or not the frame was stable (tauhost.c never
// rolls it back).
int qm1d_gs_frame(sq_ctx *c, int *stable) {
    int rc = gs_reserve(c);
    if (rc) return rc;
    const long long calls = (long long)(c->N + 1) * c->p.loops;
    const bool injected = c->inject_pending;
    c->inject_pending = false;
    EvPair *e = nullptr;
    rc = ev_begin(c, c->qstream, &e);
    if (rc) return rc;
    if (!injected)
        SQ_HIP(sq::qm1d_gs_lcg_launch(c->lcg_seed, c->N, calls, c->g_w1, c->g_w2, c->g_seeds, c->g_xi,
                                      c->g_lcg_scr, c->qstream));
    sq::Qm1dGsArgs a{};
    const int k = c->qcur;
    a.f0 = c->qf[k];
    a.x0 = c->qx[k];
    a.xx00 = c->qxx0[k];
    a.nf = c->qf[k ^ 1];
    a.nx = c->qx[k ^ 1];
    a.nxx0 = c->qxx0[k ^ 1];
    a.nfp = c->g_nfp;
    a.xi = c->g_xi;
    a.om = c->g_om;
    a.xc = c->g_xc;
    a.cand = c->g_cand;
    a.flags = c->g_flags;
    c->gs_tag = c->gs_tag == 0x7fffffff ? 1 : c->gs_tag + 1;
    a.tag = c->gs_tag;
    a.hist = c->g_hist_buf;
    a.st = c->g_st;
    a.N = c->N;
    a.pot = c->p.pot;
    a.loops = c->p.loops;
    a.runs = (int)c->runs;
    a.a = c->p.deltat;
    const float fa = (float)c->p.deltat;
    a.a2 = (double)(fa * fa);
    a.h = c->dtau;
    a.sig = c->p.C * (double)sqrtf((float)(2. * c->dtau / c->p.deltat));
    a.sigw = c->p.C * (double)sqrtf((float)(2. * c->dtau));
    a.kconst = host_intconst(c->p.pot);
    sq::Qm1dGsState st{};
    st.omega_in = c->omega;
    st.lrgEl = c->lrgEl;
    st.lrgVl = c->lrgVl;
    SQ_HIP(hipMemcpyAsync(c->g_st, &st, sizeof st, hipMemcpyHostToDevice, c->qstream));
    SQ_HIP(sq::qm1d_gs_frame_launch(a, c->qstream));
    if (e) SQ_HIP(hipEventRecord(e->b, c->qstream));
    SQ_HIP(hipMemcpyAsync(&st, c->g_st, sizeof st, hipMemcpyDeviceToHost, c->qstream));
    SQ_HIP(hipStreamSynchronize(c->qstream));
    if (st.sync_error) return fail(SQ_E_HIP, "serial frame: the scan timed out waiting for the sweep");
    c->consumed = (unsigned long long)st.consumed;
    if (!injected && st.consumed > 0)
        SQ_HIP(hipMemcpy(&c->lcg_seed, c->g_seeds + (st.consumed - 1), sizeof(unsigned long long),
                         hipMemcpyDeviceToHost));
    c->step += (unsigned long long)c->p.loops;
    c->lrgEl = st.lrgEl;
    c->lrgVl = st.lrgVl;
    c->perf.steps += st.steps_done;
    c->perf.site_updates += (long long)st.steps_done * c->N;
    *stable = st.stable;
    if (st.stable == 1) {  // tauhost.c:506-532
        c->qcur ^= 1;
        c->omega = st.omega_out;
        c->runs += c->p.loops;
    }
    return SQ_OK;
}

int qm1d_frame(sq_ctx *c, int *stable) {
    if (c->order == SQ_ORDER_SERIAL) return qm1d_gs_frame(c, stable);
    sq::Qm1dArgs a{};
    const int k = c->qcur;
    a.f = c->qf[k];
    a.x = c->qx[k];
    a.xx0 = c->qxx0[k];
    a.nf = c->qf[k ^ 1];
    a.nx = c->qx[k ^ 1];
    a.nxx0 = c->qxx0[k ^ 1];
    a.fs = c->qscr[0];
    a.xs = c->qscr[1];
    a.ds = c->qscr[2];
    a.st = c->qst;
    a.N = c->N;
    a.pot = c->p.pot;
    a.loops = c->p.loops;
    a.runs = (int)c->runs;
    a.a = c->p.deltat;
    const float fa = (float)c->p.deltat;
    a.a2 = (double)(fa * fa);
    a.h = c->dtau;
    a.sig = c->p.C * (double)sqrtf((float)(2. * c->dtau / c->p.deltat));
    a.sigw = c->p.C * (double)sqrtf((float)(2. * c->dtau));
    a.kconst = host_intconst(c->p.pot);
    a.k0 = (uint32_t)c->p.seed;
    a.k1 = (uint32_t)(c->p.seed >> 32);
    a.tick = c->step;
    const bool tables = c->N <= sq::kQm1dRegMaxN;
    if (tables) {  // the field-independent work of the frame, grid-wide ahead of the chain (qm1d_prep_launch)
        const size_t L = (size_t)c->p.loops, nq4 = (size_t)((c->N + 3) & ~3);
        if (!c->qom) {  // all tables as one unit: a failed allocation leaves none behind
            const size_t bxi = sizeof(float) * L * nq4;
            const size_t btcl = c->p.pot == 3 ? sizeof(float) * L * (size_t)(c->N + 2) : 0;
            const size_t bdd = c->p.pot == 3 ? sizeof(double) * L * (size_t)c->N : 0;
            if (bxi + btcl + bdd > sq::kQm1dTableCap)
                return fail(SQ_E_ARG, "QM1D frame tables (loops x N) exceed the device-memory cap "
                                      "(sq::kQm1dTableCap); use fewer loops per frame");
            double *om = nullptr, *dd = nullptr;
            float *xi = nullptr, *tcl = nullptr;
            hipError_t e = hipMalloc(&om, sizeof(double) * (L + 1));
            if (e == hipSuccess) e = hipMalloc(&xi, bxi);
            if (e == hipSuccess && btcl) e = hipMalloc(&tcl, btcl);
            if (e == hipSuccess && bdd) e = hipMalloc(&dd, bdd);
            if (e != hipSuccess) {
                (void)hipFree(om);
                (void)hipFree(xi);
                (void)hipFree(tcl);
                (void)hipFree(dd);
                return fail(SQ_E_HIP, std::string("QM1D frame tables: hipMalloc: ") + hipGetErrorString(e));
            }
            c->qom = om;
            c->qxi = xi;
            c->qtcl = tcl;
            c->qdd = dd;
        }
        a.om = c->qom;
        a.xi = c->qxi;
        a.tcl = c->qtcl;
        a.dd = c->qdd;
    }
    sq::Qm1dState st{};
    st.omega_in = c->omega;
    st.lrgEl = c->lrgEl;
    st.lrgVl = c->lrgVl;
    SQ_HIP(hipMemcpyAsync(c->qst, &st, sizeof st, hipMemcpyHostToDevice, c->qstream));
    // diagnostics (SQ_QM1D_STAMPS=<path>, grid kernel): per-block phase stamps of
    // the frame's first 64 steps, appended to <path> as text (block step t0..t4)
    const char *dpath = getenv("SQ_QM1D_STAMPS");
    const size_t ndbg = (size_t)sq::kQm1dStampBlocks * 64 * 5;  // the kernel stamps no block past these
    struct DbgFree {  // every return path below frees the stamp buffer
        unsigned long long *&p;
        ~DbgFree() {
            if (p) (void)hipFree(p);
        }
    } dbg_free{a.dbg};
    if (dpath && c->N > sq::kQm1dRegMaxN) {
        SQ_HIP(hipMalloc(&a.dbg, ndbg * sizeof(unsigned long long)));
        SQ_HIP(hipMemsetAsync(a.dbg, 0, ndbg * sizeof(unsigned long long), c->qstream));
    }
    EvPair *e = nullptr;
    int rc = ev_begin(c, c->qstream, &e);
    if (rc) return rc;
    if (tables) SQ_HIP(sq::qm1d_prep_launch(a, c->qstream));
    SQ_HIP(sq::qm1d_frame_launch(a, c->qstream));
    if (e) SQ_HIP(hipEventRecord(e->b, c->qstream));
    SQ_HIP(hipMemcpyAsync(&st, c->qst, sizeof st, hipMemcpyDeviceToHost, c->qstream));
    SQ_HIP(hipStreamSynchronize(c->qstream));
    if (a.dbg) {
        std::vector<unsigned long long> h(ndbg);
        SQ_HIP(hipMemcpy(h.data(), a.dbg, ndbg * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE *fp = fopen(dpath, "a")) {
            for (size_t q = 0; q < ndbg / 5; ++q)
                if (h[5 * q])
                    fprintf(fp, "%zu %zu %llu %llu %llu %llu %llu\n", q / 64, q % 64, h[5 * q], h[5 * q + 1],
                            h[5 * q + 2], h[5 * q + 3], h[5 * q + 4]);
            fclose(fp);
        }
    }
    if (st.sync_error)  // qm1d_frame_grid: a grid barrier gave up; nothing of the frame is adopted
        return fail(SQ_E_HIP, "QM1D grid barrier timeout: a block of qm1d_frame_grid never arrived "
                              "(the frame is void, the state is the frame start)");
    c->step += (unsigned long long)c->p.loops;
    c->lrgEl = st.lrgEl;
    c->lrgVl = st.lrgVl;
    c->perf.steps += st.steps_done;
    c->perf.site_updates += (long long)st.steps_done * c->N;
    *stable = st.stable;
    if (st.stable == 1) {  // tauhost.c:506-532
        c->qcur ^= 1;
        c->omega = st.omega_out;
        c->runs += c->p.loops;
    }
    return SQ_OK;
}

void adapt(sq_ctx *c, int stable) {  // tauhost.c:523-529,537-541
    if (!c->p.adapt_dtau) return;
    if (stable == 1) {
        if (c->stab_cnt > 10) {
            c->stab_cnt = 0;
            c->dtau /= 0.950;
        }
        c->stab_cnt++;
    } else {
        c->dtau *= 0.950;
        c->stab_cnt = 0;
    }
}

// max phi and max |phi| over the whole lattice (all slabs, all ranks).
int phi4_field_max(sq_ctx *c, float *mx_phi, float *mx_abs) {
    unsigned int m[2] = {0, 0};
    for (auto &s : c->slabs) {
        unsigned int t[2];
        SQ_HIP(sq::phi4_moments_launch(plane0(c, s, c->cur), (long long)s.nz * (long long)plane_floats(c), c->dacc,
                                       c->dmax, c->dpart, s.sA));
        int rc = rank_allreduce(c, c->dmax, 2, sq::P2pRed::kMaxU32, s.sA);
        if (rc) return rc;
        SQ_HIP(hipMemcpyAsync(t, c->dmax, sizeof t, hipMemcpyDeviceToHost, s.sA));
        SQ_HIP(hipStreamSynchronize(s.sA));
        m[0] = std::max(m[0], t[0]);
        m[1] = std::max(m[1], t[1]);
    }
    memcpy(mx_abs, &m[0], sizeof(float));
    *mx_phi = unord_f32(m[1]);
    return SQ_OK;
}

// The stability heuristic of tau_kernel.cl:135-143, restated for the 3-D
// lattice from per-step records: step j has a new leader when
// its maximum M_j exceeds T (the maximum of the step before, carried across
// frames); the frame is unstable at the first leader whose drift increment
// D_j = |phi' - phi - sigma xi| at the maximum exceeds V, the running maximum
// of |phi| of the steps before.  T and V are updated through that step (the
// reference breaks after it) and never rolled back.
int stab_rule(float &T, float &V, const float *M, const float *D, const float *A, int n) {
    for (int j = 0; j < n; ++j) {
        const bool fired = M[j] > T && D[j] > V;
        T = M[j];
        V = std::max(V, A[j]);
        if (fired) return j;
    }
    return -1;
}

// The frame snapshot: allocated padded like the slab's buffers, so the three
// can swap roles (three-buffer device frames); snap = its interior.
int ensure_snap(sq_ctx *c, Slab &s) {
    if (s.snap_pad) return SQ_OK;
    const size_t bytes = (size_t)(s.nz + 2 * c->gpad) * plane_floats(c) * sizeof(float);
    SQ_HIP(hipMalloc(&s.snap_pad, bytes));
    s.snap = s.snap_pad + (size_t)c->gpad * plane_floats(c);
    return SQ_OK;
}

int phi4_frame(sq_ctx *c, int *stable) {
    const size_t plane = plane_floats(c);
    // one slab without an exchange: every launch of the frame is on stream A,
    // so stream order replaces the joins around the set-up
    const bool one_stream = c->slabs.size() == 1 && c->p.comm == SQ_COMM_NONE;
    int rc = one_stream ? SQ_OK : phi4_join(c);
    if (rc) return rc;
    if (!c->stab_init) {  // the first frame's leader value and running max: the field itself
        rc = phi4_field_max(c, &c->stab_T, &c->stab_V);
        if (rc) return rc;
        c->stab_init = true;
    }
    const size_t nrec = (size_t)sq::kStabSlots * (size_t)c->p.loops;
    if (!c->frame_rec_zero)  // records and guard flag (normally cleared behind the previous read-back)
        SQ_HIP(hipMemsetAsync(c->frame_cur, 0, c->frame_bytes, c->slabs[0].sA));
    c->frame_rec_zero = false;
    // frame-start snapshot, kept on device: a one-stream frame that starts
    // with a fused pair has that launch store its input's interior (every
    // site once, nontemporal), otherwise a device copy
    const bool snap_in_kernel = one_stream && c->tbz > 0 && c->p.loops >= 2;
    for (auto &s : c->slabs) {
        const size_t bytes = (size_t)s.nz * plane * sizeof(float);
        rc = ensure_snap(c, s);
        if (rc) return rc;
        if (snap_in_kernel)
            c->snap_next = s.snap;
        else
            SQ_HIP(hipMemcpyAsync(s.snap, plane0(c, s, c->cur), bytes, hipMemcpyDeviceToDevice, s.sA));
    }
    rc = one_stream ? SQ_OK : phi4_join(c);
    if (rc) return rc;
    c->in_frame = true;
    c->kstage_pending = false;  // frames stage their exchanges by copy
    c->frame_step0 = c->step;
    // the agreed value: a rollback restores it on every rank alike (an
    // unagreed local value would let a rank with fin = 1 take the guard's fast
    // path on a neighbour's unguarded ghost planes after the rollback)
    rc = fin_agree(c);
    if (rc) return rc;
    const bool fin0 = c->field_finite;
    rc = phi4_steps(c, c->p.loops);
    c->in_frame = false;
    c->snap_next = nullptr;
    if (rc) return rc;
    rc = one_stream ? SQ_OK : phi4_join(c);
    if (rc) return rc;
    Slab &s0 = c->slabs[0];
    if (per_rank(c->p.comm) && c->p.nranks > 1) {
        const bool grp = c->p.comm == SQ_COMM_RCCL;
        if (grp) SQ_NCCLW(c, ncclGroupStart());
        rc = rank_allreduce(c, c->flag, 1, sq::P2pRed::kMaxI32, s0.sA);
        if (!rc) rc = rank_allreduce(c, c->st_md, nrec, sq::P2pRed::kMaxU64, s0.sA);
        if (!rc) rc = rank_allreduce(c, c->st_a, nrec, sq::P2pRed::kMaxU32, s0.sA);
        if (grp) SQ_NCCLW(c, ncclGroupEnd());
        if (rc) return rc;
    }
    // one read-back of the records and the flag into pinned memory
    SQ_HIP(hipMemcpyAsync(c->frame_host, c->frame_cur, c->frame_bytes, hipMemcpyDeviceToHost, s0.sA));
    // clear the records for the next frame behind the read-back (stream order), off its start
    SQ_HIP(hipMemsetAsync(c->frame_cur, 0, c->frame_bytes, s0.sA));
    c->frame_rec_zero = true;
    SQ_HIP(hipStreamSynchronize(s0.sA));
    rc = gate_check(c, true);  // a timed-out rim chunk: no verdict from a corrupt field
    if (rc) return rc;
    const char *hb = static_cast<const char *>(c->frame_host);
    const unsigned long long *md = reinterpret_cast<const unsigned long long *>(hb);
    const unsigned int *am = reinterpret_cast<const unsigned int *>(hb + nrec * sizeof(unsigned long long));
    const int h = *reinterpret_cast<const int *>(hb + nrec * (sizeof(unsigned long long) + sizeof(unsigned int)));
    const int L = c->p.loops;
    c->rec_M.assign(L, 0.f);
    c->rec_D.assign(L, 0.f);
    c->rec_A.assign(L, 0.f);
    for (int j = 0; j < L; ++j) {
        unsigned long long k = 0;
        unsigned int a = 0;
        for (int i = 0; i < sq::kStabSlots; ++i) {
            k = std::max(k, md[(size_t)j * sq::kStabSlots + i]);
            a = std::max(a, am[(size_t)j * sq::kStabSlots + i]);
        }
        c->rec_M[j] = unord_f32((unsigned int)(k >> 32));
        const unsigned int db = (unsigned int)k;
        memcpy(&c->rec_D[j], &db, sizeof(float));
        memcpy(&c->rec_A[j], &a, sizeof(float));
    }
    c->stab_fired = stab_rule(c->stab_T, c->stab_V, c->rec_M.data(), c->rec_D.data(), c->rec_A.data(), L);
    *stable = (h == 0 && c->stab_fired < 0) ? 1 : 0;
    if (!*stable) {  // rollback from the device snapshot; the noise counter is NOT rewound,
                     // so a retried frame draws fresh noise (as the reference's LCG state)
        c->field_finite = fin0;
        for (auto &s : c->slabs)
            SQ_HIP(hipMemcpyAsync(plane0(c, s, c->cur), s.snap, (size_t)s.nz * plane * sizeof(float),
                                  hipMemcpyDeviceToDevice, s.sA));
        rc = phi4_join(c);
        if (rc) return rc;
    }
    return SQ_OK;
}

// Frames back to back under the device controller: per frame
// the launches of phi4_frame (snapshot from the first fused launch, the frame
// instances with the guard flag and the records), then phi4_frame_ctl_kernel
// (record fold, stab_rule, Δτ) and phi4_rollback_kernel (a no-op when
// stable); the launches of frame f+1 read the coefficients frame f's
// controller wrote.  One read-back at the end of the batch.  Bit-identical to
// the host path (phi4_frame + adapt) in field, verdicts, Δτ, T/V and records.
// One slab without an exchange; other decompositions (and loops < 1, a field
// not yet through the guard, SQ_FRAME_HOST=1) take the host path per frame.
int phi4_frames_dev(sq_ctx *c, int n, int *stable, double *dtau_out) {
    const int L = c->p.loops;
    const bool one_stream = c->slabs.size() == 1 && c->p.comm == SQ_COMM_NONE;
    const char *fh = getenv("SQ_FRAME_HOST");
    const bool host_only = !one_stream || L < 1 || c->st_md == nullptr || (fh && atoi(fh) != 0) ||
                           ((size_t)c->slabs[0].nz * plane_floats(c)) % 4 != 0;
    int f = 0;
    while (f < n && (host_only || !c->field_finite)) {  // host path (rollback restores fin0 = false)
        int rc = phi4_frame(c, &stable[f]);
        if (rc) return rc;
        adapt(c, stable[f]);
        if (dtau_out) dtau_out[f] = c->dtau;
        ++f;
    }
    if (f == n) return SQ_OK;
    Slab &s0 = c->slabs[0];
    const hipStream_t st = s0.sA;
    const size_t plane = plane_floats(c), nfl = (size_t)s0.nz * plane;
    if (!c->stab_init) {
        int rc = phi4_field_max(c, &c->stab_T, &c->stab_V);
        if (rc) return rc;
        c->stab_init = true;
    }
    if (!c->ctl || !c->ctl_host || !c->rec_dev) {  // all three, or none after a failure
        (void)hipFree(c->ctl);
        (void)hipFree(c->rec_dev);
        if (c->ctl_host) (void)hipHostFree(c->ctl_host);
        c->ctl = nullptr;
        c->rec_dev = nullptr;
        c->ctl_host = nullptr;
        SQ_HIP(hipMalloc(&c->ctl, 2 * sizeof(sq::FrameCtl)));
        SQ_HIP(hipHostMalloc(&c->ctl_host, sizeof(sq::FrameCtl), hipHostMallocDefault));
        SQ_HIP(hipMalloc(&c->rec_dev, 3 * sizeof(float) * (size_t)L));
    }
    {
        int rc = ensure_snap(c, s0);
        if (rc) return rc;
    }
    const int m = n - f;
    if (m > c->fr_cap) {
        (void)hipFree(c->fr_stable);
        (void)hipFree(c->fr_dtau);
        if (c->fr_stable_h) (void)hipHostFree(c->fr_stable_h);
        if (c->fr_dtau_h) (void)hipHostFree(c->fr_dtau_h);
        c->fr_stable = nullptr;  // a failed allocation below must not leave freed pointers for sq_destroy
        c->fr_dtau = nullptr;
        c->fr_stable_h = nullptr;
        c->fr_dtau_h = nullptr;
        c->fr_cap = 0;
        SQ_HIP(hipMalloc(&c->fr_stable, sizeof(int) * (size_t)m));
        SQ_HIP(hipMalloc(&c->fr_dtau, sizeof(double) * (size_t)m));
        SQ_HIP(hipHostMalloc(&c->fr_stable_h, sizeof(int) * (size_t)m, hipHostMallocDefault));
        SQ_HIP(hipHostMalloc(&c->fr_dtau_h, sizeof(double) * (size_t)m, hipHostMallocDefault));
        c->fr_cap = m;
    }
    // the controller starts from the host's state (a caller may have set Δτ or T/V)
    sq::FrameCtl &h = *c->ctl_host;
    memset(&h, 0, sizeof h);
    h.dtau = c->dtau;
    h.C = c->p.C;
    const float hf = (float)c->dtau;  // as phi4_base_args
    h.coef[0] = hf;
    h.coef[1] = (float)(sqrt(2.0 * (double)hf) * c->p.C);
    h.coef[2] = (float)(sqrt(2.0 * (double)hf) * c->p.C * sq::kSqrt2Ln2);
    h.T = c->stab_T;
    h.V = c->stab_V;
    h.stab_cnt = c->stab_cnt;
    h.adapt = c->p.adapt_dtau ? 1 : 0;
    h.stable = 1;
    h.fired = -1;
    // three buffers (the slab's two and the padded snapshot allocation): a
    // frame never writes the buffer it starts from, so that buffer is its
    // rollback -- no snapshot store, no copy back (SQ_FRAME_TRI=0: off)
    const char *ft = getenv("SQ_FRAME_TRI");
    const bool tri = c->tbz > 0 && L >= 2 && !(ft && atoi(ft) == 0);
    if (tri) {
        c->tri_bufs[0] = s0.buf[c->cur];
        c->tri_bufs[1] = s0.buf[c->cur ^ 1];
        c->tri_bufs[2] = s0.snap_pad;
        h.tri = 1;
        h.bs = 0;
        h.bw0 = 1;
        h.bw1 = 2;
        h.nl_odd = ((L / 2) + (L & 1)) & 1;  // launches per frame: the pairs and an odd last step
    }
    c->spec_bs = 0;  // the guess starts from the roles the controller starts from
    c->spec_bw0 = 1;
    c->spec_bw1 = 2;
    {
        const char *fs = getenv("SQ_FRAME_SPEC");
        c->tri_spec = !(fs && atoi(fs) == 0);
    }
    SQ_HIP(hipMemcpyAsync(c->ctl, c->ctl_host, sizeof h, hipMemcpyHostToDevice, st));
    // the active record set must start zero; each frame-end launch clears the
    // other one, which the next frame then uses
    if (!c->frame_rec_zero) SQ_HIP(hipMemsetAsync(c->frame_cur, 0, c->frame_bytes, st));
    const bool snap_in_kernel = c->tbz > 0 && L >= 2;
    // frame i > 0's first fused launch takes frame i-1's end (FrameFoldArgs):
    // frames of 4..kFoldMaxL steps (the launch after the first, a fused pair
    // too, clears the folded set); SQ_FRAME_FOLD=0 keeps one end launch per frame
    const char *ff = getenv("SQ_FRAME_FOLD");
    const bool fold = snap_in_kernel && L >= 4 && L <= sq::kFoldMaxL && !(ff && atoi(ff) == 0);
    // diagnostic only (profiles/r04/frames/): no snapshot store, so a rolled-back
    // frame restores garbage -- prices the store on stable frames
    const char *dns = getenv("SQ_DIAG_NO_SNAP");
    const bool diag_no_snap = dns && atoi(dns) != 0;
    c->tri = tri;
    for (int i = 0; i < m; ++i) {
        if (tri)
            c->snap_next = nullptr;
        else if (snap_in_kernel)
            c->snap_next = diag_no_snap ? nullptr : s0.snap;
        else
            SQ_HIP(hipMemcpyAsync(s0.snap, plane0(c, s0, c->cur), nfl * sizeof(float), hipMemcpyDeviceToDevice, st));
        c->in_frame = true;
        c->kstage_pending = false;  // frames stage their exchanges by copy
        c->dev_frames = true;
        c->ctl_cur = c->ctl + (i & 1);
        c->frame_step0 = c->step;
        c->frame_tk = 0;
        c->clr_armed = false;
        if (fold && i == 0 && m > 1) {
            // the other record set still holds the previous batch's last frame:
            // frame 0's second launch clears it for frame 1
            const int cur_set = c->rec_set;
            use_rec_set(c, cur_set ^ 1);
            c->clr_next = sq::RecClear{c->st_md, c->st_a, c->flag, L * sq::kStabSlots};
            use_rec_set(c, cur_set);
            c->clr_first = true;
        }
        int rc = phi4_steps(c, L);
        if (tri) {  // the next frame's roles if this one is stable (frame_decide's rotation)
            const int fin = h.nl_odd ? c->spec_bw0 : c->spec_bw1;
            const int third = 3 - c->spec_bs - fin;
            c->spec_bw1 = c->spec_bs;
            c->spec_bs = fin;
            c->spec_bw0 = third;
        }
        c->in_frame = false;
        c->dev_frames = false;
        c->snap_next = nullptr;
        c->fold_next = sq::FrameFoldArgs{};
        c->clr_armed = false;
        c->clr_first = false;
        if (rc) {
            c->tri = false;
            return rc;
        }
        if (fold && i + 1 < m) {
            // frame i+1's first launch decides frame i: it folds this record
            // set and writes ctl[(i+1)&1]; frame i+1 accumulates into the other
            // set (cleared by frame i's second launch)
            sq::FrameFoldArgs fa{};
            fa.cin = c->ctl + (i & 1);
            fa.cout = c->ctl + ((i + 1) & 1);
            fa.md = c->st_md;
            fa.am = c->st_a;
            fa.flag = c->flag;
            fa.rec = c->rec_dev;
            fa.stable_out = c->fr_stable + i;
            fa.dtau_out = c->fr_dtau + i;
            fa.snap = s0.snap;
            fa.L = L;
            sq::RecClear cl{};
            cl.md = c->st_md;
            cl.am = c->st_a;
            cl.flag = c->flag;
            cl.n = L * sq::kStabSlots;
            use_rec_set(c, c->rec_set ^ 1);
            c->fold_next = fa;
            c->clr_next = cl;
            continue;
        }
        sq::FrameEndArgs e{};
        e.cin = c->ctl + (i & 1);
        e.cout = c->ctl + ((i + 1) & 1);
        e.md = c->st_md;
        e.am = c->st_a;
        e.flag = c->flag;
        const int cur_set = c->rec_set;
        use_rec_set(c, cur_set ^ 1);
        e.md_next = c->st_md;
        e.am_next = c->st_a;
        e.flag_next = c->flag;
        e.L = L;
        e.rec = c->rec_dev;
        e.stable_out = c->fr_stable + i;
        e.dtau_out = c->fr_dtau + i;
        e.dst = reinterpret_cast<float4 *>(plane0(c, s0, c->cur));
        e.snap = reinterpret_cast<const float4 *>(s0.snap);
        e.n4 = tri ? 0 : (long long)(nfl / 4);  // three buffers: the rollback is the next start buffer
        SQ_HIP(sq::phi4_frame_end_launch(e, st));
        c->perf.kernel_launches += 1;
    }
    c->tri = false;
    c->frame_rec_zero = true;  // the active set is the one the last frame-end launch cleared
    SQ_HIP(hipMemcpyAsync(c->ctl_host, c->ctl + (m & 1), sizeof h, hipMemcpyDeviceToHost, st));
    SQ_HIP(hipMemcpyAsync(c->fr_stable_h, c->fr_stable, sizeof(int) * (size_t)m, hipMemcpyDeviceToHost, st));
    SQ_HIP(hipMemcpyAsync(c->fr_dtau_h, c->fr_dtau, sizeof(double) * (size_t)m, hipMemcpyDeviceToHost, st));
    SQ_HIP(hipMemcpyAsync(c->frame_host, c->rec_dev, 3 * sizeof(float) * (size_t)L, hipMemcpyDeviceToHost, st));
    SQ_HIP(hipStreamSynchronize(st));
    for (int i = 0; i < m; ++i) {
        stable[f + i] = c->fr_stable_h[i];
        if (dtau_out) dtau_out[f + i] = c->fr_dtau_h[i];
    }
    c->dtau = h.dtau;
    c->stab_cnt = h.stab_cnt;
    c->stab_T = h.T;
    c->stab_V = h.V;
    c->stab_fired = h.fired;
    if (tri) {  // the field is the start buffer of the frame after the batch: make it buf[0]
        if (h.bs < 0 || h.bs > 2) return fail(SQ_E_STATE, "device frames: corrupt buffer rotation");
        float *b[3] = {c->tri_bufs[h.bs], c->tri_bufs[(h.bs + 1) % 3], c->tri_bufs[(h.bs + 2) % 3]};
        s0.buf[0] = b[0];
        s0.buf[1] = b[1];
        s0.snap_pad = b[2];
        s0.snap = b[2] + (size_t)c->gpad * plane;
        c->cur = 0;
    }
    const float *r = static_cast<const float *>(c->frame_host);
    c->rec_M.assign(r, r + L);
    c->rec_D.assign(r + L, r + 2 * L);
    c->rec_A.assign(r + 2 * L, r + 3 * L);
    return SQ_OK;
}

}  // namespace

extern "C" {

void sq_params_init(sq_params *p) {
    memset(p, 0, sizeof *p);
    p->struct_size = (int)sizeof(sq_params);
    p->model = SQ_MODEL_QM1D;
    p->dims[0] = 200;
    p->dims[1] = 1;
    p->dims[2] = 1;
    p->deltat = 0.02;
    p->deltatau = 0.002;
    p->pot = 3;
    p->C = 1.0;
    p->loops = 1000;
    p->seed = 0x5EEDull;
    p->m2 = 1.0;
    p->lambda = 1.0;
    p->clamp = 1000.0;
    p->device = 0;
    p->adapt_dtau = 1;
    p->comm = SQ_COMM_NONE;
    p->nranks = 1;
    p->rank = 0;
    p->nslabs = 1;
}

const char *sq_last_error(void) { return g_err.c_str(); }
int sq_abi_version(void) { return SQ_ABI_VERSION; }

int sq_device_count(int *n) {
    int k = 0;
    hipError_t e = hipGetDeviceCount(&k);
    if (e != hipSuccess) k = 0;
    *n = k;
    return SQ_OK;
}

int sq_create(const sq_params *p, sq_ctx **out) {
    if (!p || !out) return fail(SQ_E_ARG, "null argument");
    *out = nullptr;
    if (p->struct_size != (int)sizeof(sq_params)) return fail(SQ_E_ARG, "sq_params size mismatch");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    if (p->device < 0 || p->device >= ndev) return fail(SQ_E_ARG, "device ordinal out of range");
    if (!(p->deltatau > 0)) return fail(SQ_E_ARG, "deltatau must be > 0");
    DeviceGuard g(p->device);
    sq_ctx *c = new sq_ctx();
    c->p = *p;
    c->dev = p->device;
    c->dtau = p->deltatau;
    int rc = p->model == SQ_MODEL_PHI4 ? create_phi4(c) : p->model == SQ_MODEL_QM1D ? create_qm1d(c)
                                                                                      : fail(SQ_E_ARG, "unknown model");
    if (rc) {
        std::string msg = g_err;
        sq_destroy(c);
        g_err = msg;
        return rc;
    }
    *out = c;
    return SQ_OK;
}

int sq_destroy(sq_ctx *c) {
    if (!c) return SQ_OK;
    DeviceGuard g(c->dev);
    bool p2p_drained = true;
    if (c->p2p_ready && c->xchg_seq > 0 && !c->slabs.empty() && c->slabs[0].sB) {
        // P2P: our staged copy may still be read by a neighbour that is behind;
        // free it only after both have acknowledged the last exchange (bounded
        // wait: a peer that died leaves the buffers mapped, not a hang)
        // (exchanges do not acknowledge one by one, phi4_block: the last one is
        // acknowledged here, behind our own pulls of it on the exchange stream)
        hipStream_t sB = c->slabs[0].sB;
        const int P = c->p.nranks, r = c->p.rank;
        const int up = (r + 1) % P, dn = (r + P - 1) % P;
        // with the exchange in order on stream A (SQ_XCHG_ON_A) our last pulls
        // ran there: the acknowledgements on stream B must follow them (the
        // hand-shake's bounded poll ends stream A's work even if a peer died)
        (void)hipStreamSynchronize(c->slabs[0].sA);
        if (hipStreamWriteValue32(sB, c->peers[dn].mbox + kMbAckFromUp, c->xchg_seq, 0) != hipSuccess ||
            hipStreamWriteValue32(sB, c->peers[up].mbox + kMbAckFromDn, c->xchg_seq, 0) != hipSuccess ||
            wait_seq(sB, c->mbox + kMbAckFromDn, c->xchg_seq) != hipSuccess ||
            wait_seq(sB, c->mbox + kMbAckFromUp, c->xchg_seq) != hipSuccess)
            p2p_drained = false;
        const auto t0 = std::chrono::steady_clock::now();
        while (p2p_drained && hipStreamQuery(sB) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) p2p_drained = false;
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    if (!p2p_drained) return SQ_OK;  // leak rather than free memory a peer may still read
    for (auto &s : c->slabs) {
        if (s.sA) (void)hipStreamSynchronize(s.sA);
        if (s.sB) (void)hipStreamSynchronize(s.sB);
    }
    for (Peer &q : c->peers)
        if (q.mapped) {
            (void)hipIpcCloseMemHandle(q.stage);
            (void)hipIpcCloseMemHandle(q.mbox);
            (void)hipIpcCloseMemHandle(q.coll);
        }
    (void)hipFree(c->mbox);
    (void)hipFree(c->coll);
    (void)hipFree(c->gate_word);
    (void)hipFree(c->gate_err);
    (void)hipFree(c->run_flags);
    (void)hipFree(c->kstage_ctr);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (auto &s : c->slabs) {
        (void)hipFree(s.buf[0]);
        (void)hipFree(s.buf[1]);
        (void)hipFree(s.snap_pad);
        if (s.sA) (void)hipStreamDestroy(s.sA);
        if (s.sB) (void)hipStreamDestroy(s.sB);
        if (s.evC) (void)hipEventDestroy(s.evC);
        if (s.evE) (void)hipEventDestroy(s.evE);
        if (s.evS) (void)hipEventDestroy(s.evS);
        for (hipEvent_t e : s.evk)
            if (e) (void)hipEventDestroy(e);
        (void)hipFree(s.stage);
    }
    for (int k = 0; k < 2; ++k) {
        (void)hipFree(c->qf[k]);
        (void)hipFree(c->qx[k]);
        (void)hipFree(c->qxx0[k]);
    }
    (void)hipFree(c->qst);
    for (double *q : c->qscr) (void)hipFree(q);
    (void)hipFree(c->qom);
    (void)hipFree(c->qdd);
    (void)hipFree(c->qxi);
    (void)hipFree(c->qtcl);
    for (double *q : {c->g_xi, c->g_om, c->g_xc, c->g_hist_buf, c->g_nfp}) (void)hipFree(q);
    (void)hipFree(c->g_w1);
    (void)hipFree(c->g_w2);
    (void)hipFree(c->g_seeds);
    (void)hipFree(c->g_lcg_scr);
    (void)hipFree(c->g_cand);
    (void)hipFree(c->g_flags);
    (void)hipFree(c->g_st);
    if (c->frame_rec) {  // flag, st_md, st_a live in it
        (void)hipFree(c->frame_rec);
    } else {
        (void)hipFree(c->flag);
        (void)hipFree(c->st_md);
        (void)hipFree(c->st_a);
    }
    if (c->frame_host) (void)hipHostFree(c->frame_host);
    (void)hipFree(c->ctl);
    (void)hipFree(c->dstamps);
    (void)hipFree(c->rec_dev);
    (void)hipFree(c->fr_stable);
    (void)hipFree(c->fr_dtau);
    if (c->ctl_host) (void)hipHostFree(c->ctl_host);
    if (c->fr_stable_h) (void)hipHostFree(c->fr_stable_h);
    if (c->fr_dtau_h) (void)hipHostFree(c->fr_dtau_h);
    (void)hipFree(c->dacc);
    (void)hipFree(c->dpart);
    (void)hipFree(c->dslice);
    (void)hipFree(c->dtune);
    (void)hipFree(c->dmax);
    if (c->qstream) (void)hipStreamDestroy(c->qstream);
    for (auto &e : c->evpool) {
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    delete c;
    return SQ_OK;
}

int sq_upload(sq_ctx *c, const double *f, const double *x, const double *xx0, double omega, long runs) {
    if (!c || !f || !x || !xx0) return fail(SQ_E_ARG, "null argument");
    if (is_phi4(c)) return fail(SQ_E_STATE, "sq_upload is for QM1D contexts");
    DeviceGuard g(c->dev);
    const size_t bytes = sizeof(double) * (size_t)c->N;
    SQ_HIP(hipMemcpy(c->qf[c->qcur], f, bytes, hipMemcpyHostToDevice));
    SQ_HIP(hipMemcpy(c->qx[c->qcur], x, bytes, hipMemcpyHostToDevice));
    SQ_HIP(hipMemcpy(c->qxx0[c->qcur], xx0, bytes, hipMemcpyHostToDevice));
    // the reference writes newf = f once, before the first frame (tauhost.c:177-183,319-377)
    if (c->g_nfp) SQ_HIP(hipMemcpy(c->g_nfp, f, bytes, hipMemcpyHostToDevice));
    c->omega = omega;
    c->runs = runs;
    return SQ_OK;
}

int sq_download(sq_ctx *c, double *f, double *x, double *xx0, double *omega, long *runs) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (is_phi4(c)) return fail(SQ_E_STATE, "sq_download is for QM1D contexts");
    DeviceGuard g(c->dev);
    const size_t bytes = sizeof(double) * (size_t)c->N;
    if (f) SQ_HIP(hipMemcpy(f, c->qf[c->qcur], bytes, hipMemcpyDeviceToHost));
    if (x) SQ_HIP(hipMemcpy(x, c->qx[c->qcur], bytes, hipMemcpyDeviceToHost));
    if (xx0) SQ_HIP(hipMemcpy(xx0, c->qxx0[c->qcur], bytes, hipMemcpyDeviceToHost));
    if (omega) *omega = c->omega;
    if (runs) *runs = c->runs;
    return SQ_OK;
}

int sq_qm1d_get_scan(sq_ctx *c, int *lrgEl, double *lrgVl, unsigned long long *tick) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (lrgEl) *lrgEl = c->lrgEl;
    if (lrgVl) *lrgVl = c->lrgVl;
    if (tick) *tick = c->step;
    return SQ_OK;
}

int sq_qm1d_set_scan(sq_ctx *c, int lrgEl, double lrgVl, unsigned long long tick) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (is_phi4(c)) return fail(SQ_E_STATE, "QM1D only");
    if (lrgEl < 0 || lrgEl >= c->N) return fail(SQ_E_ARG, "lrgEl out of range");
    c->lrgEl = lrgEl;
    c->lrgVl = lrgVl;
    c->step = tick;
    return SQ_OK;
}

int sq_qm1d_set_ordering(sq_ctx *c, int ordering) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (is_phi4(c)) return fail(SQ_E_STATE, "QM1D only");
    if (ordering != SQ_ORDER_JACOBI && ordering != SQ_ORDER_SERIAL) return fail(SQ_E_ARG, "unknown ordering");
    if (ordering == SQ_ORDER_SERIAL) {
        if (sq::qm1d_gs_block(c->N) == 0)
            return fail(SQ_E_ARG, "SQ_ORDER_SERIAL supports 2 <= N <= " + std::to_string(sq::kQm1dGsMaxN));
        DeviceGuard g(c->dev);
        if (!c->g_nfp) {
            SQ_HIP(hipMalloc(&c->g_nfp, sizeof(double) * (size_t)c->N));
            SQ_HIP(hipMemcpy(c->g_nfp, c->qf[c->qcur], sizeof(double) * (size_t)c->N, hipMemcpyDeviceToDevice));
        }
    }
    c->order = ordering;
    return SQ_OK;
}

int sq_qm1d_set_lcg_seed(sq_ctx *c, unsigned long long seed) {
    if (!c) return fail(SQ_E_ARG, "null context");
    c->lcg_seed = seed;
    return SQ_OK;
}

int sq_qm1d_get_lcg_seed(sq_ctx *c, unsigned long long *seed) {
    if (!c || !seed) return fail(SQ_E_ARG, "null argument");
    *seed = c->lcg_seed;
    return SQ_OK;
}

int sq_qm1d_inject_noise(sq_ctx *c, const double *xi, size_t n) {
    if (!c || !xi) return fail(SQ_E_ARG, "null argument");
    if (is_phi4(c) || c->order != SQ_ORDER_SERIAL) return fail(SQ_E_STATE, "needs a QM1D context in SQ_ORDER_SERIAL");
    const size_t need = (size_t)(c->N + 1) * (size_t)c->p.loops;
    if (n < need) return fail(SQ_E_ARG, "need (N+1)*loops draws, got " + std::to_string(n));
    DeviceGuard g(c->dev);
    int rc = gs_reserve(c);
    if (rc) return rc;
    SQ_HIP(hipMemcpy(c->g_xi, xi, sizeof(double) * need, hipMemcpyHostToDevice));
    c->inject_pending = true;
    return SQ_OK;
}

int sq_qm1d_noise_consumed(sq_ctx *c, unsigned long long *n) {
    if (!c || !n) return fail(SQ_E_ARG, "null argument");
    *n = c->consumed;
    return SQ_OK;
}

int sq_run_frame(sq_ctx *c, int *stable) {
    if (!c || !stable) return fail(SQ_E_ARG, "null argument");
    DeviceGuard g(c->dev);
    const auto t0 = std::chrono::steady_clock::now();
    // one frame: the host-decided path (one read-back, 454 vs 478 us per 256^3
    // 20-step frame for the device controller's state upload and read-back);
    // sq_run_frames keeps the decisions on the device across frames
    int rc = is_phi4(c) ? gate_check(c, false) : SQ_OK;
    if (!rc) rc = is_phi4(c) ? phi4_frame(c, stable) : qm1d_frame(c, stable);
    if (rc) return rc;
    adapt(c, *stable);
    c->perf.frame_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return SQ_OK;
}

int sq_run_frames(sq_ctx *c, int nframes, int *stable, double *dtau) {
    if (!c || (!stable && nframes > 0)) return fail(SQ_E_ARG, "null argument");
    if (nframes < 0) return fail(SQ_E_ARG, "nframes < 0");
    DeviceGuard g(c->dev);
    const auto t0 = std::chrono::steady_clock::now();
    if (is_phi4(c)) {
        int rc = gate_check(c, false);
        if (!rc) rc = phi4_frames_dev(c, nframes, stable, dtau);
        if (rc) return rc;
    } else {
        for (int f = 0; f < nframes; ++f) {
            int rc = qm1d_frame(c, &stable[f]);
            if (rc) return rc;
            adapt(c, stable[f]);
            if (dtau) dtau[f] = c->dtau;
        }
    }
    c->perf.frame_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return SQ_OK;
}

int sq_step(sq_ctx *c, int nsteps) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "sq_step is for PHI4 contexts (QM1D uses sq_run_frame)");
    if (nsteps < 0) return fail(SQ_E_ARG, "nsteps < 0");
    DeviceGuard g(c->dev);
    {
        int rc = gate_check(c, false);  // a known timeout: no more steps on the corrupt field
        if (rc) return rc;
    }
    const auto t0 = std::chrono::steady_clock::now();
    EvPair *region = nullptr;
    if (c->profiling == 2 && nsteps > 0) {
        int rc = ev_take(c, &region);
        if (rc) return rc;
        SQ_HIP(hipEventRecord(region->a, c->slabs[0].sA));
    }
    {
        int rc = phi4_steps(c, nsteps);
        if (rc) return rc;
    }
    if (c->gate_err) {  // tests: SQ_DIAG_GATE_ERR=1 flags a gate timeout as tb_gate_wait would
        const char *ge = getenv("SQ_DIAG_GATE_ERR");
        if (ge && atoi(ge) != 0) SQ_HIP(hipMemsetAsync(c->gate_err, 1, 1, c->slabs[0].sA));
    }
    if (region) {
        SQ_HIP(hipEventRecord(region->b, c->slabs[0].sA));
        c->region_steps += nsteps;
    }
    c->perf.frame_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return SQ_OK;
}

int sq_phi4_block_stamps(sq_ctx *c, unsigned long long *out, int cap, int *nblocks) {
    if (!c || !out || !nblocks || cap < 1) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    if (c->slabs.size() != 1 || c->p.comm != SQ_COMM_NONE || c->tbz <= 0)
        return fail(SQ_E_STATE, "block stamps: one slab without an exchange, fused launches");
    DeviceGuard g(c->dev);
    const int need = std::max(cap, 4096);
    if (c->stamps_cap < need) {
        (void)hipFree(c->dstamps);
        c->stamps_cap = 0;
        SQ_HIP(hipMalloc(&c->dstamps, 4 * sizeof(unsigned long long) * (size_t)need));  // + the shader clock
        c->stamps_cap = need;
    }
    c->stamps_next = c->dstamps;
    c->stamps_blocks = 0;
    int rc = phi4_steps(c, 2);
    c->stamps_next = nullptr;
    if (rc) return rc;
    if (c->stamps_blocks > cap) return fail(SQ_E_ARG, "cap smaller than the launch's blocks");
    SQ_HIP(hipMemcpyAsync(out, c->dstamps, 2 * sizeof(unsigned long long) * (size_t)c->stamps_blocks,
                          hipMemcpyDeviceToHost, c->slabs[0].sA));
    SQ_HIP(hipStreamSynchronize(c->slabs[0].sA));
    *nblocks = c->stamps_blocks;
    return SQ_OK;
}

int sq_phi4_block_clocks(sq_ctx *c, unsigned long long *out, int cap, int *nblocks) {
    if (!c || !out || !nblocks || cap < 1) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    if (c->dstamps == nullptr || c->stamps_blocks < 1) return fail(SQ_E_STATE, "no sq_phi4_block_stamps launch yet");
    if (c->stamps_blocks > cap) return fail(SQ_E_ARG, "cap smaller than the launch's blocks");
    DeviceGuard g(c->dev);
    const size_t n = 2 * (size_t)c->stamps_blocks;  // written behind the 2 x blocks constant-clock stamps
    SQ_HIP(hipMemcpyAsync(out, c->dstamps + n, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost,
                          c->slabs[0].sA));
    SQ_HIP(hipStreamSynchronize(c->slabs[0].sA));
    *nblocks = c->stamps_blocks;
    return SQ_OK;
}

int sq_sync(sq_ctx *c) {
    if (!c) return fail(SQ_E_ARG, "null context");
    DeviceGuard g(c->dev);
    if (c->qstream) SQ_HIP(hipStreamSynchronize(c->qstream));
    int rc = phi4_join(c);
    if (rc) return rc;
    return gate_check(c, true);  // a gated rim chunk gave up waiting for its exchange: sticky
}

int sq_slab(sq_ctx *c, long long *nz_local, long long *z0) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    long long n = 0;
    for (auto &s : c->slabs) n += s.nz;
    if (nz_local) *nz_local = n;
    if (z0) *z0 = c->slabs[0].z0;
    return SQ_OK;
}

int sq_phi4_tile(sq_ctx *c, int out[4]) {
    if (!c || !out) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    out[0] = c->geom.qx;
    out[1] = c->geom.r;
    out[2] = c->zc;
    out[3] = c->geom.v;
    return SQ_OK;
}

int sq_phi4_kernel(sq_ctx *c, char *name, size_t cap) {
    if (!c || !name || cap == 0) return fail(SQ_E_ARG, "bad argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    // the template arguments phi4_step_launch picks for the interior launch
    // (rocprofv3 prints the kernel under exactly this name)
    const bool ms = c->Lx / (4 * c->geom.qx * c->geom.v) > 1;
    const bool nz = (float)(sqrt(2.0 * (double)(float)c->dtau) * c->p.C) != 0.0f;
    const int pf = c->geom.pf;
    if (c->tbz > 0 && c->tbz_pin)
        snprintf(name, cap, "phi4_tb2_kernel<%s> (2 steps per launch) z=%d", nz ? "true" : "false", c->tbz);
    else if (c->tbz > 0)
        snprintf(name, cap, "phi4_tb2_kernel<%s> (2 steps per launch) one round of %d blocks", nz ? "true" : "false",
                 c->tb_blocks);
    else
        snprintf(name, cap, "phi4_step_kernel<%d, %d, %d, %s, %s, %d> zc=%d", c->geom.qx, c->geom.r, c->geom.v,
                 ms ? "true" : "false", nz ? "true" : "false", pf, c->zc);
    return SQ_OK;
}

int sq_phi4_ghost(sq_ctx *c, int *active, int *allocated) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    if (active) *active = c->p.comm == SQ_COMM_NONE ? 0 : c->gz;
    if (allocated) *allocated = c->p.comm == SQ_COMM_NONE ? 0 : c->gpad;
    return SQ_OK;
}

int sq_phi4_schedule(sq_ctx *c, int *core_pairs, int *rims_b, int *tuned) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    const bool slab = c->p.comm != SQ_COMM_NONE;
    if (core_pairs) *core_pairs = slab ? c->core_pairs : 0;
    if (rims_b) *rims_b = slab && c->rims_b ? 1 : 0;
    if (tuned) *tuned = c->g_tuned ? 1 : 0;
    return SQ_OK;
}

int sq_phi4_edge_first(sq_ctx *c, int *edge_first) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    if (edge_first) *edge_first = c->p.comm != SQ_COMM_NONE && c->edge_first ? 1 : 0;
    return SQ_OK;
}

int sq_phi4_exchange_stream(sq_ctx *c, int *in_order, int *kstaged) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    const bool slab = c->p.comm == SQ_COMM_P2P || c->p.comm == SQ_COMM_RCCL;
    if (in_order) *in_order = slab && c->xchg_on_a ? 1 : 0;
    if (kstaged) *kstaged = c->p.comm == SQ_COMM_P2P && kstage_on(c) ? 1 : 0;
    return SQ_OK;
}

int sq_phi4_stability(sq_ctx *c, double state[2], int *fired_step, float *M, float *D, float *A, int n) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    if (n < 0 || (n > 0 && (!M || !D || !A))) return fail(SQ_E_ARG, "bad record arguments");
    if (n > (int)c->rec_M.size()) return fail(SQ_E_ARG, "n exceeds the last frame's steps");
    if (state) {
        state[0] = c->stab_T;
        state[1] = c->stab_V;
    }
    if (fired_step) *fired_step = c->stab_fired;
    for (int j = 0; j < n; ++j) {
        M[j] = c->rec_M[j];
        D[j] = c->rec_D[j];
        A[j] = c->rec_A[j];
    }
    return SQ_OK;
}

}  // extern "C"

namespace sq {
int frame_state_get(const sq_ctx *c, FrameState *fs) {
    if (!c || !fs) return fail(SQ_E_ARG, "null argument");
    fs->T = c->stab_T;
    fs->V = c->stab_V;
    fs->init = c->stab_init ? 1 : 0;
    fs->stab_cnt = c->stab_cnt;
    return SQ_OK;
}
int frame_state_set(sq_ctx *c, const FrameState &fs) {
    if (!c) return fail(SQ_E_ARG, "null argument");
    if (fs.stab_cnt < 0) return fail(SQ_E_ARG, "stab_cnt must be >= 0");
    c->stab_T = fs.T;
    c->stab_V = fs.V;
    c->stab_init = fs.init != 0;
    c->stab_cnt = fs.stab_cnt;
    return SQ_OK;
}
}  // namespace sq

extern "C" {

int sq_phi4_set_stability(sq_ctx *c, double T, double V) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    c->stab_T = (float)T;
    c->stab_V = (float)V;
    c->stab_init = true;
    return SQ_OK;
}

int sq_phi4_block_plan(int nz, int ghost, int g, int fuse2, int edge_first, int core_pairs, int rims_b,
                       sq_block_op *ops, int cap, int *nops) {
    if (!nops || (cap > 0 && !ops)) return fail(SQ_E_ARG, "null argument");
    if (nz < 1 || ghost < 1 || g < 1 || g > ghost || ghost > nz) return fail(SQ_E_ARG, "need 1 <= g <= ghost <= nz");
    if (core_pairs < 0) return fail(SQ_E_ARG, "core_pairs must be >= 0");
    const std::vector<sq_block_op> v = block_plan(nz, ghost, g, fuse2 != 0, edge_first != 0, core_pairs, rims_b != 0);
    *nops = (int)v.size();
    if ((int)v.size() > cap) return fail(SQ_E_ARG, "cap too small: need " + std::to_string(v.size()));
    std::copy(v.begin(), v.end(), ops);
    return SQ_OK;
}

int sq_phi4_pick_ghost(const double *ms, int n) {
    int best = 0;
    for (int k = 1; k < n; ++k)
        if (ms[k] < ms[best]) best = k;
    return best;
}

int sq_upload_field(sq_ctx *c, const float *phi, size_t count) {
    if (!c || !phi) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    DeviceGuard g(c->dev);
    const size_t plane = plane_floats(c);
    size_t need = 0;
    for (auto &s : c->slabs) need += (size_t)s.nz * plane;
    if (count != need) return fail(SQ_E_ARG, "field size mismatch");
    SQ_HIP(hipDeviceSynchronize());
    {
        int rc = gate_reset(c);
        if (rc) return rc;
    }
    size_t off = 0;
    for (auto &s : c->slabs) {
        SQ_HIP(hipMemcpy(plane0(c, s, c->cur), phi + off, (size_t)s.nz * plane * sizeof(float),
                         hipMemcpyHostToDevice));
        off += (size_t)s.nz * plane;
    }
    c->field_finite = false;  // the caller's values (NaN / inf / beyond the clamp allowed) meet the full guard
    c->fin_sync = true;
    return SQ_OK;
}

int sq_download_field(sq_ctx *c, float *phi, size_t count) {
    if (!c || !phi) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    DeviceGuard g(c->dev);
    const size_t plane = plane_floats(c);
    size_t need = 0;
    for (auto &s : c->slabs) need += (size_t)s.nz * plane;
    if (count != need) return fail(SQ_E_ARG, "field size mismatch");
    int rc = phi4_join(c);
    if (!rc) rc = gate_check(c, true);
    if (rc) return rc;
    size_t off = 0;
    for (auto &s : c->slabs) {
        SQ_HIP(hipMemcpy(phi + off, plane0(c, s, c->cur), (size_t)s.nz * plane * sizeof(float),
                         hipMemcpyDeviceToHost));
        off += (size_t)s.nz * plane;
    }
    return SQ_OK;
}

int sq_init_field(sq_ctx *c, float amp) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    DeviceGuard g(c->dev);
    int rc = phi4_join(c);
    if (!rc) rc = gate_reset(c);
    if (rc) return rc;
    for (auto &s : c->slabs)
        SQ_HIP(sq::phi4_init_launch(plane0(c, s, c->cur), c->Lx, c->Ly, s.nz, s.z0, (uint32_t)c->p.seed,
                                    (uint32_t)(c->p.seed >> 32), amp, s.sA));
    c->field_finite = std::isfinite(amp) && std::fabs(amp) * 8.0f < (float)c->p.clamp;
    c->fin_sync = true;
    return phi4_join(c);
}

int sq_init_field_hash(sq_ctx *c, double amp, unsigned long long key) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    if (!std::isfinite(amp) || std::fabs(amp) > 1e30) return fail(SQ_E_ARG, "amp must be finite");
    DeviceGuard g(c->dev);
    int rc = phi4_join(c);
    if (!rc) rc = gate_reset(c);
    if (rc) return rc;
    for (auto &s : c->slabs)
        SQ_HIP(sq::phi4_init_hash_launch(plane0(c, s, c->cur), c->Lx, c->Ly, s.nz, s.z0, key, amp, s.sA));
    c->field_finite = std::fabs(amp) < c->p.clamp;  // |phi| <= |amp| < clamp: every site finite and unclamped
    c->fin_sync = true;
    return phi4_join(c);
}

int sq_moments(sq_ctx *c, double out[3]) {
    if (!c || !out) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    DeviceGuard g(c->dev);
    int rc = observe_join(c);
    if (rc) return rc;
    const size_t plane = plane_floats(c);
    out[0] = out[1] = out[2] = 0;
    for (auto &s : c->slabs) {
        SQ_HIP(sq::phi4_moments_launch(plane0(c, s, c->cur), (long long)s.nz * (long long)plane,
                                       c->dacc, c->dmax, c->dpart, s.sA));
        double acc[2];
        unsigned int mx;
        SQ_HIP(hipMemcpyAsync(acc, c->dacc, sizeof acc, hipMemcpyDeviceToHost, s.sA));
        SQ_HIP(hipMemcpyAsync(&mx, c->dmax, sizeof mx, hipMemcpyDeviceToHost, s.sA));
        SQ_HIP(hipStreamSynchronize(s.sA));
        float fm;
        memcpy(&fm, &mx, sizeof fm);
        out[0] += acc[0];
        out[1] += acc[1];
        out[2] = std::max(out[2], (double)fm);
    }
    return SQ_OK;
}

int sq_get_params(sq_ctx *c, sq_params *out) {
    if (!c || !out) return fail(SQ_E_ARG, "null argument");
    *out = c->p;
    out->deltatau = c->dtau;
    return SQ_OK;
}

int sq_set_dtau(sq_ctx *c, double dtau) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (!(dtau > 0) || !std::isfinite(dtau) || (is_phi4(c) && dtau > 1e20))
        return fail(SQ_E_ARG, "dtau must be finite, > 0 (and <= 1e20 for PHI4: the guard's drift bound)");
    c->dtau = dtau;
    return SQ_OK;
}
int sq_get_dtau(sq_ctx *c, double *dtau) {
    if (!c || !dtau) return fail(SQ_E_ARG, "null argument");
    *dtau = c->dtau;
    return SQ_OK;
}
int sq_get_step(sq_ctx *c, unsigned long long *step) {
    if (!c || !step) return fail(SQ_E_ARG, "null argument");
    *step = c->step;
    return SQ_OK;
}
int sq_set_step(sq_ctx *c, unsigned long long step) {
    if (!c) return fail(SQ_E_ARG, "null context");
    c->step = step;
    return SQ_OK;
}

int sq_correlator(sq_ctx *c, double *out, int n) {
    if (!c || !out || n < 0) return fail(SQ_E_ARG, "bad argument");
    DeviceGuard g(c->dev);
    if (!is_phi4(c)) {
        if (n > c->N) return fail(SQ_E_ARG, "n > N");
        std::vector<double> x(c->N), xx0(c->N);
        int rc = sq_download(c, nullptr, x.data(), xx0.data(), nullptr, nullptr);
        if (rc) return rc;
        const int mid = c->N / 2;
        for (int i = 0; i < n; ++i) out[i] = xx0[i] - x[i] * x[mid];  // tauhost.c:519-521
        return SQ_OK;
    }
    if (n > c->Lz) return fail(SQ_E_ARG, "n > Lz");
    if (c->p.comm == SQ_COMM_P2P && !c->p2p_ready)
        return fail(SQ_E_STATE, "SQ_COMM_P2P context not connected (sq_p2p_connect)");
    int rc = observe_join(c);
    if (rc) return rc;
    // slice sums S(z) of the whole lattice: every slab writes its planes into a
    // zeroed global-length array; across ranks one RCCL sum all-reduce (the
    // per-frame collective of SURVEY.md §8e)
    const long long Lz = c->Lz;
    std::vector<double> S((size_t)Lz, 0.0);
    if (!c->dslice) SQ_HIP(hipMalloc(&c->dslice, sizeof(double) * (size_t)Lz));
    double *d = c->dslice;
    hipStream_t s0 = c->slabs[0].sA;
    hipError_t e = hipMemsetAsync(d, 0, sizeof(double) * (size_t)Lz, s0);
    for (auto &s : c->slabs) {  // one slab: stream order alone, one synchronisation below
        if (e == hipSuccess && s.sA != s0) e = hipStreamSynchronize(s0);
        if (e == hipSuccess) e = sq::phi4_slices_launch(plane0(c, s, c->cur), c->Lx, c->Ly, s.nz, d + s.z0, s.sA);
        if (e == hipSuccess && s.sA != s0) e = hipStreamSynchronize(s.sA);
    }
    if (e == hipSuccess && per_rank(c->p.comm) && c->p.nranks > 1) {
        // disjoint z ranges, zeros elsewhere: the sum is exact in any order
        if (int rc = rank_allreduce(c, d, (size_t)Lz, sq::P2pRed::kSumF64, s0)) return rc;
    }
    if (e == hipSuccess) e = hipMemcpyAsync(S.data(), d, sizeof(double) * (size_t)Lz, hipMemcpyDeviceToHost, s0);
    if (e == hipSuccess) e = hipStreamSynchronize(s0);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    const double vol = (double)c->Lx * c->Ly * (double)Lz;
    for (int t = 0; t < n; ++t) {  // z ascending, the wrap without a modulo per term
        double acc = 0;
        for (long long z = 0; z < Lz - t; ++z) acc += S[z] * S[z + t];
        for (long long z = Lz - t; z < Lz; ++z) acc += S[z] * S[z + t - Lz];
        out[t] = acc / vol;
    }
    return SQ_OK;
}

int sq_set_profiling(sq_ctx *c, int on) {
    if (!c) return fail(SQ_E_ARG, "null context");
    if (on < 0 || on > 2) return fail(SQ_E_ARG, "profiling mode must be 0, 1 or 2");
    int rc = flush_events(c);
    if (rc) return rc;
    c->profiling = on;
    return SQ_OK;
}

int sq_perf(sq_ctx *c, sq_perf_t *out) {
    if (!c || !out) return fail(SQ_E_ARG, "null argument");
    DeviceGuard g(c->dev);
    int rc = flush_events(c);
    if (rc) return rc;
    *out = c->perf;
    return SQ_OK;
}

int sq_perf_reset(sq_ctx *c) {
    if (!c) return fail(SQ_E_ARG, "null context");
    DeviceGuard g(c->dev);
    int rc = flush_events(c);
    if (rc) return rc;
    c->perf = sq_perf_t{};
    c->kstat.clear();
    return SQ_OK;
}

int sq_phi4_launch_info(sq_ctx *c, char *name, size_t cap, long long *grid_threads, long long *launches) {
    if (!c || !name || cap == 0) return fail(SQ_E_ARG, "bad argument");
    if (!is_phi4(c)) return fail(SQ_E_STATE, "PHI4 only");
    name[0] = 0;
    uint64_t best = 0;
    long long n = 0;
    for (const auto &kv : c->kstat)  // most launches; ties: the larger grid (the map is ordered by id)
        if (kv.second > n || (kv.second == n && sq::phi4_kernel_id_grid(kv.first) > sq::phi4_kernel_id_grid(best))) {
            best = kv.first;
            n = kv.second;
        }
    if (n > 0) {
        if ((best & 3) == 3)
            sq::phi4_run_kernel_id_name(best, name, cap);
        else
            sq::phi4_kernel_id_name(best, name, cap);
    }
    if (grid_threads) *grid_threads = n > 0 ? (long long)sq::phi4_kernel_id_grid(best) : 0;
    if (launches) *launches = n;
    return SQ_OK;
}

int sq_set_noise(sq_ctx *c, double C) {
    if (!c) return fail(SQ_E_ARG, "null context");
    // the PHI4 guard fast path bounds |sigma xi| by 16 sqrt(2 dtau) |C| (create_phi4), dtau <= 1e20
    if (!std::isfinite(C) || std::fabs(C) > 1e12) return fail(SQ_E_ARG, "C must be finite, |C| <= 1e12");
    if (is_phi4(c)) {  // create_phi4's bound with the new C at the current dtau
        const double cl = c->p.clamp, h = c->dtau;
        const double drift = 12.0 * cl + std::fabs(c->p.m2) * cl + std::fabs(c->p.lambda) / 6.0 * cl * cl * cl;
        if (!(h * drift + cl + 16.0 * sqrt(2.0 * h) * std::fabs(C) < 1e30))
            return fail(SQ_E_ARG, "C too large for the guard's fast path at this dtau (dtau * drift + noise >= 1e30)");
    }
    c->p.C = C;
    return SQ_OK;
}

int sq_comm_unique_id(unsigned char out[128]) {
    if (!out) return fail(SQ_E_ARG, "null argument");
    ncclUniqueId id;
    SQ_NCCL(ncclGetUniqueId(&id));
    memset(out, 0, 128);
    memcpy(out, id.internal, sizeof(id.internal));
    return SQ_OK;
}

int sq_p2p_handle(sq_ctx *c, unsigned char out[SQ_P2P_HANDLE_BYTES]) {
    if (!c || !out) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c) || c->p.comm != SQ_COMM_P2P) return fail(SQ_E_STATE, "not an SQ_COMM_P2P context");
    DeviceGuard g(c->dev);
    P2pBlob b{};
    b.magic = kP2pMagic;
    b.version = SQ_ABI_VERSION;
    b.rank = c->p.rank;
    b.nranks = c->p.nranks;
    b.Lx = c->Lx;
    b.Ly = c->Ly;
    b.gpad = c->gpad;
    b.loops = c->p.loops;
    b.gz = c->gz;
    b.gauto = c->g_auto ? 1 : 0;
    b.ef_auto = c->ef_auto ? 1 : 0;
    b.k_auto = c->k_auto ? 1 : 0;
    b.edge_first = c->edge_first ? 1 : 0;
    b.core_pairs = c->core_pairs;
    b.rims_b = c->rims_b ? 1 : 0;
    b.a_auto = c->a_auto ? 1 : 0;
    b.on_a = c->xchg_on_a ? 1 : 0;
    b.kstage = c->kstage_env;
    b.Lz = c->Lz;
    b.coll_cap = (long long)c->coll_cap;
    b.seed = c->p.seed;
    SQ_HIP(hipIpcGetMemHandle(&b.stage, c->slabs[0].stage));
    SQ_HIP(hipIpcGetMemHandle(&b.mbox, c->mbox));
    SQ_HIP(hipIpcGetMemHandle(&b.coll, c->coll));
    memset(out, 0, SQ_P2P_HANDLE_BYTES);
    memcpy(out, &b, sizeof b);
    return SQ_OK;
}

int sq_p2p_connect(sq_ctx *c, const unsigned char *handles, int nranks) {
    if (!c || !handles) return fail(SQ_E_ARG, "null argument");
    if (!is_phi4(c) || c->p.comm != SQ_COMM_P2P) return fail(SQ_E_STATE, "not an SQ_COMM_P2P context");
    if (nranks != c->p.nranks) return fail(SQ_E_ARG, "handle count != nranks");
    if (c->p2p_ready && nranks > 1) return fail(SQ_E_STATE, "already connected");
    if (nranks == 1) return SQ_OK;
    std::vector<P2pBlob> bl(nranks);
    for (int q = 0; q < nranks; ++q) {  // validate every blob before mapping anything
        memcpy(&bl[q], handles + (size_t)q * SQ_P2P_HANDLE_BYTES, sizeof(P2pBlob));
        const P2pBlob &b = bl[q];
        if (b.magic != kP2pMagic || b.version != SQ_ABI_VERSION) return fail(SQ_E_ARG, "not a P2P handle blob");
        if (b.rank != q || b.nranks != nranks)
            return fail(SQ_E_ARG, "handle " + std::to_string(q) + " belongs to rank " + std::to_string(b.rank) +
                                      " of " + std::to_string(b.nranks) + " (blobs must be in rank order)");
        if (b.Lx != c->Lx || b.Ly != c->Ly || b.Lz != c->Lz || b.gpad != c->gpad ||
            b.coll_cap != (long long)c->coll_cap || b.seed != c->p.seed)
            return fail(SQ_E_ARG, "rank " + std::to_string(q) + " was created for a different lattice, ghost depth or seed");
        // the exchanges move gz planes and the frame collectives loops records:
        // ranks that disagree would hang in a wait or fold mismatched records
        if (b.loops != c->p.loops || b.gz != c->gz || b.gauto != (c->g_auto ? 1 : 0))
            return fail(SQ_E_ARG, "rank " + std::to_string(q) + " has different loops (" + std::to_string(b.loops) +
                                      "), active ghost depth (" + std::to_string(b.gz) + ") or ghost tuning (SQ_GHOST)");
        if (b.ef_auto != (c->ef_auto ? 1 : 0) || b.k_auto != (c->k_auto ? 1 : 0) ||
            b.edge_first != (c->edge_first ? 1 : 0) || b.core_pairs != c->core_pairs || b.rims_b != (c->rims_b ? 1 : 0) ||
            b.a_auto != (c->a_auto ? 1 : 0) || b.on_a != (c->xchg_on_a ? 1 : 0) || b.kstage != c->kstage_env)
            return fail(SQ_E_ARG, "rank " + std::to_string(q) + " has a different block schedule (SQ_EDGE_FIRST, "
                                      "SQ_CORE_PAIRS, SQ_RIMS_B, SQ_XCHG_ON_A, SQ_P2P_KSTAGE must be set alike on every rank)");
    }
    DeviceGuard g(c->dev);
    for (int q = 0; q < nranks; ++q) {
        if (q == c->p.rank) continue;
        Peer pr{};
        void *a = nullptr, *m = nullptr, *k = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&a, bl[q].stage, hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle(&m, bl[q].mbox, hipIpcMemLazyEnablePeerAccess);
        if (e == hipSuccess) e = hipIpcOpenMemHandle(&k, bl[q].coll, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            for (void *v : {a, m, k})
                if (v) (void)hipIpcCloseMemHandle(v);
            for (Peer &o : c->peers)
                if (o.mapped) {
                    (void)hipIpcCloseMemHandle(o.stage);
                    (void)hipIpcCloseMemHandle(o.mbox);
                    (void)hipIpcCloseMemHandle(o.coll);
                    o = Peer{};
                }
            return fail(SQ_E_COMM, std::string("hipIpcOpenMemHandle (rank ") + std::to_string(q) + "): " +
                                       hipGetErrorString(e));
        }
        pr.stage = static_cast<float *>(a);
        pr.mbox = static_cast<unsigned int *>(m);
        pr.coll = static_cast<unsigned char *>(k);
        pr.mapped = true;
        c->peers[q] = pr;
    }
    c->p2p_ready = true;
    return SQ_OK;
}

int sq_selftest_normals(int device, unsigned long long seed, unsigned int stream,
                        unsigned long long quad0, unsigned long long step, float *out, size_t nquads) {
    if (!out) return fail(SQ_E_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    float *d = nullptr;
    SQ_HIP(hipMalloc(&d, nquads * 4 * sizeof(float)));
    hipError_t e = sq::selftest_normals_launch(d, nquads, quad0, stream, step, (uint32_t)seed,
                                               (uint32_t)(seed >> 32), nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d, nquads * 4 * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_selftest_dpp(int device, float *out64x2) {
    if (!out64x2) return fail(SQ_E_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    float *d = nullptr;
    SQ_HIP(hipMalloc(&d, 128 * sizeof(float)));
    hipError_t e = sq::selftest_dpp_launch(d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out64x2, d, 128 * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_selftest_dpp_mix(int device, int mode, int blocks, int iters, unsigned int *errs64) {
    if (!errs64 || mode < 0 || mode > 3 || blocks < 1 || blocks > 65536 || iters < 1)
        return fail(SQ_E_ARG, "bad dpp_mix arguments");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    unsigned *d = nullptr;
    float *sink = nullptr;
    SQ_HIP(hipMalloc(&d, 64 * sizeof(unsigned)));
    hipError_t e = hipMalloc(&sink, 1024 * sizeof(float));
    if (e == hipSuccess) e = hipMemset(d, 0, 64 * sizeof(unsigned));
    if (e == hipSuccess) e = sq::selftest_dpp_mix_launch(mode, blocks, iters, d, sink, nullptr);
    if (e == hipSuccess) e = hipMemcpy(errs64, d, 64 * sizeof(unsigned), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    (void)hipFree(sink);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_selftest_philox(int device, const unsigned int ctr[4], const unsigned int key[2],
                       unsigned int out[4]) {
    if (!ctr || !key || !out) return fail(SQ_E_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    uint32_t h[6] = {ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]};
    uint32_t *d = nullptr;
    SQ_HIP(hipMalloc(&d, 10 * sizeof(uint32_t)));
    hipError_t e = hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = sq::selftest_philox_launch(d, d + 6, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d + 6, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_selftest_libm(int device, int fn, const float *x, float *y, long long n) {
    if (!x || !y || n < 0 || fn < 0 || fn > 2) return fail(SQ_E_ARG, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    if (n == 0) return SQ_OK;
    DeviceGuard g(device);
    float *d = nullptr;
    SQ_HIP(hipMalloc(&d, 2 * (size_t)n * sizeof(float)));
    hipError_t e = hipMemcpy(d, x, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = sq::selftest_libm_launch(fn, d, d + n, n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(y, d + n, (size_t)n * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_selftest_bm_tables(int device, float *out) {
    if (!out) return fail(SQ_E_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    const size_t bytes = 4 * ((size_t)1 << 23) * sizeof(float);
    float *d = nullptr;
    SQ_HIP(hipMalloc(&d, bytes));
    hipError_t e = sq::selftest_bm_tables_launch(d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_selftest_lcg(int device, unsigned long long seed, int N, int loops, unsigned int *w1,
                    unsigned int *w2, unsigned long long *seeds, double *xi, int generator) {
    if (!w1 || !w2 || !seeds || !xi || N < 1 || loops < 1) return fail(SQ_E_ARG, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    const long long n = (long long)(N + 1) * loops;
    char *d = nullptr;
    SQ_HIP(hipMalloc(&d, (size_t)n * 24 + 8 * sq::kLcgScratch));
    uint32_t *dw1 = (uint32_t *)d, *dw2 = dw1 + n;
    unsigned long long *ds = (unsigned long long *)(dw2 + n);
    double *dx = (double *)(ds + n);
    unsigned long long *scr = generator == 1 ? (unsigned long long *)(dx + n) : nullptr;
    hipError_t e = sq::qm1d_gs_lcg_launch(seed, N, n, dw1, dw2, ds, dx, scr, nullptr);
    if (e == hipSuccess) e = hipMemcpy(w1, dw1, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(w2, dw2, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(seeds, ds, n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(xi, dx, n * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SQ_E_HIP, hipGetErrorString(e));
    return SQ_OK;
}

int sq_copy_bandwidth(int device, size_t bytes, int iters, double *gbps) {
    if (!gbps || iters < 1 || bytes < 1024) return fail(SQ_E_ARG, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SQ_E_NODEV, "no HIP device");
    DeviceGuard g(device);
    const size_t n4 = bytes / 16;
    float4 *a = nullptr, *b = nullptr;
    SQ_HIP(hipMalloc(&a, n4 * 16));
    SQ_HIP(hipMalloc(&b, n4 * 16));
    SQ_HIP(hipMemset(a, 0, n4 * 16));
    hipEvent_t e0, e1;
    SQ_HIP(hipEventCreate(&e0));
    SQ_HIP(hipEventCreate(&e1));
    double best = 0;
    for (int nt = 0; nt < 2; ++nt) {
        SQ_HIP(sq::copy_launch(a, b, n4, nt != 0, nullptr));
        SQ_HIP(hipEventRecord(e0, nullptr));
        for (int i = 0; i < iters; ++i)
            SQ_HIP(sq::copy_launch((i & 1) ? b : a, (i & 1) ? a : b, n4, nt != 0, nullptr));
        SQ_HIP(hipEventRecord(e1, nullptr));
        SQ_HIP(hipEventSynchronize(e1));
        float ms = 0;
        SQ_HIP(hipEventElapsedTime(&ms, e0, e1));
        best = std::max(best, 2.0 * (double)n4 * 16.0 * iters / (ms * 1e-3) / 1e9);
    }
    *gbps = best;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    return SQ_OK;
}

}  // extern "C"
