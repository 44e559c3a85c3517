// tauhost.cpp -- drop-in replacement for the reference executable tauhost.o
// (tauhost.c, built by `gcc tauhost.c -o tauhost.o -lOpenCL`, README.md:8),
// driven unchanged by taumain.py:132:
//
//   ./tauhost.o N dt dtau frames potID C dev fps inTime loops startFile endFile endAccuracy
//
// Same positional arguments (tauhost.c:31-43), same initial state from the
// unseeded glibc rand() (:84-102), same start-file parser (:103-173), same
// stdout frame line (:485-501), same end file (:562-581) and the same error
// messages / exit code 1 (:105-107,564-566).  The OpenCL set-up and the
// per-frame kernel/read-back/rollback (:187-560) are one sq_run_frame() call
// on the MI355X.  Differences, all documented in DESIGN.md: `dev` is a HIP
// device ordinal (taken modulo the device count, since taumain.py hard-codes
// the OpenCL platform index 2); no tau_kernel.cl is read from the cwd; the
// kernel runs the reference's own serial order (Gauss-Seidel sweep, its
// shared-seed LCG seeded from the same rand() draw, :185; SQ_ORDER_SERIAL in
// stochquant.h) for N <= 4096, and the Jacobi order with Philox noise keyed by
// that draw above (SQ_ORDER=jacobi forces it; SQ_SEED overrides the key).
// SQ_MODEL=phi4 (+ SQ_SHAPE, SQ_M2, SQ_LAMBDA) runs the 3-D lattice behind the
// same arguments (run_phi4 below).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/stochquant.h"

namespace {

std::chrono::steady_clock::time_point t_start;
constexpr int kSerialMaxN = 4096;  // SQ_ORDER_SERIAL's limit (sq_qm1d_set_ordering)

double absol(double v) { return v <= 0 ? -v : v; }

// tauhost.c:103-173: lines split at '\n', tokens at '|'; line i < N holds
// xavg|xx0|x|f, line N (omega) is ignored, line N+1 the recorded length,
// line N+2 the last Δτ (capped at argv Δτ).
bool read_start(const char *path, int N, double deltatau, std::vector<double> &xavg,
                std::vector<double> &xx0, std::vector<double> &x, std::vector<double> &f,
                int &recSimlgth, double &dtautmp) {
    FILE *fp = fopen(path, "r");
    if (!fp) return false;
    std::string line;
    int i = 0, ch;
    while ((ch = fgetc(fp)) != EOF) {
        if (ch != '\n') {
            line.push_back((char)ch);
            continue;
        }
        std::vector<char> buf(line.begin(), line.end());
        buf.push_back('\0');
        char *tok;
        if (i == N + 1) {
            tok = strtok(buf.data(), "|");
            recSimlgth = tok ? atoi(tok) : 0;
        } else if (i == N + 2) {
            tok = strtok(buf.data(), "|");
            dtautmp = tok ? atof(tok) : 0;
            if (dtautmp > deltatau) dtautmp = deltatau;
        } else if (i < N) {
            double *dst[4] = {&xavg[i], &xx0[i], &x[i], &f[i]};
            tok = strtok(buf.data(), "|");
            for (int k = 0; k < 4; ++k) {
                *dst[k] = tok ? atof(tok) : 0;
                tok = strtok(nullptr, "|");
            }
        }
        line.clear();
        ++i;
    }
    fclose(fp);
    return true;
}

int die(const char *what, sq_ctx *ctx) {
    fprintf(stderr, "tauhost: %s: %s\n", what, sq_last_error());
    if (ctx) sq_destroy(ctx);
    return 1;
}

// SQ_PERF_JSON=<path>: one JSON perf record per run (SURVEY.md §5 "Metrics"):
// steps, site updates, time inside the frames, the rate, final Δτ.
void write_perf(sq_ctx *ctx, const char *model, int frames, double wall_s) {
    const char *path = getenv("SQ_PERF_JSON");
    if (!path) return;
    sq_perf_t pf;
    double dt = 0;
    if (sq_perf(ctx, &pf) != SQ_OK || sq_get_dtau(ctx, &dt) != SQ_OK) return;
    FILE *fp = fopen(path, "w");
    if (!fp) return;
    const double s = pf.frame_ms * 1e-3;
    fprintf(fp,
            "{\"model\": \"%s\", \"frames\": %d, \"steps\": %lld, \"site_updates\": %lld, "
            "\"frame_seconds\": %.6f, \"wall_seconds\": %.6f, \"site_updates_per_s\": %.6g, "
            "\"deltatau_final\": %.17g}\n",
            model, frames, pf.steps, pf.site_updates, s, wall_s, s > 0 ? (double)pf.site_updates / s : 0.0, dt);
    fclose(fp);
}

double env_double(const char *name, double dflt) {
    const char *s = getenv(name);
    return s ? atof(s) : dflt;
}

// SQ_MODEL=phi4: the 3-D north-star lattice behind the same 13 arguments
// (SURVEY.md §5 "Config / flag system": extensions via env).  Shape from
// SQ_SHAPE=LxxLyxLz (default N x N x N), V = m2/2 phi^2 + lambda/24 phi^4
// from SQ_M2 / SQ_LAMBDA (default 1, 1); deltat and potID are unused (a = 1).
// The printed line is the analogue of the reference's log|xavg| (the running
// connected correlator of its chain, tauhost.c:485-501,519-521): the running
// mean over stable frames of the zero-momentum time-slice correlator,
// connected, log|C(t)| for t = 1..Lz-1, then Δτ and the percentage, in the
// reference's formats, so taumain.py parses and plots it unchanged.
// startFile / endFile are binary checkpoints (sq_load_field / sq_save_field:
// <file> .npy + <file>.json); a resumed Δτ is capped at argv Δτ (:131-136).
int run_phi4(int N, double deltatau, int frames, double C, int dev, int fps, int loops,
             const char *startFile, const char *endFile, unsigned long long seed) {
    long long L[3] = {N, N, N};
    if (const char *sh = getenv("SQ_SHAPE")) {
        if (sscanf(sh, "%lldx%lldx%lld", &L[0], &L[1], &L[2]) != 3) {
            fprintf(stderr, "tauhost: SQ_SHAPE must be LxxLyxLz\n");
            return 1;
        }
    }
    sq_params p;
    sq_params_init(&p);
    p.model = SQ_MODEL_PHI4;
    for (int k = 0; k < 3; ++k) p.dims[k] = L[k];
    p.deltatau = deltatau;
    p.C = C;
    p.loops = loops;
    p.seed = seed;
    p.device = dev;
    p.m2 = env_double("SQ_M2", 1.0);
    p.lambda = env_double("SQ_LAMBDA", 1.0);
    p.adapt_dtau = 1;
    sq_ctx *ctx = nullptr;
    if (sq_create(&p, &ctx) != SQ_OK) return die("sq_create", nullptr);
    if (strcmp(startFile, "0") == 0) {
        if (sq_init_field(ctx, (float)sqrt(2. * deltatau)) != SQ_OK) return die("sq_init_field", ctx);  // as :91-100
    } else {
        if (sq_load_field(ctx, startFile, 1) != SQ_OK) {
            fprintf(stderr, "Failed to read Input.\n");
            sq_destroy(ctx);
            return 1;
        }
        double d = 0;
        sq_get_dtau(ctx, &d);
        if (d > deltatau) sq_set_dtau(ctx, deltatau);
    }
    const int Lz = (int)L[2];
    const double V = (double)L[0] * (double)L[1] * (double)L[2];
    std::vector<double> corr(Lz), cbar(Lz, 0.0);
    double sbar = 0;  // running mean of the slice sum S(z)
    long nstable = 0;
    double dtautmp = 0;
    sq_get_dtau(ctx, &dtautmp);
    for (int j = 0; j < frames; ++j) {
        if (j % fps == 0) {
            for (int t = 1; t < Lz; ++t) {
                printf(" % -.20f |", log(absol(cbar[t] - (double)Lz * sbar * sbar / V)));
                if (t == Lz - 1) {
                    printf("% -.20f | ", dtautmp);
                    printf("% -.2f\n", 100. * ((double)j + 1) / (double)frames);
                }
            }
        }
        int stable = 0;
        if (sq_run_frame(ctx, &stable) != SQ_OK) return die("sq_run_frame", ctx);
        if (stable == 1) {
            double m[3];
            if (sq_correlator(ctx, corr.data(), Lz) != SQ_OK) return die("sq_correlator", ctx);
            if (sq_moments(ctx, m) != SQ_OK) return die("sq_moments", ctx);
            ++nstable;
            for (int t = 0; t < Lz; ++t) cbar[t] += (corr[t] - cbar[t]) / (double)nstable;
            sbar += (m[0] / Lz - sbar) / (double)nstable;
        }
        sq_get_dtau(ctx, &dtautmp);
        fflush(stdout);
    }
    if (strcmp(endFile, "0") != 0 && sq_save_field(ctx, endFile) != SQ_OK) {
        fprintf(stderr, "Failed to write to Output.\n");
        sq_destroy(ctx);
        return 1;
    }
    write_perf(ctx, "phi4", frames,
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
    sq_destroy(ctx);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    t_start = std::chrono::steady_clock::now();
    if (argc < 14) {
        fprintf(stderr,
                "usage: %s N deltat deltatau frames potID C dev fps inTime loops startFile|0 "
                "endFile|0 endAccuracy\n",
                argv[0]);
        return 1;
    }
    const int N = atoi(argv[1]);
    const double deltat = atof(argv[2]);
    const double deltatau = atof(argv[3]);
    const int frames = atoi(argv[4]);
    const int potID = atoi(argv[5]);
    const double C = atof(argv[6]);
    int dev = atoi(argv[7]);
    const int fps = atoi(argv[8]);
    const int loops = atoi(argv[10]);
    const char *startFile = argv[11];
    const char *endFile = argv[12];
    const int endAccuracy = atoi(argv[13]);
    if (N < 2 || fps < 1 || loops < 1 || frames < 0) {
        fprintf(stderr, "tauhost: need N >= 2, fps >= 1, loops >= 1\n");
        return 1;
    }
    if (const char *m = getenv("SQ_MODEL")) {
        if (strcmp(m, "phi4") == 0) {
            unsigned long long seed = (unsigned long long)abs(rand());
            if (const char *s = getenv("SQ_SEED")) seed = strtoull(s, nullptr, 0);
            int ndev = 0;
            sq_device_count(&ndev);
            if (ndev < 1) {
                fprintf(stderr, "tauhost: no HIP device\n");
                return 1;
            }
            if (const char *s = getenv("SQ_DEVICE")) dev = atoi(s);
            dev = ((dev % ndev) + ndev) % ndev;
            return run_phi4(N, deltatau, frames, C, dev, fps, loops, startFile, endFile, seed);
        }
        if (strcmp(m, "qm1d") != 0) {
            fprintf(stderr, "tauhost: SQ_MODEL must be qm1d or phi4\n");
            return 1;
        }
    }
    const int midpt = N / 2;
    int recSimlgth = 0;
    double dtautmp = deltatau;
    std::vector<double> f(N, 0.0), x(N, 0.0), xx0(N, 0.0), xavg(N, 0.0);

    double v1 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);  // :84-89
    double v2 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
    double omega = sqrt(2. * deltatau) * sin(2. * 3.14 * v2) * sqrt(-2. * log(v1)) + deltat * (double)(N / 2);
    while (omega > N * deltat) omega -= deltat;

    if (strcmp(startFile, "0") == 0) {  // :91-102
        for (int i = 0; i < N; ++i) {
            v1 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
            v2 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
            f[i] = sqrt(2. * deltatau) * cos(2. * 3.14 * v2) * sqrt(-2. * log(v1));
        }
    } else if (!read_start(startFile, N, deltatau, xavg, xx0, x, f, recSimlgth, dtautmp)) {
        fprintf(stderr, "Failed to read Input.\n");
        return 1;
    }
    unsigned long long seed = (unsigned long long)abs(rand());  // :185
    if (const char *s = getenv("SQ_SEED")) seed = strtoull(s, nullptr, 0);

    int ndev = 0;
    sq_device_count(&ndev);
    if (ndev < 1) {
        fprintf(stderr, "tauhost: no HIP device\n");
        return 1;
    }
    if (const char *s = getenv("SQ_DEVICE")) dev = atoi(s);
    dev = ((dev % ndev) + ndev) % ndev;

    sq_params p;
    sq_params_init(&p);
    p.model = SQ_MODEL_QM1D;
    p.dims[0] = N;
    p.deltat = deltat;
    p.deltatau = dtautmp;
    p.pot = potID;
    p.C = C;
    p.loops = loops;
    p.seed = seed;
    p.device = dev;
    p.adapt_dtau = 1;
    sq_ctx *ctx = nullptr;
    if (sq_create(&p, &ctx) != SQ_OK) return die("sq_create", nullptr);
    // The reference's own serial order (its Gauss-Seidel sweep and shared-seed
    // LCG, seeded from the same rand() draw as the reference, tauhost.c:185) is
    // the default wherever it is supported (N <= 4096, every taumain.py preset):
    // it reproduces the reference's trajectory (to 1 ulp of its float
    // transcendentals) and is also the faster frame at those sizes (DESIGN.md
    // §4.1).  Larger chains (config C1's 32,768 sites) and SQ_ORDER=jacobi run
    // the Jacobi / Philox frame.
    bool serial = N <= kSerialMaxN;
    if (const char *o = getenv("SQ_ORDER")) {
        if (strcmp(o, "serial") == 0) {
            serial = true;
        } else if (strcmp(o, "jacobi") == 0) {
            serial = false;
        } else {
            fprintf(stderr, "tauhost: SQ_ORDER must be jacobi or serial\n");
            sq_destroy(ctx);
            return 1;
        }
    }
    if (serial) {
        if (sq_qm1d_set_ordering(ctx, SQ_ORDER_SERIAL) != SQ_OK) return die("sq_qm1d_set_ordering", ctx);
        if (sq_qm1d_set_lcg_seed(ctx, seed) != SQ_OK) return die("sq_qm1d_set_lcg_seed", ctx);
    }
    if (sq_upload(ctx, f.data(), x.data(), xx0.data(), omega, recSimlgth) != SQ_OK)
        return die("sq_upload", ctx);

    long runs = recSimlgth;  // :477
    for (int j = 0; j < frames; ++j) {
        if (j % fps == 0) {  // :485-501 (prints the xavg of the last stable frame)
            for (int i = 1; i < N; ++i) {
                printf(" % -.20f |", log(absol(xavg[i])));
                if (i == N - 1) {
                    printf("% -.20f | ", dtautmp);
                    printf("% -.2f\n", 100. * ((double)j + 1) / (double)frames);
                }
            }
        }
        int stable = 0;
        if (sq_run_frame(ctx, &stable) != SQ_OK) return die("sq_run_frame", ctx);
        if (stable == 1) {  // :506-532
            if (sq_download(ctx, f.data(), x.data(), xx0.data(), &omega, &runs) != SQ_OK)
                return die("sq_download", ctx);
            for (int i = 0; i < N; ++i) xavg[i] = (xx0[i] - x[i] * x[midpt]);
        }
        sq_get_dtau(ctx, &dtautmp);
        fflush(stdout);
    }
    if (strcmp(endFile, "0") != 0) {  // :562-581
        FILE *fp = fopen(endFile, "w");
        if (!fp) {
            fprintf(stderr, "Failed to write to Output.\n");
            sq_destroy(ctx);
            return 1;
        }
        for (int i = 0; i < N; ++i) {
            fprintf(fp, "% -*a| % -*a| % -*a| % -*a", endAccuracy, xavg[i], endAccuracy, xx0[i],
                    endAccuracy, x[i], endAccuracy, f[i]);
            fprintf(fp, "\n");
        }
        fprintf(fp, "% -*a|omega\n", endAccuracy, omega);
        fprintf(fp, "%*d|N\n", endAccuracy, (int)(runs + recSimlgth));  // double count kept
        fprintf(fp, "% -*e|deltaTau\n", endAccuracy, dtautmp);
        fclose(fp);
    }
    write_perf(ctx, "qm1d", frames,
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
    sq_destroy(ctx);
    return 0;
}
