/*
 * orc_tauhost.c -- restatement of the reference host program tauhost.c main()
 * (TEST INFRASTRUCTURE ONLY, see sq_oracle.h) with the OpenCL device replaced
 * by the serial restatement of time_dev (orc_serial_launch).
 *
 * Mirrors, in order: argv parsing tauhost.c:31-43; initial state from the
 * unseeded glibc rand() :84-102; start-file parser :103-173; state copies and
 * shared seed :177-185; frame loop with print / stable read-back / Δτ
 * adaptation / rollback :479-560; end file :562-581.  The OpenCL plumbing
 * (:187-453) has no observable effect under a serialising runtime and is
 * omitted.  Known reference quirks are kept on purpose: the omega line of the
 * start file is ignored (:122-124), N in the end file is runs+recSimlgth
 * (double count, :577), lrgEl/lrgVl/newf/seed are never rolled back.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "sq_oracle.h"

static double absol(double v) { return v <= 0 ? -v : v; }

/* Start-file parser, tauhost.c:103-173 (line-by-line, tokens split at '|'). */
static int read_start_file(const char *path, int N, double deltatau, double *xavg, double *xx0,
                           double *x, double *f, int *recSimlgth, double *dtautmp)
{
    FILE *fp = fopen(path, "r");
    if (!fp) return -1;
    char *buf = NULL;
    size_t len = 0, cap = 0;
    int i = 0, ch;
    while ((ch = fgetc(fp)) != EOF) {
        if (ch == '\n') {
            char *line = (char *)malloc(len + 1);
            memcpy(line, buf, len);
            line[len] = 0;
            char *tok;
            if (i == N + 1) { tok = strtok(line, "|"); *recSimlgth = tok ? atoi(tok) : 0; }
            if (i == N + 2) {
                tok = strtok(line, "|");
                *dtautmp = tok ? atof(tok) : 0;
                if (*dtautmp > deltatau) *dtautmp = deltatau;
            }
            if (i < N) {
                tok = strtok(line, "|"); xavg[i] = tok ? atof(tok) : 0;
                tok = strtok(NULL, "|"); xx0[i] = tok ? atof(tok) : 0;
                tok = strtok(NULL, "|"); x[i] = tok ? atof(tok) : 0;
                tok = strtok(NULL, "|"); f[i] = tok ? atof(tok) : 0;
            }
            free(line);
            len = 0;
            ++i;
        } else {
            if (len + 1 > cap) { cap = cap ? 2 * cap : 64; buf = (char *)realloc(buf, cap); }
            buf[len++] = (char)ch;
        }
    }
    free(buf);
    fclose(fp);
    return 0;
}

int orc_tauhost_main(int argc, const char **argv, FILE *out)
{
    if (argc < 14) { fprintf(stderr, "usage: tauhost N dt dtau frames potID C dev fps inTime loops start end acc\n"); return 2; }
    const int N = atoi(argv[1]);
    const double deltat = atof(argv[2]);
    const double deltatau = atof(argv[3]);
    const int frames = atoi(argv[4]);
    const int potID = atoi(argv[5]);
    const double C = atof(argv[6]);
    const int fps = atoi(argv[8]);
    const int loops = atoi(argv[10]);
    const char *startFile = argv[11];
    const char *endFile = argv[12];
    const int endAccuracy = atoi(argv[13]);
    const int midpt = N / 2;
    int recSimlgth = 0;
    double dtautmp = deltatau;

    double *f = (double *)calloc((size_t)N, sizeof(double));
    double *x = (double *)calloc((size_t)N, sizeof(double));
    double *xx0 = (double *)calloc((size_t)N, sizeof(double));
    double *xavg = (double *)calloc((size_t)N, sizeof(double));
    double *nf = (double *)calloc((size_t)N, sizeof(double));
    double *nx = (double *)calloc((size_t)N, sizeof(double));
    double *nxx0 = (double *)calloc((size_t)N, sizeof(double));

    /* :84-89 */
    double v1 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
    double v2 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
    double omega = sqrt(2. * deltatau) * sin(2. * 3.14 * v2) * sqrt(-2. * log(v1)) + deltat * (double)(N / 2);
    while (omega > N * deltat) omega -= deltat;

    if (strcmp(startFile, "0") == 0) {                            /* :91-102 */
        for (int i = 0; i < N; ++i) {
            v1 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
            v2 = (double)(rand() + 1.) / ((double)(RAND_MAX) + 1.);
            f[i] = sqrt(2. * deltatau) * cos(2. * 3.14 * v2) * sqrt(-2. * log(v1));
            xavg[i] = 0;
        }
        recSimlgth = 0;
    } else if (read_start_file(startFile, N, deltatau, xavg, xx0, x, f, &recSimlgth, &dtautmp) != 0) {
        fprintf(stderr, "Failed to read Input.\n");
        return 1;
    }
    for (int i = 0; i < N; ++i) { nf[i] = f[i]; nx[i] = x[i]; nxx0[i] = xx0[i]; }   /* :177-183 */

    orc_serial_dev d;
    memset(&d, 0, sizeof d);
    d.N = N; d.pot = potID; d.loops = loops; d.a = deltat; d.c = C;
    d.seed = (uint64_t)abs(rand());                                /* :185 */
    d.stable = 1; d.dtau = dtautmp; d.lrgEl = 0; d.lrgVl = 0; d.runs = recSimlgth;
    d.f = (double *)malloc(sizeof(double) * N); d.x = (double *)malloc(sizeof(double) * N);
    d.xx0 = (double *)malloc(sizeof(double) * N); d.nf = (double *)malloc(sizeof(double) * N);
    d.nx = (double *)malloc(sizeof(double) * N); d.nxx0 = (double *)malloc(sizeof(double) * N);
    memcpy(d.f, f, sizeof(double) * N); memcpy(d.x, x, sizeof(double) * N);
    memcpy(d.xx0, xx0, sizeof(double) * N); memcpy(d.nf, nf, sizeof(double) * N);
    memcpy(d.nx, nx, sizeof(double) * N); memcpy(d.nxx0, nxx0, sizeof(double) * N);
    d.omega = omega;

    int stabCnt = 0;
    int runs = recSimlgth;                                          /* :477 */
    for (int j = 0; j < frames; ++j) {
        orc_serial_launch(&d);                                      /* :481-483 */
        for (int i = 0; i < N; ++i) {                               /* :485-501 */
            if (i != 0 && j % fps == 0) {
                fprintf(out, " % -.20f |", log(absol(xavg[i])));
                if (i == N - 1) {
                    fprintf(out, "% -.20f | ", dtautmp);
                    fprintf(out, "% -.2f\n", 100. * ((double)j + 1) / (double)frames);
                }
            }
        }
        if (d.stable == 1) {                                        /* :504-532 */
            memcpy(f, d.nf, sizeof(double) * N);
            memcpy(x, d.nx, sizeof(double) * N);
            memcpy(xx0, d.nxx0, sizeof(double) * N);
            omega = d.omega;
            for (int i = 0; i < N; ++i) xavg[i] = (xx0[i] - x[i] * x[midpt]);
            if (stabCnt > 10) { stabCnt = 0; dtautmp /= 0.950; d.dtau = dtautmp; }
            stabCnt++;
            runs += loops;
        } else {                                                    /* :533-545 */
            dtautmp = d.dtau;
            dtautmp *= 0.950;
            stabCnt = 0;
            d.dtau = dtautmp;
            d.stable = 1;
        }
        memcpy(d.f, f, sizeof(double) * N);                         /* :550-554 */
        memcpy(d.x, x, sizeof(double) * N);
        memcpy(d.xx0, xx0, sizeof(double) * N);
        d.omega = omega;
        d.runs = runs;
        fflush(out);
    }
    int rc = 0;
    if (strcmp(endFile, "0") != 0) {                                /* :562-581 */
        FILE *fp = fopen(endFile, "w");
        if (!fp) { fprintf(stderr, "Failed to write to Output.\n"); rc = 1; }
        else {
            for (int i = 0; i < N; ++i) {
                fprintf(fp, "% -*a| % -*a| % -*a| % -*a", endAccuracy, xavg[i], endAccuracy, xx0[i],
                        endAccuracy, x[i], endAccuracy, f[i]);
                fprintf(fp, "\n");
            }
            fprintf(fp, "% -*a|omega\n", endAccuracy, omega);
            fprintf(fp, "%*d|N\n", endAccuracy, runs + recSimlgth);
            fprintf(fp, "% -*e|deltaTau\n", endAccuracy, dtautmp);
            fclose(fp);
        }
    }
    free(f); free(x); free(xx0); free(xavg); free(nf); free(nx); free(nxx0);
    free(d.f); free(d.x); free(d.xx0); free(d.nf); free(d.nx); free(d.nxx0);
    return rc;
}
