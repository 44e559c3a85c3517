// Feasibility probe for a peer-pointer (IPC) halo transport between two
// processes: IPC export of device and signal memory, cross-process stream
// write/wait of a flag, and D2D copies from a peer's buffer.  Usage:
//   ipc_probe <dir>      (forks two ranks before any HIP call)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/wait.h>
#include <thread>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "rank %d: %s -> %s\n", rank, #x, hipGetErrorString(e_)); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

struct Handles {
    hipIpcMemHandle_t buf, sig, plain;
};

static bool wait_file(const std::string &p, void *out, size_t n) {
    for (int i = 0; i < 20000; ++i) {
        FILE *f = fopen(p.c_str(), "rb");
        if (f) {
            size_t r = fread(out, 1, n, f);
            fclose(f);
            if (r == n) return true;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return false;
}

static int run(int rank, const std::string &dir) {
    const size_t n = 4 << 20;
    int dev = 0;
    CK(hipSetDevice(dev));
    int can = -1;
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev));
    printf("rank %d: CanUseStreamWaitValue = %d\n", rank, can);
    float *buf;
    CK(hipMalloc(&buf, n));
    std::vector<float> h(n / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i * 3 + rank);
    CK(hipMemcpy(buf, h.data(), n, hipMemcpyHostToDevice));
    void *sig = nullptr, *plain = nullptr;
    hipError_t em = hipExtMallocWithFlags(&sig, 8, hipMallocSignalMemory);
    printf("rank %d: signal memory (8 B): %s\n", rank, hipGetErrorString(em));
    if (em != hipSuccess) sig = nullptr;
    CK(hipMalloc(&plain, 4096));
    if (sig) CK(hipMemset(sig, 0, 8));
    CK(hipMemset(plain, 0, 4096));
    Handles mine{};
    CK(hipIpcGetMemHandle(&mine.buf, buf));
    hipError_t es = sig ? hipIpcGetMemHandle(&mine.sig, sig) : hipErrorInvalidValue;
    printf("rank %d: IPC export of signal memory: %s\n", rank, hipGetErrorString(es));
    CK(hipIpcGetMemHandle(&mine.plain, plain));
    {
        std::string tmp = dir + "/h" + std::to_string(rank) + ".tmp", fin = dir + "/h" + std::to_string(rank) + ".bin";
        FILE *f = fopen(tmp.c_str(), "wb");
        fwrite(&mine, sizeof mine, 1, f);
        fclose(f);
        rename(tmp.c_str(), fin.c_str());
    }
    Handles peer{};
    if (!wait_file(dir + "/h" + std::to_string(1 - rank) + ".bin", &peer, sizeof peer)) {
        fprintf(stderr, "rank %d: no peer handles\n", rank);
        return 1;
    }
    void *pbuf = nullptr, *psig = nullptr, *pplain = nullptr;
    CK(hipIpcOpenMemHandle(&pbuf, peer.buf, hipIpcMemLazyEnablePeerAccess));
    if (es == hipSuccess) {
        hipError_t eo = hipIpcOpenMemHandle(&psig, peer.sig, hipIpcMemLazyEnablePeerAccess);
        printf("rank %d: IPC open of peer signal memory: %s\n", rank, hipGetErrorString(eo));
        if (eo != hipSuccess) psig = nullptr;
    }
    CK(hipIpcOpenMemHandle(&pplain, peer.plain, hipIpcMemLazyEnablePeerAccess));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

    // 1. copy the peer's buffer and check it
    float *dst;
    CK(hipMalloc(&dst, n));
    CK(hipMemcpyAsync(dst, pbuf, n, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
    std::vector<float> got(n / 4);
    CK(hipMemcpy(got.data(), dst, n, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < got.size(); ++i) bad += got[i] != (float)(i * 3 + (1 - rank));
    printf("rank %d: peer copy mismatches = %zu\n", rank, bad);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 200; ++i) CK(hipMemcpyAsync(dst, pbuf, n, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 200;
    printf("rank %d: 4 MiB peer-pointer copy %.1f us (%.1f GB/s)\n", rank, us, n / us / 1e3);

    // 2. ping-pong through flags: write the peer's flag, wait on our own
    for (int mode = 0; mode < 2; ++mode) {
        void *own = mode == 0 ? sig : plain;
        void *rem = mode == 0 ? psig : pplain;
        if (!rem || !own) {
            printf("rank %d: mode %d skipped\n", rank, mode);
            continue;
        }
        const int iters = 2000;
        auto a = std::chrono::steady_clock::now();
        for (int i = 1; i <= iters; ++i) {
            if (rank == 0) {
                CK(hipStreamWriteValue32(st, rem, (uint32_t)i, 0));
                CK(hipStreamWaitValue32(st, own, (uint32_t)i, hipStreamWaitValueGte, 0xFFFFFFFFu));
            } else {
                CK(hipStreamWaitValue32(st, own, (uint32_t)i, hipStreamWaitValueGte, 0xFFFFFFFFu));
                CK(hipStreamWriteValue32(st, rem, (uint32_t)i, 0));
            }
        }
        CK(hipStreamSynchronize(st));
        double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count() / iters;
        printf("rank %d: %s flags: round trip %.2f us\n", rank, mode == 0 ? "signal" : "plain", rt);
        CK(hipMemsetAsync(own, 0, 4, st));
        CK(hipStreamSynchronize(st));
        // both ranks reset before the next mode
        std::string p = dir + "/m" + std::to_string(mode) + "_" + std::to_string(rank);
        FILE *f = fopen(p.c_str(), "wb");
        fwrite(&mode, 4, 1, f);
        fclose(f);
        int dummy;
        if (!wait_file(dir + "/m" + std::to_string(mode) + "_" + std::to_string(1 - rank), &dummy, 4)) return 1;
    }
    CK(hipIpcCloseMemHandle(pbuf));
    if (psig) CK(hipIpcCloseMemHandle(psig));
    CK(hipIpcCloseMemHandle(pplain));
    printf("rank %d: done\n", rank);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    std::string dir = argv[1];
    pid_t kids[2];
    for (int r = 0; r < 2; ++r) {
        kids[r] = fork();
        if (kids[r] == 0) {
            fflush(stdout);
            int rc = run(r, dir);
            fflush(stdout);
            _exit(rc);
        }
    }
    int rc = 0;
    for (int r = 0; r < 2; ++r) {
        int s = 0;
        waitpid(kids[r], &s, 0);
        if (!WIFEXITED(s) || WEXITSTATUS(s) != 0) rc = 1;
    }
    printf("probe rc=%d\n", rc);
    return rc;
}
