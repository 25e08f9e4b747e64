// rccl_capture_probe.cpp -- diagnostic: the RCCL call pattern the partitioned
// step graph captures (dw_kernels.hip neighbourExchange / flagExchange), on
// one rank: a group of ncclSend + ncclRecv (here to the rank itself, the only
// peer one device offers) and an ncclAllReduce(max) captured into a HIP graph,
// instantiated once and replayed; every replay's received values and reduced
// flag are checked.  Exit 0 when all replays match.
//   hipcc -O2 -o tools/rccl_capture_probe tools/rccl_capture_probe.cpp -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

static double secs()
{
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            return 2;                                                           \
        }                                                                       \
    } while (0)
#define NK(x)                                                                   \
    do {                                                                        \
        ncclResult_t r_ = (x);                                                  \
        if (r_ != ncclSuccess) {                                                \
            printf("%s: %s\n", #x, ncclGetErrorString(r_));                     \
            return 3;                                                           \
        }                                                                       \
    } while (0)

int main(int argc, char** argv)
{
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int kRep = argc > 1 ? atoi(argv[1]) : 16;
    // teardown order: "graphs" (default) destroys every graph that captured
    // RCCL work before the communicator; "comm" destroys the communicator
    // while the timing graphs still exist (the round-5 order of this probe)
    const bool commFirst = argc > 2 && strcmp(argv[2], "comm") == 0;
    const size_t n = 4 * 2828;                    // a 4M strip boundary: 2 x 1414 links x 4 doubles
    const char* ifn = getenv("NCCL_SOCKET_IFNAME");
    printf("[%.3f s] start: %d repetitions, NCCL_SOCKET_IFNAME=%s\n", secs(), kRep, ifn ? ifn : "(unset)");
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    printf("[%.3f s] unique id (bootstrap root listening)\n", secs());
    ncclComm_t comm;
    NK(ncclCommInitRank(&comm, 1, id, 0));
    printf("[%.3f s] communicator initialised\n", secs());
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    double *snd, *rcv;
    int* flag;
    CK(hipMalloc(&snd, n * sizeof(double)));
    CK(hipMalloc(&rcv, n * sizeof(double)));
    CK(hipMalloc(&flag, sizeof(int)));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    NK(ncclGroupStart());
    NK(ncclSend(snd, n, ncclDouble, 0, comm, s));
    NK(ncclRecv(rcv, n, ncclDouble, 0, comm, s));
    NK(ncclGroupEnd());
    NK(ncclAllReduce(flag, flag, 1, ncclInt32, ncclMax, comm, s));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("[%.3f s] single pattern captured\n", secs());
    std::vector<double> h(n), back(n);
    int bad = 0;
    for (int rep = 0; rep < 50; rep++) {
        for (size_t i = 0; i < n; i++) h[i] = rep * 1.0e6 + (double)i;
        const int fv = rep & 1;
        CK(hipMemcpyAsync(snd, h.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(flag, &fv, sizeof(int), hipMemcpyHostToDevice, s));
        CK(hipMemsetAsync(rcv, 0, n * sizeof(double), s));
        CK(hipGraphLaunch(ge, s));
        int fo = -1;
        CK(hipMemcpyAsync(back.data(), rcv, n * sizeof(double), hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(&fo, flag, sizeof(int), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        for (size_t i = 0; i < n; i++)
            if (back[i] != h[i]) { bad++; break; }
        if (fo != fv) bad++;
    }
    printf("[%.3f s] 50 replays checked: %d mismatches\n", secs(), bad);
    // timing: the pattern, and its two parts alone, each captured kRep times
    // in one graph (the cost inside a graph, as the step graph has it, not
    // that of a graph launch)
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeGraph = [&](hipGraphExec_t x, float* us) -> int {
        for (int rep = 0; rep < 5; rep++) CK(hipGraphLaunch(x, s));
        CK(hipEventRecord(a, s));
        for (int rep = 0; rep < 50; rep++) CK(hipGraphLaunch(x, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        *us = 1000.f * ms / (50 * kRep);
        return 0;
    };
    hipGraph_t gr[3];
    hipGraphExec_t gx[3];
    for (int v = 0; v < 3; v++) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < kRep; r++) {
            if (v != 2) {
                NK(ncclGroupStart());
                NK(ncclSend(snd, n, ncclDouble, 0, comm, s));
                NK(ncclRecv(rcv, n, ncclDouble, 0, comm, s));
                NK(ncclGroupEnd());
            }
            if (v != 1) NK(ncclAllReduce(flag, flag, 1, ncclInt32, ncclMax, comm, s));
        }
        CK(hipStreamEndCapture(s, &gr[v]));
        CK(hipGraphInstantiate(&gx[v], gr[v], nullptr, nullptr, 0));
        printf("[%.3f s] variant %d captured (%d repetitions)\n", secs(), v, kRep);
    }
    float tAll = 0.f, tX = 0.f, tF = 0.f;
    if (timeGraph(gx[2], &tF)) return 2;
    printf("all-reduce alone timed\n");
    if (timeGraph(gx[1], &tX)) return 2;
    printf("send/recv alone timed\n");
    if (timeGraph(gx[0], &tAll)) return 2;
    printf("captured send/recv (%zu doubles) + all-reduce, 50 checked replays: %d mismatches\n", n, bad);
    printf("inside a graph, per occurrence: both %.2f us, send/recv alone %.2f us, all-reduce alone %.2f us\n", tAll, tX, tF);
    printf("[%.3f s] teardown (%s first)\n", secs(), commFirst ? "communicator" : "graphs");
    if (commFirst) {
        ncclCommDestroy(comm);
        printf("[%.3f s] communicator destroyed\n", secs());
    }
    for (int v = 0; v < 3; v++) {
        (void)hipGraphExecDestroy(gx[v]);
        (void)hipGraphDestroy(gr[v]);
    }
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    printf("[%.3f s] graphs destroyed\n", secs());
    if (!commFirst) {
        ncclCommDestroy(comm);
        printf("[%.3f s] communicator destroyed\n", secs());
    }
    return bad ? 1 : 0;
}
