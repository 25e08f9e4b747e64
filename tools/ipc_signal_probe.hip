// tools/ipc_signal_probe.hip -- diagnostic only (not part of the engine).
// What the IPC transport's per-Picard-iteration signalling costs (DESIGN.md
// section 6), without the routing kernels around it.  Two "ranks" exchange
// exactly what the engine's exchange kernels exchange -- G ghost granules
// ({seq << 32 | payload}, 8-byte system-scope stores into the peer's
// uncached region, polled with system-scope loads) and one flag granule per
// rank -- inside captured HIP graphs of N iterations each, launched on both
// ranks at once.  Per iteration:
//   base : work, work, bump           (no waits: the launch floor)
//   flag : work, work, flag           (the convergence-flag exchange alone)
//   split: work, post, wait, work, flag   (the engine's k_ipc_pack / k_ipc_unpack / k_ipc_flag)
//   fused: work, xchg, work, flag     (pack and unpack in one launch)
//   fold : work, xchg, work+flag      (the flag posted and awaited by the
//                                      node pass's last workgroup)
// The cost of the signalling is (variant - base) / N per iteration.
//
//   thread mode (default, `ipc_signal_probe thread G`): one process, the two ranks on two HIP streams of
//     one device (concurrent hardware queues of one process);
//   proc mode: `ipc_signal_probe proc R DIR [G]` for R = 0, 1 started together,
//     two processes on the same device, regions exchanged through
//     hipIpcGetMemHandle / hipIpcOpenMemHandle (files in DIR), as the engine
//     does with one process per rank.
// Every wait is bounded (2 s): a failed variant reports "timeout", never hangs.
//   hipcc --offload-arch=gfx950 -O3 ipc_signal_probe.hip -o ipc_signal_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned long long u64;
constexpr int kBlock = 256;
constexpr long long kDeadline = 200000000LL;      // wall_clock64 ticks (100 MHz): 2 s

struct Side {
    u64* mine;      // this rank's region: [ghost granules | flag granule]
    u64* peer;      // the other rank's region (same layout)
    unsigned* ctl;  // [0] exchange number, [1] failure
    int* work;
};

__device__ __forceinline__ u64 ld(const u64* w) { return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void st(u64* w, unsigned seq, unsigned v)
{
    __hip_atomic_store(w, ((u64)seq << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ bool waitSeq(const u64* w, unsigned seq, unsigned* ctl)
{
    const u64 t0 = wall_clock64();
    for (unsigned it = 0;; it++) {
        if ((unsigned)(ld(w) >> 32) == seq) return true;
        if ((it & 15) == 15 && (long long)(wall_clock64() - t0) > kDeadline) {
            ctl[1] = 1;
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
__global__ void k_work(Side s) { if (threadIdx.x == 0) s.work[blockIdx.x] += 1; }
__global__ void k_post(Side s, int G)
{
    const unsigned seq = s.ctl[0] + 1;
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < G; g += gridDim.x * kBlock) st(s.peer + g, seq, (unsigned)g);
}
__global__ void k_wait(Side s, int G)
{
    const unsigned seq = s.ctl[0] + 1;
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < G; g += gridDim.x * kBlock)
        if (!waitSeq(s.mine + g, seq, s.ctl)) return;
}
__global__ void k_xchg(Side s, int G)
{
    const unsigned seq = s.ctl[0] + 1;
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < G; g += gridDim.x * kBlock) st(s.peer + g, seq, (unsigned)g);
    for (int g = blockIdx.x * kBlock + threadIdx.x; g < G; g += gridDim.x * kBlock)
        if (!waitSeq(s.mine + g, seq, s.ctl)) return;
}
// one wave: post the flag, wait for the peer's, advance the exchange number
__global__ void k_flag(Side s, int G)
{
    const unsigned seq = s.ctl[0] + 1;
    if (threadIdx.x == 0) {
        st(s.peer + G, seq, 1u);
        if (waitSeq(s.mine + G, seq, s.ctl)) s.ctl[0] = seq;
    }
}
__global__ void k_bump(Side s) { if (threadIdx.x == 0) s.ctl[0] += 1; }
// the node pass with the flag folded in: every workgroup does its work; the
// last one to finish (a device-scope arrival count) posts the flag and waits
// for the peer's -- one waiting workgroup, no launch of its own
__global__ void k_work_flag(Side s, int G)
{
    __shared__ int last;
    if (threadIdx.x == 0) s.work[blockIdx.x] += 1;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(&s.ctl[2], 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    s.ctl[2] = 0;
    const unsigned seq = s.ctl[0] + 1;
    st(s.peer + G, seq, 1u);
    if (waitSeq(s.mine + G, seq, s.ctl)) s.ctl[0] = seq;
}

enum { V_BASE, V_FLAG, V_SPLIT, V_FUSED, V_FOLD, V_COUNT };
static const char* kName[V_COUNT] = {"base", "flag", "split", "fused", "fold"};

static hipGraphExec_t capture(hipStream_t st, const Side& s, int v, int N, int G, int grid)
{
    hipGraph_t g;
    hipGraphExec_t x;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; i++) {
        hipLaunchKernelGGL(k_work, dim3(grid), dim3(kBlock), 0, st, s);
        if (v == V_SPLIT) {
            hipLaunchKernelGGL(k_post, dim3(grid), dim3(kBlock), 0, st, s, G);
            hipLaunchKernelGGL(k_wait, dim3(grid), dim3(kBlock), 0, st, s, G);
        } else if (v == V_FUSED || v == V_FOLD) {
            hipLaunchKernelGGL(k_xchg, dim3(grid), dim3(kBlock), 0, st, s, G);
        }
        if (v == V_FOLD) {
            hipLaunchKernelGGL(k_work_flag, dim3(grid), dim3(kBlock), 0, st, s, G);
            continue;
        }
        hipLaunchKernelGGL(k_work, dim3(grid), dim3(kBlock), 0, st, s);
        if (v == V_BASE) hipLaunchKernelGGL(k_bump, dim3(1), dim3(64), 0, st, s);
        else hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, s, G);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    return x;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// proc mode helpers: publish this rank's handle, read the peer's
static void publish(const char* dir, int r, const hipIpcMemHandle_t& h)
{
    std::string tmp = std::string(dir) + "/h" + std::to_string(r) + ".tmp", fin = std::string(dir) + "/h" + std::to_string(r) + ".bin";
    FILE* f = fopen(tmp.c_str(), "wb");
    fwrite(&h, sizeof h, 1, f);
    fclose(f);
    rename(tmp.c_str(), fin.c_str());
}
static bool fetch(const char* dir, int r, hipIpcMemHandle_t* h)
{
    std::string fin = std::string(dir) + "/h" + std::to_string(r) + ".bin";
    for (int t = 0; t < 1000; t++) {
        FILE* f = fopen(fin.c_str(), "rb");
        if (f) {
            bool ok = fread(h, sizeof *h, 1, f) == 1;
            fclose(f);
            if (ok) return true;
        }
        usleep(10000);
    }
    return false;
}
// a file barrier between the two processes (before each timed variant)
static bool fileBarrier(const char* dir, int r, int k)
{
    std::string me = std::string(dir) + "/b" + std::to_string(r) + "_" + std::to_string(k);
    std::string other = std::string(dir) + "/b" + std::to_string(1 - r) + "_" + std::to_string(k);
    FILE* f = fopen(me.c_str(), "w");
    if (f) fclose(f);
    for (int t = 0; t < 2000; t++) {
        if (access(other.c_str(), F_OK) == 0) return true;
        usleep(1000);
    }
    return false;
}

int main(int argc, char** argv)
{
    setvbuf(stdout, nullptr, _IONBF, 0);
    const bool proc = argc > 1 && strcmp(argv[1], "proc") == 0;
    const int rank = proc && argc > 2 ? atoi(argv[2]) : 0;
    const char* dir = proc && argc > 3 ? argv[3] : "/tmp";
    const int N = 50, reps = 20;
    // ghost granules per rank per exchange; default a 4M strip boundary:
    // 2828 links x 4 values x 2 granules (thread mode: argv[2]; proc: argv[4])
    const int G = proc ? (argc > 4 ? atoi(argv[4]) : 4 * 2 * 2828) : (argc > 2 ? atoi(argv[2]) : 4 * 2 * 2828);
    const int grid = 64;
    const int nr = proc ? 1 : 2;                  // ranks driven by this process
    Side s[2];
    hipStream_t st[2];
    u64* region[2] = {nullptr, nullptr};
    const size_t bytes = (size_t)(G + 64) * 8;
    for (int r = 0; r < 2; r++) {
        if (proc && r != rank) continue;
        CK(hipExtMallocWithFlags((void**)&region[r], bytes, hipDeviceMallocUncached));
        CK(hipMemset(region[r], 0, bytes));
    }
    if (proc) {
        hipIpcMemHandle_t h, hp;
        CK(hipIpcGetMemHandle(&h, region[rank]));
        publish(dir, rank, h);
        if (!fetch(dir, 1 - rank, &hp)) { printf("rank %d: no peer handle\n", rank); return 1; }
        void* p = nullptr;
        CK(hipIpcOpenMemHandle(&p, hp, hipIpcMemLazyEnablePeerAccess));
        region[1 - rank] = (u64*)p;
    }
    for (int i = 0; i < nr; i++) {
        const int r = proc ? rank : i;
        s[i].mine = region[r];
        s[i].peer = region[1 - r];
        CK(hipMalloc(&s[i].ctl, 64));
        CK(hipMemset(s[i].ctl, 0, 64));
        CK(hipMalloc(&s[i].work, grid * sizeof(int)));
        CK(hipMemset(s[i].work, 0, grid * sizeof(int)));
        CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    }
    CK(hipDeviceSynchronize());
    printf("mode %s%s: %d iterations per graph, %d ghost granules per rank per exchange, grid %d x %d\n",
           proc ? "proc rank " : "thread", proc ? std::to_string(rank).c_str() : "", N, G, grid, kBlock);
    double us[V_COUNT] = {0, 0, 0, 0, 0};
    int barrierNo = 0;
    for (int v = 0; v < V_COUNT; v++) {
        hipGraphExec_t x[2];
        for (int i = 0; i < nr; i++) x[i] = capture(st[i], s[i], v, N, G, grid);
        double best = 1e30;
        bool failed = false;
        for (int rep = 0; rep < reps + 3 && !failed; rep++) {
            if (proc && !fileBarrier(dir, rank, barrierNo++)) { printf("rank %d: peer lost\n", rank); return 1; }
            const double t0 = now();
            for (int i = 0; i < nr; i++) CK(hipGraphLaunch(x[i], st[i]));
            for (int i = 0; i < nr; i++) CK(hipStreamSynchronize(st[i]));
            const double t = now() - t0;
            unsigned c[2];
            for (int i = 0; i < nr; i++) {
                CK(hipMemcpy(c, s[i].ctl, 8, hipMemcpyDeviceToHost));
                if (c[1]) failed = true;
            }
            if (rep >= 3) best = std::min(best, t);
        }
        for (int i = 0; i < nr; i++) CK(hipGraphExecDestroy(x[i]));
        us[v] = failed ? -1.0 : 1e6 * best / N;
        if (failed) printf("  %-5s timeout (a wait reached its 2 s deadline)\n", kName[v]);
        else printf("  %-5s %8.2f us per iteration (best of %d graph launches)\n", kName[v], us[v], reps);
        if (failed) break;
    }
    if (us[V_BASE] > 0)
        for (int v = 1; v < V_COUNT; v++)
            if (us[v] > 0) printf("  signalling cost, %-5s: %6.2f us per iteration\n", kName[v], us[v] - us[V_BASE]);
    for (int i = 0; i < nr; i++) CK(hipStreamDestroy(st[i]));
    if (proc) CK(hipIpcCloseMemHandle(region[1 - rank]));
    return 0;
}
