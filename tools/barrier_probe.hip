// tools/barrier_probe.hip -- diagnostic only (not part of the engine).
// What a phase boundary costs on this GPU, for the design of the compacted
// Picard iterations k >= 2:
//  (a) a kernel boundary inside a captured graph (R back-to-back launches of
//      a small phase kernel),
//  (b) a grid barrier inside one persistent launch with agent-scope
//      release / acquire fences (buffer_wbl2 sc1 / buffer_inv sc1 on gfx950),
//  (c) a forked side kernel joined two phases later (a concurrent graph
//      branch, e.g. for the outfall depths),
// each phase writing F bytes of "compact state" (spread over the grid) and
// reading another workgroup's values of the previous phase (so the data
// really crosses workgroups / XCDs, and is checked).
//   hipcc --offload-arch=gfx950 -O3 barrier_probe.hip -o barrier_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Ctl {
    unsigned bar;
    int err;
};

// one phase: thread t (of nthr) owns doubles [t*per, (t+1)*per) of one half
// of buf (phases alternate halves); it reads the values another workgroup's
// thread wrote in the previous phase (other half) and writes its own, value =
// phase + index
__device__ __forceinline__ int phaseWork(double* buf, int per, int nthr, int tid, int r)
{
    int bad = 0;
    if (per == 0) return 0;
    const size_t half = (size_t)per * nthr;
    const double* in = buf + ((r + 1) & 1) * half;
    double* out = buf + (r & 1) * half;
    const int src = (tid + 64 * 37 + 1) % nthr;           // another workgroup
    for (int q = 0; q < per; q++) {
        const size_t i = (size_t)src * per + q;
        const double v = in[i];
        if (r > 0 && v != (double)(r - 1) + (double)i) bad++;
    }
    for (int q = 0; q < per; q++) {
        const size_t i = (size_t)tid * per + q;
        out[i] = (double)r + (double)i;
    }
    return bad;
}

__device__ __forceinline__ void gridBarrier(Ctl* c, unsigned target)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(&c->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(&c->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) { c->err = 1; break; }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__global__ void k_persist(Ctl* c, double* buf, int per, int rounds, int* bad)
{
    const int nthr = gridDim.x * blockDim.x, tid = blockIdx.x * blockDim.x + threadIdx.x;
    int b = 0;
    unsigned target = 0;
    for (int r = 0; r < rounds; r++) {
        b += phaseWork(buf, per, nthr, tid, r);
        target += gridDim.x;
        gridBarrier(c, target);
    }
    if (b) atomicAdd(bad, b);
}

__global__ void k_phase(double* buf, int per, int r, int* bad)
{
    const int nthr = gridDim.x * blockDim.x, tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = phaseWork(buf, per, nthr, tid, r);
    if (b) atomicAdd(bad, b);
}

// (c) fork/join inside a captured graph: a main chain of `rounds` phase
// kernels, and a side kernel per phase forked after main phase i (on a second
// stream) and joined before main phase i + 2 -- what a concurrent branch costs
__global__ void k_side(double* buf, int r, int* bad)
{
    if (threadIdx.x == 0 && blockIdx.x == 0 && buf[r & 1023] < -1.0) atomicAdd(bad, 1);
}

static int forkJoin(hipStream_t s, hipStream_t s2, double* buf, int* bad, int wgs, int per, int rounds, float* msOut,
                    bool withSide)
{
    std::vector<hipEvent_t> fork(rounds), join(rounds);
    for (int r = 0; r < rounds; r++) {
        CK(hipEventCreateWithFlags(&fork[r], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&join[r], hipEventDisableTiming));
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < rounds; r++) {
        if (withSide && r >= 2) CK(hipStreamWaitEvent(s, join[r - 2], 0));
        hipLaunchKernelGGL(k_phase, dim3(wgs), dim3(256), 0, s, buf, per, r, bad);
        if (withSide) {
            CK(hipEventRecord(fork[r], s));
            CK(hipStreamWaitEvent(s2, fork[r], 0));
            hipLaunchKernelGGL(k_side, dim3(1), dim3(64), 0, s2, buf, r, bad);
            CK(hipEventRecord(join[r], s2));
        }
    }
    if (withSide)
        for (int r = rounds - 2; r < rounds; r++) CK(hipStreamWaitEvent(s, join[r], 0));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
    }
    *msOut = best;
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return 0;
}

int main()
{
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    printf("CUs %d\n", cus);
    Ctl* c;
    double* buf;
    int* bad;
    const size_t maxBytes = 128ull << 20;      // two halves
    CK(hipMalloc(&c, sizeof(Ctl)));
    CK(hipMalloc(&buf, maxBytes));
    CK(hipMalloc(&bad, sizeof(int)));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = 64;
    const int blockSz = 256;
    {
        hipStream_t s2;
        CK(hipStreamCreate(&s2));
        for (int wgs : {64, 256}) {
            float a = 0, b = 0;
            if (forkJoin(s, s2, buf, bad, wgs, 4, rounds, &a, false) || forkJoin(s, s2, buf, bad, wgs, 4, rounds, &b, true))
                return 1;
            printf("graph chain of %d phases (%d wgs): %.2f us/phase; with a forked side kernel per phase joined two "
                   "phases later: %.2f us/phase\n", rounds, wgs, 1000.0f * a / rounds, 1000.0f * b / rounds);
            fflush(stdout);
        }
    }
    for (int wgs : {8, 32, 64, 128, 256}) {
        for (size_t foot : {(size_t)0, (size_t)256 << 10, (size_t)2 << 20, (size_t)16 << 20}) {
            const int nthr = wgs * blockSz;
            const int per = (int)(foot / 8 / nthr);
            if (foot && per == 0) continue;
            // (b) persistent launch with grid barriers
            float msP = 1e30f;
            int hbad = 0;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipMemsetAsync(c, 0, sizeof(Ctl), s));
                CK(hipMemsetAsync(bad, 0, sizeof(int), s));
                CK(hipEventRecord(e0, s));
                hipLaunchKernelGGL(k_persist, dim3(wgs), dim3(blockSz), 0, s, c, buf, per, rounds, bad);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < msP) msP = ms;
                int b = 0;
                CK(hipMemcpy(&b, bad, sizeof(int), hipMemcpyDeviceToHost));
                hbad += b;
            }
            Ctl hc;
            CK(hipMemcpy(&hc, c, sizeof(Ctl), hipMemcpyDeviceToHost));
            // (a) the same phases as a captured graph of launches
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int r = 0; r < rounds; r++)
                hipLaunchKernelGGL(k_phase, dim3(wgs), dim3(blockSz), 0, s, buf, per, r, bad);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            float msG = 1e30f;
            int gbad = 0;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipMemsetAsync(bad, 0, sizeof(int), s));
                CK(hipEventRecord(e0, s));
                CK(hipGraphLaunch(ge, s));
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < msG) msG = ms;
                int b = 0;
                CK(hipMemcpy(&b, bad, sizeof(int), hipMemcpyDeviceToHost));
                gbad += b;
            }
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
            printf("wgs %4d footprint %6zu KB: persistent %.2f us/phase (bad %d, err %d) | graph %.2f us/phase (bad %d)\n",
                   wgs, foot >> 10, 1000.0f * msP / rounds, hbad, hc.err, 1000.0f * msG / rounds, gbad);
            fflush(stdout);
        }
    }
    return 0;
}
