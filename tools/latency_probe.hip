// tools/latency_probe.hip -- diagnostic only (not part of the engine).
// Calibrates what a short Picard iteration (a few thousand conduits or nodes)
// can cost on this GPU: the duration of an empty kernel at the engine's grid
// sizes, and the latency of one dependent global load (pointer chase over a
// 256 MB random cycle, i.e. out of L2 and mostly out of the MALL).
//   hipcc --offload-arch=gfx950 -O3 latency_probe.hip -o latency_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

__global__ void k_empty(int* sink)
{
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 1;
}

__global__ void k_chase(const int* next, int hops, int start, int* out)
{
    if (threadIdx.x != 0) return;
    int i = start + blockIdx.x * 977;
    for (int h = 0; h < hops; h++) i = next[i];
    out[blockIdx.x] = i;
}

static float timed(void (*launch)(hipEvent_t, hipEvent_t), int reps)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; r++) {
        launch(a, b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        sum += ms;
        if (ms < best) best = ms;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return 1000.0f * sum / reps;
}

static int* gSink;
static int* gNext;
static int gGrid, gHops;

int main()
{
    (void)hipMalloc(&gSink, 1 << 20);
    for (int grid : {1, 256, 768, 1024, 2048, 4096}) {
        gGrid = grid;
        float us = timed([](hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL(k_empty, dim3(gGrid), dim3(256), 0, 0, a, b, 0, gSink);
        }, 50);
        printf("empty kernel, %5d blocks of 256: %.2f us (kernel execution, ext events)\n", grid, us);
    }
    const int n = 64 << 20;                           // 64M ints = 256 MB
    std::vector<int> perm(n);
    std::iota(perm.begin(), perm.end(), 0);
    std::mt19937 rng(20250215);
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<int> next(n);
    for (int i = 0; i < n; i++) next[perm[i]] = perm[(i + 1) % n];
    (void)hipMalloc(&gNext, (size_t)n * sizeof(int));
    (void)hipMemcpy(gNext, next.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice);
    for (int hops : {1, 8, 64}) {
        for (int grid : {1, 256}) {
            gHops = hops;
            gGrid = grid;
            float us = timed([](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL(k_chase, dim3(gGrid), dim3(64), 0, 0, a, b, 0, (const int*)gNext, gHops, 12345,
                                      gSink);
            }, 20);
            printf("pointer chase, %2d dependent loads, %3d blocks: %.2f us\n", hops, grid, us);
        }
    }
    return 0;
}
