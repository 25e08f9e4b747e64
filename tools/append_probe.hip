// tools/append_probe.hip -- diagnostic only (not part of the engine).
// What does appending ~4,000 scattered nodes to one list cost in a kernel that
// scans 500k nodes (k_node's unconverged list at Picard iterations k >= 2)?
//   mode 0: no list (scan only)
//   mode 1: one returning agent-scope atomicAdd per wave that has listed nodes
//           (the engine's waveAppend)
//   mode 2: one atomicAdd per workgroup (LDS aggregation first)
//   mode 3: no atomics: each 256-node chunk writes its own segment and count
//   hipcc --offload-arch=gfx950 -O3 append_probe.hip -o append_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <random>
#include <vector>

constexpr int kBlock = 256;

template <int kMode>
__global__ __launch_bounds__(kBlock) void k_scan(const unsigned char* mark, int n, int* count, int* list,
                                                 int* segCount)
{
    __shared__ int wbase[kBlock / 64 + 1];
    const int nthr = gridDim.x * kBlock;
    for (int base = blockIdx.x * kBlock; base < n; base += nthr) {
        const int i = base + threadIdx.x;
        const bool me = i < n && mark[i];
        const unsigned long long m = __ballot(me);
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        if (kMode == 1) {
            if (m) {
                int leader = __ffsll((long long)m) - 1, b = 0;
                if (lane == leader) b = atomicAdd(count, __popcll(m));
                b = __shfl(b, leader, 64);
                if (me) list[b + __popcll(m & ((1ull << lane) - 1ull))] = i;
            }
        } else if (kMode == 2 || kMode == 3) {
            if (lane == 0) wbase[w] = __popcll(m);
            __syncthreads();
            if (threadIdx.x == 0) {
                int s = 0;
                for (int x = 0; x < kBlock / 64; x++) { int c = wbase[x]; wbase[x] = s; s += c; }
                wbase[kBlock / 64] = s;
                if (kMode == 2) wbase[kBlock / 64] = s ? atomicAdd(count, s) : 0;
                else segCount[base / kBlock] = s;
            }
            __syncthreads();
            const int off = (kMode == 2) ? wbase[kBlock / 64] : base;
            if (me) list[off + wbase[w] + __popcll(m & ((1ull << lane) - 1ull))] = i;
            __syncthreads();
        }
    }
}

int main()
{
    const int n = 499850;
    int *count, *list, *seg;
    unsigned char* mark;
    (void)hipMalloc(&count, 64);
    (void)hipMalloc(&list, n * sizeof(int));
    (void)hipMalloc(&seg, (n / kBlock + 1) * sizeof(int));
    (void)hipMalloc(&mark, n);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::mt19937 rng(7);
    for (int listed : {0, 1000, 4200, 20000}) {
        for (int pattern = 0; pattern < 2; pattern++) {     // 0 scattered, 1 clustered (a square of the 707 grid)
            std::vector<unsigned char> h(n, 0);
            if (pattern == 0) {
                for (int c = 0; c < listed;) { int i = rng() % n; if (!h[i]) { h[i] = 1; c++; } }
            } else {
                int side = 1; while (side * side < listed) side++;
                for (int c = 0, r = 300; c < listed; r++)
                    for (int x = 300; x < 300 + side && c < listed; x++, c++) h[r * 707 + x] = 1;
            }
            (void)hipMemcpy(mark, h.data(), n, hipMemcpyHostToDevice);
            for (int mode = 0; mode < 4; mode++) {
                for (int grid : {1024, 2048}) {
                    float sum = 0;
                    const int reps = 30;
                    for (int r = 0; r < reps; r++) {
                        (void)hipMemset(count, 0, 64);
                        switch (mode) {
                        case 0: hipExtLaunchKernelGGL(k_scan<0>, dim3(grid), dim3(kBlock), 0, 0, a, b, 0, mark, n, count, list, seg); break;
                        case 1: hipExtLaunchKernelGGL(k_scan<1>, dim3(grid), dim3(kBlock), 0, 0, a, b, 0, mark, n, count, list, seg); break;
                        case 2: hipExtLaunchKernelGGL(k_scan<2>, dim3(grid), dim3(kBlock), 0, 0, a, b, 0, mark, n, count, list, seg); break;
                        case 3: hipExtLaunchKernelGGL(k_scan<3>, dim3(grid), dim3(kBlock), 0, 0, a, b, 0, mark, n, count, list, seg); break;
                        }
                        (void)hipEventSynchronize(b);
                        float ms;
                        (void)hipEventElapsedTime(&ms, a, b);
                        if (r >= 5) sum += ms;
                    }
                    printf("listed %6d %-9s mode %d grid %4d: %6.2f us\n", listed, pattern ? "clustered" : "scattered",
                           mode, grid, 1000.f * sum / (reps - 5));
                }
            }
        }
    }
    return 0;
}
