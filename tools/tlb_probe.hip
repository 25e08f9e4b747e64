// tools/tlb_probe.hip -- diagnostic only (not part of the engine).
// A sparse Picard iteration touches a few thousand scattered nodes and links,
// each reading ~30 separate SoA arrays.  Does touching many arrays (pages)
// per item cost more than the same number of loads from one array?
//   mode 0: R dependent rounds, each 32 loads at one random index from 32 arrays
//   mode 1: R dependent rounds, each 32 loads at 32 random indices of array 0
//   mode 2: R dependent rounds, each 32 loads at 32 adjacent indices of array 0
//   mode 3: R dependent rounds, each 1 load (array 0)
// Active items: one lane in every `stride` threads of a 2048 x 256 grid.
//   hipcc --offload-arch=gfx950 -O3 tlb_probe.hip -o tlb_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <vector>

constexpr int kArrays = 32;
constexpr int kN = 1 << 20;          // doubles per array (8 MB)

struct Arrs { const double* a[kArrays]; };

__device__ __forceinline__ unsigned hashu(unsigned x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int kMode>
__global__ __launch_bounds__(256) void k_probe(Arrs A, int rounds, int stride, double* out)
{
    const unsigned tid = blockIdx.x * 256 + threadIdx.x;
    if (tid % stride) return;
    unsigned idx = hashu(tid) % kN;
    double acc = 0.0;
    for (int r = 0; r < rounds; r++) {
        double s = 0.0;
        if (kMode == 0) {
#pragma unroll
            for (int a = 0; a < kArrays; a++) s += A.a[a][idx];
        } else if (kMode == 1) {
#pragma unroll
            for (int a = 0; a < kArrays; a++) s += A.a[0][hashu(idx + a) % kN];
        } else if (kMode == 2) {
#pragma unroll
            for (int a = 0; a < kArrays; a++) s += A.a[0][(idx + a) % kN];
        } else {
            s = A.a[0][idx];
        }
        acc += s;
        idx = hashu(idx + (unsigned)(s != 12345.0)) % kN;     // next round depends on this one
    }
    out[tid] = acc;
}

int main()
{
    Arrs A;
    std::vector<double> h(kN, 1.0);
    for (int a = 0; a < kArrays; a++) {
        double* p;
        (void)hipMalloc(&p, kN * sizeof(double));
        (void)hipMemcpy(p, h.data(), kN * sizeof(double), hipMemcpyHostToDevice);
        A.a[a] = p;
    }
    double* out;
    (void)hipMalloc(&out, 2048 * 256 * sizeof(double));
    // a large buffer streamed between launches, so the probe's lines are not L2-resident
    double* big;
    const size_t nb = (size_t)512 << 20;
    (void)hipMalloc(&big, nb);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int stride : {128, 32}) {
        for (int rounds : {1, 4}) {
            for (int mode = 0; mode < 4; mode++) {
                float sum = 0;
                const int reps = 12;
                for (int r = 0; r < reps; r++) {
                    (void)hipMemsetAsync(big, r, nb, 0);
                    switch (mode) {
                    case 0: hipExtLaunchKernelGGL(k_probe<0>, dim3(2048), dim3(256), 0, 0, e0, e1, 0, A, rounds, stride, out); break;
                    case 1: hipExtLaunchKernelGGL(k_probe<1>, dim3(2048), dim3(256), 0, 0, e0, e1, 0, A, rounds, stride, out); break;
                    case 2: hipExtLaunchKernelGGL(k_probe<2>, dim3(2048), dim3(256), 0, 0, e0, e1, 0, A, rounds, stride, out); break;
                    case 3: hipExtLaunchKernelGGL(k_probe<3>, dim3(2048), dim3(256), 0, 0, e0, e1, 0, A, rounds, stride, out); break;
                    }
                    (void)hipEventSynchronize(e1);
                    float ms;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    if (r >= 2) sum += ms;
                }
                printf("items %6d rounds %d mode %d: %7.2f us\n", 2048 * 256 / stride, rounds, mode,
                       1000.f * sum / (reps - 2));
            }
        }
    }
    return 0;
}
