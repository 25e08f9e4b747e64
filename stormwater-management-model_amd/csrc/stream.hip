// stream.hip -- the achievable HBM bandwidth of this GPU ("measure
// the achievable peak with a STREAM-triad HIP kernel on the box and report
// both"): a[i] = b[i] + s c[i] over fp64 arrays far larger than the 256 MB
// MALL, 16-byte lanes, timed with HIP events around back-to-back launches
// outside any profiler.  bench.py reports it beside the 8 TB/s spec as
// roofline.peak_measured.  Measurement only; no routing state is touched.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/swmm5_mi355x.h"

namespace {

__global__ __launch_bounds__(256) void k_triad(double2* __restrict__ a, const double2* __restrict__ b,
                                               const double2* __restrict__ c, double s, long n2)
{
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const double2 x = b[i], y = c[i];
        a[i] = make_double2(x.x + s * y.x, x.y + s * y.y);
    }
}

__global__ __launch_bounds__(256) void k_copy(double2* __restrict__ a, const double2* __restrict__ b, long n2)
{
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) a[i] = b[i];
}

}  // namespace

// out[0] triad GB/s (best launch), out[1] triad GB/s (average), out[2] copy
// GB/s (best), out[3] bytes per triad launch.  nDoubles per array (even);
// returns 0 or a HIP error code (negated).
extern "C" int DLLEXPORT swmmx_streamTriad(long nDoubles, int reps, double* out)
{
    if (!out || nDoubles < 2 || reps < 1) return -1;
    const long n2 = nDoubles / 2;
    const size_t bytes = (size_t)n2 * sizeof(double2);
    double2 *a = nullptr, *b = nullptr, *c = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    auto ck = [&](hipError_t e) {
        if (e != hipSuccess && !rc) rc = -(int)e;
        return rc == 0;
    };
    int dev = 0, cus = 1;
    if (ck(hipGetDevice(&dev)) && ck(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) &&
        ck(hipMalloc(&a, bytes)) && ck(hipMalloc(&b, bytes)) && ck(hipMalloc(&c, bytes)) &&
        ck(hipStreamCreate(&st)) && ck(hipEventCreate(&e0)) && ck(hipEventCreate(&e1)) &&
        ck(hipMemsetAsync(a, 0, bytes, st)) && ck(hipMemsetAsync(b, 0, bytes, st)) &&
        ck(hipMemsetAsync(c, 0, bytes, st))) {
        // a resident grid of 8 workgroups per CU, grid-stride
        const int grid = 8 * std::max(cus, 1);
        double best = 0.0, sum = 0.0, bestCopy = 0.0;
        hipLaunchKernelGGL(k_triad, dim3(grid), dim3(256), 0, st, a, b, c, 3.0, n2);   // warm-up
        for (int r = 0; r < reps && rc == 0; r++) {
            ck(hipEventRecord(e0, st));
            hipLaunchKernelGGL(k_triad, dim3(grid), dim3(256), 0, st, a, b, c, 3.0, n2);
            ck(hipEventRecord(e1, st));
            ck(hipEventSynchronize(e1));
            float ms = 0.0f;
            ck(hipEventElapsedTime(&ms, e0, e1));
            const double gbs = 3.0 * (double)bytes / (ms * 1e-3) / 1e9;
            best = std::max(best, gbs);
            sum += gbs;
        }
        for (int r = 0; r < reps && rc == 0; r++) {
            ck(hipEventRecord(e0, st));
            hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, st, a, b, n2);
            ck(hipEventRecord(e1, st));
            ck(hipEventSynchronize(e1));
            float ms = 0.0f;
            ck(hipEventElapsedTime(&ms, e0, e1));
            bestCopy = std::max(bestCopy, 2.0 * (double)bytes / (ms * 1e-3) / 1e9);
        }
        out[0] = best;
        out[1] = sum / reps;
        out[2] = bestCopy;
        out[3] = 3.0 * (double)bytes;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (c) (void)hipFree(c);
    return rc;
}
