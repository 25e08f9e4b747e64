// pmc_calib.hip -- calibration of the FETCH_SIZE / WRITE_SIZE counters on gfx950
// for the access widths the routing kernels use (8-byte fp64 per lane).
//
// Three kernels with exactly known HBM traffic, each launched 5 times:
//   k_read8   every lane loads one double per grid-stride round   (N*8 bytes read)
//   k_read16  every lane loads one double2                        (N*8 bytes read)
//   k_write8  every lane stores one double                        (N*8 bytes written)
// N = 2^28 doubles = 2 GiB per buffer (far above the 256 MiB Infinity Cache), so
// every byte comes from / goes to HBM.  The per-dispatch counter value divided
// by N*8 is the correction factor bench.py applies to the engine's kernels.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -o run -- ./tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_read8(const double* __restrict__ x, size_t n, double* out)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += x[i];
    if (s == 12345.678) out[blockIdx.x] = s;   // never true: keeps the loads, writes nothing
}
__global__ __launch_bounds__(256) void k_read16(const double2* __restrict__ x, size_t n2, double* out)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        double2 v = x[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_write8(double* __restrict__ x, size_t n)
{
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) x[i] = (double)i;
}

int main()
{
    const size_t n = (size_t)1 << 28;
    double *a = nullptr, *o = nullptr;
    if (hipMalloc(&a, n * sizeof(double)) != hipSuccess || hipMalloc(&o, 65536 * sizeof(double)) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 0, n * sizeof(double));
    const int grid = 256 * 8;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[3] = {"k_read8", "k_read16", "k_write8"};
    for (int k = 0; k < 3; k++) {
        float ms = 0.f;
        for (int r = 0; r < 5; r++) {
            (void)hipEventRecord(e0, 0);
            if (k == 0) hipLaunchKernelGGL(k_read8, dim3(grid), dim3(256), 0, 0, a, n, o);
            if (k == 1) hipLaunchKernelGGL(k_read16, dim3(grid), dim3(256), 0, 0, (const double2*)a, n / 2, o);
            if (k == 2) hipLaunchKernelGGL(k_write8, dim3(grid), dim3(256), 0, 0, a, n);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            ms += t;
        }
        printf("%s: %zu bytes per launch, %.1f us avg, %.0f GB/s\n", names[k], n * 8, 1000.0 * ms / 5,
               n * 8 / (ms / 5 * 1e-3) / 1e9);
    }
    (void)hipFree(a);
    (void)hipFree(o);
    return 0;
}
