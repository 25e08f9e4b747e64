// tools/outfall_latency.hip -- single-thread latency probe of the root finders
// used by link_setOutfallDepth (normal + critical depth of a circular conduit).
// Diagnostic only; not part of the engine.  Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../stormwater-management-model_amd/csrc
//         outfall_latency.hip -o outfall_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include "xsect.h"
using namespace swx;

__global__ void probe(const double* tables, const double* qs, int n, double* out, long long* cyc)
{
    __shared__ double ct[5 * SWX_CIRC_N];
    for (int i = threadIdx.x; i < 5 * SWX_CIRC_N; i += blockDim.x) ct[i] = tables[i];
    __syncthreads();
    if (threadIdx.x != 0) return;
    Geom x{};
    x.type = G_CIRCULAR;
    x.yFull = 8.0; x.wMax = 8.0; x.ywMax = 4.0;
    x.aFull = 3.141592654 / 4.0 * 64.0;
    x.rFull = 2.0;
    x.sFull = x.aFull * pow(x.rFull, 2. / 3.);
    x.sMax = 1.08 * x.sFull;
    double beta = 1.486 / 0.013 * sqrt(0.002);
    for (int i = 0; i < n; i++) {
        double q = qs[i];
        long long t0 = clock64();
        double s = q / beta;
        double a = getAofS(x, s, ct);
        long long t1 = clock64();
        double yn = getYofA(x, a, ct);
        long long t2 = clock64();
        double yc = getYcrit(x, q, ct);
        long long t3 = clock64();
        out[3 * i] = a; out[3 * i + 1] = yn; out[3 * i + 2] = yc;
        cyc[3 * i] = t1 - t0; cyc[3 * i + 1] = t2 - t1; cyc[3 * i + 2] = t3 - t2;
    }
}

int main()
{
    const int n = 8;
    double hq[n] = {0.01, 0.1, 0.5, 1.0, 2.0, 5.0, 20.0, 100.0};
    double *dq, *dout, *dt;
    long long* dc;
    (void)hipMalloc(&dq, sizeof hq); (void)hipMalloc(&dout, 3 * n * 8); (void)hipMalloc(&dc, 3 * n * 8);
    (void)hipMalloc(&dt, sizeof SWX_CIRC_TABLES);
    (void)hipMemcpy(dq, hq, sizeof hq, hipMemcpyHostToDevice);
    (void)hipMemcpy(dt, SWX_CIRC_TABLES, sizeof SWX_CIRC_TABLES, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; rep++) {
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dt, dq, n, dout, dc);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
        double ho[3 * n]; long long hc[3 * n];
        (void)hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
        (void)hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        printf("rep %d kernel %.1f us\n", rep, ms * 1000);
        for (int i = 0; i < n; i++)
            printf("q=%7.2f  AofS %6lld cyc  YofA %6lld cyc  Ycrit %6lld cyc   (a=%.4g yn=%.4g yc=%.4g)\n", hq[i],
                   hc[3 * i], hc[3 * i + 1], hc[3 * i + 2], ho[3 * i], ho[3 * i + 1], ho[3 * i + 2]);
    }
    return 0;
}
