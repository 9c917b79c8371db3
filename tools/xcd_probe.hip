// xcd_probe.hip -- does an XCD-contiguous block->tile mapping help the
// double-sum K=2 combine at large nreduce (TLB reach per XCD)?  Not part of
// the product.  Build: hipcc --offload-arch=gfx950 -O3 xcd_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int B = 256, U = 4;

// REMAP 0: tile = blockIdx.x (the shipped kernel); 1: the 8 XCDs (blocks
// are dealt round-robin, blockIdx.x % 8) each stream one contiguous eighth
template <int REMAP>
__global__ __launch_bounds__(B) void k(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    size_t tile = blockIdx.x;
    if (REMAP) tile = (size_t) (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
    size_t t = tile * (B * U) + threadIdx.x;
    if (t + (size_t) (U - 1) * B < nv) {
        d2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = __builtin_nontemporal_load(a + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) y[u] = __builtin_nontemporal_load(b + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) __builtin_nontemporal_store(x[u] + y[u], out + t + u * B);
    }
}

template <int REMAP>
static double run(d2 *o, d2 *a, d2 *b, size_t nv, int reps)
{
    const size_t grid = nv / (B * U);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < reps + 3; r++) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k<REMAP>, dim3((unsigned) grid), dim3(B), 0, 0, o, a, b, nv);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2] * 1e3;
}

__global__ void fill(double *p, size_t n, double v)
{
    for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t) gridDim.x * blockDim.x)
        p[i] = v + (double) (i & 1023) * 1e-3;
}

int main()
{
    for (int lg = 24; lg <= 28; lg++) {
        const size_t n = (size_t) 1 << lg, nv = n / 2;
        for (int trial = 0; trial < 2; trial++) {
            double *a, *b, *o;
            CHK(hipMalloc(&a, n * 8));
            CHK(hipMalloc(&b, n * 8));
            CHK(hipMalloc(&o, n * 8));
            hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a, n, 1.0);
            hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, n, 2.0);
            hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, o, n, 0.0);
            CHK(hipDeviceSynchronize());
            const double bytes = 3.0 * n * 8;
            for (int rep = 0; rep < 2; rep++) {
                double t0 = run<0>((d2 *) o, (d2 *) a, (d2 *) b, nv, 15);
                double t1 = run<1>((d2 *) o, (d2 *) a, (d2 *) b, nv, 15);
                printf("{\"nreduce_log2\": %d, \"trial\": %d, \"tile_us\": %.1f, \"tile_frac\": %.4f, "
                       "\"xcd_us\": %.1f, \"xcd_frac\": %.4f}\n", lg, trial, t0,
                       bytes / (t0 * 1e-6) / 8e12, t1, bytes / (t1 * 1e-6) / 8e12);
                fflush(stdout);
            }
            CHK(hipFree(a));
            CHK(hipFree(b));
            CHK(hipFree(o));
        }
    }
    return 0;
}
