// tlb_probe.hip -- the shipped combine shape (double sum, K = 2, tiles of
// 256 x 4 vectors) at 2^26 and 2^28 elements, for PMC passes on address
// translation (UTCL1) counters: do arrays of >= 1 GiB lose rate to TLB
// misses?  Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int B = 256, U = 4;

__global__ __launch_bounds__(B) void tile(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    size_t t = (size_t) blockIdx.x * (B * U) + threadIdx.x;
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

int main()
{
    for (int lg : {26, 28}) {
        const size_t n = (size_t) 1 << lg, nv = n / 2;
        double *a, *b, *o;
        CHK(hipMalloc(&a, n * 8));
        CHK(hipMalloc(&b, n * 8));
        CHK(hipMalloc(&o, n * 8));
        CHK(hipMemset(a, 0, n * 8));
        CHK(hipMemset(b, 0, n * 8));
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0));
        CHK(hipEventCreate(&e1));
        for (int r = 0; r < 4; r++) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(tile, dim3((unsigned) (nv / (B * U))), dim3(B), 0, 0, (d2 *) o,
                               (const d2 *) a, (const d2 *) b, nv);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"log2n\": %d, \"rep\": %d, \"us\": %.1f, \"frac\": %.4f}\n", lg, r, ms * 1e3,
                   3.0 * n * 8 / (ms * 1e-3) / 8e12);
        }
        CHK(hipFree(a));
        CHK(hipFree(b));
        CHK(hipFree(o));
    }
    return 0;
}
