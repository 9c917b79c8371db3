// pcie_kernel_probe.hip -- can kernels moving pinned host memory over PCIe
// (zero-copy loads/stores, as the fused staged path does) beat the DMA
// copies of the STAGED path, especially with both directions at once (DMA
// measured 57 GB/s one way, 28.7 GB/s each way together,
// profiles/r01_pcie_probe.json)?  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 pcie_kernel_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// grid-stride 16-B copy; U vectors in flight per lane
template <int U>
__global__ __launch_bounds__(256) void copy_k(u4 *dst, const u4 *src, size_t nv)
{
    const size_t stride = (size_t) gridDim.x * 256 * U;
    for (size_t base = (size_t) blockIdx.x * 256 * U + threadIdx.x; base < nv; base += stride) {
        u4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (base + (size_t) u * 256 < nv) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
        for (int u = 0; u < U; u++)
            if (base + (size_t) u * 256 < nv) __builtin_nontemporal_store(v[u], dst + base + u * 256);
    }
}

// one launch, both directions: first half of the grid reads host, second writes host
template <int U>
__global__ __launch_bounds__(256) void both_k(u4 *dd, const u4 *hs, u4 *hd, const u4 *ds, size_t nv)
{
    const unsigned half = gridDim.x / 2;
    const bool rd = blockIdx.x < half;
    const unsigned b = rd ? blockIdx.x : blockIdx.x - half;
    u4 *dst = rd ? dd : hd;
    const u4 *src = rd ? hs : ds;
    const size_t stride = (size_t) half * 256 * U;
    for (size_t base = (size_t) b * 256 * U + threadIdx.x; base < nv; base += stride) {
        u4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (base + (size_t) u * 256 < nv) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
        for (int u = 0; u < U; u++)
            if (base + (size_t) u * 256 < nv) __builtin_nontemporal_store(v[u], dst + base + u * 256);
    }
}

struct Ctx {
    u4 *h_in, *h_out, *d_in, *d_out;
    size_t nv;
    int grid;
    hipStream_t s1, s2;
};

static double timeit(Ctx *c, void (*fn)(Ctx *))
{
    fn(c);
    CHK(hipDeviceSynchronize());
    double best = 1e30;
    for (int r = 0; r < 5; r++) {
        hipEvent_t a, b;
        CHK(hipEventCreate(&a));
        CHK(hipEventCreate(&b));
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a, nullptr));
        fn(c);
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(b, nullptr));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        best = std::min(best, ms * 1e-3);
        CHK(hipEventDestroy(a));
        CHK(hipEventDestroy(b));
    }
    return best;
}

static void k_read(Ctx *c)
{
    hipLaunchKernelGGL(copy_k<4>, dim3(c->grid), dim3(256), 0, c->s1, c->d_in, c->h_in, c->nv);
}
static void k_write(Ctx *c)
{
    hipLaunchKernelGGL(copy_k<4>, dim3(c->grid), dim3(256), 0, c->s1, c->h_out, c->d_out, c->nv);
}
static void k_two(Ctx *c)
{
    hipLaunchKernelGGL(copy_k<4>, dim3(c->grid), dim3(256), 0, c->s1, c->d_in, c->h_in, c->nv);
    hipLaunchKernelGGL(copy_k<4>, dim3(c->grid), dim3(256), 0, c->s2, c->h_out, c->d_out, c->nv);
}
static void k_one(Ctx *c)
{
    hipLaunchKernelGGL(both_k<4>, dim3(2 * c->grid), dim3(256), 0, c->s1, c->d_in, c->h_in,
                       c->h_out, c->d_out, c->nv);
}
static void dma_two(Ctx *c)
{
    CHK(hipMemcpyAsync(c->d_in, c->h_in, c->nv * 16, hipMemcpyHostToDevice, c->s1));
    CHK(hipMemcpyAsync(c->h_out, c->d_out, c->nv * 16, hipMemcpyDeviceToHost, c->s2));
}
static hipStream_t g_s3, g_s4;
static void dma_four(Ctx *c)  // two PEs' worth: 2 H2D + 2 D2H streams, halves
{
    const size_t h = c->nv * 8;
    CHK(hipMemcpyAsync(c->d_in, c->h_in, h, hipMemcpyHostToDevice, c->s1));
    CHK(hipMemcpyAsync((char *) c->d_in + h, (char *) c->h_in + h, h, hipMemcpyHostToDevice, g_s3));
    CHK(hipMemcpyAsync(c->h_out, c->d_out, h, hipMemcpyDeviceToHost, c->s2));
    CHK(hipMemcpyAsync((char *) c->h_out + h, (char *) c->d_out + h, h, hipMemcpyDeviceToHost, g_s4));
}
static void dma_chunked(Ctx *c)  // 32 MiB chunks alternating, two streams
{
    const size_t ch = (size_t) 32 << 20, tot = c->nv * 16;
    for (size_t o = 0; o < tot; o += ch) {
        CHK(hipMemcpyAsync((char *) c->d_in + o, (char *) c->h_in + o, ch, hipMemcpyHostToDevice, c->s1));
        CHK(hipMemcpyAsync((char *) c->h_out + o, (char *) c->d_out + o, ch, hipMemcpyDeviceToHost, c->s2));
    }
}
static void mix(Ctx *c)  // DMA in, kernel out
{
    CHK(hipMemcpyAsync(c->d_in, c->h_in, c->nv * 16, hipMemcpyHostToDevice, c->s1));
    hipLaunchKernelGGL(copy_k<4>, dim3(c->grid), dim3(256), 0, c->s2, c->h_out, c->d_out, c->nv);
}

int main()
{
    const size_t bytes = (size_t) 1 << 30;
    Ctx c;
    c.nv = bytes / 16;
    CHK(hipHostMalloc((void **) &c.h_in, bytes, hipHostMallocMapped));
    CHK(hipHostMalloc((void **) &c.h_out, bytes, hipHostMallocMapped));
    CHK(hipMalloc((void **) &c.d_in, bytes));
    CHK(hipMalloc((void **) &c.d_out, bytes));
    CHK(hipMemset(c.d_out, 1, bytes));
    for (size_t i = 0; i < bytes / 4; i += 1024) ((unsigned *) c.h_in)[i] = (unsigned) i;
    CHK(hipStreamCreateWithFlags(&c.s1, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));
    const double GB = 1e9;
    for (int grid : {64, 256, 1024, 4096}) {
        c.grid = grid;
        double tr = timeit(&c, k_read), tw = timeit(&c, k_write);
        double t2 = timeit(&c, k_two), t1 = timeit(&c, k_one);
        printf("{\"grid\": %d, \"kernel_read_GBs\": %.1f, \"kernel_write_GBs\": %.1f, "
               "\"kernel_both_two_launches_each_way_GBs\": %.1f, "
               "\"kernel_both_one_launch_each_way_GBs\": %.1f}\n",
               grid, bytes / tr / GB, bytes / tw / GB, bytes / t2 / GB, bytes / t1 / GB);
        fflush(stdout);
    }
    c.grid = 1024;
    CHK(hipStreamCreateWithFlags(&g_s3, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&g_s4, hipStreamNonBlocking));
    double td = timeit(&c, dma_two), tm = timeit(&c, mix);
    double t4 = timeit(&c, dma_four), tc = timeit(&c, dma_chunked);
    printf("{\"dma_both_each_way_GBs\": %.1f, \"dma_in_kernel_out_each_way_GBs\": %.1f, "
           "\"dma_four_streams_each_way_GBs\": %.1f, \"dma_32MiB_chunks_each_way_GBs\": %.1f}\n",
           bytes / td / GB, bytes / tm / GB, bytes / t4 / GB, bytes / tc / GB);
    return 0;
}
