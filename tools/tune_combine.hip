// tune_combine.hip -- design-space sweep for the double-sum K=2 combine
// (BASELINE config 2 shape) on one MI355X.  Not part of the product: it
// times variants of the streaming kernel so the shipped one can be chosen
// from measurements.  Build: hipcc --offload-arch=gfx950 -O3 tune_combine.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

enum { LD_PLAIN = 0, LD_NT = 1 };
enum { ST_PLAIN = 0, ST_NT = 1 };

template <int LD>
__device__ __forceinline__ d2 ld(const d2 *p)
{
    if (LD == LD_NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <int ST>
__device__ __forceinline__ void st(d2 *p, d2 v)
{
    if (ST == ST_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// one-shot grid: block covers B*U consecutive vectors
template <int B, int U, int LD, int ST>
__global__ __launch_bounds__(B) void k_tile(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    size_t t = (size_t) blockIdx.x * (B * U) + threadIdx.x;
    if (t + (size_t) (U - 1) * B < nv) {
        d2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = ld<LD>(a + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) y[u] = ld<LD>(b + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) st<ST>(out + t + u * B, x[u] + y[u]);
    } else {
        for (int u = 0; u < U; u++)
            if (t + u * B < nv) st<ST>(out + t + u * B, ld<LD>(a + t + u * B) + ld<LD>(b + t + u * B));
    }
}

// grid-stride over tiles with a fixed grid
template <int B, int U, int LD, int ST>
__global__ __launch_bounds__(B) void k_stride(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    const size_t tile = (size_t) B * U;
    for (size_t base = (size_t) blockIdx.x * tile; base < nv; base += (size_t) gridDim.x * tile) {
        size_t t = base + threadIdx.x;
        if (base + tile <= nv) {
            d2 x[U], y[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = ld<LD>(a + t + u * B);
#pragma unroll
            for (int u = 0; u < U; u++) y[u] = ld<LD>(b + t + u * B);
#pragma unroll
            for (int u = 0; u < U; u++) st<ST>(out + t + u * B, x[u] + y[u]);
        } else {
            for (int u = 0; u < U; u++)
                if (t + u * B < nv) st<ST>(out + t + u * B, ld<LD>(a + t + u * B) + ld<LD>(b + t + u * B));
        }
    }
}

// per-thread contiguous chunk (each lane streams its own 16*U bytes)
template <int B, int U, int LD, int ST>
__global__ __launch_bounds__(B) void k_contig(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    size_t t = ((size_t) blockIdx.x * B + threadIdx.x) * U;
    if (t + U <= nv) {
        d2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = ld<LD>(a + t + u);
#pragma unroll
        for (int u = 0; u < U; u++) y[u] = ld<LD>(b + t + u);
#pragma unroll
        for (int u = 0; u < U; u++) st<ST>(out + t + u, x[u] + y[u]);
    } else {
        for (int u = 0; u < U; u++)
            if (t + u < nv) st<ST>(out + t + u, ld<LD>(a + t + u) + ld<LD>(b + t + u));
    }
}

// loads interleaved a0 b0 a1 b1 ... (the product kernel's issue order)
template <int B, int U>
__global__ __launch_bounds__(B) void k_tile_ilv(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    size_t t = (size_t) blockIdx.x * (B * U) + threadIdx.x;
    if (t + (size_t) (U - 1) * B < nv) {
        d2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            x[u] = __builtin_nontemporal_load(a + t + u * B);
            y[u] = __builtin_nontemporal_load(b + t + u * B);
        }
#pragma unroll
        for (int u = 0; u < U; u++) __builtin_nontemporal_store(x[u] + y[u], out + t + u * B);
    } else {
        for (int u = 0; u < U; u++)
            if (t + u * B < nv)
                __builtin_nontemporal_store(a[t + u * B] + b[t + u * B], out + t + u * B);
    }
}

// persistent grid, software-pipelined: the next tile's loads are in flight
// while the current tile is added and stored
template <int B, int U>
__global__ __launch_bounds__(B) void k_pipe(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    const size_t tile = (size_t) B * U;
    const size_t step = (size_t) gridDim.x * tile;
    size_t base = (size_t) blockIdx.x * tile;
    d2 x[U], y[U];
    auto load = [&](size_t bs, d2 *xx, d2 *yy) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t j = bs + threadIdx.x + u * B;
            if (j < nv) {
                xx[u] = __builtin_nontemporal_load(a + j);
                yy[u] = __builtin_nontemporal_load(b + j);
            }
        }
    };
    if (base < nv) load(base, x, y);
    for (; base < nv; base += step) {
        d2 xn[U], yn[U];
        const size_t nb = base + step;
        if (nb < nv) load(nb, xn, yn);
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t j = base + threadIdx.x + u * B;
            if (j < nv) __builtin_nontemporal_store(x[u] + y[u], out + j);
        }
#pragma unroll
        for (int u = 0; u < U; u++) { x[u] = xn[u]; y[u] = yn[u]; }
    }
}

// 32-byte per lane per load (two dwordx4 to adjacent addresses)
template <int B, int U>
__global__ __launch_bounds__(B) void k_wide(d2 *out, const d2 *a, const d2 *b, size_t nv)
{
    size_t t = ((size_t) blockIdx.x * (B * U) + threadIdx.x) * 2;
    if (t + (size_t) (U - 1) * B * 2 + 1 < nv) {
        d2 x[2 * U], y[2 * U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            x[2 * u] = __builtin_nontemporal_load(a + t + u * 2 * B);
            x[2 * u + 1] = __builtin_nontemporal_load(a + t + u * 2 * B + 1);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            y[2 * u] = __builtin_nontemporal_load(b + t + u * 2 * B);
            y[2 * u + 1] = __builtin_nontemporal_load(b + t + u * 2 * B + 1);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            __builtin_nontemporal_store(x[2 * u] + y[2 * u], out + t + u * 2 * B);
            __builtin_nontemporal_store(x[2 * u + 1] + y[2 * u + 1], out + t + u * 2 * B + 1);
        }
    } else {
        for (size_t j = t; j < nv && j < t + (size_t) U * 2 * B; j += 1) (void) 0;
        for (int u = 0; u < U; u++)
            for (int h = 0; h < 2; h++) {
                size_t j = t + u * 2 * B + h;
                if (j < nv) out[j] = a[j] + b[j];
            }
    }
}

typedef void (*kfn)(d2 *, const d2 *, const d2 *, size_t);

extern "C" int osgpu_combine(int type, int op, void *target, const void *const *srcs, int nsrc,
                             size_t nelems, void *hip_stream);

struct Variant {
    const char *name;
    kfn f;
    int block, per_block;  // vectors per block (tile kernels) or 0
    int stride_blocks;     // >0: fixed grid
};

int main(int argc, char **argv)
{
    size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (64ull << 20);  // doubles
    int reps = argc > 2 ? atoi(argv[2]) : 30;
    size_t nv = n / 2;
    d2 *a, *b, *o;
    CHK(hipMalloc(&a, n * 8));
    CHK(hipMalloc(&b, n * 8));
    CHK(hipMalloc(&o, n * 8));
    CHK(hipMemset(a, 0x3f, n * 8));
    CHK(hipMemset(b, 0x3f, n * 8));
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Variant> v = {
        {"tile B256 U4 nt/nt", k_tile<256, 4, LD_NT, ST_NT>, 256, 1024, 0},
        {"tile B256 U4 plain/nt", k_tile<256, 4, LD_PLAIN, ST_NT>, 256, 1024, 0},
        {"tile B256 U4 plain/plain", k_tile<256, 4, LD_PLAIN, ST_PLAIN>, 256, 1024, 0},
        {"tile B256 U4 nt/plain", k_tile<256, 4, LD_NT, ST_PLAIN>, 256, 1024, 0},
        {"tile B256 U2 nt/nt", k_tile<256, 2, LD_NT, ST_NT>, 256, 512, 0},
        {"tile B256 U8 nt/nt", k_tile<256, 8, LD_NT, ST_NT>, 256, 2048, 0},
        {"tile B512 U4 nt/nt", k_tile<512, 4, LD_NT, ST_NT>, 512, 2048, 0},
        {"tile B1024 U2 nt/nt", k_tile<1024, 2, LD_NT, ST_NT>, 1024, 2048, 0},
        {"tile B128 U4 nt/nt", k_tile<128, 4, LD_NT, ST_NT>, 128, 512, 0},
        {"tile B256 U1 nt/nt", k_tile<256, 1, LD_NT, ST_NT>, 256, 256, 0},
        {"stride B256 U4 nt/nt x4/CU", k_stride<256, 4, LD_NT, ST_NT>, 256, 1024, 4},
        {"stride B256 U4 nt/nt x8/CU", k_stride<256, 4, LD_NT, ST_NT>, 256, 1024, 8},
        {"stride B256 U4 nt/nt x16/CU", k_stride<256, 4, LD_NT, ST_NT>, 256, 1024, 16},
        {"stride B512 U4 nt/nt x8/CU", k_stride<512, 4, LD_NT, ST_NT>, 512, 2048, 8},
        {"stride B256 U8 nt/nt x8/CU", k_stride<256, 8, LD_NT, ST_NT>, 256, 2048, 8},
        {"stride B256 U4 plain/nt x8/CU", k_stride<256, 4, LD_PLAIN, ST_NT>, 256, 1024, 8},
        {"contig B256 U4 nt/nt", k_contig<256, 4, LD_NT, ST_NT>, 256, 1024, 0},
        {"contig B256 U2 nt/nt", k_contig<256, 2, LD_NT, ST_NT>, 256, 512, 0},
        {"tile-ilv B256 U4", k_tile_ilv<256, 4>, 256, 1024, 0},
        {"tile-ilv B256 U8", k_tile_ilv<256, 8>, 256, 2048, 0},
        {"pipe B256 U2 x4/CU", k_pipe<256, 2>, 256, 512, 4},
        {"pipe B256 U2 x8/CU", k_pipe<256, 2>, 256, 512, 8},
        {"pipe B256 U4 x4/CU", k_pipe<256, 4>, 256, 1024, 4},
        {"pipe B512 U2 x4/CU", k_pipe<512, 2>, 512, 1024, 4},
        {"wide B256 U2", k_wide<256, 2>, 256, 1024, 0},
        {"wide B256 U1", k_wide<256, 1>, 256, 512, 0},
    };
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const double bytes = 3.0 * n * 8;
    printf("n=%zu doubles, %d CUs, bytes/launch=%.0f\n", n, cus, bytes);
    for (int pass = 0; pass < 2; pass++) {
        for (auto &x : v) {
            size_t grid = x.stride_blocks ? (size_t) x.stride_blocks * cus
                                          : (nv + x.per_block - 1) / x.per_block;
            for (int w = 0; w < 3; w++)
                hipLaunchKernelGGL(x.f, dim3(grid), dim3(x.block), 0, 0, o, a, b, nv);
            CHK(hipDeviceSynchronize());
            std::vector<float> ms(reps);
            for (int r = 0; r < reps; r++) {
                CHK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(x.f, dim3(grid), dim3(x.block), 0, 0, o, a, b, nv);
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                CHK(hipEventElapsedTime(&ms[r], e0, e1));
            }
            std::sort(ms.begin(), ms.end());
            double med = ms[reps / 2] * 1e-3, best = ms[0] * 1e-3;
            if (pass == 1)
                printf("%-32s grid=%7zu  med %8.1f us  %7.1f GB/s (%.1f%% of 8 TB/s)  best %7.1f GB/s\n",
                       x.name, grid, med * 1e6, bytes / med / 1e9, bytes / med / 8e12 * 100,
                       bytes / best / 1e9);
        }
    }
    // the shipped kernel through the library's C ABI, same buffers / stream
    {
        const void *srcs[2] = {a, b};
        for (int w = 0; w < 3; w++) osgpu_combine(5, 0, o, srcs, 2, n, nullptr);
        CHK(hipDeviceSynchronize());
        hipStream_t s;
        CHK(hipStreamCreate(&s));
        std::vector<float> ms(reps);
        for (int r = 0; r < reps; r++) {
            CHK(hipEventRecord(e0, s));
            osgpu_combine(5, 0, o, srcs, 2, n, s);
            CHK(hipEventRecord(e1, s));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms[r], e0, e1));
        }
        std::sort(ms.begin(), ms.end());
        double med = ms[reps / 2] * 1e-3, best = ms[0] * 1e-3;
        printf("%-32s grid=%7s  med %8.1f us  %7.1f GB/s (%.1f%% of 8 TB/s)  best %7.1f GB/s\n",
               "PRODUCT osgpu_combine", "-", med * 1e6, bytes / med / 1e9,
               bytes / med / 8e12 * 100, bytes / best / 1e9);
    }
    // verify last variant output
    std::vector<double> h(16);
    CHK(hipMemcpy(h.data(), o, 128, hipMemcpyDeviceToHost));
    printf("check %g\n", h[0]);
    return 0;
}
