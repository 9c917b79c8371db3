// D2H / H2D / duplex copy rate over time, around a burst of HBM streaming
// work: does the DMA rate depend on what the GPU did just before (clock and
// power state)?  One JSON line per sample.  Not part of the product.
//   hipcc --offload-arch=gfx950 -O2 tools/d2h_timeline.hip -o tools/d2h_timeline
//   tools/d2h_timeline [load_seconds=3] [after_seconds=4]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void stream_copy(const float4 *__restrict__ a, float4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n;
         i += (size_t) gridDim.x * blockDim.x)
        b[i] = a[i];
}

// device <-> host copy by kernel (mapped pinned host memory): 16-B vector
// loads and stores, grid-stride
__global__ void kcopy(const float4 *__restrict__ a, float4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n;
         i += (size_t) gridDim.x * blockDim.x)
        b[i] = a[i];
}

int main(int argc, char **argv)
{
    const double load_s = argc > 1 ? atof(argv[1]) : 3.0;
    const double after_s = argc > 2 ? atof(argv[2]) : 4.0;
    const size_t nb = (size_t) 64 << 20;
    const size_t big = (size_t) 2 << 30;
    char *h_in, *h_out, *d_in, *d_out, *x, *y;
    CK(hipHostMalloc((void **) &h_in, nb, hipHostMallocMapped));
    CK(hipHostMalloc((void **) &h_out, nb, hipHostMallocMapped));
    char *hd_in = nullptr, *hd_out = nullptr;
    CK(hipHostGetDevicePointer((void **) &hd_in, h_in, 0));
    CK(hipHostGetDevicePointer((void **) &hd_out, h_out, 0));
    const int kgrid = argc > 3 ? atoi(argv[3]) : 256;
    CK(hipMalloc((void **) &d_in, nb));
    CK(hipMalloc((void **) &d_out, nb));
    CK(hipMalloc((void **) &x, big));
    CK(hipMalloc((void **) &y, big));
    CK(hipMemset(x, 1, big));
    hipStream_t si, so, sk;
    CK(hipStreamCreateWithFlags(&si, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&so, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    const double t0 = now();
    auto sample = [&](const char *phase) {
        double a = now();
        CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, so));
        CK(hipStreamSynchronize(so));
        double b = now();
        CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
        CK(hipStreamSynchronize(si));
        double c = now();
        CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
        CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, so));
        CK(hipStreamSynchronize(si));
        CK(hipStreamSynchronize(so));
        double d = now();
        kcopy<<<kgrid, 256, 0, so>>>((const float4 *) d_out, (float4 *) hd_out, nb / 16);
        CK(hipStreamSynchronize(so));
        double e = now();
        kcopy<<<kgrid, 256, 0, si>>>((const float4 *) hd_in, (float4 *) d_in, nb / 16);
        CK(hipStreamSynchronize(si));
        double f = now();
        kcopy<<<kgrid, 256, 0, si>>>((const float4 *) hd_in, (float4 *) d_in, nb / 16);
        kcopy<<<kgrid, 256, 0, so>>>((const float4 *) d_out, (float4 *) hd_out, nb / 16);
        CK(hipStreamSynchronize(si));
        CK(hipStreamSynchronize(so));
        double g = now();
        CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
        kcopy<<<kgrid, 256, 0, so>>>((const float4 *) d_out, (float4 *) hd_out, nb / 16);
        CK(hipStreamSynchronize(si));
        CK(hipStreamSynchronize(so));
        double h = now();
        printf("{\"t\": %.3f, \"phase\": \"%s\", \"d2h_GBs\": %.1f, \"h2d_GBs\": %.1f, "
               "\"duplex_each_way_GBs\": %.1f, \"kd2h_GBs\": %.1f, \"kh2d_GBs\": %.1f, "
               "\"kduplex_each_way_GBs\": %.1f, \"dma_in_kernel_out_each_way_GBs\": %.1f}\n",
               a - t0, phase, nb / (b - a) / 1e9, nb / (c - b) / 1e9, nb / (d - c) / 1e9,
               nb / (e - d) / 1e9, nb / (f - e) / 1e9, nb / (g - f) / 1e9, nb / (h - g) / 1e9);
        fflush(stdout);
    };
    // idle start
    while (now() - t0 < 1.5) sample("start");
    // HBM streaming load on its own stream, sampled concurrently
    const double l0 = now();
    while (now() - l0 < load_s) {
        for (int k = 0; k < 4; k++)
            stream_copy<<<4096, 256, 0, sk>>>((const float4 *) x, (float4 *) y, big / 16);
        sample("under_load");
        CK(hipStreamSynchronize(sk));
    }
    const double a0 = now();
    while (now() - a0 < after_s) sample("after_load");
    return 0;
}
