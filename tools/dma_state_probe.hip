// What moves the GPU's DMA device-to-host rate between its two levels
// (28-30 GB/s and 56-57 GB/s, tools/d2h_timeline.hip)?  Runs a script of
// phases given on the command line and samples the DMA rates during the
// sampling phases.  Tokens:
//   d<sec>  DMA samples only (64 MiB D2H, H2D, then both at once)
//   s<sec>  sleep (GPU idle)
//   l<sec>  heavy HBM streaming load (2 GiB copy kernels back to back)
//   b<ms>   a burst of that load lasting <ms> milliseconds
// One JSON line per sample: {"step", "token", "t", "d2h_GBs", ...}.
// Not part of the product.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

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

int main(int argc, char **argv)
{
    const size_t nb = (size_t) 64 << 20;
    const size_t big = (size_t) 2 << 30;
    char *h_in, *h_out, *d_in, *d_out, *x, *y;
    CK(hipHostMalloc((void **) &h_in, nb, 0));
    CK(hipHostMalloc((void **) &h_out, nb, 0));
    CK(hipMalloc((void **) &d_in, nb));
    CK(hipMalloc((void **) &d_out, nb));
    CK(hipMalloc((void **) &x, big));
    CK(hipMalloc((void **) &y, big));
    CK(hipMemset(x, 1, big));
    hipStream_t si, so, sk;
    CK(hipStreamCreateWithFlags(&si, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&so, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    const double t0 = now();
    for (int a = 1; a < argc; a++) {
        const char kind = argv[a][0];
        const double v = atof(argv[a] + 1);
        const double p0 = now();
        if (kind == 's') {
            std::this_thread::sleep_for(std::chrono::duration<double>(v));
        } else if (kind == 'l' || kind == 'b') {
            const double dur = kind == 'l' ? v : v / 1e3;
            while (now() - p0 < dur) {
                stream_copy<<<4096, 256, 0, sk>>>((const float4 *) x, (float4 *) y, big / 16);
                CK(hipStreamSynchronize(sk));
            }
        } else if (kind == 'd') {
            while (now() - p0 < v) {
                double q0 = now();
                CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, so));
                CK(hipStreamSynchronize(so));
                double q1 = now();
                CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
                CK(hipStreamSynchronize(si));
                double q2 = now();
                CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, si));
                CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, so));
                CK(hipStreamSynchronize(si));
                CK(hipStreamSynchronize(so));
                double q3 = now();
                printf("{\"step\": %d, \"token\": \"%s\", \"t\": %.3f, \"d2h_GBs\": %.1f, "
                       "\"h2d_GBs\": %.1f, \"duplex_each_way_GBs\": %.1f}\n",
                       a, argv[a], q0 - t0, nb / (q1 - q0) / 1e9, nb / (q2 - q1) / 1e9,
                       nb / (q3 - q2) / 1e9);
                fflush(stdout);
            }
        }
    }
    return 0;
}
