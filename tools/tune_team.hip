// tune_team.hip -- design sweep for the owner-computes team kernel
// (csrc/team.hip) at P = 2, 4, 8 members, double sum in every member's own
// fold order, against the same-mix copy ceiling (P ranges copied in one
// launch: P read + P write streams over the same bytes).  Not part of the
// product.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/tune_team.hip -o tools/tune_team
//   ./tools/tune_team [n_per_array] [reps] [passes]
// One JSON line per (variant, P, pass): average launch time (one HIP event
// pair around reps launches back to back), fraction of 8 TB/s for 2*P*n*8
// bytes, and the ratio to the copy kernel.  Inputs: uniform [1, 2) doubles.
//
// Variant knobs (template parameters):
//   U      16-B vectors per input per lane
//   G      of them loaded per round before the fold (U % G == 0)
//   PMAJ   load issue order inside a round: 0 vector-major (for u: for p,
//          the shipped order), 1 input-major (for p: for u)
//   WAVE   lane -> vector map: 0 block-strided (vector t0 + u*BLOCK, the
//          shipped map: a wave touches U pieces of 1 KiB per input), 1
//          wave-contiguous (a wave owns 64*U consecutive vectors per input)
//   BLOCK  workgroup size
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#pragma clang fp contract(off)

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

union DVec {
    u32x4 v;
    double e[2];
};

template <int P>
struct Ptrs {
    const double *src[P];
    double *dst[P];
};

template <int P>
__device__ __forceinline__ void fold_store(const DVec (&in)[P], const Ptrs<P> &a, size_t j)
{
    DVec out[P];
#pragma unroll
    for (int w = 0; w < 2; w++) {
#pragma unroll
        for (int q = 0; q < P; q++) {
            double acc = in[q].e[w];
#pragma unroll
            for (int k = 0; k < P; k++)
                if (k != q) acc = acc + in[k].e[w];
            out[q].e[w] = acc;
        }
    }
#pragma unroll
    for (int q = 0; q < P; q++)
        __builtin_nontemporal_store(out[q].v, reinterpret_cast<u32x4 *>(a.dst[q]) + j);
}

template <int P, int U, int G, int PMAJ, int WAVE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void team_kernel(Ptrs<P> a, size_t nvec)
{
    static_assert(U % G == 0, "G must divide U");
    const size_t tile = (size_t) blockIdx.x * BLOCK * U;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    auto idx = [&](int u) -> size_t {
        return WAVE ? tile + (size_t) wave * 64 * U + (size_t) u * 64 + lane
                    : tile + (size_t) u * BLOCK + threadIdx.x;
    };
    if (tile + (size_t) BLOCK * U <= nvec) {
#pragma unroll
        for (int g = 0; g < U; g += G) {
            DVec in[G][P];
            if (PMAJ) {
#pragma unroll
                for (int p = 0; p < P; p++)
#pragma unroll
                    for (int u = 0; u < G; u++)
                        in[u][p].v = __builtin_nontemporal_load(
                            reinterpret_cast<const u32x4 *>(a.src[p]) + idx(g + u));
            } else {
#pragma unroll
                for (int u = 0; u < G; u++)
#pragma unroll
                    for (int p = 0; p < P; p++)
                        in[u][p].v = __builtin_nontemporal_load(
                            reinterpret_cast<const u32x4 *>(a.src[p]) + idx(g + u));
            }
#pragma unroll
            for (int u = 0; u < G; u++) fold_store<P>(in[u], a, idx(g + u));
        }
        return;
    }
    for (int u = 0; u < U; u++) {
        const size_t j = idx(u);
        if (j < nvec) {
            DVec in[P];
#pragma unroll
            for (int p = 0; p < P; p++)
                in[p].v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.src[p]) + j);
            fold_store<P>(in, a, j);
        }
    }
}

// the same-mix ceiling: P ranges, each block copies U*256 vectors of one range
template <int P>
__global__ __launch_bounds__(256) void copy_kernel(Ptrs<P> a, size_t nvec, unsigned per_range)
{
    const int r = blockIdx.x / per_range;
    const size_t base = (size_t) (blockIdx.x % per_range) * 256 * 4 + threadIdx.x;
    u32x4 v[4];
    const u32x4 *s = reinterpret_cast<const u32x4 *>(a.src[r]);
    u32x4 *d = reinterpret_cast<u32x4 *>(a.dst[r]);
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (base + u * 256 < nvec) v[u] = __builtin_nontemporal_load(s + base + u * 256);
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (base + u * 256 < nvec) __builtin_nontemporal_store(v[u], d + base + u * 256);
}

// the same ranges with every range streaming at once: block b copies a tile
// of range b % P (the team kernel's 2P concurrent streams, no fold)
template <int P>
__global__ __launch_bounds__(256) void copy_interleaved_kernel(Ptrs<P> a, size_t nvec)
{
    const int r = blockIdx.x % P;
    const size_t base = (size_t) (blockIdx.x / P) * 256 * 4 + threadIdx.x;
    u32x4 v[4];
    const u32x4 *s = reinterpret_cast<const u32x4 *>(a.src[r]);
    u32x4 *d = reinterpret_cast<u32x4 *>(a.dst[r]);
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (base + u * 256 < nvec) v[u] = __builtin_nontemporal_load(s + base + u * 256);
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (base + u * 256 < nvec) __builtin_nontemporal_store(v[u], d + base + u * 256);
}

// uniform [1, 2) doubles from a hash of (array, index): data like the bench's
__global__ void fill_kernel(double *p, size_t n, unsigned seed)
{
    for (size_t i = (size_t) blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t) gridDim.x * 256) {
        unsigned long long z = (i + 1) * 0x9e3779b97f4a7c15ull + seed * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        z ^= z >> 31;
        p[i] = __longlong_as_double((long long) (0x3ff0000000000000ull | (z >> 12)));
    }
}

static size_t g_n;
static int g_reps;
static double *g_buf[16];

template <typename F>
static double median_us(F launch)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) launch();
    // one event pair around reps launches back to back (bench.py's timing)
    float ms = 0;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < g_reps; i++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1e3 / g_reps;
}

template <int P>
static Ptrs<P> ptrs()
{
    Ptrs<P> a;
    for (int p = 0; p < P; p++) {
        a.src[p] = g_buf[p];
        a.dst[p] = g_buf[8 + p];
    }
    return a;
}

template <int P>
static double copy_us()
{
    const size_t nvec = g_n / 2;
    const unsigned per = (unsigned) ((nvec + 1023) / 1024);
    Ptrs<P> a = ptrs<P>();
    return median_us([&] {
        hipLaunchKernelGGL(copy_kernel<P>, dim3(per * P), dim3(256), 0, 0, a, nvec, per);
    });
}

template <int P>
static double copy_il_us()
{
    const size_t nvec = g_n / 2;
    const unsigned per = (unsigned) ((nvec + 1023) / 1024);
    Ptrs<P> a = ptrs<P>();
    return median_us([&] {
        hipLaunchKernelGGL(copy_interleaved_kernel<P>, dim3(per * P), dim3(256), 0, 0, a, nvec);
    });
}

static bool check(int P)
{
    // element 12345 of every target: member q's fold order
    const size_t i = 12345 % g_n;
    double x[8], r;
    for (int p = 0; p < P; p++) CK(hipMemcpy(&x[p], g_buf[p] + i, 8, hipMemcpyDeviceToHost));
    for (int q = 0; q < P; q++) {
        double acc = x[q];
        for (int k = 0; k < P; k++)
            if (k != q) acc = acc + x[k];
        CK(hipMemcpy(&r, g_buf[8 + q] + i, 8, hipMemcpyDeviceToHost));
        if (r != acc) return false;
    }
    return true;
}

template <int P, int U, int G, int PMAJ, int WAVE, int BLOCK>
static void run(double cus)
{
    const size_t nvec = g_n / 2;
    const size_t blocks = (nvec + (size_t) BLOCK * U - 1) / ((size_t) BLOCK * U);
    Ptrs<P> a = ptrs<P>();
    for (int p = 0; p < P; p++) CK(hipMemset(g_buf[8 + p], 0, g_n * 8));
    const double us = median_us([&] {
        hipLaunchKernelGGL((team_kernel<P, U, G, PMAJ, WAVE, BLOCK>), dim3((unsigned) blocks),
                           dim3(BLOCK), 0, 0, a, nvec);
    });
    const double B = 2.0 * P * g_n * 8;
    printf("{\"P\": %d, \"U\": %d, \"G\": %d, \"pmaj\": %d, \"wave\": %d, \"block\": %d, "
           "\"us\": %.2f, \"frac\": %.4f, \"copy_us\": %.2f, \"copy_frac\": %.4f, "
           "\"of_copy\": %.4f, \"ok\": %s}\n",
           P, U, G, PMAJ, WAVE, BLOCK, us, B / us / 8e6, cus, B / cus / 8e6, cus / us,
           check(P) ? "true" : "false");
    fflush(stdout);
}

template <int P>
static void sweep()
{
    const double c = copy_us<P>();
    run<P, 1, 1, 0, 0, 256>(c);
    run<P, 2, 2, 0, 0, 256>(c);
    run<P, 2, 2, 1, 0, 256>(c);
    run<P, 2, 2, 0, 1, 256>(c);
    run<P, 2, 1, 0, 0, 256>(c);
    run<P, 4, 4, 0, 0, 256>(c);
    run<P, 4, 4, 1, 0, 256>(c);
    run<P, 4, 4, 0, 1, 256>(c);
    run<P, 4, 2, 0, 0, 256>(c);
    run<P, 4, 1, 0, 0, 256>(c);
    run<P, 2, 2, 0, 0, 512>(c);
    run<P, 4, 4, 0, 0, 512>(c);
    run<P, 2, 2, 0, 0, 128>(c);
    run<P, 4, 4, 0, 0, 128>(c);
    if (P <= 2) {
        run<P, 8, 8, 0, 0, 256>(c);
        run<P, 8, 4, 0, 0, 256>(c);
    }
    const double c2 = copy_us<P>();   // the ceiling again: drift over the sweep
    printf("{\"P\": %d, \"copy_us_end\": %.2f}\n", P, c2);
}

template <int P, int U, int G>
static void layout_trial(int k)
{
    const size_t nvec = g_n / 2;
    const size_t blocks = (nvec + (size_t) 256 * U - 1) / ((size_t) 256 * U);
    Ptrs<P> a = ptrs<P>();
    const double cb = copy_us<P>(), ci = copy_il_us<P>();
    const double us = median_us([&] {
        hipLaunchKernelGGL((team_kernel<P, U, G, 0, 0, 256>), dim3((unsigned) blocks), dim3(256), 0,
                           0, a, nvec);
    });
    const double B = 2.0 * P * g_n * 8;
    printf("{\"trial\": %d, \"P\": %d, \"team_frac\": %.4f, \"copy_blocked_frac\": %.4f, "
           "\"copy_interleaved_frac\": %.4f, \"team_of_interleaved\": %.4f, \"src0\": \"%p\"}\n",
           k, P, B / us / 8e6, B / cb / 8e6, B / ci / 8e6, ci / us, (void *) g_buf[0]);
    fflush(stdout);
}

int main(int argc, char **argv)
{
    g_n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (size_t) 64 << 20;
    g_reps = argc > 2 ? atoi(argv[2]) : 20;
    for (int i = 0; i < 16; i++) {
        CK(hipMalloc(&g_buf[i], g_n * 8));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, g_buf[i], g_n, (unsigned) i);
    }
    CK(hipDeviceSynchronize());
    const int passes = argc > 3 ? atoi(argv[3]) : 2;
    if (argc > 4 && !strcmp(argv[4], "layouts")) {
        // placement trials: every array freed and allocated again, then the
        // shipped team shape, the blocked copy and the interleaved copy
        for (int k = 0; k < passes; k++) {
            for (int i = 0; i < 16; i++) CK(hipFree(g_buf[i]));
            for (int i = 0; i < 16; i++) {
                CK(hipMalloc(&g_buf[i], g_n * 8));
                hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, g_buf[i], g_n,
                                   (unsigned) (i + 16 * k));
            }
            CK(hipDeviceSynchronize());
            layout_trial<2, 4, 4>(k);
            layout_trial<4, 4, 4>(k);
            layout_trial<8, 4, 2>(k);
        }
        return 0;
    }
    for (int k = 0; k < passes; k++) {
        sweep<2>();
        sweep<4>();
        sweep<8>();
    }
    return 0;
}
