// tune_ns.hip -- variants of the K=2 double-sum combine at the north-star
// size (nreduce = 128 Mi, 1 GiB per array) on one MI355X.  Not part of the
// product: it measures which load/store cache policy, occupancy and staging
// form moves the most bytes, so the shipped kernel can follow the data.
// Build: hipcc --offload-arch=gfx950 -O3 tune_ns.hip -o tune_ns
// Run:   ./tune_ns [n_doubles] [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CHK(x)                                                                 \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

constexpr int B = 256;

// cache-policy bits on the vector memory instructions (gfx950 mnemonics)
__device__ __forceinline__ u4 ld_nt(const void *p)
{
    u4 v;
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ u4 ld_sc1(const void *p)
{
    u4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ u4 ld_sc1nt(const void *p)
{
    u4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1 nt" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ u4 ld_plain(const void *p)
{
    u4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st_nt(void *p, u4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off nt" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc0sc1(void *p, u4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1nt(void *p, u4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_plain(void *p, u4 v)
{
    asm volatile("global_store_dwordx4 %0, %1, off" : : "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ u4 addv(u4 x, u4 y)
{
    union { u4 u; d2 d; } a, b;
    a.u = x;
    b.u = y;
    a.d = a.d + b.d;
    return a.u;
}

typedef u4 (*ldf)(const void *);
typedef void (*stf)(void *, u4);

// one-shot tile kernel with explicit policies; extern LDS caps occupancy
template <int U, u4 (*LD)(const void *), void (*ST)(void *, u4)>
__global__ __launch_bounds__(B) void k_pol(u4 *out, const u4 *a, const u4 *b, size_t nv)
{
    extern __shared__ char cap[];
    (void) cap;
    const size_t t = (size_t) blockIdx.x * (B * U) + threadIdx.x;
    if (t + (size_t) (U - 1) * B < nv) {
        u4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = LD(a + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) y[u] = LD(b + t + u * B);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; u++) ST(out + t + u * B, addv(x[u], y[u]));
    } else {
        for (int u = 0; u < U; u++) {
            const size_t j = t + (size_t) u * B;
            if (j < nv) out[j] = addv(a[j], b[j]);
        }
    }
}

// the shipped form (compiler builtins), for reference in the same binary
template <int U>
__global__ __launch_bounds__(B) void k_builtin(u4 *out, const u4 *a, const u4 *b, size_t nv)
{
    extern __shared__ char cap[];
    (void) cap;
    const size_t t = (size_t) blockIdx.x * (B * U) + threadIdx.x;
    if (t + (size_t) (U - 1) * B < nv) {
        u4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = __builtin_nontemporal_load(a + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) y[u] = __builtin_nontemporal_load(b + t + u * B);
#pragma unroll
        for (int u = 0; u < U; u++) __builtin_nontemporal_store(addv(x[u], y[u]), out + t + u * B);
    } else {
        for (int u = 0; u < U; u++) {
            const size_t j = t + (size_t) u * B;
            if (j < nv) out[j] = addv(a[j], b[j]);
        }
    }
}

// LDS-DMA staging: global_load_lds_dwordx4 (nt) of both inputs into the
// wave's LDS slice, then ds_read, add, nt store
template <int U, int AUX>
__global__ __launch_bounds__(B) void k_glds(u4 *out, const u4 *a, const u4 *b, size_t nv)
{
    __shared__ u4 lds[2 * U * B];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t t = (size_t) blockIdx.x * (B * U) + threadIdx.x;
    if (t + (size_t) (U - 1) * B < nv) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void *) (a + t + u * B),
                (__attribute__((address_space(3))) void *) &lds[(2 * u) * B + wave * 64], 16, 0,
                AUX);
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void *) (b + t + u * B),
                (__attribute__((address_space(3))) void *) &lds[(2 * u + 1) * B + wave * 64], 16,
                0, AUX);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; u++) {
            const u4 x = lds[(2 * u) * B + wave * 64 + lane];
            const u4 y = lds[(2 * u + 1) * B + wave * 64 + lane];
            __builtin_nontemporal_store(addv(x, y), out + t + u * B);
        }
    } else {
        for (int u = 0; u < U; u++) {
            const size_t j = t + (size_t) u * B;
            if (j < nv) out[j] = addv(a[j], b[j]);
        }
    }
}

typedef void (*kfn)(u4 *, const u4 *, const u4 *, size_t);

struct Variant {
    const char *name;
    kfn f;
    int U;
    int lds;  // dynamic LDS bytes (caps workgroups per CU)
};

int main(int argc, char **argv)
{
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (128ull << 20);  // doubles
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const size_t nv = n / 2;
    // ALLOC: 0 hipMalloc x3, 1 hipExtMallocWithFlags(Contiguous) x3, 2 one
    // hipMalloc carved in three, 3 virtual-memory chunks (hipMemCreate of
    // CHUNK bytes, as osgpu_heap_create builds heaps) mapped back to back
    const int alloc = getenv("ALLOC") ? atoi(getenv("ALLOC")) : 0;
    const char *only = getenv("VARIANTS");  // comma list of indices, or all
    u4 *a, *b, *o;
    const size_t S = n * 8;
    if (alloc == 1) {
        CHK(hipExtMallocWithFlags((void **) &a, S, hipDeviceMallocContiguous));
        CHK(hipExtMallocWithFlags((void **) &b, S, hipDeviceMallocContiguous));
        CHK(hipExtMallocWithFlags((void **) &o, S, hipDeviceMallocContiguous));
    } else if (alloc == 2) {
        char *p;
        CHK(hipMalloc((void **) &p, 3 * S));
        a = (u4 *) p;
        b = (u4 *) (p + S);
        o = (u4 *) (p + 2 * S);
    } else if (alloc == 3) {
        const size_t chunk = getenv("CHUNK") ? strtoull(getenv("CHUNK"), 0, 0) : (1ull << 30);
        hipMemAllocationProp prop;
        memset(&prop, 0, sizeof(prop));
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        void *va;
        CHK(hipMemAddressReserve(&va, 3 * S, 2 << 20, nullptr, 0));
        for (size_t off = 0; off < 3 * S; off += chunk) {
            hipMemGenericAllocationHandle_t h;
            const size_t len = std::min(chunk, 3 * S - off);
            CHK(hipMemCreate(&h, len, &prop, 0));
            CHK(hipMemMap((char *) va + off, len, 0, h, 0));
        }
        hipMemAccessDesc d;
        memset(&d, 0, sizeof(d));
        d.location.type = hipMemLocationTypeDevice;
        d.location.id = 0;
        d.flags = hipMemAccessFlagsProtReadWrite;
        CHK(hipMemSetAccess(va, 3 * S, &d, 1));
        a = (u4 *) va;
        b = (u4 *) ((char *) va + S);
        o = (u4 *) ((char *) va + 2 * S);
    } else {
        CHK(hipMalloc(&a, S));
        CHK(hipMalloc(&b, S));
        CHK(hipMalloc(&o, S));
    }
    CHK(hipMemset(a, 0x3f, n * 8));
    CHK(hipMemset(b, 0x3f, n * 8));
    std::vector<Variant> v = {
        {"builtin nt/nt U4 (shipped)", k_builtin<4>, 4, 0},
        {"asm nt/nt U4", k_pol<4, ld_nt, st_nt>, 4, 0},
        {"asm nt/sc0sc1 U4", k_pol<4, ld_nt, st_sc0sc1>, 4, 0},
        {"asm nt/sc1nt U4", k_pol<4, ld_nt, st_sc1nt>, 4, 0},
        {"asm sc1/nt U4", k_pol<4, ld_sc1, st_nt>, 4, 0},
        {"asm sc1nt/nt U4", k_pol<4, ld_sc1nt, st_nt>, 4, 0},
        {"asm sc1nt/sc1nt U4", k_pol<4, ld_sc1nt, st_sc1nt>, 4, 0},
        {"asm plain/nt U4", k_pol<4, ld_plain, st_nt>, 4, 0},
        {"asm nt/plain U4", k_pol<4, ld_nt, st_plain>, 4, 0},
        {"builtin U4 max 6 WG/CU", k_builtin<4>, 4, 160 * 1024 / 6},
        {"builtin U4 max 4 WG/CU", k_builtin<4>, 4, 160 * 1024 / 4},
        {"builtin U4 max 3 WG/CU", k_builtin<4>, 4, 160 * 1024 / 3},
        {"builtin U4 max 2 WG/CU", k_builtin<4>, 4, 160 * 1024 / 2},
        {"builtin U8 max 4 WG/CU", k_builtin<8>, 8, 160 * 1024 / 4},
        {"builtin U8 max 2 WG/CU", k_builtin<8>, 8, 160 * 1024 / 2},
        {"glds nt U4", k_glds<4, 2>, 4, 0},
        {"glds default U4", k_glds<4, 0>, 4, 0},
        {"glds nt U2", k_glds<2, 2>, 2, 0},
        {"glds nt U8", k_glds<8, 2>, 8, 0},
    };
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const double bytes = 3.0 * n * 8;
    printf("n=%zu doubles, bytes/launch=%.0f, alloc=%d\n", n, bytes, alloc);
    for (int pass = 0; pass < 2; pass++) {
        for (size_t vi = 0; vi < v.size(); vi++) {
            auto &x = v[vi];
            if (only) {
                char key[16];
                snprintf(key, sizeof(key), ",%zu,", vi);
                char list[256];
                snprintf(list, sizeof(list), ",%s,", only);
                if (!strstr(list, key)) continue;
            }
            const size_t per = (size_t) B * x.U;
            const size_t grid = (nv + per - 1) / per;
            for (int w = 0; w < 3; w++)
                hipLaunchKernelGGL(x.f, dim3(grid), dim3(B), x.lds, 0, o, a, b, nv);
            CHK(hipGetLastError());
            CHK(hipDeviceSynchronize());
            std::vector<float> ms(reps);
            for (int r = 0; r < reps; r++) {
                CHK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(x.f, dim3(grid), dim3(B), x.lds, 0, o, a, b, nv);
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                CHK(hipEventElapsedTime(&ms[r], e0, e1));
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[reps / 2] * 1e-3, best = ms[0] * 1e-3;
            // correctness: 0x3f3f... + itself
            std::vector<double> h(4);
            CHK(hipMemcpy(h.data(), (char *) o + (n * 8) / 2, 32, hipMemcpyDeviceToHost));
            double want;
            unsigned long long bits = 0x3f3f3f3f3f3f3f3full;
            memcpy(&want, &bits, 8);
            want += want;
            if (pass == 1)
                printf("{\"variant\": \"%s\", \"alloc\": %d, \"n\": %zu, \"us\": %.1f, "
                       "\"frac\": %.4f, \"best_frac\": %.4f, \"ok\": %s}\n",
                       x.name, alloc, n, med * 1e6, bytes / med / 8e12, bytes / best / 8e12,
                       h[0] == want ? "true" : "false");
            fflush(stdout);
        }
    }
    return 0;
}
