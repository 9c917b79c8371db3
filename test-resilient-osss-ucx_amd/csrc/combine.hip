// combine.hip -- the reduce-to-all combine as gfx950 streaming kernels.
//
// out[i] = op(...op(op(in[0][i], in[1][i]), in[2][i])..., in[K-1][i])
//
// This is the element-wise fold of src/reductions.c:79-111 (copy source,
// then fold every peer's source in PE order) with the 64-element pWrk bounce
// and the per-element indirect call removed: every input is streamed once
// from HBM (local or a peer GPU's over xGMI), the accumulator never leaves
// registers, and the target is written once.  HBM bytes per element:
// (K + 1) * sizeof(T) -- the roofline quantity reported by bench.py.
//
// Shape (MI355X: 256 CUs, 64-wide waves, 16-B global_load_dwordx4):
//  * one 16-byte vector per lane per load; a 256-thread workgroup covers
//    256*U consecutive vectors of every input, so each wave-instruction is a
//    fully coalesced 1 KiB access;
//  * all K*U loads of a lane are issued before the fold, so a lane keeps
//    K*U*16 B in flight (K=2, U=4: 128 B/lane, 32 KiB per workgroup);
//  * the result is stored nontemporal (it is not re-read by this kernel);
//  * the head/tail elements that do not fill a 16-B vector (unaligned start,
//    ragged n) are folded by the first lanes of workgroup 0, so one launch
//    covers any n.
#include <hip/hip_runtime.h>
#include <atomic>
#include <stdint.h>
#include <stddef.h>

#include "elem_ops.hpp"
#include "combine.hpp"

#pragma clang fp contract(off)

namespace osgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
union Vec16 {
    u32x4 v;
    T e[16 / sizeof(T)];
};

template <typename T, int K>
struct Inputs {
    const T *p[K];
};

constexpr int kBlock = 256;

// above 6 inputs: vectors per input in flight per round (U = kUK8 in all);
// G = U keeps every load of the tile in flight at once (G = 2 and 1 were
// measured no faster: tools/combine_variants.py)
constexpr int kCombineG8 = kUK8;

// lanes per vector-tile unroll: keep K*U*4 VGPRs of payload modest
template <int K>
struct Unroll {
    static constexpr int value = K <= 2 ? kUK2 : (K <= 4 ? kUK4 : kUK8);
};

template <typename T, int OP, int K>
__device__ __forceinline__ T fold_scalar(const Inputs<T, K> &in, size_t i)
{
    T x[K];
#pragma unroll
    for (int k = 0; k < K; k++) x[k] = in.p[k][i];
    T acc = x[0];
#pragma unroll
    for (int k = 1; k < K; k++) acc = Elem<T, OP>::f(acc, x[k]);
    return acc;
}

// the branch-free fold (elem_ops.hpp Fast), redone with the exact one only
// for a vector whose result holds a NaN part: no branch per element
template <typename T, int OP, int K>
__device__ __forceinline__ void fold_vec(Vec16<T> (&x)[K], Vec16<T> &out)
{
    constexpr int W = 16 / sizeof(T);
    using F = Fast<T, OP>;
    bool bad = false;
#pragma unroll
    for (int w = 0; w < W; w++) {
        T acc = x[0].e[w];
#pragma unroll
        for (int k = 1; k < K; k++) acc = F::f(acc, x[k].e[w]);
        out.e[w] = acc;
        bad = bad || F::bad(acc);
    }
    if (F::kChecked && __builtin_expect(bad, 0)) {
#pragma unroll
        for (int w = 0; w < W; w++) {
            T acc = x[0].e[w];
#pragma unroll
            for (int k = 1; k < K; k++) acc = Elem<T, OP>::f(acc, x[k].e[w]);
            out.e[w] = acc;
        }
    }
}

// Vector body over [head, head + nvec*W) plus the scalar edges.
template <typename T, int OP, int K>
__global__ __launch_bounds__(kBlock) void combine_vec_kernel(
    T *out, Inputs<T, K> in, size_t nvec, size_t head, size_t tail_start,
    int nedge)
{
    constexpr int U = Unroll<K>::value;
    constexpr int W = 16 / sizeof(T);
    const size_t tid = (size_t) blockIdx.x * (kBlock * U) + threadIdx.x;

    // edges: head elements [0, head) and tail [tail_start, tail_start + ...)
    if (blockIdx.x == 0 && (int) threadIdx.x < nedge) {
        size_t e = threadIdx.x < head ? threadIdx.x : tail_start + (threadIdx.x - head);
        out[e] = fold_scalar<T, OP, K>(in, e);
    }

    const u32x4 *src[K];
#pragma unroll
    for (int k = 0; k < K; k++) src[k] = reinterpret_cast<const u32x4 *>(in.p[k] + head);
    u32x4 *dst = reinterpret_cast<u32x4 *>(out + head);
    (void) W;

    if (tid + (size_t) (U - 1) * kBlock < nvec) {
        // the loads of G vectors of every input in flight before their folds
        // (G = U: all K*U of them; above 6 inputs kCombineG8)
        constexpr int G = K <= 6 ? U : kCombineG8;
        static_assert(G >= 1 && G <= U && U % G == 0, "kCombineG8 must divide U");
#pragma unroll
        for (int g = 0; g < U; g += G) {
            Vec16<T> x[G][K];
#pragma unroll
            for (int u = 0; u < G; u++)
#pragma unroll
                for (int k = 0; k < K; k++)
                    x[u][k].v = __builtin_nontemporal_load(&src[k][tid + (size_t) (g + u) * kBlock]);
#pragma unroll
            for (int u = 0; u < G; u++) {
                Vec16<T> r;
                fold_vec<T, OP, K>(x[u], r);
                __builtin_nontemporal_store(r.v, &dst[tid + (size_t) (g + u) * kBlock]);
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t j = tid + (size_t) u * kBlock;
            if (j < nvec) {
                Vec16<T> x[K], r;
#pragma unroll
                for (int k = 0; k < K; k++) x[k].v = __builtin_nontemporal_load(&src[k][j]);
                fold_vec<T, OP, K>(x, r);
                __builtin_nontemporal_store(r.v, &dst[j]);
            }
        }
    }
}

// LDS-staged form (2 <= K <= kCombineLdsMaxK): K
// waves per workgroup, a tile of 64*U 16-B vectors of every input.  Wave k
// streams input k's tile into LDS (one read stream per wave, like the copy
// kernel and team_lds_kernel); after the barrier the K waves fold the tile
// from LDS in input order and store it, each a contiguous 1 KiB per
// instruction.  HBM bytes as combine_vec_kernel.  Timed against it in one
// process on the same fresh arrays (tools/combine_inproc_ab.py, 6
// allocations each, profiles/r05_combine_lds_ab.jsonl): double sum K = 2
// 1.04x with U = 2 (0.824 against 0.792 of 8 TB/s median; 1.02x with
// U = 4), K = 3 and 4 1.02x with U = 4 (U = 2: 1.01x, 0.98x); float / int
// sum 1.02x / 1.04x, long xor 1.01x, double max 1.00x at K = 2; K = 5 and
// 8 (32 Mi doubles) 1.04x and 1.07x with U = 4 (U = 2: 1.01x, 1.05x); at
// 8 / 64 / 128 Mi doubles, K = 2: 1.07x / 1.04x / 1.04x.
constexpr int kCombineLdsMaxK = 8;
#ifndef OSGPU_COMBINE_LDS_U2
#define OSGPU_COMBINE_LDS_U2 2  // vectors per lane per input at K = 2 (the headline kernel)
#endif
constexpr int kCombineLdsU = 4;  // ... at K = 3 .. 8
// (Round 6, in one process on the same arrays, 6 allocations each,
// profiles/r06_combine_glds_ab.jsonl: the tile staged by LDS-DMA --
// global_load_lds_dwordx4, no VGPR round trip -- 1.005x at U = 2 (min
// 0.997x), 0.985x at U = 4, 0.975x at U = 8; register staging at U = 4
// 0.979x.  Within noise at best: the register staging ships.  Several
// tiles per workgroup, the next tile's loads in flight during this one's
// fold (profiles/r06_combine_tpw_ab.jsonl): 2 tiles 0.979x, 4 tiles 0.912x,
// 4 strided tiles 0.922x, 4 tiles of U = 1 0.993x -- one tile per
// workgroup, a one-shot grid, ships.)

template <typename T, int OP, int K, int U>
__global__ __launch_bounds__(64 * K) void combine_lds_kernel(T *out, Inputs<T, K> in, size_t nvec,
                                                              size_t head, size_t tail_start,
                                                              int nedge)
{
    constexpr int V = 64 * U;  // vectors per input per tile
    __shared__ u32x4 tile[K][V];
    if (blockIdx.x == 0 && (int) threadIdx.x < nedge) {
        size_t e = threadIdx.x < head ? threadIdx.x : tail_start + (threadIdx.x - head);
        out[e] = fold_scalar<T, OP, K>(in, e);
    }
    const int w = __builtin_amdgcn_readfirstlane((int) (threadIdx.x >> 6));
    const int lane = (int) (threadIdx.x & 63);
    const size_t base = (size_t) blockIdx.x * V;
    const bool whole = base + V <= nvec;
    const T *pw = in.p[0];
#pragma unroll
    for (int k = 1; k < K; k++)
        if (w == k) pw = in.p[k];
    const u32x4 *src = reinterpret_cast<const u32x4 *>(pw + head);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        if (whole || base + u * 64 + lane < nvec)
            v[u] = __builtin_nontemporal_load(src + base + u * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; u++) tile[w][u * 64 + lane] = v[u];
    __syncthreads();
    u32x4 *dst = reinterpret_cast<u32x4 *>(out + head);
    for (int j = (int) threadIdx.x; j < V; j += 64 * K) {
        if (!whole && base + j >= nvec) continue;
        Vec16<T> x[K], r;
#pragma unroll
        for (int k = 0; k < K; k++) x[k].v = tile[k][j];
        fold_vec<T, OP, K>(x, r);
        __builtin_nontemporal_store(r.v, dst + base + j);
    }
}

// Element-granular fallback for inputs whose 16-byte phases differ.
template <typename T, int OP, int K>
__global__ __launch_bounds__(kBlock) void combine_scalar_kernel(T *out, Inputs<T, K> in,
                                                                size_t n)
{
    const size_t stride = (size_t) gridDim.x * kBlock;
    for (size_t i = (size_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = fold_scalar<T, OP, K>(in, i);
}

// ------------------------------------------------------------------ launch

static std::atomic<size_t> g_launch_threads{kMaxLaunchThreads};
size_t max_launch_threads() { return g_launch_threads.load(std::memory_order_relaxed); }
void set_max_launch_threads(size_t n) { g_launch_threads.store(n, std::memory_order_relaxed); }

template <typename T, int OP, int K>
static hipError_t launch_k(T *out, const T *const *srcs, size_t n, hipStream_t s)
{
    Inputs<T, K> in;
    uintptr_t phase = (uintptr_t) out & 15;
    bool same_phase = (phase % sizeof(T)) == 0;
    for (int k = 0; k < K; k++) {
        in.p[k] = srcs[k];
        if (((uintptr_t) srcs[k] & 15) != phase) same_phase = false;
    }
    if (!same_phase || sizeof(T) > 16) {
        size_t blocks = (n + kBlock - 1) / kBlock;
        if (blocks > 8192) blocks = 8192;
        if (blocks == 0) blocks = 1;
        hipLaunchKernelGGL((combine_scalar_kernel<T, OP, K>), dim3((unsigned) blocks),
                           dim3(kBlock), 0, s, out, in, n);
        return hipGetLastError();
    }
    constexpr int W = 16 / sizeof(T);
    constexpr int U = Unroll<K>::value;
    size_t head = phase ? (16 - phase) / sizeof(T) : 0;
    if (head > n) head = n;
    size_t nvec = (n - head) / W;
    size_t tail_start = head + nvec * W;
    int nedge = (int) (head + (n - tail_start));
    // tiles of V vectors, one per workgroup of `threads`; at most
    // max_launch_threads() per launch (combine.hpp): the first launch takes the
    // edges, the others the next runs of tiles through shifted pointers
    auto launch = [&](size_t V, unsigned threads, auto kernel) -> hipError_t {
        size_t tiles = (nvec + V - 1) / V;
        if (tiles == 0) tiles = 1;
        const size_t lim = max_launch_threads() / threads;
        const size_t per_launch = lim ? lim : 1;
        for (size_t t0 = 0; t0 < tiles; t0 += per_launch) {
            const size_t nt = tiles - t0 < per_launch ? tiles - t0 : per_launch;
            const size_t nv = nvec - t0 * V < nt * V ? nvec - t0 * V : nt * V;
            if (t0 == 0) {
                hipLaunchKernelGGL(kernel, dim3((unsigned) nt), dim3(threads), 0, s, out, in, nv,
                                   head, tail_start, nedge);
            } else {
                const size_t off = head + t0 * V * W;
                Inputs<T, K> ic;
                for (int k = 0; k < K; k++) ic.p[k] = in.p[k] + off;
                hipLaunchKernelGGL(kernel, dim3((unsigned) nt), dim3(threads), 0, s, out + off, ic, nv,
                                   (size_t) 0, (size_t) 0, 0);
            }
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    if constexpr (K >= 2 && K <= kCombineLdsMaxK) {
        constexpr int UL = K == 2 ? OSGPU_COMBINE_LDS_U2 : kCombineLdsU;
        return launch((size_t) 64 * UL, 64 * K, combine_lds_kernel<T, OP, K, UL>);
    }
    return launch((size_t) kBlock * U, kBlock, combine_vec_kernel<T, OP, K>);
}

constexpr int kMaxK = 8;

template <typename T, int OP>
static hipError_t launch_op(void *out_, const void *const *srcs_, int k, size_t n,
                            hipStream_t s)
{
    T *out = static_cast<T *>(out_);
    const T *const *srcs = reinterpret_cast<const T *const *>(srcs_);
    // fold in chunks of at most kMaxK inputs: out = fold(srcs[0..7]), then
    // out = fold(out, srcs[8..14]), ... -- left-to-right order is preserved
    const T *chunk[kMaxK];
    int done = 0;
    hipError_t err = hipSuccess;
    while (done < k && err == hipSuccess) {
        int m = 0;
        if (done > 0) chunk[m++] = out;
        while (m < kMaxK && done < k) chunk[m++] = srcs[done++];
        switch (m) {
        case 1: err = launch_k<T, OP, 1>(out, chunk, n, s); break;
        case 2: err = launch_k<T, OP, 2>(out, chunk, n, s); break;
        case 3: err = launch_k<T, OP, 3>(out, chunk, n, s); break;
        case 4: err = launch_k<T, OP, 4>(out, chunk, n, s); break;
        case 5: err = launch_k<T, OP, 5>(out, chunk, n, s); break;
        case 6: err = launch_k<T, OP, 6>(out, chunk, n, s); break;
        case 7: err = launch_k<T, OP, 7>(out, chunk, n, s); break;
        default: err = launch_k<T, OP, 8>(out, chunk, n, s); break;
        }
    }
    return err;
}

template <typename T>
static hipError_t launch_int(int op, void *out, const void *const *srcs, int k, size_t n,
                             hipStream_t s)
{
    switch (op) {
    case OP_SUM: return launch_op<T, OP_SUM>(out, srcs, k, n, s);
    case OP_PROD: return launch_op<T, OP_PROD>(out, srcs, k, n, s);
    case OP_AND: return launch_op<T, OP_AND>(out, srcs, k, n, s);
    case OP_OR: return launch_op<T, OP_OR>(out, srcs, k, n, s);
    case OP_XOR: return launch_op<T, OP_XOR>(out, srcs, k, n, s);
    case OP_MAX: return launch_op<T, OP_MAX>(out, srcs, k, n, s);
    case OP_MIN: return launch_op<T, OP_MIN>(out, srcs, k, n, s);
    }
    return hipErrorInvalidValue;
}

template <typename T>
static hipError_t launch_real(int op, void *out, const void *const *srcs, int k, size_t n,
                              hipStream_t s)
{
    switch (op) {
    case OP_SUM: return launch_op<T, OP_SUM>(out, srcs, k, n, s);
    case OP_PROD: return launch_op<T, OP_PROD>(out, srcs, k, n, s);
    case OP_MAX: return launch_op<T, OP_MAX>(out, srcs, k, n, s);
    case OP_MIN: return launch_op<T, OP_MIN>(out, srcs, k, n, s);
    }
    return hipErrorInvalidValue;
}

template <typename T>
static hipError_t launch_cplx(int op, void *out, const void *const *srcs, int k, size_t n,
                              hipStream_t s)
{
    switch (op) {
    case OP_SUM: return launch_op<T, OP_SUM>(out, srcs, k, n, s);
    case OP_PROD: return launch_op<T, OP_PROD>(out, srcs, k, n, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_combine(int type, int op, void *out, const void *const *srcs, int k,
                          size_t n, hipStream_t s)
{
    if (k < 1 || out == nullptr) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    switch (type) {
    case T_SHORT: return launch_int<int16_t>(op, out, srcs, k, n, s);
    case T_INT: return launch_int<int32_t>(op, out, srcs, k, n, s);
    case T_LONG:
    case T_LONGLONG: return launch_int<int64_t>(op, out, srcs, k, n, s);
    case T_FLOAT: return launch_real<float>(op, out, srcs, k, n, s);
    case T_DOUBLE: return launch_real<double>(op, out, srcs, k, n, s);
    case T_COMPLEXF: return launch_cplx<cfloat>(op, out, srcs, k, n, s);
    case T_COMPLEXD: return launch_cplx<cdouble>(op, out, srcs, k, n, s);
    case T_LONGDOUBLE: return launch_longdouble(op, out, srcs, k, n, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace osgpu
