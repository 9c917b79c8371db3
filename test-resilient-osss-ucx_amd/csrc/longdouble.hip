// longdouble.hip -- shmem_longdouble_{sum,prod,max,min}_to_all combine on gfx950.
//
// The reference folds `long double` with x87 instructions (fadd / fmul /
// fcomi from src/shmemu/miscops.c:30,98 compiled for x86-64), i.e. 80-bit
// extended precision: 64-bit significand with an explicit integer bit,
// 15-bit exponent, round-to-nearest-even, gradual underflow.  The GPU has
// no such type, so this file is a bit-exact x87 soft-float:
//
//   * encodings: zero, denormal (e=0, J=0), pseudo-denormal (e=0, J=1; the
//     same value as e=1), normal, infinity, QNaN/SNaN; "unsupported"
//     encodings (unnormal: 0<e<0x7fff with J=0; pseudo-infinity/pseudo-NaN:
//     e=0x7fff with J=0) are invalid operands;
//   * add/mul: exact 128-bit intermediate, one RNE rounding to 64 bits (or
//     to the denormal grid), overflow to infinity;
//   * NaN results (probed through the reference's own compiled ops, see
//     tests/test_oracle.py and DESIGN.md): an invalid operand or invalid
//     operation gives the default NaN ffff:c000000000000000 (even beside a
//     NaN operand); otherwise the NaN with the larger 64-bit significand wins,
//     quieted; equal significands -> positive sign;
//   * min/max: `a<b?a:b` / `a>b?a:b` with fcomi semantics: any NaN or
//     unsupported operand is unordered (-> b), +0 == -0, selection returns
//     the original encoding.
// Storage: 16 bytes per element (x86-64 ABI); bytes 10..15 are padding and
// are written as zero.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "combine.hpp"
#include "x87.hpp"

namespace osgpu {
namespace x87 {

__device__ __forceinline__ X80 load(const unsigned char *p)
{
    const uint64_t *q = reinterpret_cast<const uint64_t *>(p);
    return X80{q[0], (uint32_t) (q[1] & 0xffffu)};
}

__device__ __forceinline__ void store(unsigned char *p, X80 x)
{
    uint64_t *q = reinterpret_cast<uint64_t *>(p);
    q[0] = x.m;
    q[1] = (uint64_t) (x.se & 0xffffu);          // padding bytes written as zero
}

template <int OP>
__device__ __forceinline__ X80 apply(X80 a, X80 b)
{
    if (OP == 0) return add(a, b);
    if (OP == 1) return mul(a, b);
    if (OP == 5) return less(b, a) ? a : b;      // max: a > b ? a : b
    return less(a, b) ? a : b;                   // min: a < b ? a : b
}

constexpr int kMaxIn = 8;

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ X80 unpack(u64x2 v) { return X80{v.x, (uint32_t) (v.y & 0xffffu)}; }
__device__ __forceinline__ u64x2 pack(X80 x)
{
    u64x2 v;
    v.x = x.m;
    v.y = (unsigned long long) (x.se & 0xffffu);  // padding bytes written as zero
    return v;
}

template <int K>
struct LdVecInputs {
    const u64x2 *p[K];
};

// elements in flight per lane for 3..8 inputs (soft-float registers)
constexpr int kLdUK8 = 4;

// 16-byte aligned arrays: one dwordx4 per element per input, U elements per
// lane with every load issued before the soft-float fold
template <int OP, int K>
__global__ __launch_bounds__(256) void ld_vec_kernel(u64x2 *out, LdVecInputs<K> in, size_t n)
{
    constexpr int U = K <= 2 ? 4 : kLdUK8;
    const size_t base = (size_t) blockIdx.x * (256 * U) + threadIdx.x;
    u64x2 raw[U][K];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t) u * 256;
        if (i < n) {
#pragma unroll
            for (int k = 0; k < K; k++) raw[u][k] = __builtin_nontemporal_load(in.p[k] + i);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t) u * 256;
        if (i < n) {
            X80 acc = unpack(raw[u][0]);
#pragma unroll
            for (int k = 1; k < K; k++) acc = apply<OP>(acc, unpack(raw[u][k]));
            __builtin_nontemporal_store(pack(acc), out + i);
        }
    }
}

template <int OP>
static hipError_t ld_vec_launch(int K, void *out, const void *const *srcs, size_t n,
                                hipStream_t s)
{
#define LDV(KK)                                                                \
    case KK: {                                                                 \
        LdVecInputs<KK> in;                                                    \
        for (int k = 0; k < KK; k++) in.p[k] = (const u64x2 *) srcs[k];        \
        constexpr int U = KK <= 2 ? 4 : kLdUK8;                                     \
        size_t blocks = (n + 256 * U - 1) / (256 * U);                         \
        hipLaunchKernelGGL((ld_vec_kernel<OP, KK>), dim3((unsigned) (blocks ? blocks : 1)), \
                           dim3(256), 0, s, (u64x2 *) out, in, n);             \
        return hipGetLastError();                                              \
    }
    switch (K) {
        LDV(1) LDV(2) LDV(3) LDV(4) LDV(5) LDV(6) LDV(7) LDV(8)
    }
#undef LDV
    return hipErrorInvalidValue;
}

struct LdInputs {
    const unsigned char *p[kMaxIn];
};

template <int OP>
__global__ __launch_bounds__(256) void ld_combine_kernel(unsigned char *out, LdInputs in,
                                                         int k, size_t n)
{
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        X80 acc = load(in.p[0] + 16 * i);
        for (int j = 1; j < k; j++) acc = apply<OP>(acc, load(in.p[j] + 16 * i));
        store(out + 16 * i, acc);
    }
}

}  // namespace x87

hipError_t launch_longdouble(int op, void *out, const void *const *srcs, int k, size_t n,
                             hipStream_t s)
{
    if (op != 0 && op != 1 && op != 5 && op != 6) return hipErrorInvalidValue;
    for (int j = 0; j < k; j++)
        if (((uintptr_t) srcs[j] & 7) != 0) return hipErrorInvalidValue;
    if (((uintptr_t) out & 7) != 0) return hipErrorInvalidValue;
    size_t blocks = (n + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    if (blocks == 0) blocks = 1;
    // chunks of up to 8 inputs, left to right: out = fold(out, next 7 ...)
    int done = 0;
    bool first = true;
    while (done < k) {
        x87::LdInputs in;
        int m = 0;
        if (!first) in.p[m++] = (const unsigned char *) out;
        while (m < x87::kMaxIn && done < k) in.p[m++] = (const unsigned char *) srcs[done++];
        first = false;
        bool aligned16 = ((uintptr_t) out & 15) == 0;
        for (int j = 0; j < m; j++) aligned16 = aligned16 && ((uintptr_t) in.p[j] & 15) == 0;
        if (aligned16) {  // the usual case: x86-64 long double arrays are 16-B aligned
            const void *vp[x87::kMaxIn];
            for (int j = 0; j < m; j++) vp[j] = in.p[j];
            hipError_t e;
            switch (op) {
            case 0: e = x87::ld_vec_launch<0>(m, out, vp, n, s); break;
            case 1: e = x87::ld_vec_launch<1>(m, out, vp, n, s); break;
            case 5: e = x87::ld_vec_launch<5>(m, out, vp, n, s); break;
            default: e = x87::ld_vec_launch<6>(m, out, vp, n, s); break;
            }
            if (e != hipSuccess) return e;
            continue;
        }
        switch (op) {
        case 0: hipLaunchKernelGGL(x87::ld_combine_kernel<0>, dim3((unsigned) blocks), dim3(256), 0, s,
                                   (unsigned char *) out, in, m, n); break;
        case 1: hipLaunchKernelGGL(x87::ld_combine_kernel<1>, dim3((unsigned) blocks), dim3(256), 0, s,
                                   (unsigned char *) out, in, m, n); break;
        case 5: hipLaunchKernelGGL(x87::ld_combine_kernel<5>, dim3((unsigned) blocks), dim3(256), 0, s,
                                   (unsigned char *) out, in, m, n); break;
        default: hipLaunchKernelGGL(x87::ld_combine_kernel<6>, dim3((unsigned) blocks), dim3(256), 0, s,
                                    (unsigned char *) out, in, m, n); break;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

namespace x87 {

struct LdTeam {
    const unsigned char *src[kMaxTeam];
    unsigned char *dst[kMaxTeam];
};

// owner-computes form (team.hip): every PE's own fold order, P(P-1) soft
// ops per element; P is a template parameter so the P inputs stay in
// registers.  sum / prod: x87.hpp team_fold_sum_prod (P-1 folds advanced
// in rounds); max / min: team_fold_minmax (P key compares, then every
// member's pick among the tied extremes).
// VEC: 16-byte aligned arrays (the x86-64 layout), one dwordx4 per element.
// At least 4 waves per SIMD (<= 128 VGPRs): the 8-member sum's rounds want
// 132, and 3 waves per SIMD cost the same-sign sums 6-7 % (interleaved A/B,
// profiles/r03_ld_variants.jsonl).
#ifndef OSGPU_LD_WAVES
#define OSGPU_LD_WAVES 4
#endif
template <int OP, int P, bool VEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OSGPU_LD_WAVES))) void ld_team_kernel(
    LdTeam a, size_t n)
{
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        X80 x[P], r[P];
#pragma unroll
        for (int p = 0; p < P; p++)
            x[p] = VEC ? unpack(__builtin_nontemporal_load(
                             reinterpret_cast<const u64x2 *>(a.src[p]) + i))
                       : load(a.src[p] + 16 * i);
        if (OP == 0 || OP == 1) {
            team_fold_sum_prod<OP, P>(x, r);
        } else if (P > 2) {
            team_fold_minmax<OP, P>(x, r);
        } else {  // two members: one compare each
            r[0] = apply<OP>(x[0], x[1]);
            r[1] = apply<OP>(x[1], x[0]);
        }
#pragma unroll
        for (int q = 0; q < P; q++) {
            if (VEC)
                __builtin_nontemporal_store(pack(r[q]), reinterpret_cast<u64x2 *>(a.dst[q]) + i);
            else
                store(a.dst[q] + 16 * i, r[q]);
        }
    }
}

template <int OP>
hipError_t ld_team_launch(int P, bool vec, const LdTeam &a, size_t n, unsigned blocks,
                          hipStream_t s)
{
    switch (P) {
#define LDT(PP)                                                                \
    case PP:                                                                   \
        if (vec)                                                               \
            hipLaunchKernelGGL((ld_team_kernel<OP, PP, true>), dim3(blocks), dim3(256), 0, s, a, n); \
        else                                                                   \
            hipLaunchKernelGGL((ld_team_kernel<OP, PP, false>), dim3(blocks), dim3(256), 0, s, a, n); \
        return hipGetLastError();
        LDT(2) LDT(3) LDT(4) LDT(5) LDT(6) LDT(7) LDT(8)
#undef LDT
    }
    return hipErrorInvalidValue;
}

}  // namespace x87

hipError_t launch_team_longdouble(int op, int P, void *const *dsts, const void *const *srcs,
                                  size_t n, hipStream_t s)
{
    if (P < 2 || P > kMaxTeam) return hipErrorInvalidValue;
    x87::LdTeam a;
    bool vec = true;
    for (int p = 0; p < P; p++) {
        a.src[p] = (const unsigned char *) srcs[p];
        a.dst[p] = (unsigned char *) dsts[p];
        if ((((uintptr_t) srcs[p]) | ((uintptr_t) dsts[p])) & 7) return hipErrorInvalidValue;
        vec = vec && ((((uintptr_t) srcs[p]) | ((uintptr_t) dsts[p])) & 15) == 0;
    }
    size_t blocks = (n + 255) / 256;
    blocks = blocks > 16384 ? 16384 : (blocks ? blocks : 1);
    switch (op) {
    case 0: return x87::ld_team_launch<0>(P, vec, a, n, (unsigned) blocks, s);
    case 1: return x87::ld_team_launch<1>(P, vec, a, n, (unsigned) blocks, s);
    case 5: return x87::ld_team_launch<5>(P, vec, a, n, (unsigned) blocks, s);
    case 6: return x87::ld_team_launch<6>(P, vec, a, n, (unsigned) blocks, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace osgpu
