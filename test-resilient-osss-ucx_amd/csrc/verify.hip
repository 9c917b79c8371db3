// verify.hip -- full-size parity checks on the GPU, without copying the
// arrays to the host: a checksum of a whole array (so "checksum of the
// target == combination of the sources' checksums" can be checked at
// BASELINE sizes) and a bitwise compare of two arrays.
//
// Shape: a grid-stride 16-B streaming pass (HBM-bound, like the combine),
// each lane folding into a 64-bit register; wavefront reduction with
// cross-lane shuffles (compare: a ballot + popcount per wave); one partial
// per wave staged in LDS; one atomic per workgroup into the result.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "combine.hpp"

namespace osgpu {

namespace {

constexpr int kVBlock = 256;
constexpr int kWaves = kVBlock / 64;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix64(uint64_t z)  // splitmix64 finaliser
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// fold element value v (zero-extended; 16-byte elements pre-mixed to one
// word) at index idx into the lane's accumulator
template <int MODE>
__device__ __forceinline__ uint64_t fold_elem(uint64_t acc, uint64_t v, size_t idx)
{
    if (MODE == CK_SUM) return acc + v;
    if (MODE == CK_XOR) return acc ^ v;
    return acc + mix64(v + 0x9e3779b97f4a7c15ull * (uint64_t) (idx + 1));  // CK_HASH
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ uint64_t wave_xor(uint64_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
    return v;
}

// wave reduction, per-wave partials in LDS, one atomic per workgroup
template <int MODE>
__device__ __forceinline__ void block_publish(uint64_t acc, unsigned long long *out)
{
    __shared__ uint64_t part[kWaves];
    acc = MODE == CK_XOR ? wave_xor(acc) : wave_sum(acc);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) part[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = part[0];
        for (int w = 1; w < kWaves; w++) t = MODE == CK_XOR ? (t ^ part[w]) : (t + part[w]);
        if (MODE == CK_XOR) atomicXor(out, (unsigned long long) t);
        else atomicAdd(out, (unsigned long long) t);
    }
}

// fold the W = 16 / ES elements of vector j
template <int ES, int MODE>
__device__ __forceinline__ uint64_t fold_vec(uint64_t acc, u32x4 v, size_t j)
{
    if (ES == 2) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            acc = fold_elem<MODE>(acc, v[k] & 0xffffu, j * 8 + 2 * k);
            acc = fold_elem<MODE>(acc, v[k] >> 16, j * 8 + 2 * k + 1);
        }
    } else if (ES == 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) acc = fold_elem<MODE>(acc, v[k], j * 4 + k);
    } else if (ES == 8) {
        acc = fold_elem<MODE>(acc, (uint64_t) v[0] | (uint64_t) v[1] << 32, j * 2);
        acc = fold_elem<MODE>(acc, (uint64_t) v[2] | (uint64_t) v[3] << 32, j * 2 + 1);
    } else {
        const uint64_t lo = (uint64_t) v[0] | (uint64_t) v[1] << 32;
        const uint64_t hi = (uint64_t) v[2] | (uint64_t) v[3] << 32;
        acc = fold_elem<MODE>(acc, lo ^ mix64(hi), j);
    }
    return acc;
}

// ES: element bytes.  Elements are read 16 B at a time when the array is
// 16-B aligned (the body), byte-assembled otherwise and for the tail.
template <int ES, int MODE>
__global__ __launch_bounds__(kVBlock) void checksum_kernel(const unsigned char *p, size_t n,
                                                           unsigned long long *out)
{
    constexpr int W = 16 / ES;
    const size_t tid = (size_t) blockIdx.x * kVBlock + threadIdx.x;
    const size_t stride = (size_t) gridDim.x * kVBlock;
    uint64_t acc = 0;
    const bool vec = ((uintptr_t) p & 15) == 0;
    const size_t nvec = vec ? n / W : 0;
    // tiles of kVBlock * 4 consecutive vectors per workgroup, four vectors
    // in flight per lane; the last partial tile one vector at a time
    const u32x4 *vp = reinterpret_cast<const u32x4 *>(p);
    constexpr size_t kTile = (size_t) kVBlock * 4;
    const size_t full = nvec / kTile;
    for (size_t t = blockIdx.x; t < full; t += gridDim.x) {
        const size_t j0 = t * kTile + threadIdx.x;
        u32x4 w[4];
#pragma unroll
        for (int u = 0; u < 4; u++) w[u] = __builtin_nontemporal_load(vp + j0 + u * kVBlock);
#pragma unroll
        for (int u = 0; u < 4; u++) acc = fold_vec<ES, MODE>(acc, w[u], j0 + u * kVBlock);
    }
    for (size_t j = full * kTile + tid; j < nvec; j += stride)
        acc = fold_vec<ES, MODE>(acc, __builtin_nontemporal_load(vp + j), j);
    for (size_t i = nvec * W + tid; i < n; i += stride) {
        const unsigned char *e = p + i * ES;
        uint64_t v = 0;
        if (ES == 16) {
            uint64_t lo = 0, hi = 0;
            for (int b = 0; b < 8; b++) lo |= (uint64_t) e[b] << (8 * b);
            for (int b = 0; b < 8; b++) hi |= (uint64_t) e[8 + b] << (8 * b);
            v = lo ^ mix64(hi);
        } else {
            for (int b = 0; b < ES; b++) v |= (uint64_t) e[b] << (8 * b);
        }
        acc = fold_elem<MODE>(acc, v, i);
    }
    block_publish<MODE>(acc, out);
}

// Bitwise compare: out[0] += differing 16-B vectors (differing bytes for an
// unaligned pair), out[1] = min byte offset of a difference (~0 if none).
__global__ __launch_bounds__(kVBlock) void compare_kernel(const unsigned char *a,
                                                          const unsigned char *b, size_t nbytes,
                                                          unsigned long long *out)
{
    const size_t tid = (size_t) blockIdx.x * kVBlock + threadIdx.x;
    const size_t stride = (size_t) gridDim.x * kVBlock;
    const bool vec = (((uintptr_t) a | (uintptr_t) b) & 15) == 0;
    const size_t nvec = vec ? nbytes / 16 : 0;
    uint64_t bad = 0, first = ~0ull;
    auto check = [&](const u32x4 &x, const u32x4 &y, size_t j) {
        const bool diff = x[0] != y[0] || x[1] != y[1] || x[2] != y[2] || x[3] != y[3];
        const uint64_t m = __ballot(diff);  // the wave's differing vectors
        if ((threadIdx.x & 63) == 0) bad += (uint64_t) __popcll(m);
        if (diff && j * 16 < first) first = j * 16;
    };
    const u32x4 *va = reinterpret_cast<const u32x4 *>(a), *vb = reinterpret_cast<const u32x4 *>(b);
    constexpr size_t kTile = (size_t) kVBlock * 2;  // two vectors of each array in flight
    const size_t full = nvec / kTile;
    for (size_t t = blockIdx.x; t < full; t += gridDim.x) {
        const size_t j0 = t * kTile + threadIdx.x;
        const u32x4 x0 = __builtin_nontemporal_load(va + j0), y0 = __builtin_nontemporal_load(vb + j0);
        const u32x4 x1 = __builtin_nontemporal_load(va + j0 + kVBlock);
        const u32x4 y1 = __builtin_nontemporal_load(vb + j0 + kVBlock);
        check(x0, y0, j0);
        check(x1, y1, j0 + kVBlock);
    }
    for (size_t j = full * kTile + tid; j < nvec; j += stride)
        check(__builtin_nontemporal_load(va + j), __builtin_nontemporal_load(vb + j), j);
    for (size_t i = nvec * 16 + tid; i < nbytes; i += stride)
        if (a[i] != b[i]) {
            bad++;
            if (i < first) first = i;
        }
    block_publish<CK_SUM>(bad, out);
    if (first != ~0ull) atomicMin(out + 1, (unsigned long long) first);
}

unsigned grid_for(size_t work)
{
    size_t g = (work + kVBlock - 1) / kVBlock;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;  // 16 workgroups per CU, then grid-stride
    return (unsigned) g;
}

template <int ES>
hipError_t launch_ck(int mode, const void *p, size_t n, unsigned long long *out, hipStream_t s)
{
    const unsigned g = grid_for(n * ES / 16 + 1);
    const unsigned char *q = static_cast<const unsigned char *>(p);
    switch (mode) {
    case CK_SUM:
        hipLaunchKernelGGL((checksum_kernel<ES, CK_SUM>), dim3(g), dim3(kVBlock), 0, s, q, n, out);
        break;
    case CK_XOR:
        hipLaunchKernelGGL((checksum_kernel<ES, CK_XOR>), dim3(g), dim3(kVBlock), 0, s, q, n, out);
        break;
    case CK_HASH:
        hipLaunchKernelGGL((checksum_kernel<ES, CK_HASH>), dim3(g), dim3(kVBlock), 0, s, q, n,
                           out);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_checksum(int elem_bytes, int mode, const void *p, size_t n,
                           unsigned long long *out, hipStream_t s)
{
    switch (elem_bytes) {
    case 2: return launch_ck<2>(mode, p, n, out, s);
    case 4: return launch_ck<4>(mode, p, n, out, s);
    case 8: return launch_ck<8>(mode, p, n, out, s);
    case 16: return launch_ck<16>(mode, p, n, out, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_compare(const void *a, const void *b, size_t nbytes, unsigned long long *out,
                          hipStream_t s)
{
    hipLaunchKernelGGL(compare_kernel, dim3(grid_for(nbytes / 16 + 1)), dim3(kVBlock), 0, s,
                       static_cast<const unsigned char *>(a), static_cast<const unsigned char *>(b),
                       nbytes, out);
    return hipGetLastError();
}

}  // namespace osgpu
