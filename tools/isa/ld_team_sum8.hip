#include <hip/hip_runtime.h>
#include <stdint.h>
#include "x87.hpp"
using namespace osgpu::x87;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
struct LdTeam { const unsigned char *src[8]; unsigned char *dst[8]; };
__device__ __forceinline__ X80 unpack(u64x2 v) { return X80{v.x, (uint32_t) (v.y & 0xffffu)}; }
__device__ __forceinline__ u64x2 pack(X80 x) { u64x2 v; v.x = x.m; v.y = (unsigned long long) (x.se & 0xffffu); return v; }
template <int OP, int P>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void ldk(LdTeam a, size_t n)
{
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        X80 x[P], r[P];
#pragma unroll
        for (int p = 0; p < P; p++) x[p] = unpack(__builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(a.src[p]) + i));
        team_fold_sum_prod<OP, P>(x, r);
#pragma unroll
        for (int q = 0; q < P; q++) __builtin_nontemporal_store(pack(r[q]), reinterpret_cast<u64x2 *>(a.dst[q]) + i);
    }
}
template __global__ void ldk<0, 8>(LdTeam, size_t);
