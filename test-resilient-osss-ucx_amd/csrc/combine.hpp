// combine.hpp -- internal interface between the C-ABI layer and the kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>

namespace osgpu {

// type codes (same numbering as include/osgpu_reduce.h OSGPU_T_*)
enum TypeCode {
    T_SHORT = 0, T_INT, T_LONG, T_LONGLONG, T_FLOAT, T_DOUBLE, T_LONGDOUBLE,
    T_COMPLEXF, T_COMPLEXD, T_NTYPES
};

// out[i] = fold(op, srcs[0][i], srcs[1][i], ..., srcs[k-1][i]) for i < n,
// enqueued on stream s.  All pointers are device-accessible (local HBM or a
// peer GPU's HBM mapped into this process).  `out` may alias srcs[0].
hipError_t launch_combine(int type, int op, void *out, const void *const *srcs, int k,
                          size_t n, hipStream_t s);

// x87 80-bit extended combine (soft-float on the GPU), longdouble.hip
hipError_t launch_longdouble(int op, void *out, const void *const *srcs, int k, size_t n,
                             hipStream_t s);

}  // namespace osgpu
