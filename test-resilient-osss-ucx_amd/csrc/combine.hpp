// combine.hpp -- internal interface between the C-ABI layer and the kernels.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>

// 16-byte vectors in flight per lane per input: for <= 2, <= 4 and <= 8
// inputs (register budget vs bytes in flight; see tools/tune_combine.hip)
#ifndef OSGPU_U_K2
#define OSGPU_U_K2 4
#endif
#ifndef OSGPU_U_K4
#define OSGPU_U_K4 4
#endif
#ifndef OSGPU_U_K8
#define OSGPU_U_K8 2
#endif

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

// Owner-computes team combine over an active set of P PEs (2 <= P <= 8):
// for i < n, dsts[q][i] = fold of srcs[*][i] in PE q's order (q first, then
// ascending, skipping q).  srcs/dsts indexed by position in the active set
// and already offset to this PE's shard.
constexpr int kMaxTeam = 8;
hipError_t launch_team(int type, int op, int P, void *const *dsts, const void *const *srcs,
                       size_t n, hipStream_t s);
hipError_t launch_team_longdouble(int op, int P, void *const *dsts, const void *const *srcs,
                                  size_t n, hipStream_t s);

// Byte copy of up to kMaxCopySegs independent ranges in one launch (copy.hip):
// the data movement of broadcast / collect / fcollect / alltoall.  Sources may
// be peer HBM.  Zero-length segments are skipped; more than kMaxCopySegs
// non-empty segments is an error (callers batch).
constexpr int kMaxCopySegs = 8;
struct CopySeg {
    const void *src;
    void *dst;
    size_t bytes;
};
hipError_t launch_copy(const CopySeg *segs, int nseg, hipStream_t s);

// x87 80-bit extended combine (soft-float on the GPU), longdouble.hip
hipError_t launch_longdouble(int op, void *out, const void *const *srcs, int k, size_t n,
                             hipStream_t s);

}  // namespace osgpu
