// host_fold.hip -- the fold of a SMALL reduce-to-all call whose arrays live
// in host symmetric-heap memory, on the calling PE's own thread.
//
// The reference's whole algorithm for such a call is a CPU loop
// (src/reductions.c:79-111: copy the source into the target, barrier, pull
// every other PE's source with a blocking 64-element shmem_getmem and fold it
// through an indirect call per element, barrier).  For 1 Ki ints that loop
// takes 4-7 us; the GPU paths cannot come below a kernel launch whose
// completion the host sees (6.4 us for an empty kernel, DESIGN_HISTORY.md
// 10) plus the PCIe legs: the fused one-launch staged path takes 15-17 us.
// So while a PE pulls at most host_fold_max_bytes() from its peers
// (shmem_reduce.cpp run_host_fold) a host-heap call is folded here: one
// shmem_getmem per peer of its whole source, and a direct (inlined, not
// indirect) fold in the reference's per-PE order.
//
// The element ops are the SAME definitions the kernels use (elem_ops.hpp
// functors, x87.hpp soft-float for long double), compiled for the host: the
// results are bit-identical to the GPU paths' (tests/test_gpu_parity.py
// test_host_fold_matches_golden and tests/test_multiproc.py
// test_host_staged_processes check both against the golden vectors), not
// merely to the host compiler's view of the C operators.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "combine.hpp"
#include "elem_ops.hpp"
#include "x87.hpp"

#pragma clang fp contract(off)

namespace osgpu {
namespace {

template <typename T, int OP>
void fold_n(void *acc_v, const void *in_v, size_t n)
{
    T *acc = static_cast<T *>(acc_v);
    const T *in = static_cast<const T *>(in_v);
    for (size_t i = 0; i < n; i++) acc[i] = Elem<T, OP>::f(acc[i], in[i]);
}

// long double: 16-byte slots, value in bytes 0..9, padding written as zero
// (as longdouble.hip stores it)
template <int OP>
void fold_ld(void *acc_v, const void *in_v, size_t n)
{
    uint64_t *acc = static_cast<uint64_t *>(acc_v);
    const uint64_t *in = static_cast<const uint64_t *>(in_v);
    for (size_t i = 0; i < n; i++) {
        const x87::X80 a{acc[2 * i], (uint32_t) (acc[2 * i + 1] & 0xffffu)};
        const x87::X80 b{in[2 * i], (uint32_t) (in[2 * i + 1] & 0xffffu)};
        x87::X80 r;
        if (OP == OP_SUM) r = x87::add(a, b);
        else if (OP == OP_PROD) r = x87::mul(a, b);
        else if (OP == OP_MAX) r = x87::less(b, a) ? a : b;  // a > b ? a : b
        else r = x87::less(a, b) ? a : b;                     // a < b ? a : b
        acc[2 * i] = r.m;
        acc[2 * i + 1] = (uint64_t) (r.se & 0xffffu);
    }
}

typedef void (*FoldFn)(void *, const void *, size_t);

template <typename T>
FoldFn int_fn(int op)
{
    switch (op) {
    case OP_SUM: return fold_n<T, OP_SUM>;
    case OP_PROD: return fold_n<T, OP_PROD>;
    case OP_AND: return fold_n<T, OP_AND>;
    case OP_OR: return fold_n<T, OP_OR>;
    case OP_XOR: return fold_n<T, OP_XOR>;
    case OP_MAX: return fold_n<T, OP_MAX>;
    case OP_MIN: return fold_n<T, OP_MIN>;
    }
    return nullptr;
}

template <typename T>
FoldFn real_fn(int op)
{
    switch (op) {
    case OP_SUM: return fold_n<T, OP_SUM>;
    case OP_PROD: return fold_n<T, OP_PROD>;
    case OP_MAX: return fold_n<T, OP_MAX>;
    case OP_MIN: return fold_n<T, OP_MIN>;
    }
    return nullptr;
}

template <typename T>
FoldFn cplx_fn(int op)
{
    switch (op) {
    case OP_SUM: return fold_n<T, OP_SUM>;
    case OP_PROD: return fold_n<T, OP_PROD>;
    }
    return nullptr;
}

FoldFn ld_fn(int op)
{
    switch (op) {
    case OP_SUM: return fold_ld<OP_SUM>;
    case OP_PROD: return fold_ld<OP_PROD>;
    case OP_MAX: return fold_ld<OP_MAX>;
    case OP_MIN: return fold_ld<OP_MIN>;
    }
    return nullptr;
}

FoldFn fold_fn(int type, int op)
{
    switch (type) {
    case T_SHORT: return int_fn<int16_t>(op);
    case T_INT: return int_fn<int32_t>(op);
    case T_LONG:
    case T_LONGLONG: return int_fn<int64_t>(op);
    case T_FLOAT: return real_fn<float>(op);
    case T_DOUBLE: return real_fn<double>(op);
    case T_COMPLEXF: return cplx_fn<cfloat>(op);
    case T_COMPLEXD: return cplx_fn<cdouble>(op);
    case T_LONGDOUBLE: return ld_fn(op);
    }
    return nullptr;
}

}  // namespace

bool host_fold_supported(int type, int op) { return fold_fn(type, op) != nullptr; }

// acc[i] = op(acc[i], in[i]) for i < n, elements of `type`
bool host_fold(int type, int op, void *acc, const void *in, size_t n)
{
    const FoldFn f = fold_fn(type, op);
    if (!f) return false;
    f(acc, in, n);
    return true;
}

}  // namespace osgpu
