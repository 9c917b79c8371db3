// x87_check.hip -- TEST INFRASTRUCTURE: the GPU's x87 soft-float
// (csrc/x87.hpp) compiled for the HOST, so tests/test_x87_softfloat.py can
// compare it bit for bit with the reference's own x87 long double ops on
// millions of inputs without a GPU.
#include <stddef.h>
#include <stdint.h>
#include "../../test-resilient-osss-ucx_amd/csrc/x87.hpp"

using namespace osgpu::x87;

static X80 ld(const unsigned char *p)
{
    uint64_t m, se = 0;
    __builtin_memcpy(&m, p, 8);
    __builtin_memcpy(&se, p + 8, 2);
    return X80{m, (uint32_t) se};
}

extern "C" int x87check_op(int op, const void *a, const void *b, void *out, size_t n)
{
    const unsigned char *A = (const unsigned char *) a, *B = (const unsigned char *) b;
    unsigned char *O = (unsigned char *) out;
    for (size_t i = 0; i < n; i++) {
        X80 x = ld(A + 16 * i), y = ld(B + 16 * i), r;
        switch (op) {
        case 0: r = add(x, y); break;
        case 1: r = mul(x, y); break;
        case 5: r = less(y, x) ? x : y; break;
        case 6: r = less(x, y) ? x : y; break;
        default: return -1;
        }
        __builtin_memset(O + 16 * i, 0, 16);
        __builtin_memcpy(O + 16 * i, &r.m, 8);
        uint16_t se = (uint16_t) r.se;
        __builtin_memcpy(O + 16 * i + 8, &se, 2);
    }
    return 0;
}
