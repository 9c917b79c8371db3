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
        case 10: {  // the near-exponent rounds' add: add_near where it applies, else add
            XU ua = unpack_u(x), ub = unpack_u(y), ur;
            const uint32_t EA = ua.e > ub.e ? ua.e : ub.e;  // add_near's precondition
            r = normal_u(ua) && normal_u(ub) && EA >= 30 && EA <= kEmax - 2 && add_near(ua, ub, &ur)
                    ? pack_u(ur) : add(x, y);
            break;
        }
        case 11: {  // the same-sign near rounds' add, where the signs agree
            XU ua = unpack_u(x), ub = unpack_u(y), ur;
            r = ua.s == ub.s && normal_u(ua) && normal_u(ub) && ua.e <= kEmax - 2 &&
                        ub.e <= kEmax - 2 && add_same_near(ua, ub, &ur)
                    ? pack_u(ur) : add(x, y);
            break;
        }
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

// every member's result of a P-PE sum / prod / max / min, as the team kernel
// folds them (x87.hpp team_fold_sum_prod, team_fold_minmax): srcs[p] and dsts[p] are arrays of n 16-B
// elements
template <int OP, int P>
static void team_p(const unsigned char *const *srcs, unsigned char *const *dsts, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        X80 x[P], r[P];
        for (int p = 0; p < P; p++) x[p] = ld(srcs[p] + 16 * i);
        if (OP == 0 || OP == 1)
            team_fold_sum_prod<OP, P>(x, r);
        else
            team_fold_minmax<OP, P>(x, r);
        for (int p = 0; p < P; p++) {
            unsigned char *o = dsts[p] + 16 * i;
            __builtin_memset(o, 0, 16);
            __builtin_memcpy(o, &r[p].m, 8);
            uint16_t se = (uint16_t) r[p].se;
            __builtin_memcpy(o + 8, &se, 2);
        }
    }
}

extern "C" int x87check_team(int op, int P, const void *const *srcs, void *const *dsts, size_t n)
{
    const unsigned char *const *S = (const unsigned char *const *) srcs;
    unsigned char *const *D = (unsigned char *const *) dsts;
#define TP(PP)                                                                 \
    case PP:                                                                   \
        if (op == 0) team_p<0, PP>(S, D, n);                                   \
        else if (op == 1) team_p<1, PP>(S, D, n);                              \
        else if (op == 5) team_p<5, PP>(S, D, n);                              \
        else team_p<6, PP>(S, D, n);                                           \
        return 0;
    if (op != 0 && op != 1 && op != 5 && op != 6) return -1;
    switch (P) { TP(2) TP(3) TP(4) TP(5) TP(6) TP(7) TP(8) }
#undef TP
    return -1;
}
