/*
 * oracle_ops.c -- CPU restatement of the reference's element operations.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Build: -O2 -ffp-contract=off,
 * no -ffast-math, no -march (baseline x86-64 SSE2, like the reference).
 *
 * The reference ops are one-line C functions (src/reductions.c calls them
 * through a function pointer per element, src/reductions.c:95-96,105-106):
 *   sum/prod   a+b, a*b                   src/shmemu/miscops.c:12-39
 *   and/or/xor a&b, a|b, a^b              src/shmemu/miscops.c:46-73
 *   min/max    a<b?a:b, a>b?a:b           src/shmemu/miscops.c:80-105
 * `a` is the running accumulator, `b` the incoming peer element.
 *
 * Floating point is restated as an explicit model rather than "whatever the
 * compiler emits", so the same model can be written down for the GPU:
 *   - non-NaN results: IEEE-754 binary32/64, round-to-nearest-even, no FMA
 *     contraction, subnormals kept (x86-64 SSE with default MXCSR);
 *   - NaN results follow the SSE rule for a two-operand instruction whose
 *     first source is `a`: a NaN `a` is returned quieted, else a NaN `b` is
 *     returned quieted, else (invalid operation) the default NaN, which on x86
 *     is the NEGATIVE quiet NaN 0xFFF8... / 0xFFC00000.  The compiled
 *     reference emits `addsd %xmm1,%xmm0` (first source = a) for a+b, see
 *     `objdump -d miscops.o`.
 *   - complex product: GCC expands `a*b` inline and calls libgcc
 *     __muldc3/__mulsc3 when the real OR imaginary part of the inline result
 *     is NaN (`ucomisd x,y; jp` in the compiled shmemu_prod_complex{d,f}_func);
 *     __mul?c3 (libgcc2.c, GCC 11.4) is restated with the operand order of
 *     its compiled body.
 *   - long double: native x87 arithmetic of this host == the reference's.
 * Integers: two's-complement wrap (the reference relies on gcc's wrapping
 * codegen for signed overflow; short is promoted to int and truncated).
 */
#include "oracle.h"

#include <complex.h>
#include <math.h>
#include <string.h>

size_t oracle_type_size(int type)
{
    switch (type) {
    case OR_SHORT: return sizeof(short);
    case OR_INT: return sizeof(int);
    case OR_LONG: return sizeof(long);
    case OR_LONGLONG: return sizeof(long long);
    case OR_FLOAT: return sizeof(float);
    case OR_DOUBLE: return sizeof(double);
    case OR_LONGDOUBLE: return sizeof(long double);
    case OR_COMPLEXF: return sizeof(float _Complex);
    case OR_COMPLEXD: return sizeof(double _Complex);
    default: return 0;
    }
}

/* src/reductions.c:248-297: which (type, op) pairs exist */
int oracle_has_op(int type, int op)
{
    if (type < 0 || type >= OR_NTYPES || op < 0 || op >= OR_NOPS) return 0;
    switch (op) {
    case OR_SUM: case OR_PROD: return 1;
    case OR_AND: case OR_OR: case OR_XOR: return type <= OR_LONGLONG;
    case OR_MAX: case OR_MIN: return type <= OR_LONGDOUBLE;
    }
    return 0;
}

/* ---------------- SSE NaN model (binary64 / binary32) ---------------- */

static inline uint64_t bits_d(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double from_d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static inline uint32_t bits_f(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static inline float from_f(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }

static inline int nan_d(double x) { return (bits_d(x) & 0x7fffffffffffffffull) > 0x7ff0000000000000ull; }
static inline int nan_f(float x) { return (bits_f(x) & 0x7fffffffu) > 0x7f800000u; }
static inline int inf_d(double x) { return (bits_d(x) & 0x7fffffffffffffffull) == 0x7ff0000000000000ull; }
static inline int inf_f(float x) { return (bits_f(x) & 0x7fffffffu) == 0x7f800000u; }

#define QBIT_D 0x0008000000000000ull
#define QBIT_F 0x00400000u
#define DEFNAN_D 0xfff8000000000000ull
#define DEFNAN_F 0xffc00000u

static inline double sse_fix_d(double r, double a, double b)
{
    if (!nan_d(r)) return r;
    if (nan_d(a)) return from_d(bits_d(a) | QBIT_D);
    if (nan_d(b)) return from_d(bits_d(b) | QBIT_D);
    return from_d(DEFNAN_D);
}

static inline float sse_fix_f(float r, float a, float b)
{
    if (!nan_f(r)) return r;
    if (nan_f(a)) return from_f(bits_f(a) | QBIT_F);
    if (nan_f(b)) return from_f(bits_f(b) | QBIT_F);
    return from_f(DEFNAN_F);
}

/* volatile-free: -ffp-contract=off guarantees separate roundings */
static inline double add_d(double a, double b) { return sse_fix_d(a + b, a, b); }
static inline double sub_d(double a, double b) { return sse_fix_d(a - b, a, b); }
static inline double mul_d(double a, double b) { return sse_fix_d(a * b, a, b); }
static inline float add_f(float a, float b) { return sse_fix_f(a + b, a, b); }
static inline float sub_f(float a, float b) { return sse_fix_f(a - b, a, b); }
static inline float mul_f(float a, float b) { return sse_fix_f(a * b, a, b); }

static inline double copysign_d(double mag, double sgn)
{
    return from_d((bits_d(mag) & 0x7fffffffffffffffull) | (bits_d(sgn) & 0x8000000000000000ull));
}
static inline float copysign_f(float mag, float sgn)
{
    return from_f((bits_f(mag) & 0x7fffffffu) | (bits_f(sgn) & 0x80000000u));
}

/*
 * libgcc2.c __muldc3 (GCC 11.4), operand order of the compiled body:
 *   ac=a*c bd=b*d ad=a*d bc=c*b ; x=ac-bd ; y=ad+bc
 *   recovery: x=(a*c-b*d)*INF ; y=INF*(a*d+b*c)
 */
#define DEF_MULC3(SUF, T, ADD, SUB, MUL, ISNAN, ISINF, CPS)                    \
    static void mulc3_##SUF(T a, T b, T c, T d, T *xr, T *yr)                  \
    {                                                                          \
        const T one = 1, zero = 0, inf = (T)INFINITY;                          \
        T ac = MUL(a, c), bd = MUL(b, d), ad = MUL(a, d), bc = MUL(c, b);      \
        T x = SUB(ac, bd), y = ADD(ad, bc);                                    \
        if (ISNAN(x) && ISNAN(y)) {                                            \
            int recalc = 0;                                                    \
            if (ISINF(a) || ISINF(b)) {                                        \
                a = CPS(ISINF(a) ? one : zero, a);                             \
                b = CPS(ISINF(b) ? one : zero, b);                             \
                if (ISNAN(c)) c = CPS(zero, c);                                \
                if (ISNAN(d)) d = CPS(zero, d);                                \
                recalc = 1;                                                    \
            }                                                                  \
            if (ISINF(c) || ISINF(d)) {                                        \
                c = CPS(ISINF(c) ? one : zero, c);                             \
                d = CPS(ISINF(d) ? one : zero, d);                             \
                if (ISNAN(a)) a = CPS(zero, a);                                \
                if (ISNAN(b)) b = CPS(zero, b);                                \
                recalc = 1;                                                    \
            }                                                                  \
            if (!recalc && (ISINF(ac) || ISINF(bd) || ISINF(ad) || ISINF(bc))) { \
                if (ISNAN(a)) a = CPS(zero, a);                                \
                if (ISNAN(b)) b = CPS(zero, b);                                \
                if (ISNAN(c)) c = CPS(zero, c);                                \
                if (ISNAN(d)) d = CPS(zero, d);                                \
                recalc = 1;                                                    \
            }                                                                  \
            if (recalc) {                                                      \
                x = MUL(SUB(MUL(a, c), MUL(b, d)), inf);                       \
                y = MUL(inf, ADD(MUL(a, d), MUL(b, c)));                       \
            }                                                                  \
        }                                                                      \
        *xr = x;                                                               \
        *yr = y;                                                               \
    }                                                                          \
    /* GCC's inline expansion of complex `*` (miscops.c:19-21 at :38-39):     \
       plain products; any NaN part -> libcall.  Payloads of the inline path  \
       never escape, so plain IEEE ops suffice there. */                      \
    static void cmul_##SUF(T a, T b, T c, T d, T *xr, T *yr)                   \
    {                                                                          \
        T x = a * c - b * d;                                                   \
        T y = a * d + b * c;                                                   \
        if (ISNAN(x) || ISNAN(y)) {                                            \
            mulc3_##SUF(a, b, c, d, &x, &y);                                   \
        }                                                                      \
        *xr = x;                                                               \
        *yr = y;                                                               \
    }

DEF_MULC3(d, double, add_d, sub_d, mul_d, nan_d, inf_d, copysign_d)
DEF_MULC3(f, float, add_f, sub_f, mul_f, nan_f, inf_f, copysign_f)

/* ---------------- elementwise driver ---------------- */

#define INT_OPS(T, UT)                                                         \
    do {                                                                       \
        const T *A = (const T *) a, *B = (const T *) b;                        \
        T *O = (T *) out;                                                      \
        for (size_t i = 0; i < n; i++) {                                       \
            T x = A[i], y = B[i], r;                                           \
            switch (op) {                                                      \
            case OR_SUM: r = (T) (UT) ((UT) x + (UT) y); break;                \
            case OR_PROD: r = (T) (UT) ((UT) x * (UT) y); break;               \
            case OR_AND: r = x & y; break;                                     \
            case OR_OR: r = x | y; break;                                      \
            case OR_XOR: r = x ^ y; break;                                     \
            case OR_MAX: r = x > y ? x : y; break;                             \
            default: r = x < y ? x : y; break;                                 \
            }                                                                  \
            O[i] = r;                                                          \
        }                                                                      \
    } while (0)

#define FP_OPS(T, ADD, MUL)                                                    \
    do {                                                                       \
        const T *A = (const T *) a, *B = (const T *) b;                        \
        T *O = (T *) out;                                                      \
        for (size_t i = 0; i < n; i++) {                                       \
            T x = A[i], y = B[i], r;                                           \
            switch (op) {                                                      \
            case OR_SUM: r = ADD(x, y); break;                                 \
            case OR_PROD: r = MUL(x, y); break;                                \
            case OR_MAX: r = x > y ? x : y; break;                             \
            default: r = x < y ? x : y; break;                                 \
            }                                                                  \
            O[i] = r;                                                          \
        }                                                                      \
    } while (0)

static inline long double add_ld(long double x, long double y) { return x + y; }
static inline long double mul_ld(long double x, long double y) { return x * y; }

int oracle_op(int type, int op, const void *a, const void *b, void *out,
              size_t n)
{
    if (!oracle_has_op(type, op)) return -1;
    switch (type) {
    case OR_SHORT:
        /* short arithmetic happens in int and is truncated (C promotion);
           the low 16 bits of 32-bit unsigned arithmetic are identical */
        INT_OPS(short, uint32_t);
        break;
    case OR_INT: INT_OPS(int, uint32_t); break;
    case OR_LONG: INT_OPS(long, uint64_t); break;
    case OR_LONGLONG: INT_OPS(long long, uint64_t); break;
    case OR_FLOAT: FP_OPS(float, add_f, mul_f); break;
    case OR_DOUBLE: FP_OPS(double, add_d, mul_d); break;
    case OR_LONGDOUBLE: FP_OPS(long double, add_ld, mul_ld); break;
    case OR_COMPLEXF: {
        const float *A = (const float *) a, *B = (const float *) b;
        float *O = (float *) out;
        for (size_t i = 0; i < n; i++) {
            float ar = A[2 * i], ai = A[2 * i + 1], br = B[2 * i], bi = B[2 * i + 1];
            float xr, xi;
            /* the compiled shmemu_sum_complexf_func adds the imaginary parts
               as b.im + a.im (`addss -0x4(%rsp),%xmm0`, xmm0 = b.im): the
               first source -- and so the surviving NaN -- is b's */
            if (op == OR_SUM) { xr = add_f(ar, br); xi = add_f(bi, ai); }
            else cmul_f(ar, ai, br, bi, &xr, &xi);
            O[2 * i] = xr;
            O[2 * i + 1] = xi;
        }
        break;
    }
    case OR_COMPLEXD: {
        const double *A = (const double *) a, *B = (const double *) b;
        double *O = (double *) out;
        for (size_t i = 0; i < n; i++) {
            double ar = A[2 * i], ai = A[2 * i + 1], br = B[2 * i], bi = B[2 * i + 1];
            double xr, xi;
            if (op == OR_SUM) { xr = add_d(ar, br); xi = add_d(ai, bi); }
            else cmul_d(ar, ai, br, bi, &xr, &xi);
            O[2 * i] = xr;
            O[2 * i + 1] = xi;
        }
        break;
    }
    default: return -1;
    }
    return 0;
}
