// elem_ops.hpp -- device element operations of the reduce-to-all combine.
//
// Each functor is op(acc, in) with `acc` the running accumulator (the first
// operand), exactly like the reference's function-pointer fold
// `write_to[ti] = (*the_op)(write_to[ti], pWrk[j])` (src/reductions.c:95-96)
// over the one-line ops of src/shmemu/miscops.c:12-105.
//
// The floating-point model (documented in DESIGN.md, section "Numerics"):
//  * non-NaN results: IEEE-754 RNE, subnormals kept, never contracted (this
//    file is compiled with -ffp-contract=off and the pragma below);
//  * NaN results reproduce the x86-64 SSE rule of the reference build: the
//    first source operand's NaN (quieted) wins, then the second's, and an
//    invalid operation yields the NEGATIVE default NaN (0xFFF8.. / 0xFFC0..);
//  * min/max are compare + select (`a<b?a:b`), never v_min/v_max, so NaNs and
//    signed zeros resolve to the right operand exactly like the reference;
//  * complex product = GCC's inline expansion + libgcc __mul{s,d}c3 (C99
//    Annex G recovery) as compiled for the reference (operand orders from the
//    disassembly, see oracle/oracle_ops.c);
//  * integers wrap modulo 2^w (unsigned arithmetic, no UB).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

// host + device: the kernels, and the host fold of small host-heap calls
// (host_fold.hip) -- one definition of every element op for both
#define OSGPU_EHD __host__ __device__ __forceinline__

namespace osgpu {

struct cfloat { float re, im; };
struct cdouble { double re, im; };

// ---------------------------------------------------------------- bit utils
OSGPU_EHD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
OSGPU_EHD double dbl(uint64_t u) { return __builtin_bit_cast(double, u); }
OSGPU_EHD uint32_t bits(float x) { return __builtin_bit_cast(uint32_t, x); }
OSGPU_EHD float flt(uint32_t u) { return __builtin_bit_cast(float, u); }

OSGPU_EHD bool isnan_(double x) { return (bits(x) << 1) > (0x7ff0000000000000ull << 1); }
OSGPU_EHD bool isnan_(float x) { return (bits(x) << 1) > (0x7f800000u << 1); }
OSGPU_EHD bool isinf_(double x) { return (bits(x) << 1) == (0x7ff0000000000000ull << 1); }
OSGPU_EHD bool isinf_(float x) { return (bits(x) << 1) == (0x7f800000u << 1); }

OSGPU_EHD double quiet(double x) { return dbl(bits(x) | 0x0008000000000000ull); }
OSGPU_EHD float quiet(float x) { return flt(bits(x) | 0x00400000u); }
OSGPU_EHD double defnan(double) { return dbl(0xfff8000000000000ull); }
OSGPU_EHD float defnan(float) { return flt(0xffc00000u); }

// SSE NaN selection for `r = a OP b` with first source a.  The branch is
// taken only when r is NaN, so the streaming fast path pays one compare.
template <typename F>
OSGPU_EHD F sse(F r, F a, F b)
{
    if (__builtin_expect(r != r, 0)) {
        r = isnan_(a) ? quiet(a) : (isnan_(b) ? quiet(b) : defnan(a));
    }
    return r;
}
template <typename F> OSGPU_EHD F add(F a, F b) { return sse<F>(a + b, a, b); }
template <typename F> OSGPU_EHD F sub(F a, F b) { return sse<F>(a - b, a, b); }
template <typename F> OSGPU_EHD F mul(F a, F b) { return sse<F>(a * b, a, b); }

template <typename F>
OSGPU_EHD F copysign_(F mag, F sgn);
template <>
OSGPU_EHD double copysign_(double m, double s)
{
    return dbl((bits(m) & 0x7fffffffffffffffull) | (bits(s) & 0x8000000000000000ull));
}
template <>
OSGPU_EHD float copysign_(float m, float s)
{
    return flt((bits(m) & 0x7fffffffu) | (bits(s) & 0x80000000u));
}

// libgcc2.c __mul{s,d}c3, GCC 11.4, with the operand order of its compiled
// body: ac=a*c bd=b*d ad=a*d bc=c*b; x=ac-bd; y=ad+bc; recovery
// x=(a*c-b*d)*inf, y=inf*(a*d+b*c).  Reached only when the inline product
// has a NaN part, so it lives off the fast path.
template <typename F>
struct CPair {
    F x, y;
};
// returned by value (in registers): no stack frame on the fast path's kernels
template <typename F>
__host__ __device__ __attribute__((noinline)) CPair<F> mulc3(F a, F b, F c, F d)
{
    const F one = 1, zero = 0, inf = __builtin_huge_val();
    F ac = mul(a, c), bd = mul(b, d), ad = mul(a, d), bc = mul(c, b);
    F x = sub(ac, bd), y = add(ad, bc);
    if (isnan_(x) && isnan_(y)) {
        bool recalc = false;
        if (isinf_(a) || isinf_(b)) {
            a = copysign_(isinf_(a) ? one : zero, a);
            b = copysign_(isinf_(b) ? one : zero, b);
            if (isnan_(c)) c = copysign_(zero, c);
            if (isnan_(d)) d = copysign_(zero, d);
            recalc = true;
        }
        if (isinf_(c) || isinf_(d)) {
            c = copysign_(isinf_(c) ? one : zero, c);
            d = copysign_(isinf_(d) ? one : zero, d);
            if (isnan_(a)) a = copysign_(zero, a);
            if (isnan_(b)) b = copysign_(zero, b);
            recalc = true;
        }
        if (!recalc && (isinf_(ac) || isinf_(bd) || isinf_(ad) || isinf_(bc))) {
            if (isnan_(a)) a = copysign_(zero, a);
            if (isnan_(b)) b = copysign_(zero, b);
            if (isnan_(c)) c = copysign_(zero, c);
            if (isnan_(d)) d = copysign_(zero, d);
            recalc = true;
        }
        if (recalc) {
            x = mul(sub(mul(a, c), mul(b, d)), inf);
            y = mul(inf, add(mul(a, d), mul(b, c)));
        }
    }
    return CPair<F>{x, y};
}

// --------------------------------------------------------------- functors
// Integer ops run on the unsigned image so overflow wraps (miscops.c:12-39
// compiled by gcc wraps; short is promoted to int and truncated, whose low
// 16 bits equal 16-bit wrapping arithmetic).
template <typename T> struct Unsigned;
// int16 runs in 32-bit unsigned (low 16 bits identical, no int-promotion UB)
template <> struct Unsigned<int16_t> { using type = uint32_t; };
template <> struct Unsigned<int32_t> { using type = uint32_t; };
template <> struct Unsigned<int64_t> { using type = uint64_t; };

enum OpCode { OP_SUM = 0, OP_PROD, OP_AND, OP_OR, OP_XOR, OP_MAX, OP_MIN };

template <typename T, int OP> struct Elem;

// integers ---------------------------------------------------------------
template <typename T> struct Elem<T, OP_SUM> {
    OSGPU_EHD static T f(T a, T b)
    {
        using U = typename Unsigned<T>::type;
        return (T) (U) ((U) a + (U) b);
    }
};
template <typename T> struct Elem<T, OP_PROD> {
    OSGPU_EHD static T f(T a, T b)
    {
        using U = typename Unsigned<T>::type;
        return (T) (U) ((U) a * (U) b);
    }
};
template <typename T> struct Elem<T, OP_AND> { OSGPU_EHD static T f(T a, T b) { return a & b; } };
template <typename T> struct Elem<T, OP_OR> { OSGPU_EHD static T f(T a, T b) { return a | b; } };
template <typename T> struct Elem<T, OP_XOR> { OSGPU_EHD static T f(T a, T b) { return a ^ b; } };
// compare + select: exact for every type, including NaN / signed zero
template <typename T> struct Elem<T, OP_MAX> { OSGPU_EHD static T f(T a, T b) { return a > b ? a : b; } };
template <typename T> struct Elem<T, OP_MIN> { OSGPU_EHD static T f(T a, T b) { return a < b ? a : b; } };

// real floating point ------------------------------------------------------
template <> struct Elem<float, OP_SUM> { OSGPU_EHD static float f(float a, float b) { return add(a, b); } };
template <> struct Elem<float, OP_PROD> { OSGPU_EHD static float f(float a, float b) { return mul(a, b); } };
template <> struct Elem<double, OP_SUM> { OSGPU_EHD static double f(double a, double b) { return add(a, b); } };
template <> struct Elem<double, OP_PROD> { OSGPU_EHD static double f(double a, double b) { return mul(a, b); } };

// complex ----------------------------------------------------------------
// complexd sum: compiled as addsd %xmm3,%xmm1 ; addsd %xmm2,%xmm0 (a first)
template <> struct Elem<cdouble, OP_SUM> {
    OSGPU_EHD static cdouble f(cdouble a, cdouble b)
    {
        return cdouble{add(a.re, b.re), add(a.im, b.im)};
    }
};
// complexf sum: the compiled body adds the imaginary parts as b.im + a.im
template <> struct Elem<cfloat, OP_SUM> {
    OSGPU_EHD static cfloat f(cfloat a, cfloat b)
    {
        return cfloat{add(a.re, b.re), add(b.im, a.im)};
    }
};
template <typename C, typename F>
OSGPU_EHD C cmul(C p, C q)
{
    F a = p.re, b = p.im, c = q.re, d = q.im;
    F x = a * c - b * d;   // inline fast path; any NaN part -> libgcc path
    F y = a * d + b * c;
    if (__builtin_expect(x != x || y != y, 0)) {
        const CPair<F> r = mulc3<F>(a, b, c, d);
        x = r.x;
        y = r.y;
    }
    return C{x, y};
}
template <> struct Elem<cdouble, OP_PROD> {
    OSGPU_EHD static cdouble f(cdouble a, cdouble b) { return cmul<cdouble, double>(a, b); }
};
template <> struct Elem<cfloat, OP_PROD> {
    OSGPU_EHD static cfloat f(cfloat a, cfloat b) { return cmul<cfloat, float>(a, b); }
};

// ------------------------------------------------------- branch-free folds
// Fast<T, OP>::f is Elem<T, OP>::f without its NaN handling (the SSE rule,
// the complex product's libgcc recovery): one instruction stream with no
// branch per element, so a streaming kernel keeps every load in flight.
// It differs from Elem::f only where that result has a NaN part, and a NaN
// part, once there, stays through every later + and * of a fold (x + NaN,
// x * NaN and both complex formulas give NaN in it).  So a fold whose FINAL
// value has no NaN part (Fast::bad false) is bit-identical to the exact
// fold; kernels test the final values of a tile and recompute the tile with
// Elem::f only where some lane's is flagged.  Ops without NaN handling
// (integers, min/max, which never produce a NaN of their own) are exact:
// kChecked = false and the test compiles away.
template <typename T, int OP> struct Fast {
    static constexpr bool kChecked = false;
    OSGPU_EHD static T f(T a, T b) { return Elem<T, OP>::f(a, b); }
    OSGPU_EHD static bool bad(T) { return false; }
};
template <typename F, int OP> struct FastReal {
    static constexpr bool kChecked = true;
    OSGPU_EHD static F f(F a, F b) { return OP == OP_SUM ? a + b : a * b; }
    OSGPU_EHD static bool bad(F r) { return r != r; }
};
template <> struct Fast<float, OP_SUM> : FastReal<float, OP_SUM> {};
template <> struct Fast<float, OP_PROD> : FastReal<float, OP_PROD> {};
template <> struct Fast<double, OP_SUM> : FastReal<double, OP_SUM> {};
template <> struct Fast<double, OP_PROD> : FastReal<double, OP_PROD> {};
template <> struct Fast<cdouble, OP_SUM> {
    static constexpr bool kChecked = true;
    OSGPU_EHD static cdouble f(cdouble a, cdouble b)
    {
        return cdouble{a.re + b.re, a.im + b.im};
    }
    OSGPU_EHD static bool bad(cdouble r) { return r.re != r.re || r.im != r.im; }
};
template <> struct Fast<cfloat, OP_SUM> {
    static constexpr bool kChecked = true;
    OSGPU_EHD static cfloat f(cfloat a, cfloat b)
    {
        return cfloat{a.re + b.re, b.im + a.im};  // the compiled order, as Elem
    }
    OSGPU_EHD static bool bad(cfloat r) { return r.re != r.re || r.im != r.im; }
};
template <typename C, typename F> struct FastCplxProd {
    static constexpr bool kChecked = true;
    OSGPU_EHD static C f(C p, C q)
    {
        return C{p.re * q.re - p.im * q.im, p.re * q.im + p.im * q.re};  // cmul's inline form
    }
    OSGPU_EHD static bool bad(C r) { return r.re != r.re || r.im != r.im; }
};
template <> struct Fast<cdouble, OP_PROD> : FastCplxProd<cdouble, double> {};
template <> struct Fast<cfloat, OP_PROD> : FastCplxProd<cfloat, float> {};

}  // namespace osgpu
