// x87.hpp -- bit-exact x87 80-bit extended arithmetic (host + device).
// Used by longdouble.hip on the GPU; the identical code is compiled for the
// host only by tests/support (to check it against the reference's own x87
// ops on millions of inputs before it runs on an MI355X).
// See longdouble.hip for the semantics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef OSGPU_HD
#define OSGPU_HD __host__ __device__
#endif

namespace osgpu {
namespace x87 {

typedef unsigned __int128 u128;

struct X80 {
    uint64_t m;   // significand, bit 63 = explicit integer bit J
    uint32_t se;  // bit 15 sign, bits 0..14 biased exponent
};

enum Cls { C_ZERO, C_FIN, C_INF, C_QNAN, C_SNAN, C_BAD };

constexpr int kBias = 16383;
constexpr uint32_t kEmax = 0x7fff;

OSGPU_HD inline X80 defnan() { return X80{0xC000000000000000ull, 0xFFFFu}; }

OSGPU_HD inline Cls classify(X80 x)
{
    const uint32_t e = x.se & kEmax;
    const bool j = (x.m >> 63) != 0;
    if (e == kEmax) {
        if (!j) return C_BAD;                      // pseudo-infinity / pseudo-NaN
        if ((x.m << 1) == 0) return C_INF;
        return ((x.m >> 62) & 1) ? C_QNAN : C_SNAN;
    }
    if (e == 0) return x.m == 0 ? C_ZERO : C_FIN;    // denormal or pseudo-denormal
    return j ? C_FIN : C_BAD;                        // unnormal is unsupported
}

OSGPU_HD inline bool is_nan(Cls c) { return c == C_QNAN || c == C_SNAN; }

OSGPU_HD inline int clz128(u128 v)
{
    const uint64_t hi = (uint64_t) (v >> 64), lo = (uint64_t) v;
    return hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
}

// NaN propagation with at least one NaN operand and no unsupported one
OSGPU_HD inline X80 nan_pick(X80 a, Cls ca, X80 b, Cls cb)
{
    X80 r;
    if (is_nan(ca) && is_nan(cb)) {
        if (a.m > b.m) r = a;
        else if (b.m > a.m) r = b;
        else r = X80{a.m, (a.se & b.se)};        // tie: positive if either is
    } else {
        r = is_nan(ca) ? a : b;
    }
    r.m |= 1ull << 62;                           // quiet
    return r;
}

// Round a value sign * S * 2^(E - bias - 127), S normalised with bit 127 set
// (or S == 0), to x87 extended and encode it.
OSGPU_HD inline X80 round_pack(uint32_t sign, int E, u128 S)
{
    if (S == 0) return X80{0, sign << 15};
    if (E < 1) {                                 // gradual underflow
        const int sh = 1 - E;
        if (sh >= 128) {
            S = 1;                               // sticky only
        } else {
            const bool sticky = (S << (128 - sh)) != 0;
            S = (S >> sh) | (u128) (sticky ? 1 : 0);
        }
        E = 1;
    }
    uint64_t hi = (uint64_t) (S >> 64);
    const uint64_t lo = (uint64_t) S;
    const bool half = (lo >> 63) != 0;
    const bool rest = (lo << 1) != 0;
    if (half && (rest || (hi & 1))) {
        hi += 1;
        if (hi == 0) {                           // carried out of 64 bits
            hi = 1ull << 63;
            E += 1;
        }
    }
    if (E >= (int) kEmax) return X80{1ull << 63, (sign << 15) | kEmax};  // overflow -> inf
    const uint32_t e = (hi >> 63) ? (uint32_t) E : 0u;                    // denormal if J=0
    return X80{hi, (sign << 15) | e};
}

// The general add: every encoding, exact 128-bit intermediate, one RNE
// rounding (below).
OSGPU_HD __attribute__((noinline)) inline X80 add_general(X80 a, X80 b);

// Unpacked operand of the fast add: significand, biased exponent and sign
// in their own registers, so a fold that feeds one add's result to the next
// (and reuses each input P-1 times) does not re-extract them every time.
struct XU {
    uint64_t m;
    uint32_t e;  // biased exponent, 0..0x7fff
    uint32_t s;  // sign, 0 or 1
};

OSGPU_HD inline XU unpack_u(X80 x) { return XU{x.m, x.se & kEmax, (x.se >> 15) & 1}; }
OSGPU_HD inline X80 pack_u(XU x) { return X80{x.m, (x.s << 15) | x.e}; }

// add of two NORMAL operands (0 < biased exponent < 0x7fff, J set) whose
// exponents differ by less than 64 (or by 66 and more: the smaller is then
// below the rounding bit and the RNE result is the larger) and whose result
// stays normal -- what every soft-float add of ordinary data is: the same
// exact-then-round computation as add_general, on 64-bit halves, with the
// data-dependent choices (swap, add or subtract, carry or renormalise, round
// up) made by selects so the lanes of a wave run one instruction stream.
// false: not covered (gaps of 64 and 65, cancellation into the low half,
// underflow) -- add_general takes it.  Bit-identical by construction (same
// aligned operand, same rounding) and by test (tests/test_x87_softfloat.py
// compiles this header for the host).
OSGPU_HD inline bool add_normal(XU a, XU b, XU *r)
{
    const bool swap = b.e > a.e || (b.e == a.e && b.m > a.m);  // |A| >= |B|
    const uint64_t ma = swap ? b.m : a.m, mb = swap ? a.m : b.m;
    const int EA = (int) (swap ? b.e : a.e);
    const int d = EA - (int) (swap ? a.e : b.e);
    const uint32_t sign = swap ? b.s : a.s;
    if (d >= 66) {
        *r = XU{ma, (uint32_t) EA, sign};
        return true;
    }
    if (d >= 64) return false;
    const bool same = a.s == b.s;
    // B = mb * 2^-d as 64.64 fixed point, exact for d < 64
    const uint64_t bh = mb >> d;
    const uint64_t bl = d ? mb << ((64 - d) & 63) : 0;
    const uint64_t hs = ma + bh;
    const bool c = same && hs < ma;  // carry out of bit 127
    uint64_t hi = same ? hs : ma - bh - (bl != 0 ? 1 : 0);
    uint64_t lo = same ? bl : 0 - bl;
    if (!same && hi == 0) return false;  // cancellation into the low half
    // renormalise: right by one on a carry, left by lz after a subtraction
    const int lz = same ? 0 : __builtin_clzll(hi);
    const uint64_t hr = (hi >> 1) | (1ull << 63), lr = (lo >> 1) | (hi << 63) | (lo & 1);
    const uint64_t hl = lz ? (hi << lz) | (lo >> ((64 - lz) & 63)) : hi, ll = lo << lz;
    hi = c ? hr : hl;
    lo = c ? lr : ll;
    int E = EA + (c ? 1 : -lz);
    if (E < 1) return false;  // gradual underflow
    // round to nearest even at bit 64
    const bool up = (lo >> 63) && ((lo << 1) != 0 || (hi & 1));
    hi += up ? 1 : 0;
    const bool wrap = up && hi == 0;  // carried out of 64 bits
    hi = wrap ? (1ull << 63) : hi;
    E += wrap ? 1 : 0;
    const bool inf = E >= (int) kEmax;
    *r = XU{inf ? (1ull << 63) : hi, inf ? kEmax : (uint32_t) E, sign};
    return true;
}

// The fast form when it applies, else the general add (out of line: a fold
// of P inputs makes P(P-1) adds, and the rarely taken general path inlined
// into each of them made a long double team kernel of 24 K instructions,
// beyond the instruction cache).
OSGPU_HD inline XU add_u(XU a, XU b)
{
    XU r;
    if (a.e - 1u < kEmax - 1u && b.e - 1u < kEmax - 1u && ((a.m & b.m) >> 63) &&
        add_normal(a, b, &r))
        return r;
    return unpack_u(add_general(pack_u(a), pack_u(b)));
}

OSGPU_HD inline X80 add(X80 a, X80 b) { return pack_u(add_u(unpack_u(a), unpack_u(b))); }

OSGPU_HD __attribute__((noinline)) inline X80 add_general(X80 a, X80 b)
{
    const Cls ca = classify(a), cb = classify(b);
    if (ca == C_BAD || cb == C_BAD) return defnan();
    if (is_nan(ca) || is_nan(cb)) return nan_pick(a, ca, b, cb);
    const uint32_t sa = (a.se >> 15) & 1, sb = (b.se >> 15) & 1;
    if (ca == C_INF || cb == C_INF) {
        if (ca == C_INF && cb == C_INF) return sa == sb ? a : defnan();
        return ca == C_INF ? a : b;
    }
    if (ca == C_ZERO && cb == C_ZERO) return X80{0, (sa & sb) << 15};
    int Ea = (int) (a.se & kEmax), Eb = (int) (b.se & kEmax);
    Ea = Ea ? Ea : 1;
    Eb = Eb ? Eb : 1;
    uint64_t ma = a.m, mb = b.m;
    uint32_t sign = sa;
    if (cb == C_ZERO) { mb = 0; Eb = Ea; }
    if (ca == C_ZERO) { ma = 0; Ea = Eb; }
    // order by magnitude: |a| >= |b|
    if (Eb > Ea || (Eb == Ea && mb > ma)) {
        uint64_t tm = ma; ma = mb; mb = tm;
        int te = Ea; Ea = Eb; Eb = te;
        sign = sb;
    }
    const int d = Ea - Eb;
    const u128 A = (u128) ma << 64;
    u128 B = (u128) mb << 64;
    if (d >= 128) {
        B = (mb != 0) ? 1 : 0;
    } else if (d > 0) {
        const bool sticky = (B << (128 - d)) != 0;
        B = (B >> d) | (u128) (sticky ? 1 : 0);
    }
    int E = Ea;
    u128 S;
    if (sa == sb) {
        S = A + B;
        if (S < A) {                             // carry out of bit 127
            S = (S >> 1) | (S & 1) | ((u128) 1 << 127);
            E += 1;
        }
    } else {
        S = A - B;
        if (S == 0) return X80{0, 0};            // exact cancellation: +0 (RNE)
    }
    const int lz = clz128(S);
    S <<= lz;
    E -= lz;
    // value = S * 2^(E - bias - 127): the exponent convention above treats
    // the 128-bit S as significand bits 127..0 with J at 127
    return round_pack(sign, E, S);
}

OSGPU_HD __attribute__((noinline)) inline X80 mul_general(X80 a, X80 b);

// mul of two NORMAL operands whose product stays normal: the exact 128-bit
// product of two significands with J set lies in [2^126, 2^128), so the
// renormalising shift is 0 or 1 (a select), then one RNE rounding at bit 64
// -- the general path's computation without its classification and
// variable shifts.  Everything else goes to mul_general.
OSGPU_HD inline XU mul_u(XU a, XU b)
{
    if (a.e - 1u < kEmax - 1u && b.e - 1u < kEmax - 1u && ((a.m & b.m) >> 63)) {
        const u128 P = (u128) a.m * (u128) b.m;
        uint64_t hi = (uint64_t) (P >> 64), lo = (uint64_t) P;
        const bool top = (hi >> 63) != 0;
        const uint64_t h1 = (hi << 1) | (lo >> 63), l1 = lo << 1;
        hi = top ? hi : h1;
        lo = top ? lo : l1;
        // a.m*2^(Ea-bias-63) * b.m*2^(Eb-bias-63) = S * 2^(E-bias-127)
        int E = (int) a.e + (int) b.e - kBias + (top ? 1 : 0);
        if (E >= 1) {
            const bool up = (lo >> 63) && ((lo << 1) != 0 || (hi & 1));
            hi += up ? 1 : 0;
            const bool wrap = up && hi == 0;
            hi = wrap ? (1ull << 63) : hi;
            E += wrap ? 1 : 0;
            const bool inf = E >= (int) kEmax;
            return XU{inf ? (1ull << 63) : hi, inf ? kEmax : (uint32_t) E, a.s ^ b.s};
        }
    }
    return unpack_u(mul_general(pack_u(a), pack_u(b)));
}

OSGPU_HD inline X80 mul(X80 a, X80 b) { return pack_u(mul_u(unpack_u(a), unpack_u(b))); }

OSGPU_HD __attribute__((noinline)) inline X80 mul_general(X80 a, X80 b)
{
    const Cls ca = classify(a), cb = classify(b);
    if (ca == C_BAD || cb == C_BAD) return defnan();
    if (is_nan(ca) || is_nan(cb)) return nan_pick(a, ca, b, cb);
    const uint32_t s = ((a.se ^ b.se) >> 15) & 1;
    if (ca == C_INF || cb == C_INF) {
        if (ca == C_ZERO || cb == C_ZERO) return defnan();
        return X80{1ull << 63, (s << 15) | kEmax};
    }
    if (ca == C_ZERO || cb == C_ZERO) return X80{0, s << 15};
    int Ea = (int) (a.se & kEmax), Eb = (int) (b.se & kEmax);
    Ea = Ea ? Ea : 1;
    Eb = Eb ? Eb : 1;
    u128 P = (u128) a.m * (u128) b.m;            // exact, nonzero
    const int lz = clz128(P);
    P <<= lz;
    // a.m*2^(Ea-bias-63) * b.m*2^(Eb-bias-63) = P * 2^(Ea+Eb-2bias-126-lz)
    //   = S * 2^(E - bias - 127)  =>  E = Ea + Eb - bias + 1 - lz
    const int E = Ea + Eb - kBias + 1 - lz;
    return round_pack(s, E, P);
}

// fcomi ordering; false when unordered (NaN or unsupported encoding)
OSGPU_HD inline bool less(X80 a, X80 b)
{
    const Cls ca = classify(a), cb = classify(b);
    if (ca == C_BAD || cb == C_BAD || is_nan(ca) || is_nan(cb)) return false;
    const bool za = ca == C_ZERO, zb = cb == C_ZERO;
    if (za && zb) return false;
    const bool na = !za && ((a.se >> 15) & 1), nb = !zb && ((b.se >> 15) & 1);
    if (na != nb) return na;
    // magnitude keys (E, m): zero < denormal/pseudo-denormal (E=1) < ...
    uint32_t ea = za ? 0 : ((a.se & kEmax) ? (a.se & kEmax) : 1);
    uint32_t eb = zb ? 0 : ((b.se & kEmax) ? (b.se & kEmax) : 1);
    const uint64_t ma = za ? 0 : a.m, mb = zb ? 0 : b.m;
    const bool mag_lt = ea < eb || (ea == eb && ma < mb);
    const bool mag_gt = ea > eb || (ea == eb && ma > mb);
    return na ? mag_gt : mag_lt;
}

}  // namespace x87
}  // namespace osgpu
