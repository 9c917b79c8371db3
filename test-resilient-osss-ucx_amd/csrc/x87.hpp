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
    uint32_t s;  // sign as a mask: 0 (+) or ~0 (-)
};

OSGPU_HD inline XU unpack_u(X80 x)
{
    return XU{x.m, x.se & kEmax, (uint32_t) ((int32_t) (x.se << 16) >> 31)};
}
OSGPU_HD inline X80 pack_u(XU x) { return X80{x.m, (x.s & 0x8000u) | x.e}; }

OSGPU_HD inline bool normal_u(XU x) { return x.e - 1u < kEmax - 1u && (x.m >> 63); }

// count of leading zeros of a 32-bit word, ~0 when it is zero (what
// v_ffbh_u32 returns; clang's ctlz would add a compare and a select)
OSGPU_HD inline uint32_t ffbh(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t f;
    asm("v_ffbh_u32 %0, %1" : "=v"(f) : "v"(x));
    return f;
#else
    return x ? (uint32_t) __builtin_clz(x) : ~0u;
#endif
}

// |a - b| + c of two values below 2^16 (one v_sad_u16)
OSGPU_HD inline uint32_t absdiff15(uint32_t a, uint32_t b, uint32_t c = 0u)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sad_u16(a, b, c);
#else
    return (a > b ? a - b : b - a) + c;
#endif
}

// a - b, 0 when b > a (v_sub_u32 with clamp)
OSGPU_HD inline uint32_t sub_sat(uint32_t a, uint32_t b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_elementwise_sub_sat(a, b);
#else
    return b > a ? 0u : a - b;
#endif
}

// add of two NORMAL operands (0 < biased exponent < 0x7fff, J set; the
// caller checks), straight-line: the data-dependent choices (swap, add or
// subtract, renormalising shift, round up) are selects, so the lanes of a
// wave -- and several independent folds of one lane -- run one instruction
// stream.  Returns false where it does not apply: exponent gaps of 63 to 65,
// cancellations of 32 bits or more (exact zero included), results below the
// normal range or overflowing, a significand of all ones rounded up to the
// next power of two; add_general then computes the result.
//
// Same exact-then-round computation as add_general, one bit lower: the
// operands sit in 128 bits with one bit of headroom (A = ma * 2^63,
// B = mb * 2^(63-d), exact for d < 64), so a carry lands in bit 127 instead
// of leaving the word, and addition and subtraction share one normalising
// left shift by clz (0 or 1 after an addition).  For d >= 66 B is dropped:
// it lies below a quarter of A's ulp and RNE returns A.
//
// Written for gfx950's issue costs (tools/valu_rate2.hip,
// profiles/r03_valu_rate2.jsonl): VOP2 and/or/xor/add/sub/lshr/ashr/not/mov
// issue in ~2.6 cycles per wave64, every compare, select, carry, 64-bit
// shift, left shift and three-operand op in ~4.5.  So the magnitude order is
// one 64-bit compare of (exponent, top word) with its rare tie flagged, the
// range flags are two unsigned compares, B's drop is an arithmetic-shift
// mask, the shift amounts use the hardware's own masking, the exponent gap
// is one v_sad_u16, and the clz of the top word needs no zero test (E
// saturates instead): only a cancellation of 32+ bits (gaps of 0 or 1 with
// 32 equal leading bits, ~2^-32 of random operands) leaves the fast path.
// 51 VALU per add against 58 (≈ 185 issue cycles against 229).
OSGPU_HD inline bool add_fast(XU a, XU b, XU *r)
{
    // |A| >= |B| by one 64-bit compare of (exponent, top significand word);
    // a tie there (same exponent, same top 32 bits) is flagged below
    const uint64_t ka = ((uint64_t) a.e << 32) | (uint32_t) (a.m >> 32);
    const uint64_t kb = ((uint64_t) b.e << 32) | (uint32_t) (b.m >> 32);
    const bool swap = kb > ka;
    const uint64_t ma = swap ? b.m : a.m;
    uint64_t mb = swap ? a.m : b.m;
    const uint32_t EA = a.e > b.e ? a.e : b.e;  // the exponents need no select
    const uint32_t d = absdiff15(a.e, b.e);
    const uint32_t sign = swap ? b.s : a.s;
    // d >= 63: B dropped -- a mask from the sign of d - 63 (d < 2^15), not a
    // compare and two selects; gaps of 63..65 are flagged below, so every
    // shift amount here is the exact gap (0..62) or shifts a zero
    const uint32_t keep = (uint32_t) ((int32_t) (d - 63u) >> 31);
    mb &= ((uint64_t) keep << 32) | keep;
    const uint64_t ah = ma >> 1, bh = mb >> ((d + 1) & 63), bl = mb << ((63 - d) & 63);
    // S = A + B, or A - B as A + ~B + 1, in 32-bit words with explicit
    // carries (A's lowest word is 0; the + 1 rides in as the first carry)
    const uint32_t M = a.s ^ b.s;  // ~0 to subtract
    const uint32_t diff = M & 1u;
    unsigned c0, c1, c2, c3;
    const uint32_t s0 = __builtin_addc((uint32_t) bl ^ M, 0u, diff, &c0);
    const uint32_t s1 = __builtin_addc((uint32_t) (bl >> 32) ^ M, (uint32_t) ma << 31, c0, &c1);
    const uint32_t s2 = __builtin_addc((uint32_t) bh ^ M, (uint32_t) ah, c1, &c2);
    const uint32_t s3 = __builtin_addc((uint32_t) (bh >> 32) ^ M, (uint32_t) (ah >> 32), c2, &c3);
    (void) c3;
    // normalise by the leading zeros of the top word: a cancellation of 32
    // bits or more (top word zero; only for gaps of 0 or 1) gives lz = ~0,
    // and E saturates to 0 (flagged by the range test; the shifted value is
    // then not used), so the shift is below 32 and only the top word of the
    // low half can reach the new high half
    const uint32_t lz = ffbh(s3);
    uint64_t hi = ((uint64_t) s3 << 32) | s2, lo = ((uint64_t) s1 << 32) | s0;
    // (the masks are the hardware's own shift-amount masks: no instruction)
    hi = (hi << (lz & 63)) | ((s1 >> 1) >> ((31u - lz) & 31));
    lo <<= lz & 63;
    const uint32_t E = sub_sat(EA + 1u, lz);  // 0 (flagged) below 1 or for lz = ~0
    // round to nearest even at bit 64: up iff lo > 2^63 - (hi & 1), i.e. iff
    // (lo | (hi & 1)) > 2^63; the carry out of hi is the wrap case (all ones
    // rounded up)
    const unsigned up = (lo | (hi & 1u)) > (1ull << 63) ? 1u : 0u;
    unsigned w1, wrap;
    const uint32_t h0 = __builtin_addc((uint32_t) hi, 0u, up, &w1);
    const uint32_t hh = __builtin_addc((uint32_t) (hi >> 32), 0u, w1, &wrap);
    *r = XU{((uint64_t) hh << 32) | h0, E, sign};
    // not covered: gaps of 63..65, E outside [1, kEmax) (one unsigned range
    // test; below the normal range, or a cancellation of 32 bits or more,
    // E is 0), all ones rounded up
    return d - 63u >= 3u && E - 1u < kEmax - 1u && !wrap && ka != kb;
}

// add_fast for two NORMAL operands of the SAME sign (the caller checks):
// an addition needs no magnitude order (it commutes exactly, so the swap is
// by exponent alone), no complement, and its sum of A = ma * 2^63 and
// B = mb * 2^(63-d) lies in [2^126, 2^128): the renormalising shift is 0 or
// 1, a select instead of a clz and three variable funnel shifts.  false:
// gaps of 63 to 65, overflow, all ones rounded up (add_general computes
// those).
OSGPU_HD inline bool add_same_fast(XU a, XU b, XU *r)
{
    const bool swap = b.e > a.e;
    const uint64_t ma = swap ? b.m : a.m;
    uint64_t mb = swap ? a.m : b.m;
    const uint32_t EA = swap ? b.e : a.e;
    const uint32_t d = absdiff15(a.e, b.e);
    // d >= 63: B dropped by a mask (add_fast); gaps of 63..65 flagged below
    const uint32_t keep = (uint32_t) ((int32_t) (d - 63u) >> 31);
    mb &= ((uint64_t) keep << 32) | keep;
    const uint64_t ah = ma >> 1, bh = mb >> ((d + 1) & 63), bl = mb << ((63 - d) & 63);
    // S = A + B in 32-bit words with explicit carries; A's lowest word is 0
    unsigned c1, c2, c3;
    const uint32_t s1 = __builtin_addc((uint32_t) (bl >> 32), (uint32_t) ma << 31, 0u, &c1);
    const uint32_t s2 = __builtin_addc((uint32_t) bh, (uint32_t) ah, c1, &c2);
    const uint32_t s3 = __builtin_addc((uint32_t) (bh >> 32), (uint32_t) (ah >> 32), c2, &c3);
    (void) c3;  // S < 2^128: no carry out (headroom)
    uint64_t hi = ((uint64_t) s3 << 32) | s2, lo = ((uint64_t) s1 << 32) | (uint32_t) bl;
    // S >= 2^127: no shift, else one -- shifts by t = 1 - top (no selects)
    const uint32_t top = s3 >> 31, t = top ^ 1u;
    hi = (hi << t) | ((s1 >> 31) & t);
    lo <<= t;
    const uint32_t E = EA + top;  // EA + 1 - lz, lz = t
    // round to nearest even at bit 64 (add_fast); the carry out of hi when
    // it is all ones is the wrap case
    const unsigned up = (lo | (hi & 1u)) > (1ull << 63) ? 1u : 0u;
    unsigned w1, wrap;
    const uint32_t h0 = __builtin_addc((uint32_t) hi, 0u, up, &w1);
    const uint32_t hh = __builtin_addc((uint32_t) (hi >> 32), 0u, w1, &wrap);
    *r = XU{((uint64_t) hh << 32) | h0, E, a.s};
    return d - 63u >= 3u && !wrap && E < kEmax;
}

// leading bits equal to the sign bit of a 32-bit word, ~0 when it is 0 or
// ~0 (what v_ffbh_i32 returns)
OSGPU_HD inline uint32_t ffbh_signed(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t f;
    asm("v_ffbh_i32 %0, %1" : "=v"(f) : "v"(x));
    return f;
#else
    const uint32_t y = (x >> 31) ? ~x : x;
    return y ? (uint32_t) __builtin_clz(y) : ~0u;
#endif
}

// low 32 bits of (hi:lo) >> (n & 31) (one v_alignbit_b32)
OSGPU_HD inline uint32_t funnel_r(uint32_t hi, uint32_t lo, uint32_t n)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, n);
#else
    return (uint32_t) ((((uint64_t) hi << 32) | lo) >> (n & 31));
#endif
}

// add_fast for two NORMAL operands whose exponents differ by at most 30
// (the caller checks nothing; false otherwise): the same exact-then-round
// sum, two bits lower -- A = ma * 2^62, B = mb * 2^(62-d) -- which buys:
//  * B's lowest word is zero (d <= 30), so the sum has three words, not
//    four: word 0 of A + ~B + 1 is 0 with carry `diff`, and that carry
//    lands in A's word 1 as an OR (ma << 30 has 30 zero bits);
//  * B's alignment is one 32-bit left shift and one 64-bit right shift, no
//    drop mask (gaps above 30 are flagged);
//  * a valid S has bit 127 clear (an addition lies below 2^127, a
//    subtraction of the smaller magnitude below 2^126), so the only
//    negative S -- a tie of (exponent, top word) with the larger low word
//    subtracted, S > -2^94 -- has a top word of all ones, and the SIGNED
//    leading-bit count (~0 for 0 and for ~0) flags it through the exponent
//    range test with the 32-bit cancellations: no tie compare;
//  * the round's low word is zero: one 32-bit carry test.
//  * bit 127 clear also makes every valid leading-zero count 1..31, so the
//    normalising left shift is two funnel shifts right by 32 - lz.
// Precondition (the caller's): 30 <= max(a.e, b.e) <= kEmax - 2, so the
// result's exponent needs no range test.  ~38 VALU per add against
// add_fast's 51 (tools/isa/count_ld_valu.sh).  false: gaps above 30,
// cancellations of 32 bits or more, negative S, all ones rounded up.
OSGPU_HD inline bool add_near(XU a, XU b, XU *r)
{
    const uint64_t ka = ((uint64_t) a.e << 32) | (uint32_t) (a.m >> 32);
    const uint64_t kb = ((uint64_t) b.e << 32) | (uint32_t) (b.m >> 32);
    const bool swap = kb > ka;
    const uint64_t ma = swap ? b.m : a.m;
    const uint64_t mb = swap ? a.m : b.m;
    const uint32_t EA = a.e > b.e ? a.e : b.e;
    const uint32_t d2 = absdiff15(a.e, b.e, 2u);  // d + 2
    const uint32_t sign = swap ? b.s : a.s;
    // B = mb * 2^(62-d) = (mb << (30-d)) * 2^32: word 1 and words 2..3
    // (30 - d = 32 - d2 under the shift's 5-bit mask)
    unsigned far;  // d2 > 32: a gap above 30, flagged
    const uint32_t b1 = (uint32_t) mb << (__builtin_subc(32u, d2, 0u, &far) & 31);
    const uint64_t bh = mb >> (d2 & 63);
    const uint64_t ah = ma >> 2;
    const uint32_t M = a.s ^ b.s;  // ~0 to subtract
    const uint32_t diff = M & 1u;
    unsigned c1, c2, c3;
    const uint32_t s1 = __builtin_addc(b1 ^ M, ((uint32_t) ma << 30) | diff, 0u, &c1);
    const uint32_t s2 = __builtin_addc((uint32_t) bh ^ M, (uint32_t) ah, c1, &c2);
    const uint32_t s3 = __builtin_addc((uint32_t) (bh >> 32) ^ M, (uint32_t) (ah >> 32), c2, &c3);
    (void) c3;
    // normalise: bit 127 is clear, so a valid lz is 1..31 and the left
    // shift of (s3, s2, s1) is two funnel shifts right by 32 - lz; ~0 (top
    // word 0, or ~0 for a negative S) borrows in E, flagged below
    const uint32_t lz = ffbh_signed(s3);
    const uint32_t rs = (0u - lz) & 31;  // 32 - lz
    const uint32_t hh0 = funnel_r(s3, s2, rs), hl0 = funnel_r(s2, s1, rs);
    const uint64_t hi = ((uint64_t) hh0 << 32) | hl0;
    const uint32_t lo1 = s1 << (lz & 31);  // the low word of lo stays 0
    // E = EA + 2 - lz lies in [EA - 29, EA + 1], inside [1, kEmax) under the
    // precondition 30 <= EA <= kEmax - 2: only lz = ~0 borrows
    unsigned low;
    const uint32_t E = __builtin_subc(EA + 2u, lz, 0u, &low);
    // RNE at bit 64, lo = lo1 * 2^32: up iff lo1 > 2^31, or lo1 == 2^31 and
    // hi is odd, i.e. iff lo1 >= K = 2^31 + 1 - (hi & 1).  In borrows: the
    // compare's borrow is !up, and hi - ~0 - borrow = hi + up word by word,
    // each borrow out the complement of the carry (the last one, !wrap)
    unsigned nup, nc, nwrap;
    (void) __builtin_subc(lo1, (~(uint32_t) hi & 1u) | 0x80000000u, 0u, &nup);
    const uint32_t h0 = __builtin_subc((uint32_t) hi, ~0u, nup, &nc);
    const uint32_t hh = __builtin_subc((uint32_t) (hi >> 32), ~0u, nc, &nwrap);
    *r = XU{((uint64_t) hh << 32) | h0, E, sign};
    return !far && !low && nwrap;
}

// add_same_fast for two NORMAL operands of the SAME sign whose exponents
// differ by at most 31 (false otherwise), by add_near's means: B's lowest
// word is zero (one 32-bit left shift, one 64-bit right shift, no drop
// mask), and the round's low word is zero (the borrow chain).  ~30 VALU per
// add against add_same_fast's ~39.  Precondition: max(a.e, b.e) <= kEmax - 2
// (E <= EA + 1 needs no range test).  false: gaps above 31, all ones rounded
// up.
OSGPU_HD inline bool add_same_near(XU a, XU b, XU *r)
{
    const bool swap = b.e > a.e;
    const uint64_t ma = swap ? b.m : a.m;
    const uint64_t mb = swap ? a.m : b.m;
    const uint32_t EA = swap ? b.e : a.e;
    const uint32_t d1 = absdiff15(a.e, b.e, 1u);  // d + 1
    unsigned far;  // d1 > 32: a gap above 31
    const uint32_t b1 = (uint32_t) mb << (__builtin_subc(32u, d1, 0u, &far) & 31);
    const uint64_t bh = mb >> (d1 & 63);
    const uint64_t ah = ma >> 1;
    unsigned c1, c2, c3;
    const uint32_t s1 = __builtin_addc(b1, (uint32_t) ma << 31, 0u, &c1);
    const uint32_t s2 = __builtin_addc((uint32_t) bh, (uint32_t) ah, c1, &c2);
    const uint32_t s3 = __builtin_addc((uint32_t) (bh >> 32), (uint32_t) (ah >> 32), c2, &c3);
    (void) c3;
    uint64_t hi = ((uint64_t) s3 << 32) | s2;
    const uint32_t top = s3 >> 31, t = top ^ 1u;
    hi = (hi << t) | ((s1 >> 31) & t);
    const uint32_t lo1 = s1 << t;
    const uint32_t E = EA + top;  // EA + 1 - lz, lz = t
    unsigned nup, nc, nwrap;
    (void) __builtin_subc(lo1, (~(uint32_t) hi & 1u) | 0x80000000u, 0u, &nup);
    const uint32_t h0 = __builtin_subc((uint32_t) hi, ~0u, nup, &nc);
    const uint32_t hh = __builtin_subc((uint32_t) (hi >> 32), ~0u, nc, &nwrap);
    *r = XU{((uint64_t) hh << 32) | h0, E, a.s};
    return !far && nwrap;
}

// true in every lane of the wave (device), or for this element (host, where
// team folds run one element at a time): a wave-uniform branch condition
OSGPU_HD inline bool wave_all(bool pred)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(!pred) == 0;
#else
    return pred;
#endif
}

// The fast form when it applies, else the general add (out of line: a fold
// of P inputs makes P(P-1) adds, and the rarely taken general path inlined
// into each of them made a long double team kernel of 24 K instructions,
// beyond the instruction cache).
OSGPU_HD inline XU add_u(XU a, XU b)
{
    XU r;
    if (normal_u(a) && normal_u(b) && add_fast(a, b, &r)) return r;
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

// mul of two NORMAL operands (the caller checks), straight-line: the exact
// 128-bit product of two significands with J set lies in [2^126, 2^128), so
// the renormalising shift is 0 or 1 (a select), then one RNE rounding at bit
// 64 -- the general path's computation without its classification and
// variable shifts.  false: the product leaves the normal range (denormal or
// infinity) or its rounding carries out of the significand; mul_general
// computes it.
OSGPU_HD inline bool mul_fast(XU a, XU b, XU *r)
{
    const u128 P = (u128) a.m * (u128) b.m;
    uint64_t hi = (uint64_t) (P >> 64), lo = (uint64_t) P;
    // no shift when P >= 2^127, else one: shifts by t = 1 - top, no selects
    const uint32_t top = (uint32_t) (hi >> 63), t = top ^ 1u;
    hi = (hi << t) | ((uint32_t) (lo >> 63) & t);
    lo <<= t;
    // a.m*2^(Ea-bias-63) * b.m*2^(Eb-bias-63) = S * 2^(E-bias-127)
    int E = (int) a.e + (int) b.e - kBias + (int) top;
    const bool low = E < 1;
    hi += lo > (1ull << 63) - (hi & 1) ? 1 : 0;  // RNE at bit 64 (add_fast)
    const bool wrap = hi == 0;
    *r = XU{hi, (uint32_t) E, a.s ^ b.s};
    return !low && !wrap && E < (int) kEmax;
}

OSGPU_HD inline XU mul_u(XU a, XU b)
{
    XU r;
    if (normal_u(a) && normal_u(b) && mul_fast(a, b, &r)) return r;
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

// The rounds of every member's fold (team_fold_sum_prod below), by the
// fast op of MODE, add_general / mul_general for the folds and lanes it
// does not cover:
//  * F_FULL: add_fast / mul_fast;
//  * F_NEAR: add_near (exponent gaps up to 30);
//  * F_SAME, F_SAME_NEAR: every input of the element carries one sign, so
//    every fold adds like signs throughout (the exact sum of two values of
//    sign s has sign s; a NaN or infinity, whose sign may differ, is never
//    normal, and a fold whose value is not normal stays on the general op)
//    -- add_same_fast, or add_same_near (gaps up to 31).
enum FoldMode { F_FULL, F_NEAR, F_SAME, F_SAME_NEAR };

// Folds F0..F1-1 through every round.
template <int OP, int P, int MODE, int F0, int F1>
OSGPU_HD __attribute__((always_inline)) inline void fold_group(const XU (&u)[P], const bool (&nrm)[P], XU (&acc)[P - 1],
                                 bool (&slow)[P - 1])
{
    constexpr int NF = P - 1;
    // the near modes' gate (team_fold_sum_prod) makes every input normal
    // and every add meet the near adds' precondition; a running sum that
    // left the normal range (a cancellation to zero or below 2^-16351) has
    // exponent 0, more than 30 below the input's: the near add flags it
    // itself, so these rounds need no `slow` / `nrm` terms
    constexpr bool NEAR = MODE == F_NEAR || MODE == F_SAME_NEAR;
#pragma unroll
    for (int t = 0; t < P - 1; t++) {
        XU res[NF];
        bool ok[NF];
        bool all = true;
#pragma unroll
        for (int f = F0; f < F1; f++) {
            const int q = f == 0 ? 0 : f + 1;
            const int j = t < q ? t : t + 1;  // q's t-th operand
            const bool fast = OP == 1 ? mul_fast(acc[f], u[j], &res[f])
                              : MODE == F_SAME ? add_same_fast(acc[f], u[j], &res[f])
                              : MODE == F_SAME_NEAR ? add_same_near(acc[f], u[j], &res[f])
                              : MODE == F_NEAR ? add_near(acc[f], u[j], &res[f])
                                               : add_fast(acc[f], u[j], &res[f]);
            ok[f] = NEAR ? fast : fast && !slow[f] && nrm[j];
            all = all && ok[f];
        }
        if (!all) {
#pragma unroll
            for (int f = F0; f < F1; f++) {
                if (!ok[f]) {
                    const int q = f == 0 ? 0 : f + 1;
                    const int j = t < q ? t : t + 1;
                    res[f] = unpack_u(OP == 0 ? add_general(pack_u(acc[f]), pack_u(u[j]))
                                              : mul_general(pack_u(acc[f]), pack_u(u[j])));
                    if (!NEAR) slow[f] = !normal_u(res[f]);
                }
            }
        }
#pragma unroll
        for (int f = F0; f < F1; f++) acc[f] = res[f];
    }
}

// The P-1 folds in two groups, each through all its rounds before the next:
// 3-4 independent chains per round are ILP enough beside the other waves of
// the SIMD, and half the adds in flight keep the 8-member sum within 4 waves'
// 128 VGPRs (10 spilled against 57 with all 7 folds per round; 1.18x the
// random-sign 8-member sum, 1.03-1.05x the same-sign ones, in one process on
// the same arrays: profiles/r06_ld_variants.jsonl).
template <int OP, int P, int MODE>
OSGPU_HD __attribute__((always_inline)) inline void fold_rounds(const XU (&u)[P], const bool (&nrm)[P], XU (&acc)[P - 1],
                                 bool (&slow)[P - 1])
{
    constexpr int H = P / 2;
    fold_group<OP, P, MODE, 0, H>(u, nrm, acc, slow);
    fold_group<OP, P, MODE, H, P - 1>(u, nrm, acc, slow);
}

// Every member's fold of a P-PE sum (OP 0) or prod (OP 1) of one element,
// each in its own order (src/reductions.c:79-111: PE q starts from its own
// x_q, then x_0, x_1, ... skipping q).  x87 add and mul are commutative bit
// for bit (same rounding of the same exact value; nan_pick is symmetric), so
// member 1's fold x1 op x0 op x2 ... equals member 0's: P-1 folds, not P.
//
// The folds advance in rounds: round t applies every fold's t-th operand
// with the straight-line fast op, so independent chains interleave in one
// instruction stream (ILP for a VALU-bound kernel; fold_rounds); only when some
// lane of the wave has an operand or result outside the fast op's range
// does the round take the slower op, for those folds and lanes.  A fold
// whose running value leaves the normal range stays on the general op
// (`slow`) until it is normal again.  The fast add is chosen once per
// element, wave-uniform branches: a sum whose inputs' biased exponents lie
// within kNearSpread of each other in every lane of the wave takes the
// near-exponent adds (a running sum stays within a few binades of its inputs
// unless it cancels by 6+ bits, and a fold that then meets a wider gap takes
// the general add for that round), the same-sign form where every input of
// every lane carries one sign; other sums take add_fast / add_same_fast.
constexpr uint32_t kNearSpread = 24;
// and whose inputs are all normal with exponents in [kNearEmin, kNearEmax]:
// every add of the fold then meets the near adds' precondition (EA >= the
// input's exponent >= 32; a running sum grows by at most one binade per
// round, 7 rounds)
constexpr uint32_t kNearEmin = 32, kNearEmax = kEmax - 16;

template <int OP, int P>
OSGPU_HD __attribute__((always_inline)) inline void team_fold_sum_prod(const X80 (&x)[P], X80 (&out)[P])
{
    constexpr int NF = P - 1;  // folds of members 0, 2, 3, ..., P-1
    XU u[P];
    bool nrm[P];
    bool same = OP == 0, allnrm = true;
    uint32_t emax = 0, emin = kEmax;
#pragma unroll
    for (int p = 0; p < P; p++) {
        u[p] = unpack_u(x[p]);
        nrm[p] = normal_u(u[p]);
        allnrm = allnrm && nrm[p];
        same = same && u[p].s == u[0].s;
        emax = u[p].e > emax ? u[p].e : emax;
        emin = u[p].e < emin ? u[p].e : emin;
    }
    XU acc[NF];
    bool slow[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) {
        const int q = f == 0 ? 0 : f + 1;
        acc[f] = u[q];
        slow[f] = !nrm[q];
    }
    const bool near = OP == 0 && wave_all(allnrm && emax - emin <= kNearSpread &&
                                          emin >= kNearEmin && emax <= kNearEmax);
    if (OP == 0 && wave_all(same)) {
        if (near)
            fold_rounds<OP, P, F_SAME_NEAR>(u, nrm, acc, slow);
        else
            fold_rounds<OP, P, F_SAME>(u, nrm, acc, slow);
    } else if (near) {
        fold_rounds<OP, P, F_NEAR>(u, nrm, acc, slow);
    } else {
        fold_rounds<OP, P, F_FULL>(u, nrm, acc, slow);
    }
#pragma unroll
    for (int f = 0; f < NF; f++) out[f == 0 ? 0 : f + 1] = pack_u(acc[f]);
    out[1] = out[0];
}

OSGPU_HD inline bool less(X80 a, X80 b);

// Every member's fold of a P-PE max (OP 5) or min (OP 6) of one element.
// The fold acc = (acc < b ? acc : b) (min; > for max, miscops.c:80-105)
// visits x_q, then x_0, x_1, ... skipping q, and keeps the LAST visited
// element with the extreme value (a tie hands over to the incoming b).  So
// with t1 = the highest index holding the extreme and t2 the next highest,
// member q gets x_t1 unless q == t1, which gets x_t2 (x_t1 if alone) -- the
// same encodings the P(P-1) compares select, from P compares.  Values are
// ordered by a 16+64-bit key (positive: 0x8000|e : m; negative:
// 0x7fff-e : ~m; zeros as +0), which is fcomi's order on zeros, denormals,
// normals and infinities.  Any NaN or unsupported / pseudo-denormal encoding
// in the element sends it to the compare-by-compare folds.
template <int OP, int P>
OSGPU_HD inline void team_fold_minmax(const X80 (&x)[P], X80 (&out)[P])
{
    uint32_t kh[P];
    uint64_t kl[P];
    bool ord = true;
#pragma unroll
    for (int p = 0; p < P; p++) {
        const uint32_t e = x[p].se & kEmax;
        const uint64_t m = x[p].m;
        const bool J = (m >> 63) != 0;
        ord = ord && (e == 0 ? !J : (e == kEmax ? m == (1ull << 63) : J));
        const bool neg = ((x[p].se >> 15) & 1) && (e | m) != 0;
        kh[p] = neg ? kEmax - e : 0x8000u | e;
        kl[p] = neg ? ~m : m;
    }
    if (!ord) {
#pragma unroll
        for (int q = 0; q < P; q++) {
            X80 acc = x[q];
#pragma unroll
            for (int j = 0; j < P; j++)
                if (j != q) {  // field by field: a select of whole structs
                               // makes the compiler address x through scratch
                    const bool keep = OP == 5 ? less(x[j], acc) : less(acc, x[j]);
                    acc.m = keep ? acc.m : x[j].m;
                    acc.se = keep ? acc.se : x[j].se;
                }
            out[q] = acc;
        }
        return;
    }
    uint32_t bh = kh[0];
    uint64_t bl = kl[0];
#pragma unroll
    for (int p = 1; p < P; p++) {
        const bool lt = kh[p] < bh || (kh[p] == bh && kl[p] < bl);
        const bool gt = kh[p] > bh || (kh[p] == bh && kl[p] > bl);
        const bool take = OP == 5 ? gt : lt;
        bh = take ? kh[p] : bh;
        bl = take ? kl[p] : bl;
    }
    // the highest index holding it (t1, value v1) and the value at the next
    // highest (v2; v1 when t1 is alone), carried along the scan
    int t1 = -1;
    bool two = false;
    X80 v1 = x[0], v2 = x[0];
#pragma unroll
    for (int p = 0; p < P; p++) {
        const bool eq = kh[p] == bh && kl[p] == bl;
        v2.m = eq && t1 >= 0 ? v1.m : v2.m;
        v2.se = eq && t1 >= 0 ? v1.se : v2.se;
        two = two || (eq && t1 >= 0);
        v1.m = eq ? x[p].m : v1.m;
        v1.se = eq ? x[p].se : v1.se;
        t1 = eq ? p : t1;
    }
    v2.m = two ? v2.m : v1.m;
    v2.se = two ? v2.se : v1.se;
#pragma unroll
    for (int q = 0; q < P; q++) {  // member q: v1 unless q == t1
        out[q].m = q == t1 ? v2.m : v1.m;
        out[q].se = q == t1 ? v2.se : v1.se;
    }
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
