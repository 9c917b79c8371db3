"""The GPU's x87 80-bit soft-float (csrc/x87.hpp), compiled for the host,
against the reference's long double ops (src/shmemu/miscops.c:30,98 compiled
for x86-64 = x87 fadd/fmul/fcomi): bit-exact on the golden grid (NaN
payloads, unnormals, pseudo-denormals, pseudo-infinities/NaNs, subnormals,
extremes) and on random raw encodings across the whole exponent range.
The same source runs on the MI355X in longdouble.hip (tests/test_gpu_parity.py).
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from support import team as T

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OPS = ((0, "sum"), (1, "prod"), (5, "max"), (6, "min"),
       (10, "sum"),   # 10: add_near where it applies (x87_check.hip), else add
       (11, "sum"))   # 11: add_same_near where the signs agree, else add


@pytest.fixture(scope="module")
def x87():
    return T.build_x87check()


def soft(L, op, a, b):
    out = np.zeros_like(a)
    assert L.x87check_op(op, a.ctypes.data, b.ctypes.data, out.ctypes.data, a.size) == 0
    return out


def raw_random(n, seed, mode):
    r = O.splitmix64(seed, n)
    r2 = O.splitmix64(seed ^ 0x77, n)
    m = r.copy()
    e = r2 & np.uint64(0x7FFF)
    if mode == "normal":
        m |= np.uint64(1 << 63)
    elif mode == "near":       # operands within 2^65 of each other around 1
        e = np.uint64(16383) + (r2 % np.uint64(130)) - np.uint64(65)
        m |= np.uint64(1 << 63)
    elif mode == "low":        # denormal / pseudo-denormal / tiny normals
        e = r2 % np.uint64(70)
        m |= np.uint64(1 << 63) * ((r2 >> np.uint64(20)) & np.uint64(1))
    elif mode == "high":       # overflow range
        e = np.uint64(0x7FFF) - (r2 % np.uint64(70))
        m |= np.uint64(1 << 63)
    s = (r2 >> np.uint64(40)) & np.uint64(1)
    se = (e | (s << np.uint64(15))).astype(np.uint16)
    arr = np.zeros((n, 16), np.uint8)
    arr[:, :8] = m.view(np.uint8).reshape(n, 8)
    arr[:, 8:10] = se.view(np.uint8).reshape(n, 2)
    return arr.reshape(-1).view(np.longdouble)


def check(L, a, b, use_ref):
    for op, name in OPS:
        want = O.value_bytes(O.op_elementwise("longdouble", name, a, b,
                                              use_ref=use_ref)).reshape(-1, 10)
        got = O.value_bytes(soft(L, op, a, b)).reshape(-1, 10)
        bad = np.nonzero((want != got).any(1))[0]
        assert bad.size == 0, f"{name}: {bad.size} mismatches, first {bad[:5]}"


def test_golden_grid(x87):
    z = np.load(os.path.join(GOLD, "ops_longdouble.npz"))
    a = O.from_value_bytes("longdouble", z["a"])
    b = O.from_value_bytes("longdouble", z["b"])
    for op, name in OPS:
        got = O.value_bytes(soft(x87, op, a, b)).reshape(-1, 10)
        want = z["out_" + name].reshape(-1, 10)
        bad = np.nonzero((want != got).any(1))[0]
        assert bad.size == 0, f"{name}: {bad.size} mismatches at {bad[:5]}"


@pytest.mark.parametrize("mode", ["normal", "any", "near", "low", "high"])
def test_random_encodings(x87, mode):
    n = 200_000
    a, b = raw_random(n, 11, mode), raw_random(n, 12, mode)
    # the oracle's long double ops are native x87 on this host == the
    # reference's; use the compiled reference itself when it is present
    check(x87, a, b, use_ref=O.ref_lib() is not None)


def test_cancellation(x87):
    x = raw_random(100_000, 21, "near")
    k = O.splitmix64(3, 100_000).astype(np.longdouble) / np.longdouble(2.0 ** 64)
    y = -x * (np.longdouble(1) + np.longdouble(2.0) ** -60 * k)
    check(x87, x, y, use_ref=O.ref_lib() is not None)


def _pairs(where, n=60_000):
    r = O.splitmix64(77, 4 * n).reshape(4, n)
    base_e = {"unit": 16383, "underflow": 3, "overflow": 0x7FFE - 1}[where]
    diffs = np.array([0, 1, 2, 3, 29, 30, 31, 32, 62, 63, 64, 65, 66, 67, 70, 120, 200], np.int64)
    d = diffs[r[0] % np.uint64(diffs.size)]
    ea = np.full(n, base_e, np.int64) + (r[1] % np.uint64(3)).astype(np.int64) - 1
    eb = np.clip(ea - d, 1, 0x7FFE)
    # significands: random, or 2^63 + small, or 2^64 - small (seams of the
    # borrow / carry cases)
    kind = r[2] % np.uint64(3)
    small = r[3] & np.uint64(0xFF)
    top = np.uint64(1 << 63)
    ma = np.where(kind == 0, r[2] | top, np.where(kind == 1, top + small,
                                                  np.uint64((1 << 64) - 1) - small))
    mb = np.where(kind == 2, r[3] | top, np.where(kind == 1, np.uint64((1 << 64) - 1) - small,
                                                  top + small))
    sa = (r[1] >> np.uint64(7)) & np.uint64(1)
    sb = (r[1] >> np.uint64(9)) & np.uint64(1)

    def pack(m, e, s):
        arr = np.zeros((n, 16), np.uint8)
        arr[:, :8] = m.astype(np.uint64).view(np.uint8).reshape(n, 8)
        se = (e.astype(np.uint64) | (s << np.uint64(15))).astype(np.uint16)
        arr[:, 8:10] = se.view(np.uint8).reshape(n, 2)
        return arr.reshape(-1).view(np.longdouble)
    return pack(ma, ea, sa), pack(mb, eb, sb)


def _deep_cancel_pairs(gap, n=120_000, seed=41):
    """Opposite-sign normal pairs near 1 whose difference cancels 7 to 31
    leading bits of the top significand word (x87.hpp add_fast's normalise
    by ffbh of the top word and its funnel shift, every lz in 0..31):
    gap 0: b's top 32-bit significand word = a's +- k; gap 1: a's top word
    0x80000000 against b's 0xFFFFFFFF - k (2a - b is then about k * 2^32);
    k = 2^j + a random part below 2^j for j in 0..24 (k in 1..2^25), the low
    words random."""
    r = O.splitmix64(seed + gap, 5 * n).reshape(5, n)
    j = (r[0] % np.uint64(25)).astype(np.uint64)
    k = (np.uint64(1) << j) + (r[1] & ((np.uint64(1) << j) - np.uint64(1)))
    top = np.uint64(1 << 31)
    if gap == 0:
        ta = top + (r[2] >> np.uint64(33)) % (np.uint64(1 << 31) - np.uint64(1 << 26)) \
            + np.uint64(1 << 25)
        up = (r[3] & np.uint64(1)).astype(bool)
        tb = np.where(up, ta + k, ta - k)
        tb = np.minimum(tb, np.uint64(0xFFFFFFFF))
    else:
        ta = np.full(n, top, np.uint64)
        tb = np.uint64(0xFFFFFFFF) - k + np.uint64(1)
    ma = (ta << np.uint64(32)) | (r[3] >> np.uint64(32))
    mb = (tb << np.uint64(32)) | (r[4] & np.uint64(0xFFFFFFFF))
    ea = np.full(n, 16383, np.uint64) + (r[2] & np.uint64(3)) - np.uint64(1)
    eb = ea - np.uint64(gap)
    sa = (r[4] >> np.uint64(40)) & np.uint64(1)
    sb = sa ^ np.uint64(1)

    def pack(m, e, sg):
        arr = np.zeros((n, 16), np.uint8)
        arr[:, :8] = m.astype(np.uint64).view(np.uint8).reshape(n, 8)
        arr[:, 8:10] = (e | (sg << np.uint64(15))).astype(np.uint16).view(np.uint8).reshape(n, 2)
        return arr.reshape(-1).view(np.longdouble)
    return pack(ma, ea, sa), pack(mb, eb, sb)


@pytest.mark.parametrize("gap", [0, 1])
def test_deep_cancellation_top_word(x87, gap):
    """add_fast's normalisation for every leading-zero count of the top
    word (only small lz were reached before): opposite signs,
    exponent gaps 0 and 1, top significand words k apart for k up to 2^25,
    both operand orders, bit-exact against the host's x87."""
    a, b = _deep_cancel_pairs(gap)
    raw = (O.value_bytes(a).reshape(-1, 10)[:, 4:8].copy().view(np.uint32).reshape(-1).astype(np.int64)
           - O.value_bytes(b).reshape(-1, 10)[:, 4:8].copy().view(np.uint32).reshape(-1).astype(np.int64))
    if gap == 0:   # the top words really differ by 1 .. 2^25
        assert (np.abs(raw) >= 1).all() and (np.abs(raw) <= 1 << 25).all()
    check(x87, a, b, use_ref=O.ref_lib() is not None)
    check(x87, b, a, use_ref=O.ref_lib() is not None)


@pytest.mark.parametrize("where", ["unit", "underflow", "overflow"])
def test_aligned_operand_boundaries(x87, where):
    """The normal-operand fast path of x87 add (x87.hpp add_fast): exponent
    differences around the 64-bit shift seams (0-3, 62-67, 70, 120, 200),
    significands next to powers of two (borrow / carry / renormalise cases),
    both signs, near 1, near the underflow threshold (results on the denormal
    grid) and near overflow -- bit-exact against the host's x87, both operand
    orders."""
    for w in (where,):
        a, b = _pairs(w)
        check(x87, a, b, use_ref=O.ref_lib() is not None)
        check(x87, b, a, use_ref=O.ref_lib() is not None)


def test_equal_and_opposite_operands(x87):
    """a + a (carry out of the significand at every exponent, up to overflow)
    and a + (-a) (exact cancellation to +0), normal, denormal and special
    encodings alike."""
    a = np.concatenate([raw_random(20_000, 31, m) for m in ("normal", "near", "low", "high",
                                                             "any")])
    raw = O.value_bytes(a).reshape(-1, 10).copy()
    raw[::2, :7] = 0            # every other significand a power of two (2^63):
    raw[::2, 7] = 0x80          # a + a carries out of the 64 bits exactly
    a = O.from_value_bytes("longdouble", raw.reshape(-1))
    neg = O.value_bytes(a).reshape(-1, 10).copy()
    neg[:, 9] ^= 0x80
    b = O.from_value_bytes("longdouble", neg.reshape(-1))
    check(x87, a, a, use_ref=O.ref_lib() is not None)
    check(x87, a, b, use_ref=O.ref_lib() is not None)


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("op", ["sum", "prod"])
def test_team_fold_rounds(x87, op, P):
    """The team kernel's fold of every member (x87.hpp team_fold_sum_prod:
    P-1 folds advanced in rounds, fast op with a general fallback per round,
    member 1 sharing member 0's fold) against the reference's per-PE fold
    order (oracle to_all), on data that sends some lanes and rounds to the
    general op: mostly normal values near 1 with cancellations, plus zeros,
    denormals, infinities, NaNs and values near overflow."""
    n = 40_000
    srcs = []
    for p in range(P):
        x = raw_random(n, 100 + p, "near")
        raw = O.value_bytes(x).reshape(-1, 10).copy()
        k = O.splitmix64(300 + p, n)
        for sel, mode in ((1, "any"), (2, "low"), (3, "high")):
            idx = np.nonzero((k % np.uint64(53)) == np.uint64(sel))[0]
            raw[idx] = O.value_bytes(raw_random(n, 500 + 7 * p + sel, mode)).reshape(-1, 10)[idx]
        srcs.append(np.ascontiguousarray(O.from_value_bytes("longdouble", raw.reshape(-1))))
    if op == "sum":             # exact cancellations against member 0's value
        neg = O.value_bytes(srcs[0]).reshape(-1, 10).copy()
        neg[:, 9] ^= 0x80
        raw1 = O.value_bytes(srcs[1]).reshape(-1, 10).copy()
        raw1[::17] = neg[::17]
        srcs[1] = np.ascontiguousarray(O.from_value_bytes("longdouble", raw1.reshape(-1)))
    want = O.to_all("longdouble", op, srcs)
    got = [np.zeros_like(srcs[0]) for _ in range(P)]
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in srcs])
    dp = (ctypes.c_void_p * P)(*[g.ctypes.data for g in got])
    assert x87.x87check_team(0 if op == "sum" else 1, P, sp, dp, n) == 0
    for q in range(P):
        w = O.value_bytes(want[q]).reshape(-1, 10)
        g = O.value_bytes(got[q]).reshape(-1, 10)
        bad = np.nonzero((w != g).any(1))[0]
        assert bad.size == 0, f"member {q}: {bad.size} mismatches at {bad[:5]}"


def test_tie_of_exponent_and_top_word(x87):
    """Operands with the same exponent and the same top 32 significand bits
    (the magnitude order's tie, x87.hpp add_fast's flag and add_near's
    negative-sum case): low words random, equal or one apart, both signs
    pairings, both operand orders."""
    n = 100_000
    r = O.splitmix64(61, 4 * n).reshape(4, n)
    hi = (r[0] | np.uint64(1 << 63)) & np.uint64(0xFFFFFFFF00000000)
    lo_a = r[1] & np.uint64(0xFFFFFFFF)
    kind = r[2] % np.uint64(3)
    lo_b = np.where(kind == 0, r[3] & np.uint64(0xFFFFFFFF),
                    np.where(kind == 1, lo_a, (lo_a + np.uint64(1)) & np.uint64(0xFFFFFFFF)))
    e = np.full(n, 16383, np.uint64) + (r[2] >> np.uint64(8)) % np.uint64(40) - np.uint64(20)
    sa = (r[3] >> np.uint64(40)) & np.uint64(1)
    sb = np.where((r[3] >> np.uint64(41)) & np.uint64(3) == 0, sa, sa ^ np.uint64(1))

    def pack(m, sg):
        arr = np.zeros((n, 16), np.uint8)
        arr[:, :8] = m.astype(np.uint64).view(np.uint8).reshape(n, 8)
        arr[:, 8:10] = (e | (sg << np.uint64(15))).astype(np.uint16).view(np.uint8).reshape(n, 2)
        return arr.reshape(-1).view(np.longdouble)
    a, b = pack(hi | lo_a, sa), pack(hi | lo_b, sb)
    check(x87, a, b, use_ref=O.ref_lib() is not None)
    check(x87, b, a, use_ref=O.ref_lib() is not None)


@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_team_fold_near(x87, P):
    """Sums whose inputs' exponents lie within x87.hpp kNearSpread of each
    other take the near-exponent rounds (add_near, falling back to
    add_general per fold and lane): random signs, exponents 2^-3..2^3 (the bench's
    data), near-cancellations of the first two operands (the running sum
    drops 20-60 binades below the next operand: gaps above 30 in later
    rounds), exact cancellations, top-word ties, and some elements whose
    inputs spread wider (the general rounds) -- against the reference's
    per-PE fold order."""
    n = 40_000
    srcs = []
    for p in range(P):
        r = O.splitmix64(1200 + p, 2 * n).reshape(2, n)
        m = r[0] | np.uint64(1 << 63)
        e = np.full(n, 16383, np.uint64) + r[1] % np.uint64(7) - np.uint64(3)
        wide = (r[1] >> np.uint64(20)) % np.uint64(11) == np.uint64(0)
        e = np.where(wide, e + (r[1] >> np.uint64(24)) % np.uint64(60), e)
        s = (r[1] >> np.uint64(40)) & np.uint64(1)
        arr = np.zeros((n, 16), np.uint8)
        arr[:, :8] = m.view(np.uint8).reshape(n, 8)
        arr[:, 8:10] = (e | (s << np.uint64(15))).astype(np.uint16).view(np.uint8).reshape(n, 2)
        srcs.append(arr.reshape(-1).view(np.longdouble).copy())
    # element k % 5 == 1: x1 = -x0 * (1 + 2^-j * u), j in 20..60; k % 5 == 2:
    # x1 = -x0 exactly; k % 5 == 3: x1 = x0's exponent and top word, opposite sign
    x0 = O.value_bytes(srcs[0]).reshape(-1, 10).copy()
    x1 = O.value_bytes(srcs[1]).reshape(-1, 10).copy()
    k = np.arange(n)
    j = 20 + (k * 7) % 41
    u = O.splitmix64(1300, n).astype(np.longdouble) / np.longdouble(2.0 ** 64)
    near = -srcs[0] * (np.longdouble(1) + np.ldexp(np.longdouble(1), -j) * u)
    nb = O.value_bytes(near).reshape(-1, 10)
    x1[k % 5 == 1] = nb[k % 5 == 1]
    neg = x0.copy()
    neg[:, 9] ^= 0x80
    x1[k % 5 == 2] = neg[k % 5 == 2]
    tie = neg.copy()
    tie[:, :4] = x1[:, :4]
    x1[k % 5 == 3] = tie[k % 5 == 3]
    srcs[1] = np.ascontiguousarray(O.from_value_bytes("longdouble", x1.reshape(-1)))
    want = O.to_all("longdouble", "sum", srcs)
    got = [np.zeros_like(srcs[0]) for _ in range(P)]
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in srcs])
    dp = (ctypes.c_void_p * P)(*[g.ctypes.data for g in got])
    assert x87.x87check_team(0, P, sp, dp, n) == 0
    for q in range(P):
        w = O.value_bytes(want[q]).reshape(-1, 10)
        g = O.value_bytes(got[q]).reshape(-1, 10)
        bad = np.nonzero((w != g).any(1))[0]
        assert bad.size == 0, f"member {q}: {bad.size} mismatches at {bad[:5]}"


def near_bounds_srcs(P, signs, n=40_000):
    """Inputs of test_team_fold_near_exponent_bounds (and its device twin in
    test_gpu_x87.py): every run of 64 elements (one wave on the GPU, where
    the fold mode is chosen per wave) draws its exponents from one window of
    25 binades -- just below the near-exponent gate (1..25, results on the
    denormal grid), at its lower edge (32..56), at its upper edge
    (kEmax-40..kEmax-16) and above it (kEmax-25..kEmax-1, overflow) --
    random or one sign, and for random signs near-cancellations
    x1 = -x0 (1 + 2^-j u), j in 20..60, in every third element."""
    lows = np.array([1, 32, 0x7FFF - 40, 0x7FFF - 25], np.uint64)
    k = np.arange(n)
    base = lows[(k // 64) % 4]
    srcs = []
    for p in range(P):
        r = O.splitmix64(1410 + p, 2 * n).reshape(2, n)
        m = r[0] | np.uint64(1 << 63)
        e = base + r[1] % np.uint64(25)
        s = (r[1] >> np.uint64(40)) & np.uint64(1) if signs == "random" else np.zeros(n, np.uint64)
        arr = np.zeros((n, 16), np.uint8)
        arr[:, :8] = m.view(np.uint8).reshape(n, 8)
        arr[:, 8:10] = (e | (s << np.uint64(15))).astype(np.uint16).view(np.uint8).reshape(n, 2)
        srcs.append(arr.reshape(-1).view(np.longdouble).copy())
    if signs == "random":
        j = 20 + (k * 7) % 41
        u = O.splitmix64(1420, n).astype(np.longdouble) / np.longdouble(2.0 ** 64)
        near = O.value_bytes(-srcs[0] * (np.longdouble(1) + np.ldexp(np.longdouble(1), -j) * u)).reshape(-1, 10)
        x1 = O.value_bytes(srcs[1]).reshape(-1, 10).copy()
        x1[k % 3 == 1] = near[k % 3 == 1]
        srcs[1] = np.ascontiguousarray(O.from_value_bytes("longdouble", x1.reshape(-1)))
    return srcs


@pytest.mark.parametrize("P", [3, 8])
@pytest.mark.parametrize("signs", ["random", "one"])
def test_team_fold_near_exponent_bounds(x87, P, signs):
    """The near-exponent rounds' gate (x87.hpp kNearEmin / kNearEmax: the
    near adds skip the result's range test), on near_bounds_srcs' windows
    below, at and above its edges, against the reference's per-PE fold
    order."""
    n = 40_000
    srcs = near_bounds_srcs(P, signs, n)
    want = O.to_all("longdouble", "sum", srcs)
    got = [np.zeros_like(srcs[0]) for _ in range(P)]
    sp = (ctypes.c_void_p * P)(*[s_.ctypes.data for s_ in srcs])
    dp = (ctypes.c_void_p * P)(*[g.ctypes.data for g in got])
    assert x87.x87check_team(0, P, sp, dp, n) == 0
    for q in range(P):
        w = O.value_bytes(want[q]).reshape(-1, 10)
        g = O.value_bytes(got[q]).reshape(-1, 10)
        bad = np.nonzero((w != g).any(1))[0]
        assert bad.size == 0, f"member {q}: {bad.size} mismatches at {bad[:5]}"


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("sign", [0, 1])
def test_team_fold_same_sign(x87, sign, P):
    """Sums whose operands all share one sign take the addition-only fast
    add (x87.hpp add_same_fast, chosen per round when every fold of every
    lane adds like signs): exponent gaps across the 64-bit seams, carries
    out of the significand (2^64 - small + 2^64 - small), values near
    overflow and on the denormal grid (general path), against the
    reference's per-PE fold order."""
    n = 40_000
    srcs = []
    for p in range(P):
        a, b = _pairs(["unit", "overflow", "underflow"][p % 3], n)
        raw = O.value_bytes(a if p % 2 else b).reshape(-1, 10).copy()
        x = O.value_bytes(raw_random(n, 700 + p, "near")).reshape(-1, 10)
        k = O.splitmix64(800 + p, n)
        pick = (k % np.uint64(3)) == np.uint64(0)
        raw[pick] = x[pick]
        raw[:, 9] = (raw[:, 9] & 0x7F) | (0x80 if sign else 0)   # one sign everywhere
        srcs.append(np.ascontiguousarray(O.from_value_bytes("longdouble", raw.reshape(-1))))
    want = O.to_all("longdouble", "sum", srcs)
    got = [np.zeros_like(srcs[0]) for _ in range(P)]
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in srcs])
    dp = (ctypes.c_void_p * P)(*[g.ctypes.data for g in got])
    assert x87.x87check_team(0, P, sp, dp, n) == 0
    for q in range(P):
        w = O.value_bytes(want[q]).reshape(-1, 10)
        g = O.value_bytes(got[q]).reshape(-1, 10)
        bad = np.nonzero((w != g).any(1))[0]
        assert bad.size == 0, f"member {q}: {bad.size} mismatches at {bad[:5]}"


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("op", ["max", "min"])
def test_team_fold_minmax(x87, op, P):
    """The team kernel's max / min (x87.hpp team_fold_minmax: one key scan,
    then each member's pick among tied extremes) against the reference's
    per-PE fold order: values from a small pool so that extremes tie across
    PEs -- +0 against -0, equal denormals, infinities, duplicated normals --
    with NaNs, pseudo-denormals and unsupported encodings in some elements
    (the compare-by-compare fold)."""
    n = 60_000
    pool = np.zeros((12, 10), np.uint8)

    def enc(m, e, sgn):
        b = np.zeros(10, np.uint8)
        b[:8] = np.frombuffer(np.uint64(m).tobytes(), np.uint8)
        b[8:10] = np.frombuffer(np.uint16(e | (sgn << 15)).tobytes(), np.uint8)
        return b
    vals = [(0, 0, 0), (0, 0, 1), (1 << 40, 0, 0), (1 << 40, 0, 1), (1 << 63, 0x7FFF, 0),
            (1 << 63, 0x7FFF, 1), (0xC000000000000000, 0x3FFF, 0), (0xC000000000000000, 0x3FFF, 1),
            (1 << 63, 1, 0), (1 << 63, 1, 1), (0x8000000000000001, 0x7FFE, 0),
            (0x8000000000000001, 0x7FFE, 1)]
    for i, v in enumerate(vals):
        pool[i] = enc(*v)
    specials = O.value_bytes(raw_random(n, 900, "any")).reshape(-1, 10)
    srcs = []
    for p in range(P):
        k = O.splitmix64(700 + p, n)
        raw = pool[(k % np.uint64(12)).astype(np.int64)].copy()
        # a narrower pool in some elements makes ties likely at every P
        narrow = (k >> np.uint64(8)) % np.uint64(3) == 0
        raw[narrow] = pool[((k[narrow] >> np.uint64(16)) % np.uint64(2)).astype(np.int64)]
        sp = (k >> np.uint64(24)) % np.uint64(29) == 0
        raw[sp] = specials[sp]
        srcs.append(np.ascontiguousarray(O.from_value_bytes("longdouble", raw.reshape(-1))))
    want = O.to_all("longdouble", op, srcs)
    got = [np.zeros_like(srcs[0]) for _ in range(P)]
    sptr = (ctypes.c_void_p * P)(*[s.ctypes.data for s in srcs])
    dptr = (ctypes.c_void_p * P)(*[g.ctypes.data for g in got])
    assert x87.x87check_team(5 if op == "max" else 6, P, sptr, dptr, n) == 0
    for q in range(P):
        w = O.value_bytes(want[q]).reshape(-1, 10)
        g = O.value_bytes(got[q]).reshape(-1, 10)
        bad = np.nonzero((w != g).any(1))[0]
        assert bad.size == 0, f"member {q}: {bad.size} mismatches at {bad[:5]}"
