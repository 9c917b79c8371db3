"""The GPU's x87 80-bit soft-float (csrc/x87.hpp), compiled for the host,
against the reference's long double ops (src/shmemu/miscops.c:30,98 compiled
for x86-64 = x87 fadd/fmul/fcomi): bit-exact on the golden grid (NaN
payloads, unnormals, pseudo-denormals, pseudo-infinities/NaNs, subnormals,
extremes) and on random raw encodings across the whole exponent range.
The same source runs on the MI355X in longdouble.hip (tests/test_gpu_parity.py).
"""
import os

import numpy as np
import pytest

import oracle as O
from support import team as T

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OPS = ((0, "sum"), (1, "prod"), (5, "max"), (6, "min"))


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
