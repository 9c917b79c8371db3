"""The x87 soft-float as it runs on the MI355X, on the same random encodings
and seams as tests/test_x87_softfloat.py (which checks the host build of
csrc/x87.hpp): the device build has its own instruction choices
(v_ffbh_u32, v_sad_u16, saturating subtract; x87.hpp clz / absdiff / sub_sat
helpers), so the device results are checked against the reference's long
double ops (src/shmemu/miscops.c:30,98, native x87 on the host) directly.

* the combine kernel (osgpu_combine, two inputs: one soft op per element)
  on 200 K random raw encodings per mode, cancellations, and the exponent-
  gap / carry / borrow seams of the fast add, both operand orders;
* the team kernel (osgpu_team_combine: every member's own fold order,
  src/reductions.c:79-111) at 5 and 8 members on random significands with
  random signs and exponents 2^-3..2^3 -- the data of the long double rate
  measurements (tools/ld_team_rate.py), where every round takes the general
  fast add -- and on the same data with one sign.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
import osgpu
from test_x87_softfloat import _deep_cancel_pairs, _pairs, near_bounds_srcs, raw_random

pytestmark = pytest.mark.gpu

OPS = ("sum", "prod", "max", "min")


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _dev(torch, arr):
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    return torch.from_numpy(raw.copy()).to("cuda:0")


def _device_ops(torch, a, b):
    """every op of a and b on the GPU (osgpu_combine, K = 2), value bytes"""
    n = a.size
    da, db = _dev(torch, a), _dev(torch, b)
    out = torch.zeros(n * 16, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    res = {}
    for op in OPS:
        osgpu.combine("longdouble", op, out.data_ptr(), [da.data_ptr(), db.data_ptr()], n,
                      st.cuda_stream)
        st.synchronize()
        res[op] = out.cpu().numpy().reshape(-1, 16)[:, :10].copy()
    return res


def _check(torch, a, b):
    got = _device_ops(torch, a, b)
    for op in OPS:
        want = O.value_bytes(O.op_elementwise("longdouble", op, a, b,
                                              use_ref=O.ref_lib() is not None)).reshape(-1, 10)
        bad = np.nonzero((want != got[op]).any(1))[0]
        assert bad.size == 0, f"{op}: {bad.size} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("mode", ["normal", "any", "near", "low", "high"])
def test_device_random_encodings(torch_cuda, mode):
    n = 200_000
    _check(torch_cuda, raw_random(n, 11, mode), raw_random(n, 12, mode))


def test_device_cancellation(torch_cuda):
    x = raw_random(100_000, 21, "near")
    k = O.splitmix64(3, 100_000).astype(np.longdouble) / np.longdouble(2.0 ** 64)
    y = -x * (np.longdouble(1) + np.longdouble(2.0) ** -60 * k)
    _check(torch_cuda, x, y)


@pytest.mark.parametrize("where", ["unit", "underflow", "overflow"])
def test_device_aligned_operand_boundaries(torch_cuda, where):
    a, b = _pairs(where)
    _check(torch_cuda, a, b)
    _check(torch_cuda, b, a)


@pytest.mark.parametrize("gap", [0, 1])
def test_device_deep_cancellation_top_word(torch_cuda, gap):
    """add_fast's normalisation for every leading-zero count of the top word
    (opposite signs, gaps 0 and 1, top words k apart, k up to 2^25) on the
    device build, both operand orders."""
    a, b = _deep_cancel_pairs(gap)
    _check(torch_cuda, a, b)
    _check(torch_cuda, b, a)


def _ld_rate_data(P, n, seed, signs):
    """tools/ld_team_rate.py's "random" / "positive" data: random 64-bit
    significands (J set), exponents 2^-3..2^3, random or positive signs"""
    srcs = []
    for p in range(P):
        m = O.splitmix64(seed + 17 * p, n) | np.uint64(1 << 63)
        r = O.splitmix64(seed + 17 * p + 5, n)
        e = (np.uint64(0x3fff - 3) + r % np.uint64(7)).astype(np.uint16)
        s = ((r >> np.uint64(20)) & np.uint64(1)).astype(np.uint16) if signs else np.zeros(n, np.uint16)
        raw = np.zeros((n, 10), np.uint8)
        raw[:, :8] = m.view(np.uint8).reshape(n, 8)
        raw[:, 8:10] = (e | (s << np.uint16(15))).astype(np.uint16).view(np.uint8).reshape(n, 2)
        srcs.append(np.ascontiguousarray(O.from_value_bytes("longdouble", raw.reshape(-1))))
    return srcs


@pytest.mark.parametrize("P", [5, 8])
@pytest.mark.parametrize("signs", [True, False], ids=["random_signs", "one_sign"])
@pytest.mark.parametrize("op", ["sum", "prod"])
def test_team_folds_rate_data(torch_cuda, P, signs, op):
    torch = torch_cuda
    n = 50_000
    srcs = _ld_rate_data(P, n, 0x1D00 + P, signs)
    want = O.to_all("longdouble", op, srcs)
    ins = [_dev(torch, x) for x in srcs]
    outs = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda:0") for _ in range(P)]
    S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in ins])
    D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in outs])
    torch.cuda.synchronize()
    L = osgpu.load()
    assert L.osgpu_team_combine(osgpu.TYPES.index("longdouble"), osgpu.OPS.index(op), P, D, S,
                                n, None) == 0
    torch.cuda.synchronize()
    for q in range(P):
        got = outs[q].cpu().numpy().reshape(-1, 16)[:, :10].reshape(-1)
        assert np.array_equal(got, O.value_bytes(want[q]).reshape(-1)), (op, P, signs, q)


@pytest.mark.parametrize("P", [3, 8])
@pytest.mark.parametrize("signs", ["random", "one"])
def test_team_folds_near_exponent_bounds(torch_cuda, P, signs):
    """The device team kernel on near_bounds_srcs: waves whose inputs sit
    below, at and above the near-exponent gate's edges (x87.hpp kNearEmin,
    kNearEmax; the fold mode is chosen per wave), with near-cancellations
    -- every member's result bit-exact against the oracle's per-PE fold."""
    torch = torch_cuda
    n = 40_000
    srcs = near_bounds_srcs(P, signs, n)
    want = O.to_all("longdouble", "sum", srcs)
    ins = [_dev(torch, x) for x in srcs]
    outs = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda:0") for _ in range(P)]
    S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in ins])
    D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in outs])
    torch.cuda.synchronize()
    L = osgpu.load()
    assert L.osgpu_team_combine(osgpu.TYPES.index("longdouble"), osgpu.OPS.index("sum"), P, D, S,
                                n, None) == 0
    torch.cuda.synchronize()
    for q in range(P):
        got = outs[q].cpu().numpy().reshape(-1, 16)[:, :10].reshape(-1)
        assert np.array_equal(got, O.value_bytes(want[q]).reshape(-1)), (P, signs, q)
