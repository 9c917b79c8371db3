"""Maximum sizes through the real entry points on the GPU.

The reference computes `const int snred = sizeof(_type) * nreduce`
(src/reductions.c:44): it overflows once an array reaches 2 GiB, and
OVERLAP_CHECK then misjudges overlap.  The drop-in keeps
64-bit sizes end to end.  These runs use nreduce up to INT_MAX (the largest
value the int argument can carry) and check results with size-independent
properties computed on the device in chunks (the oracle would take minutes
at these sizes): every element of every PE's target equals the elementwise
fold, here recomputed by torch on exactly representable inputs.
"""
import ctypes

import pytest

import osgpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _team(P, heap_bytes):
    from support import team as T
    return T.Team(P, heap_bytes, device=True)


def _fill(torch, view, seed, lo, hi, chunk=1 << 28):
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    for s in range(0, view.numel(), chunk):
        e = min(view.numel(), s + chunk)
        view[s:e] = torch.randint(lo, hi, (e - s,), device="cuda:0", generator=g,
                                  dtype=torch.int64).to(view.dtype)


@pytest.mark.parametrize("path", [osgpu.PATH_AUTO, osgpu.PATH_PULL])
def test_short_sum_int_max_elements(torch_cuda, path):
    """nreduce = INT_MAX shorts = 4 GiB per array, 2 PEs; wrap-around sums."""
    torch = torch_cuda
    n = (1 << 31) - 1
    nb = 2 * n
    toff = (nb + 4095) // 4096 * 4096
    tm = _team(2, toff + nb)
    views = [tm.buf[pe * tm.H: pe * tm.H + nb].view(torch.int16) for pe in range(2)]
    for pe in range(2):
        _fill(torch, views[pe], 11 + pe, -32768, 32768)
    tm.lib.osgpu_set_path(path)
    try:
        tm.run("short", "sum", toff, 0, n)
    finally:
        tm.lib.osgpu_set_path(osgpu.PATH_AUTO)
    torch.cuda.synchronize()
    chunk = 1 << 28
    for pe in range(2):
        tgt = tm.buf[pe * tm.H + toff: pe * tm.H + toff + nb].view(torch.int16)
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            want = (views[0][s:e].to(torch.int32) + views[1][s:e].to(torch.int32)).to(torch.int16)
            assert torch.equal(tgt[s:e], want), (pe, s)
    del tm
    torch.cuda.empty_cache()


def test_double_sum_past_2GiB(torch_cuda):
    """nreduce = 2^28 + 3 doubles (2 GiB + 24 B per array): the size at which
    the reference's int byte count wraps.  3 PEs on the team path, values
    that make every partial sum exact, so any fold order gives the same bits."""
    torch = torch_cuda
    n = (1 << 28) + 3
    nb = 8 * n
    toff = (nb + 4095) // 4096 * 4096
    P = 3
    tm = _team(P, toff + nb)
    views = [tm.buf[pe * tm.H: pe * tm.H + nb].view(torch.float64) for pe in range(P)]
    for pe in range(P):
        _fill(torch, views[pe], 21 + pe, -(1 << 20), 1 << 20)  # small integers: exact sums
    tm.run("double", "sum", toff, 0, n)
    torch.cuda.synchronize()
    chunk = 1 << 27
    for pe in range(P):
        tgt = tm.buf[pe * tm.H + toff: pe * tm.H + toff + nb].view(torch.float64)
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            want = views[0][s:e] + views[1][s:e] + views[2][s:e]
            assert torch.equal(tgt[s:e], want), (pe, s)
    del tm
    torch.cuda.empty_cache()
