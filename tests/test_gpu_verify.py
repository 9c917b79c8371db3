"""GPU verification kernels (csrc/verify.hip) and the full-size properties
they make checkable without copying arrays to the host.

* osgpu_checksum (sum / xor / position-weighted hash of the element bits)
  and osgpu_compare (differing 16-B vectors, first difference) against
  numpy restatements, aligned and misaligned, every element size.
* "Checksum of checksums" at BASELINE scale: for an integer sum the sum of
  every PE's target equals the sum of the sources' sums (mod 2^w), for xor
  the xor of xors -- on every PE's target, team and pull path.
* Floating point at full size: the team and pull paths implement the same
  per-PE fold order, so their targets must be bitwise identical.
"""
import numpy as np
import pytest

import osgpu

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _mix64(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        return z ^ (z >> np.uint64(31))


def _values(raw, es):
    """zero-extended element values as the kernel folds them (uint64)."""
    if es == 16:
        w = raw.view(np.uint64).reshape(-1, 2)
        return w[:, 0] ^ _mix64(w[:, 1].copy())
    return raw.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[es]).astype(np.uint64)


def _expect(raw, es, mode):
    v = _values(raw, es)
    with np.errstate(over="ignore"):
        if mode == osgpu.CK_SUM:
            return int(np.sum(v, dtype=np.uint64))
        if mode == osgpu.CK_XOR:
            return int(np.bitwise_xor.reduce(v)) if v.size else 0
        idx = np.arange(1, v.size + 1, dtype=np.uint64)
        return int(np.sum(_mix64(v + np.uint64(0x9e3779b97f4a7c15) * idx), dtype=np.uint64))


@pytest.mark.parametrize("t,es", [("short", 2), ("int", 4), ("double", 8), ("complexd", 16)])
@pytest.mark.parametrize("mode", [osgpu.CK_SUM, osgpu.CK_XOR, osgpu.CK_HASH])
def test_checksum_matches_numpy(torch_cuda, t, es, mode):
    torch = torch_cuda
    rng = np.random.default_rng(es * 10 + mode)
    for n in (0, 1, 7, 1000, 65537, 3 << 20):
        for off in (0, es if es < 16 else 8):
            raw = rng.integers(0, 256, n * es, dtype=np.uint8)
            buf = torch.zeros(n * es + 64, dtype=torch.uint8, device="cuda")
            if n:
                buf[off:off + n * es].copy_(torch.from_numpy(raw).cuda())
            torch.cuda.synchronize()
            got = osgpu.checksum(t, mode, buf.data_ptr() + off, n)
            assert got == _expect(raw, es, mode), (t, mode, n, off)


def test_compare_counts_and_first_offset(torch_cuda):
    torch = torch_cuda
    n = (8 << 20) + 37
    a = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device="cuda")
    b = a.clone()
    assert osgpu.compare(a.data_ptr(), b.data_ptr(), n) == (0, None)
    for pos in (n - 1, 5_000_011, 123, 16 * 1000 + 3):
        b[pos] ^= 0x40
    torch.cuda.synchronize()
    bad, first = osgpu.compare(a.data_ptr(), b.data_ptr(), n)
    assert bad == 4 and first == 123 // 16 * 16, (bad, first)
    # misaligned pair: counted in bytes
    bad, first = osgpu.compare(a.data_ptr() + 1, b.data_ptr() + 1, n - 1)
    assert bad == 4 and first == 122, (bad, first)


def _team(torch, npes, n, es):
    from support import team as T
    return T.Team(npes, 2 * n * es + 8192, device=True)


@pytest.mark.parametrize("t,op,mode,bits", [("long", "sum", osgpu.CK_SUM, 64),
                                            ("long", "xor", osgpu.CK_XOR, 64),
                                            ("int", "sum", osgpu.CK_SUM, 32)])
def test_checksum_of_checksums_full_size(torch_cuda, t, op, mode, bits):
    """BASELINE config 3 scale (32 Mi longs = 256 MiB per array) and 64 Mi
    ints, 3 PEs: every PE's target checksum equals the combination of the
    sources' checksums, team and pull path."""
    torch = torch_cuda
    es = bits // 8
    n = (256 << 20) // es
    P = 3
    tm = _team(torch, P, n, es)
    toff = (n * es + 4095) // 4096 * 4096
    dt = torch.int64 if bits == 64 else torch.int32
    g = torch.Generator(device="cuda").manual_seed(bits + mode)
    for pe in range(P):
        tm.buf[pe * tm.H:pe * tm.H + n * es].view(dt).random_(generator=g)
    torch.cuda.synchronize()
    srcs = [osgpu.checksum(t, mode, tm.ptr(pe, 0), n) for pe in range(P)]
    want = (sum(srcs) if mode == osgpu.CK_SUM else srcs[0] ^ srcs[1] ^ srcs[2])
    mod = (1 << bits) - 1
    for path in (osgpu.PATH_AUTO, osgpu.PATH_PULL):
        tm.lib.osgpu_set_path(path)
        try:
            tm.run(t, op, toff, 0, n)
        finally:
            tm.lib.osgpu_set_path(osgpu.PATH_AUTO)
        for pe in range(P):
            got = osgpu.checksum(t, mode, tm.ptr(pe, toff), n)
            assert got & mod == want & mod, (t, op, path, pe)
    del tm


def test_fp_team_and_pull_identical_full_size(torch_cuda):
    """BASELINE config 2 shape (64 Mi doubles), 3 PEs: the owner-computes
    team kernel and the pull form fold in the same per-PE order, so every
    PE's target must be bitwise identical between them (checked on the GPU
    in full), and differ between PEs where the order does."""
    torch = torch_cuda
    n, P = 64 << 20, 3
    tm = _team(torch, P, 2 * n, 8)
    toff = (n * 8 + 4095) // 4096 * 4096
    toff2 = toff + (n * 8 + 4095) // 4096 * 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    for pe in range(P):
        tm.buf[pe * tm.H:pe * tm.H + n * 8].view(torch.float64).uniform_(-1e3, 1e3, generator=g)
    torch.cuda.synchronize()
    tm.run("double", "sum", toff, 0, n)
    assert all(p == "team" for p in tm.last_paths.values())
    tm.lib.osgpu_set_path(osgpu.PATH_PULL)
    try:
        tm.run("double", "sum", toff2, 0, n)
    finally:
        tm.lib.osgpu_set_path(osgpu.PATH_AUTO)
    for pe in range(P):
        assert osgpu.compare(tm.ptr(pe, toff), tm.ptr(pe, toff2), n * 8) == (0, None), pe
    # PE 2 folds x2 + x0 + x1, PE 0 folds x0 + x1 + x2: they must differ somewhere
    bad, _ = osgpu.compare(tm.ptr(0, toff), tm.ptr(2, toff), n * 8)
    assert bad > 0
    del tm
