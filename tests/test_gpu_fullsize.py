"""BASELINE configs 4 and 5 at their full sizes on one MI355X, through the
kernel shmem_<T>_<op>_to_all dispatches for a P-PE call (the owner-computes
team kernel, osgpu_team_combine in the C ABI: one launch does every member's
shard, as the P PEs' launches do together on P GPUs).

Every member's target is checked bit for bit against the reference's fold
order for that member (src/reductions.c:79-111: PE q starts from its own
source, then PE 0, 1, ... skipping q), restated with PyTorch element-wise
IEEE operations in that order (no contraction: one rounding per operation,
the reference's SSE arithmetic for float/double) at full size, and against
the oracle (oracle/, pinned by the reference's compiled element ops) on a
64 Ki-element sample.

* config 4: double sum, nreduce = 1 Gi (8 GiB per array), 8 PEs
  (64 GiB of sources, 64 GiB of targets);
* config 5: float min / max / prod, nreduce = 128 Mi (512 MiB per array),
  8 PEs -- the device-resident part of that config (its H2D/D2H staging is
  tests/test_gpu_parity.py and test_multiproc.py).
"""
import ctypes

import pytest

import osgpu

pytestmark = pytest.mark.gpu

P = 8


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _team(torch, t, op, srcs, dsts, n):
    L = osgpu.load()
    S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs])
    D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts])
    # the inputs were written on torch's stream; a NULL stream would be the
    # library's non-blocking one, which does not wait for them
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    rc = L.osgpu_team_combine(osgpu.TYPES.index(t), osgpu.OPS.index(op), P, D, S, n,
                              ctypes.c_void_p(st))
    assert rc == 0, L.osgpu_last_error().decode()
    torch.cuda.synchronize()


def _fold(torch, op, srcs, q):
    """Member q's result in its own order (reductions.c:84-111)."""
    f = {"sum": torch.add, "prod": torch.mul,
         # a<b?a:b / a>b?a:b with a the accumulator (miscops.c:80-105)
         "min": lambda a, b: torch.where(a < b, a, b),
         "max": lambda a, b: torch.where(a > b, a, b)}[op]
    acc = srcs[q].clone()
    for j in range(P):
        if j != q:
            acc = f(acc, srcs[j])
    return acc


def _oracle_sample(torch, t, op, srcs, got, n, nsamp=1 << 16, seed=77):
    """The full-size targets against the ORACLE (oracle/, the restatement
    pinned by the reference's compiled element ops) on a sample of indices:
    every PE's sampled inputs folded by the oracle in that PE's order,
    compared bit for bit with every target at those indices (VERDICT r05
    weak 2: the PyTorch fold above is not the oracle)."""
    import numpy as np
    import oracle as O
    g = torch.Generator(device="cuda:0").manual_seed(seed)
    idx = torch.randint(0, n, (nsamp,), device="cuda:0", generator=g)
    xs = [np.ascontiguousarray(x[idx].cpu().numpy()) for x in srcs]
    want = O.to_all(t, op, xs)
    for q in range(P):
        g_ = got[q][idx].cpu().numpy()
        assert np.array_equal(g_.view(np.uint8), np.ascontiguousarray(want[q]).view(np.uint8)), \
            (t, op, q)


def _need(torch, nbytes):
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    if free < nbytes:
        pytest.skip(f"needs {nbytes >> 30} GiB of free HBM, {free >> 30} GiB free")


def test_config4_double_sum_1Gi_8_pes(torch_cuda):
    torch = torch_cuda
    n = 1 << 30
    _need(torch, (2 * P + 2) * n * 8)
    g = torch.Generator(device="cuda:0").manual_seed(4)
    srcs = [torch.empty(n, dtype=torch.float64, device="cuda:0").uniform_(1.0, 2.0, generator=g)
            for _ in range(P)]
    dsts = [torch.empty(n, dtype=torch.float64, device="cuda:0") for _ in range(P)]
    _team(torch, "double", "sum", srcs, dsts, n)
    _oracle_sample(torch, "double", "sum", srcs, dsts, n)
    for q in range(P):
        want = _fold(torch, "sum", srcs, q)
        assert torch.equal(dsts[q].view(torch.int64), want.view(torch.int64)), q
        del want
    # every member's fold starts from its own source: with 8 addends in
    # [1, 2) the orders round differently, so targets differ between members
    assert not torch.equal(dsts[0], dsts[7])
    del srcs, dsts
    torch.cuda.empty_cache()


@pytest.mark.parametrize("op,lo,hi", [("min", -1e3, 1e3), ("max", -1e3, 1e3),
                                      ("prod", 0.9, 1.1)])
def test_config5_float_128Mi_8_pes(torch_cuda, op, lo, hi):
    torch = torch_cuda
    n = 128 << 20
    _need(torch, (2 * P + 2) * n * 4)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    srcs = [torch.empty(n, dtype=torch.float32, device="cuda:0").uniform_(lo, hi, generator=g)
            for _ in range(P)]
    dsts = [torch.empty(n, dtype=torch.float32, device="cuda:0") for _ in range(P)]
    _team(torch, "float", op, srcs, dsts, n)
    _oracle_sample(torch, "float", op, srcs, dsts, n)
    for q in range(P):
        want = _fold(torch, op, srcs, q)
        assert torch.equal(dsts[q].view(torch.int32), want.view(torch.int32)), (op, q)
        del want
    del srcs, dsts
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pinned", [True, False])
def test_config5_host_staged_128Mi_8_pes(torch_cuda, pinned):
    """BASELINE config 5 as the reference places it: sources and targets in
    HOST symmetric heaps (8 PE threads, 128 Mi floats per PE), the STAGED
    path (H2D of each PE's source, the team exchange on the GPU, D2H) for
    float min, max and prod in turn, on a heap pinned with
    osgpu_host_register and on a pageable one (the library's bounce).  Every
    member's target is checked bit for bit against its own fold order
    (_fold, on the GPU)."""
    import numpy as np
    torch = torch_cuda
    from support import team as T
    n = 128 << 20
    nb = n * 4
    _need(torch, (3 * P + 2) * nb)
    L = osgpu.load()
    L.osgpu_finalize()
    tm = T.Team(P, 2 * nb + 8192, device=False)
    toff = T._align(nb)
    if pinned:
        assert L.osgpu_host_register(ctypes.c_void_p(tm.base), P * tm.H) == 0
    try:
        for op, lo, hi in (("min", -1e3, 1e3), ("max", -1e3, 1e3), ("prod", 0.9, 1.1)):
            g = torch.Generator(device="cuda:0").manual_seed(55)
            srcs = [torch.empty(n, dtype=torch.float32, device="cuda:0").uniform_(
                lo, hi, generator=g) for _ in range(P)]
            for pe in range(P):
                a = tm.hoff + pe * tm.H
                torch.from_numpy(tm.hbuf[a:a + nb].view(np.float32)).copy_(srcs[pe])
            tm.run("float", op, toff, 0, n)
            assert set(tm.last_paths.values()) == {"staged"}, tm.last_paths
            gots = [torch.from_numpy(tm.hbuf[tm.hoff + q * tm.H + toff:][:nb].view(np.float32))
                    .to("cuda:0") for q in range(P)]
            _oracle_sample(torch, "float", op, srcs, gots, n, seed=78)
            del gots
            for q in range(P):
                a = tm.hoff + q * tm.H + toff
                got = torch.from_numpy(tm.hbuf[a:a + nb].view(np.int32)).to("cuda:0")
                want = _fold(torch, op, srcs, q)
                assert torch.equal(got, want.view(torch.int32)), (op, q)
                del got, want
            del srcs
    finally:
        if pinned:
            L.osgpu_host_unregister(ctypes.c_void_p(tm.base))
        L.osgpu_finalize()
        del tm
        torch.cuda.empty_cache()
