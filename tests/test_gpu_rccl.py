"""RCCL path through the real entry points, on one GPU.

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the
only communicator a one-GPU box can build is a world of one PE.  A 1-rank
ncclAllReduce is a copy, so these runs pin the plumbing rather than the
arithmetic: communicator setup from osgpu_rccl_unique_id, the (type, op)
mapping (complex sums as 2N reals -- a wrong count would leave half the
target untouched), the overlap scratch, in-place calls, and the collectives'
ncclBroadcast / ncclAllGather.  Multi-rank arithmetic (tolerance per
DESIGN.md 3) is measured by bench.py's N>1 line on the driver's node.
"""
import ctypes

import numpy as np
import pytest

import osgpu

pytestmark = pytest.mark.gpu

RCCL_PAIRS = [(t, op) for t in ("int", "long", "longlong", "float", "double")
              for op in ("sum", "prod", "max", "min")] + [("complexf", "sum"), ("complexd", "sum")]
SIZE = {"int": 4, "long": 8, "longlong": 8, "float": 4, "double": 8, "complexf": 8,
        "complexd": 16}


@pytest.fixture(scope="module")
def rccl_team():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from support import team as T
    tm = T.Team(1, 4 << 20, device=True)
    L = tm.lib
    uid = (ctypes.c_char * 128)()
    assert L.osgpu_rccl_unique_id(uid) == 0
    rc = L.osgpu_rccl_init(1, 0, uid)
    assert rc == 0, L.osgpu_last_error()
    L.osgpu_set_path(osgpu.PATH_RCCL)
    yield tm
    L.osgpu_set_path(osgpu.PATH_AUTO)
    assert L.osgpu_rccl_finalize() == 0


def _rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("t,op", RCCL_PAIRS)
@pytest.mark.parametrize("n", [1, 1000, 65537])
def test_rccl_one_rank_is_identity(rccl_team, t, op, n):
    tm = rccl_team
    tm.activate()
    nb = n * SIZE[t]
    src = _rand_bytes(nb, n)
    if t in ("float", "double", "complexf", "complexd"):  # finite values (NaN payloads are RCCL's)
        dt = {"float": np.float32, "complexf": np.float32}.get(t, np.float64)
        src = np.random.default_rng(n).uniform(-4, 4, nb // np.dtype(dt).itemsize).astype(dt)
        src = src.view(np.uint8)
    toff = 2 << 20
    tm.write(0, 0, src)
    tm.fill(0, toff, nb, 0xA5)
    tm.run(t, op, toff, 0, n)
    # FP min/max never go to RCCL, even forced: RCCL does not resolve NaN and
    # signed-zero ties like src/shmemu/miscops.c:80-90, so the exact kernels
    # run (here the pull form over the one registered heap)
    fp_minmax = t in ("float", "double") and op in ("max", "min")
    assert tm.last_paths[0] == ("pull" if fp_minmax else "rccl")
    np.testing.assert_array_equal(tm.read(0, toff, nb), src)
    np.testing.assert_array_equal(tm.read(0, 0, nb), src)  # source untouched


@pytest.mark.parametrize("shift", [0, 8, -8])
def test_rccl_in_place_and_overlap(rccl_team, shift):
    """target == source, and targets overlapping the source by all but 8 B
    (the scratch + copy of src/reductions.c:114-119)."""
    tm = rccl_team
    tm.activate()
    n = 4099
    nb = n * 8
    base = 64 << 10
    src = np.random.default_rng(3).uniform(1, 2, n)
    tm.write(0, base, src)
    tm.run("double", "sum", base + shift, base, n)
    assert tm.last_paths[0] == "rccl"
    np.testing.assert_array_equal(tm.read(0, base + shift, nb).view(np.float64), src)


def test_rccl_collectives(rccl_team):
    """fcollect64 -> ncclAllGather; broadcast -> ncclBroadcast (the root's
    own target stays untouched, as in the reference)."""
    tm = rccl_team
    tm.activate()
    n = 3001
    src = _rand_bytes(n * 8, 7)
    toff = 256 << 10
    tm.write(0, 0, src)
    tm.fill(0, toff, n * 8, 0x5A)
    tm.run_coll("fcollect", 64, toff, 0, n)
    assert tm.last_coll_paths[0] == "rccl"
    np.testing.assert_array_equal(tm.read(0, toff, n * 8), src)
    tm.fill(0, toff, n * 8, 0x5A)
    tm.run_coll("broadcast", 64, toff, 0, n, PE_root=0)
    assert tm.last_coll_paths[0] == "rccl"
    assert (tm.read(0, toff, n * 8) == 0x5A).all()


@pytest.mark.parametrize("t,op,dt", [("int", "sum", "int32"), ("long", "prod", "int64"),
                                     ("int", "min", "int32"), ("long", "max", "int64")])
def test_auto_path_sends_integer_arrays_outside_the_heaps_to_rccl(rccl_team, t, op, dt):
    """OSGPU_PATH_AUTO with a heap registered: arrays OUTSIDE every heap of
    an integer (type, op) go to ncclAllReduce (order-independent, so
    bit-exact), the dispatch bench.py's N>1 line checks against the oracle
    across GPUs (`rccl_integer_auto`).  Here (1 rank) the result is the
    source, wrap-around values included."""
    import torch
    tm = rccl_team
    tm.activate()
    L = tm.lib
    L.osgpu_set_path(osgpu.PATH_AUTO)
    try:
        n = 100_003
        tdt = getattr(torch, dt)
        info = torch.iinfo(tdt)
        src = torch.randint(info.min, info.max, (n,), dtype=tdt, device="cuda",
                            generator=torch.Generator(device="cuda").manual_seed(9))
        dst = torch.zeros_like(src)
        torch.cuda.synchronize()
        wrk = (ctypes.c_long * 64)()
        tm.pet.pet_set_me(0)
        osgpu.to_all(t, op)(dst.data_ptr(), src.data_ptr(), n, 0, 0, 1, wrk, tm.psync_ptr(0))
        assert osgpu.last_path() == "rccl"
        assert torch.equal(dst, src)
    finally:
        L.osgpu_set_path(osgpu.PATH_RCCL)
