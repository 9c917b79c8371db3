"""Data-movement collectives -- CPU-side checks:
the oracle restatement's own invariants, the exported C ABI, and the
zero-byte calls that only synchronise (no GPU needed).  GPU parity lives in
tests/test_gpu_collectives.py."""
import os
import subprocess

import numpy as np
import pytest

import osgpu
import oracle_coll as OC
from support import team as T


def _rand(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def test_oracle_collect_is_concatenation_in_active_set_order():
    pes = OC.active_set(1, 1, 3)                      # {1, 3, 5}
    src = {pe: _rand(64, pe) for pe in range(8)}
    tgt = {pe: np.full(200, 7, np.uint8) for pe in range(8)}
    nb = {1: 12, 3: 0, 5: 40}
    out = OC.collect(src, tgt, nb, 1, 1, 3)
    cat = np.concatenate([src[1][:12], src[5][:40]])
    for pe in pes:
        assert (out[pe][:52] == cat).all() and (out[pe][52:] == 7).all()
    assert set(out) == set(pes)


def test_oracle_fcollect_blocks_and_alltoall_transpose():
    src = {pe: _rand(4 * 16, 10 + pe) for pe in range(4)}
    tgt = {pe: np.zeros(4 * 16, np.uint8) for pe in range(4)}
    f = OC.fcollect(src, tgt, 16, 0, 0, 4)
    for pe in range(4):
        for i in range(4):
            assert (f[pe][16 * i:16 * (i + 1)] == src[i][:16]).all()
    a = OC.alltoall(src, tgt, 16, 0, 0, 4)
    a_rank = OC.alltoall(src, tgt, 16, 0, 0, 4, block_index="rank")
    for me in range(4):
        assert (a[me] == a_rank[me]).all()     # PE_start 0, stride 1: identical
        for i in range(4):
            assert (a[me][16 * i:16 * (i + 1)] == src[i][16 * me:16 * (me + 1)]).all()


def test_oracle_broadcast_leaves_root_target():
    src = {pe: _rand(32, pe) for pe in range(4)}
    tgt = {pe: np.full(32, 9, np.uint8) for pe in range(4)}
    out = OC.broadcast(src, tgt, 20, 2, 0, 0, 4)
    for pe in range(4):
        if pe == 2:
            assert (out[pe] == 9).all()
        else:
            assert (out[pe][:20] == src[2][:20]).all() and (out[pe][20:] == 9).all()


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(osgpu.LIB_PATH):
        osgpu.build()
    return osgpu.load()


def test_collective_symbols_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", osgpu.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    kinds = {p[2]: p[1] for p in (l.split() for l in out.splitlines()) if len(p) == 3}
    assert len(osgpu.COLL_ENTRY_POINTS) == 8
    for e in osgpu.COLL_ENTRY_POINTS:
        assert kinds.get("p" + e) == "T", e
        assert kinds.get(e) in ("W", "V"), e


@pytest.mark.parametrize("kind", ["broadcast", "fcollect", "alltoall", "collect"])
def test_zero_byte_collectives_only_synchronise(lib, kind):
    """nelems = 0 everywhere moves nothing, touches no GPU, leaves pSync at
    SHMEM_SYNC_VALUE and still synchronises the active set."""
    tm = T.Team(3, 4096, device=False)
    before = [tm.pet.pet_barrier_calls(pe) for pe in range(3)]
    tm.run_coll(kind, 64, 0, 1024, 0, PE_root=1)
    after = [tm.pet.pet_barrier_calls(pe) for pe in range(3)]
    assert all(a > b for a, b in zip(after, before))
    assert len({a - b for a, b in zip(after, before)}) == 1  # every PE the same


def test_broadcast_rejects_root_outside_set(lib):
    code = (
        "import sys; sys.path[:0]=[%r, %r]\n"
        "from support import team as T\n"
        "tm = T.Team(2, 4096, device=False)\n"
        "tm.run_coll('broadcast', 32, 0, 1024, 4, PE_root=2)\n"
    ) % (os.path.join(os.path.dirname(__file__)),
         os.path.join(os.path.dirname(os.path.dirname(__file__)), "test-resilient-osss-ucx_amd"))
    r = subprocess.run(["python3", "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "PE_root 2 outside" in r.stderr
