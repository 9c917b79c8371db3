"""GPU parity of the data-movement collectives (broadcast / collect /
fcollect / alltoall, 32- and 64-bit) against the CPU restatement
(oracle/oracle_coll.py), called through the C ABI by threads-as-PEs.

Device-resident: every PE's heap is a registered slice of one allocation on
cuda:0 -> COPY path (pull copy kernel over peer pointers).  Host-resident:
host symmetric heaps -> STAGED path (H2D -> copy kernel over the members'
device staging -> D2H), also with tiny staging slots to force many chunks,
and the GETMEM path.  Every byte of every member's target region is compared,
including the margins the collective must not write; pSync must come back at
SHMEM_SYNC_VALUE (checked by Team)."""
import os

import numpy as np
import pytest

import osgpu
import oracle_coll as OC
from support import team as T

pytestmark = pytest.mark.gpu

SRC_OFF = 0
MARGIN = 256
MODES = ["device", "host", "staged"]  # host = auto (GETMEM when PEs share a GPU)


def host_path(mode):
    """osgpu_set_host_path for the duration of a case (staged / getmem;
    anything else: the automatic path)."""
    return osgpu.host_path(mode if mode in ("staged", "getmem") else None)


def _layout(P, max_src_bytes):
    """source at 0, target after it (+ margins), all 256-B aligned."""
    tgt_off = T._align(max_src_bytes * P + MARGIN) + MARGIN
    heap = tgt_off + T._align(max_src_bytes * P * P + 2 * MARGIN)
    return tgt_off, heap


def _fill_inputs(tm, npes, src_bytes, tgt_off, tgt_bytes, seed):
    src, tgt = {}, {}
    for pe in range(npes):
        rng = np.random.default_rng(seed * 131 + pe)
        src[pe] = rng.integers(0, 256, src_bytes, dtype=np.uint8)
        tgt[pe] = np.full(tgt_bytes + 2 * MARGIN, 0xA5, np.uint8)
        tm.write(pe, SRC_OFF, src[pe])
        tm.write(pe, tgt_off - MARGIN, tgt[pe])
    return src, tgt


def _expected(kind, src, tgt, nb, nbytes_of, root, PE_start, log, size):
    # targets in the oracle start at the margin; shift sources/targets to match
    inner = {pe: t[MARGIN:] for pe, t in tgt.items()}
    if kind == "broadcast":
        out = OC.broadcast(src, inner, nb, root, PE_start, log, size)
    elif kind == "fcollect":
        out = OC.fcollect(src, inner, nb, PE_start, log, size)
    elif kind == "alltoall":
        out = OC.alltoall(src, inner, nb, PE_start, log, size)
    else:
        out = OC.collect(src, inner, nbytes_of, PE_start, log, size)
    full = {}
    for pe, t in tgt.items():
        f = t.copy()
        if pe in out:
            f[MARGIN:] = out[pe]
        full[pe] = f
    return full


def _check(tm, npes, tgt_off, expected):
    for pe in range(npes):
        got = tm.read(pe, tgt_off - MARGIN, expected[pe].size)
        bad = np.nonzero(got != expected[pe])[0]
        assert bad.size == 0, (pe, bad[:8], got[bad[:8]], expected[pe][bad[:8]])


SETS = [  # (npes, PE_start, logPE_stride, PE_size)
    (1, 0, 0, 1), (2, 0, 0, 2), (3, 0, 0, 3), (4, 0, 0, 4), (8, 0, 0, 8),
    (8, 1, 1, 3), (6, 2, 0, 3),
]


def _counts(kind, nelems, pes, seed):
    if kind != "collect":
        return nelems
    rng = np.random.default_rng(seed)
    c = {pe: int(rng.integers(0, nelems + 1)) for pe in pes}
    c[pes[0]] = nelems                       # at least one full contribution
    if len(pes) > 2:
        c[pes[1]] = 0                        # and an empty one
    return c


def _run_case(device, kind, bits, setdef, nelems, root=0, seed=1, same_buffer=False):
    npes, PE_start, log, size = setdef
    esz = bits // 8
    pes = OC.active_set(PE_start, log, size)
    per_src = nelems * esz * (size if kind == "alltoall" else 1)
    tgt_off, heap = _layout(size, max(per_src, 16))
    tm = T.Team(npes, heap, device=device)
    tgt_bytes = max(per_src, 16) * size
    src, tgt = _fill_inputs(tm, npes, per_src, tgt_off, tgt_bytes, seed)
    counts = _counts(kind, nelems, pes, seed)
    nbytes_of = {pe: counts[pe] * esz for pe in pes} if kind == "collect" else None
    s_off = SRC_OFF
    if same_buffer:
        # source and target are the SAME symmetric object: peers must read
        # its pre-call bytes (the reference's puts race there; this
        # implementation pulls into scratch and copies after the barrier)
        for pe in range(npes):
            r = np.random.default_rng(seed * 7 + pe).integers(0, 256, tgt_bytes, dtype=np.uint8)
            tm.write(pe, tgt_off, r)
            tgt[pe][MARGIN:MARGIN + tgt_bytes] = r
            src[pe] = r[:per_src].copy()
        s_off = tgt_off
    exp = _expected(kind, src, tgt, nelems * esz, nbytes_of, root, PE_start, log, size)
    tm.run_coll(kind, bits, tgt_off, s_off, counts, PE_root=root, PE_start=PE_start,
                logPE_stride=log, PE_size=size)
    _check(tm, npes, tgt_off, exp)
    return tm


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("kind", ["broadcast", "collect", "fcollect", "alltoall"])
@pytest.mark.parametrize("bits", [32, 64])
@pytest.mark.parametrize("setdef", SETS, ids=lambda s: "P%d_s%d_l%d_n%d" % s)
def test_collective_matches_oracle(mode, kind, bits, setdef):
    with host_path(mode):
        for nelems in (1, 7, 1000, 4099):
            root = (nelems % setdef[3]) if kind == "broadcast" else 0
            _run_case(mode != "device", kind, bits, setdef, nelems, root=root,
                      seed=nelems + bits)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("kind", ["broadcast", "collect", "fcollect", "alltoall"])
def test_collective_source_is_target(mode, kind):
    """target == source (same symmetric object): peers must read pre-call
    bytes (scratch / temporary target)."""
    with host_path(mode):
        _run_case(mode != "device", kind, 64, (3, 0, 0, 3), 1001, root=1, seed=5,
                  same_buffer=True)


@pytest.mark.parametrize("kind", ["broadcast", "collect", "fcollect", "alltoall"])
def test_host_staged_many_chunks(kind):
    """16 KiB of staging per PE: thousands of chunks, ragged last chunk."""
    L = osgpu.load()
    L.osgpu_finalize()
    L.osgpu_set_stage_bytes(4096)
    try:
        with host_path("staged"):
            _run_case(False, kind, 32, (4, 0, 0, 4), 30011, root=3, seed=9)
            _run_case(False, kind, 64, (8, 1, 1, 3), 9001, root=2, seed=10)
    finally:
        L.osgpu_finalize()
        L.osgpu_set_stage_bytes(-1)


@pytest.mark.parametrize("kind", ["broadcast", "collect", "fcollect", "alltoall"])
def test_host_getmem_path(kind):
    with host_path("getmem"):
        _run_case(False, kind, 64, (3, 0, 0, 3), 3001, root=2, seed=11)


def test_collect32_dword_phases_and_byte_path():
    """collect32 with odd counts puts blocks at 4-byte (not 16-byte) phases:
    the vector path must handle any dword phase; an odd source address
    takes the byte kernel."""
    for seed in range(3):
        _run_case(True, "collect", 32, (4, 0, 0, 4), 777 + seed, seed=20 + seed)
    npes, nelems = 3, 1001
    tgt_off, heap = _layout(3, nelems * 4 + 16)
    tm = T.Team(npes, heap, device=True)
    src, tgt = _fill_inputs(tm, npes, nelems * 4 + 16, tgt_off, (nelems * 4 + 16) * 3, 30)
    shifted = {pe: s[1:] for pe, s in src.items()}
    exp = _expected("fcollect", shifted, tgt, nelems * 4, None, 0, 0, 0, 3)
    tm.run_coll("fcollect", 32, tgt_off, SRC_OFF + 1, nelems)
    _check(tm, npes, tgt_off, exp)


def test_large_fcollect_and_broadcast_properties():
    """BASELINE-scale sizes: fcollect64 of 16 Mi elements from 4 PEs (512 MiB
    target per PE), broadcast64 of 64 Mi elements; checked on the GPU block
    by block (torch.equal), not through the host."""
    import torch
    P, n = 4, 16 << 20
    nb = n * 8
    tgt_off = nb
    tm = T.Team(P, nb + P * nb, device=True)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for pe in range(P):
        lo = pe * tm.H
        tm.buf[lo:lo + nb].copy_(torch.randint(0, 256, (nb,), dtype=torch.uint8,
                                               device="cuda:0", generator=g))
    torch.cuda.synchronize()
    tm.run_coll("fcollect", 64, tgt_off, 0, n)
    torch.cuda.synchronize()
    for me in range(P):
        for i in range(P):
            blk = tm.buf[me * tm.H + tgt_off + i * nb:][:nb]
            assert torch.equal(blk, tm.buf[i * tm.H:][:nb]), (me, i)
    del tm
    P, n = 3, 64 << 20
    nb = n * 8
    tm = T.Team(P, 2 * nb, device=True)
    for pe in range(P):
        tm.buf[pe * tm.H:][:nb].fill_(pe + 1)
        tm.buf[pe * tm.H + nb:][:nb].fill_(0xEE)
    torch.cuda.synchronize()
    tm.run_coll("broadcast", 64, nb, 0, n, PE_root=1)
    torch.cuda.synchronize()
    for pe in range(P):
        t = tm.buf[pe * tm.H + nb:][:nb]
        want = 0xEE if pe == 1 else 2
        assert bool((t == want).all()), pe


def _random_case(k):
    """A seeded draw over every dimension at once: kind, width, placement
    (device / host auto / host staged), an active set of an npes job at any
    start and stride, nelems with the vector and chunk edges over-weighted,
    any root, collect's per-PE counts."""
    rng = np.random.default_rng(0xC011 + k)
    kind = ["broadcast", "collect", "fcollect", "alltoall"][rng.integers(4)]
    bits = int(rng.choice([32, 64]))
    mode = MODES[rng.integers(len(MODES))]
    log = int(rng.choice([0, 0, 1, 2]))
    step = 1 << log
    size = int(rng.integers(1, 8 // step + 1))
    start = int(rng.integers(0, 8 - (size - 1) * step))
    npes = start + (size - 1) * step + 1
    r = rng.random()
    nelems = int(rng.choice([0, 1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257])) if r < 0.4 \
        else int(rng.integers(1, 3000)) if r < 0.85 else int(rng.integers(3000, 40000))
    root = int(rng.integers(size))
    return mode, kind, bits, (npes, start, log, size), nelems, root, int(rng.integers(1 << 30))


@pytest.mark.parametrize("block", range(0, 120, 30))
def test_random_collectives(block):
    for k in range(block, block + 30):
        mode, kind, bits, setdef, nelems, root, seed = _random_case(k)
        with host_path(mode):
            _run_case(mode != "device", kind, bits, setdef, nelems, root=root, seed=seed)


@pytest.mark.parametrize("seed", range(6))
def test_copy_kernel_segment_layouts(seed):
    """osgpu_copy directly: up to 9 segments (a second launch past 8) of
    mixed sizes -- empty, below one vector, unaligned heads and tails,
    one tile, many tiles, very unequal -- at every 4-byte source phase and
    byte phases (the byte kernel).  The segments' tiles are dealt
    round-robin for as many rounds as the smallest segment has, then
    segment by segment (copy.hip); every destination byte must equal its
    source and nothing outside the ranges may change."""
    import torch
    rng = np.random.default_rng(seed)
    nseg = int(rng.integers(1, 10))
    tile = 256 * 4 * 16
    sizes = [int(rng.choice([0, 3, 15, 16, 17, 1000, tile - 1, tile, tile + 5, 3 * tile + 7,
                             int(rng.integers(1, 40 * tile))])) for _ in range(nseg)]
    pad = 64
    total = sum(s + 2 * pad for s in sizes) + 64
    src = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
    dst = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    srcs, dsts, off, want = [], [], 16, dst.clone()
    for i, s in enumerate(sizes):
        so = off + int(rng.choice([0, 4, 8, 12] if i % 3 else [1, 2, 3]))   # byte phases too
        do = off + int(rng.choice([0, 4, 8, 12]))
        srcs.append(src.data_ptr() + so)
        dsts.append(dst.data_ptr() + do)
        want[do:do + s] = src[so:so + s]
        off += s + 2 * pad
    torch.cuda.synchronize()
    osgpu.copy(dsts, srcs, sizes)
    torch.cuda.synchronize()
    assert torch.equal(dst, want), (sizes, int((dst != want).sum()))
