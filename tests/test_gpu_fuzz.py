"""Seeded random sweep of the 44 entry points on an MI355X against the oracle.

The golden set (test_gpu_parity.py) walks a fixed grid of (type, op, P, n,
tag); this draws the dimensions together at random, one case at a time, so
combinations the grid does not pair are covered too: any (type, op), an
active set of 1..8 PEs of an 8-PE job at stride 1, 2 or 4 and any start,
nreduce from 0 to ~70 K with the chunk and vector edges over-weighted, source
and target at independent element offsets (every 16-byte phase the type
allows), in-place calls, device heaps (team / pull path) and host heaps
(staged path), input distributions with NaN / Inf / signed zeros / subnormals.

Per case: every member's target bit-exact with the oracle's fold in that
member's order (src/reductions.c:79-111), non-members' targets and every
source (unless in place) untouched, pSync back at 0 (Team._on_members).
Seeds are fixed: a failure names its case and reproduces.
"""
import os

import numpy as np
import pytest

import oracle as O
import osgpu

HEAP = 8 << 20
NCASE = int(os.environ.get("OSGPU_FUZZ_CASES", "800"))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


_TEAMS = {}


def team(device):
    from support import team as T
    if device not in _TEAMS:
        _TEAMS[device] = T.Team(8, HEAP, device=device)
    tm = _TEAMS[device]
    tm.activate()
    return tm


def esize(t):
    return 16 if t == "longdouble" else O.NP_DTYPE[t]().itemsize


def value_view(t, raw):
    return O.from_value_bytes(t, raw if t != "longdouble" else
                              raw.reshape(-1, 16)[:, :10].reshape(-1))


def draw(rng, k):
    t = O.TYPES[rng.integers(len(O.TYPES))]
    ops = [op for op in O.OPS if O.has_op(t, op)]
    op = ops[rng.integers(len(ops))]
    stride = int(rng.choice([0, 0, 1, 2]))
    step = 1 << stride
    size = int(rng.integers(1, 8 // step + 1))
    start = int(rng.integers(0, 8 - (size - 1) * step))
    edges = [0, 1, 2, 15, 63, 64, 65, 127, 128, 255, 256, 257, 1023, 4095, 4097]
    r = rng.random()
    n = int(rng.choice(edges)) if r < 0.35 else int(rng.integers(1, 4096)) if r < 0.75 \
        else int(rng.integers(4096, 70000))
    s = esize(t)
    in_place = bool(rng.random() < 0.15)
    soff = 4096 + s * int(rng.integers(0, 16 // s if s < 16 else 4))
    nbytes = n * s
    toff = soff if in_place else \
        (soff + nbytes + 4095) // 4096 * 4096 + 4096 + s * int(rng.integers(0, 16 // s if s < 16 else 4))
    dists = ["mixed", "edge", "wide"] if t not in O.INT_TYPES else ["bits", "mixed", "edge"]
    if op == "prod" and t not in O.INT_TYPES:
        dists = ["prod", "edge"]
    dist = dists[rng.integers(len(dists))]
    device = bool(rng.random() < 0.75)
    path = int(rng.choice([osgpu.PATH_AUTO, osgpu.PATH_AUTO, osgpu.PATH_PULL]))
    return dict(k=k, t=t, op=op, start=start, stride=stride, size=size, n=n, soff=soff,
                toff=toff, in_place=in_place, dist=dist, device=device, path=path,
                seed=int(rng.integers(1 << 40)))


CASES = [draw(np.random.default_rng(0xF0220 + k), k) for k in range(NCASE)]


def run_case(c):
    tm = team(c["device"])
    t, n, s = c["t"], c["n"], esize(c["t"])
    nbytes = n * s
    assert c["toff"] + max(nbytes, 16) <= HEAP and c["soff"] + nbytes <= HEAP
    src = O.team_inputs(t, 8, n, c["seed"], c["dist"])
    act = O.active_set(c["start"], c["stride"], c["size"])
    for pe in range(8):
        tm.write(pe, c["soff"], src[pe])
        if not c["in_place"]:
            tm.fill(pe, c["toff"], max(nbytes, 16), 0x5A)
    before = {pe: tm.read(pe, c["soff"], nbytes).copy() for pe in range(8)}
    L = osgpu.load()
    L.osgpu_set_path(c["path"])
    try:
        tm.run(t, c["op"], c["toff"], c["soff"], n, c["start"], c["stride"], c["size"])
    finally:
        L.osgpu_set_path(osgpu.PATH_AUTO)
    want = O.to_all(t, c["op"], src, c["start"], c["stride"], c["size"])
    for pe in range(8):
        if pe in act:
            got = value_view(t, tm.read(pe, c["toff"], nbytes))
            assert np.array_equal(O.value_bytes(got), O.value_bytes(want[pe])), \
                f"case {c}: PE {pe} differs from the oracle"
            if not c["in_place"]:
                assert np.array_equal(tm.read(pe, c["soff"], nbytes), before[pe]), \
                    f"case {c}: PE {pe}'s source was modified"
        else:
            assert np.array_equal(tm.read(pe, c["soff"], nbytes), before[pe]), \
                f"case {c}: non-member PE {pe}'s source was modified"
            if not c["in_place"]:
                assert (tm.read(pe, c["toff"], max(nbytes, 16)) == 0x5A).all(), \
                    f"case {c}: non-member PE {pe}'s target was written"


@pytest.mark.gpu
@pytest.mark.parametrize("block", range(0, NCASE, 100))
def test_random_calls_match_oracle(torch_cuda, block):
    for c in CASES[block:block + 100]:
        run_case(c)


def test_draw_covers_the_space():
    # the seeded draw reaches every type, both heaps, in-place, subsets with
    # every stride, single-PE sets and empty calls (checked without a GPU)
    ks = lambda f: {f(c) for c in CASES}  # noqa: E731
    assert ks(lambda c: c["t"]) == set(O.TYPES)
    assert ks(lambda c: c["device"]) == {True, False}
    assert ks(lambda c: c["in_place"]) == {True, False}
    assert ks(lambda c: c["stride"]) == {0, 1, 2}
    assert 1 in ks(lambda c: c["size"]) and 0 in ks(lambda c: c["n"])
