"""coll_cases.py -- TEST INFRASTRUCTURE: deterministic collective cases shared
by the multi-process worker (tests/support/mp_worker.py) and the checker
(tests/test_multiproc.py).  Every rank derives its source bytes from the
case alone, so the parent can rebuild every PE's input for the oracle."""
import numpy as np

KINDS = ["broadcast", "collect", "fcollect", "alltoall"]
SENTINEL = 0xA5


def cases(world):
    """(kind, bits, nelems_of_rank(list), root)."""
    out = []
    for kind in KINDS:
        for bits in (32, 64):
            if kind == "collect":
                counts = [1001 + 7 * r if r != 1 else 0 for r in range(world)]
            else:
                counts = [1001] * world
            out.append((kind, bits, counts, world - 1))
    return out


def src_bytes(kind, bits, counts, rank, world):
    esz = bits // 8
    n = counts[rank]
    return n * esz * (world if kind == "alltoall" else 1)


def source(kind, bits, counts, rank, world):
    seed = 1000 * bits + 17 * KINDS.index(kind) + rank
    return np.random.default_rng(seed).integers(0, 256, src_bytes(kind, bits, counts, rank, world),
                                                dtype=np.uint8)


def target_bytes(kind, bits, counts, world):
    esz = bits // 8
    if kind == "collect":
        return sum(counts) * esz + 64
    if kind == "broadcast":
        return counts[0] * esz + 64
    return world * counts[0] * esz + 64


def key(kind, bits, path):
    return f"coll/{kind}/{bits}/{path}"


def expected(kind, bits, counts, root, world):
    """every rank's target (target_bytes long, sentinel-initialised) after
    the collective, from oracle_coll."""
    import oracle_coll as OC
    esz = bits // 8
    src = {r: source(kind, bits, counts, r, world) for r in range(world)}
    tb = target_bytes(kind, bits, counts, world)
    tgt = {r: np.full(tb, SENTINEL, np.uint8) for r in range(world)}
    if kind == "broadcast":
        return OC.broadcast(src, tgt, counts[0] * esz, root, 0, 0, world)
    if kind == "collect":
        return OC.collect(src, tgt, {r: counts[r] * esz for r in range(world)}, 0, 0, world)
    if kind == "fcollect":
        return OC.fcollect(src, tgt, counts[0] * esz, 0, 0, world)
    return OC.alltoall(src, tgt, counts[0] * esz, 0, 0, world)
