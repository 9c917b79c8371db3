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


# ---------------------------------------------------------------------------
# cases for the fused (one-launch) collectives across processes: every rank
# rebuilds its inputs from the case alone; the parent rebuilds every rank's
# expected target region (margins included) from oracle_coll.

MARGIN = 256
FUSED_SETS = [(2, 0, 0, 2), (3, 0, 0, 3), (4, 0, 0, 4), (4, 1, 0, 3), (4, 0, 1, 2),
              (8, 0, 0, 8), (8, 1, 1, 3), (8, 2, 0, 6)]


def _align(x, a=256):
    return (x + a - 1) // a * a


def fused_cases():
    out = []
    for kind in KINDS:
        for bits in (32, 64):
            for setdef in FUSED_SETS:
                for nelems in ((0, 1, 63, 1001, 4099) if kind == "collect" else
                               (1, 63, 1001, 4099)):
                    root = nelems % setdef[3] if kind == "broadcast" else 0
                    out.append({"kind": kind, "bits": bits, "set": setdef, "nelems": nelems,
                                "root": root, "same": False, "seed": nelems + bits})
        out.append({"kind": kind, "bits": 64, "set": (3, 0, 0, 3), "nelems": 1001, "root": 1,
                    "same": True, "seed": 5})
    return out


def fused_layout(c):
    """(per_src, tgt_off, tgt_bytes, src_off): source at 0 (or the target
    itself when `same`), target after it; all 256-B aligned."""
    npes, start, log, size = c["set"]
    esz = c["bits"] // 8
    per_src = c["nelems"] * esz * (size if c["kind"] == "alltoall" else 1)
    m = max(per_src, 16)
    tgt_off = _align(m * size + MARGIN) + MARGIN
    return per_src, tgt_off, m * size, (tgt_off if c["same"] else 0)


def fused_counts(c):
    """{pe: nelems} of every member (collect contributions differ)."""
    import oracle_coll as OC
    npes, start, log, size = c["set"]
    pes = OC.active_set(start, log, size)
    if c["kind"] != "collect":
        return {pe: c["nelems"] for pe in pes}
    rng = np.random.default_rng(c["seed"])
    cnt = {pe: int(rng.integers(0, c["nelems"] + 1)) for pe in pes}
    cnt[pes[0]] = c["nelems"]
    if len(pes) > 2:
        cnt[pes[1]] = 0
    return cnt


def fused_inputs(c, pe):
    """(source bytes, initial target region incl. margins) of PE pe."""
    per_src, tgt_off, tgt_bytes, _ = fused_layout(c)
    tgt = np.full(tgt_bytes + 2 * MARGIN, SENTINEL, np.uint8)
    if c["same"]:
        r = np.random.default_rng(c["seed"] * 7 + pe).integers(0, 256, tgt_bytes, dtype=np.uint8)
        tgt[MARGIN:MARGIN + tgt_bytes] = r
        return r[:per_src].copy(), tgt
    src = np.random.default_rng(c["seed"] * 131 + pe).integers(0, 256, per_src, dtype=np.uint8)
    return src, tgt


def fused_expected(c):
    """every PE's target region (margins included) after the call."""
    import oracle_coll as OC
    npes, start, log, size = c["set"]
    esz = c["bits"] // 8
    src, tgt = {}, {}
    for pe in range(npes):
        src[pe], tgt[pe] = fused_inputs(c, pe)
    inner = {pe: t[MARGIN:] for pe, t in tgt.items()}
    nb = c["nelems"] * esz
    k = c["kind"]
    if k == "broadcast":
        out = OC.broadcast(src, inner, nb, c["root"], start, log, size)
    elif k == "fcollect":
        out = OC.fcollect(src, inner, nb, start, log, size)
    elif k == "alltoall":
        out = OC.alltoall(src, inner, nb, start, log, size)
    else:
        cnt = fused_counts(c)
        out = OC.collect(src, inner, {pe: cnt[pe] * esz for pe in cnt}, start, log, size)
    full = {}
    for pe, t in tgt.items():
        f = t.copy()
        if pe in out:
            f[MARGIN:] = out[pe]
        full[pe] = f
    return full
