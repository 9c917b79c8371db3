"""oracle_coll.py -- CPU restatement of the reference's data-movement
collectives.  TEST INFRASTRUCTURE ONLY (same rule as oracle.py: only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it).

Byte work, so numpy on uint8 arrays.  Every PE is a dict entry
{pe: np.ndarray(uint8)} holding that PE's symmetric object; the functions
return every active PE's target after the collective, starting from the
target it had before (bytes a collective does not write keep their value).

Parity status: the reference's collectives (src/shmemc/broadcast.c,
collect.c, fcollect.c, src/alltoall.c) include src/shmemc/state.h ->
<ucp/api/ucp.h> and cannot be built here, and the reference holds no tests or
fixtures for them (Makefile.am:5), so this restatement is **parity
unpinned**: it is checked only against the source text cited below and the
OpenSHMEM 1.4 semantics those lines implement.
"""
from __future__ import annotations

import numpy as np


def active_set(PE_start: int, logPE_stride: int, PE_size: int):
    step = 1 << logPE_stride
    return [PE_start + i * step for i in range(PE_size)]


def broadcast(sources: dict, targets: dict, nbytes: int, PE_root: int,
              PE_start: int, logPE_stride: int, PE_size: int) -> dict:
    """src/shmemc/broadcast.c:29-42 (linear) / :48-250 (tree, binomial):
    PE_root is an index into the active set (:34 root = PE_root * stride +
    PE_start); every other member's target receives the root's first nbytes
    (shmemc_get(target, source, nbytes, root), :40); the root's own target is
    not written (:39 `if (me != root)`; the tree variants never put to the
    tree root, :100-116)."""
    pes = active_set(PE_start, logPE_stride, PE_size)
    root = pes[PE_root]
    out = {pe: targets[pe].copy() for pe in pes}
    for pe in pes:
        if pe != root:
            out[pe][:nbytes] = sources[root][:nbytes]
    return out


def collect(sources: dict, targets: dict, nbytes_of: dict, PE_start: int,
            logPE_stride: int, PE_size: int) -> dict:
    """src/shmemc/collect.c:24-69: the wavefront gives member i the offset
    sum(nbytes of members 0..i-1) (:32-50, pSync carries it left to right),
    then member i puts its nbytes_of[i] source bytes at that offset of every
    member's target (:52-64): every target = concatenation in active-set
    order."""
    pes = active_set(PE_start, logPE_stride, PE_size)
    cat = np.concatenate([sources[pe][:nbytes_of[pe]] for pe in pes]) if pes else \
        np.zeros(0, np.uint8)
    out = {pe: targets[pe].copy() for pe in pes}
    for pe in pes:
        out[pe][:cat.size] = cat
    return out


def fcollect(sources: dict, targets: dict, nbytes: int, PE_start: int,
             logPE_stride: int, PE_size: int) -> dict:
    """src/shmemc/fcollect.c:19-40: member vpe = (me - PE_start) >>
    logPE_stride (:27) puts its nbytes at tidx = nbytes * vpe (:28) of every
    member's target (:32-38)."""
    pes = active_set(PE_start, logPE_stride, PE_size)
    return collect(sources, targets, {pe: nbytes for pe in pes}, PE_start, logPE_stride,
                   PE_size)


def alltoall(sources: dict, targets: dict, nbytes: int, PE_start: int,
             logPE_stride: int, PE_size: int, block_index: str = "active_set") -> dict:
    """src/alltoall.c:59-82: for the i-th member pe, me gets nbytes from
    pe's source at sidx into its target at tidx = nbytes * i (:74-81).

    block_index="active_set" (the OpenSHMEM 1.4 definition, this
    implementation): sidx = nbytes * (me's active-set index).
    block_index="rank" (the reference's literal code, :76 `sidx = _size *
    nelems * proc.rank`): sidx = nbytes * me.  The two agree whenever
    PE_start = 0 and logPE_stride = 0."""
    pes = active_set(PE_start, logPE_stride, PE_size)
    out = {pe: targets[pe].copy() for pe in pes}
    for me_i, me in enumerate(pes):
        b = me_i if block_index == "active_set" else me
        for i, pe in enumerate(pes):
            out[me][i * nbytes:(i + 1) * nbytes] = sources[pe][b * nbytes:(b + 1) * nbytes]
    return out


COLL_KINDS = ["broadcast", "collect", "fcollect", "alltoall"]


def cpu_baseline(kind: str, npes: int, nb: int, root: int = 0, reps: int = 5,
                 pin: bool = True) -> float:
    """Median seconds per call of the reference loop shape (oracle_coll.c),
    one pthread per PE, nb bytes per PE contribution."""
    import ctypes
    import oracle as O
    L = O.lib()
    f = L.oracle_coll_baseline
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    sb = npes * nb if kind == "alltoall" else nb
    srcs = [np.random.default_rng(pe).integers(0, 256, sb, dtype=np.uint8) for pe in range(npes)]
    tgts = [np.empty(npes * nb, np.uint8) for _ in range(npes)]
    sp = (ctypes.c_void_p * npes)(*[s.ctypes.data for s in srcs])
    tp = (ctypes.c_void_p * npes)(*[t.ctypes.data for t in tgts])
    sec = f(COLL_KINDS.index(kind), npes, sp, tp, nb, root, reps, 1 if pin else 0)
    if sec < 0:
        raise ValueError("bad baseline arguments")
    return sec
