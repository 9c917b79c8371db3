#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE.

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py

Element arithmetic comes from the reference's own src/shmemu/miscops.c,
compiled unmodified by oracle/Makefile into oracle/_ref/libref_ops.so and
called through a function pointer per element, exactly like
src/reductions.c:95-96.  The team schedule (PE `me` folds its own source
first, then the active set PE_start + i*2^logPE_stride in ascending order
skipping itself, src/reductions.c:79-111) is restated here because
src/reductions.c itself cannot be compiled in this image (it needs UCX's
<ucp/api/ucp.h>, see oracle/oracle.h).

Outputs
  ops_<type>.npz     a, b, out_<op>: elementwise op(a[i], b[i]) on grids of
                     special values (NaN payloads, signed zeros, infinities,
                     subnormals, extremes) plus random pairs
  reduce_cases.json  reduce-to-all cases: inputs are regenerated from
                     (type, npes, nreduce, seed, dist) by oracle.gen_input;
                     expected per-PE outputs are stored as SHA-256 digests
                     (oracle.digest) plus full hex for nreduce <= 8
"""
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def ref_fn(t, op, a, b):
    return O.op_elementwise(t, op, a, b, use_ref=True)


def op_grid(t):
    """(a, b) pairs: all pairs of special values + 2000 random pairs.
    Complex: all 4-tuples over 10 component specials."""
    if t in O.CPLX:
        comp = "float" if t == "complexf" else "double"
        s = O.special_values(comp)
        pick = np.array([0, 1, 2, 3, 6, 9, 12, 13, 14, 16])  # 0,-0,1,-1,max,sub,inf,-inf,nan,nanpayload
        s = s[pick]
        idx = np.array(np.meshgrid(*[np.arange(s.size)] * 4, indexing="ij")).reshape(4, -1)
        a = np.empty(idx.shape[1], dtype=O.NP_DTYPE[t])
        b = np.empty_like(a)
        fa = a.view(s.dtype).reshape(-1, 2)
        fb = b.view(s.dtype).reshape(-1, 2)
        fa[:, 0], fa[:, 1], fb[:, 0], fb[:, 1] = s[idx[0]], s[idx[1]], s[idx[2]], s[idx[3]]
    else:
        sv = O.special_values(t)
        ia, ib = np.meshgrid(np.arange(sv.size), np.arange(sv.size), indexing="ij")
        a, b = sv[ia.ravel()], sv[ib.ravel()]
    dist = "bits" if t in O.INT_TYPES else "wide"
    ra = O.gen_input(t, 2000, 0xA11CE, dist)
    rb = O.gen_input(t, 2000, 0xB0B, dist)
    return np.concatenate([a, ra]), np.concatenate([b, rb])


def default_dist(t, op):
    if t in O.INT_TYPES:
        return "bits"
    if op == "prod":
        return "prod"
    return "mixed"


def case_seed(*parts):
    return zlib.crc32(repr(parts).encode()) * 0x100000001 & O.M64


def make_case(t, op, npes, nreduce, dist, PE_start=0, logPE_stride=0, PE_size=None,
              tag="grid"):
    if PE_size is None:
        PE_size = npes
    seed = case_seed(t, op, npes, nreduce, dist, PE_start, logPE_stride, PE_size)
    src = O.team_inputs(t, npes, nreduce, seed, dist)
    rec = dict(type=t, op=op, npes=npes, nreduce=nreduce, dist=dist, seed=seed,
               PE_start=PE_start, logPE_stride=logPE_stride, PE_size=PE_size,
               tag=tag, digests={}, hex={})
    for me in O.active_set(PE_start, logPE_stride, PE_size):
        out = O.fold_with(ref_fn, t, op, src, me, PE_start, logPE_stride, PE_size)
        rec["digests"][str(me)] = O.digest(out)
        if nreduce <= 8:
            rec["hex"][str(me)] = O.value_bytes(out).tobytes().hex()
    return rec


def main():
    O.build(ref=True)
    if O.ref_lib() is None:
        sys.exit("oracle/_ref/libref_ops.so missing: needs /root/reference")

    # ---- element-op grids
    for t in O.TYPES:
        a, b = op_grid(t)
        arrs = {"a": O.value_bytes(a), "b": O.value_bytes(b)}
        for op in O.OPS:
            if O.has_op(t, op):
                arrs["out_" + op] = O.value_bytes(ref_fn(t, op, a, b))
        np.savez_compressed(os.path.join(OUT, f"ops_{t}.npz"), **arrs)

    # ---- reduce-to-all cases
    cases = []
    Ns = [0, 1, 63, 64, 65, 127, 1000, 4097]
    for t, op in O.ALL_PAIRS:
        d = default_dist(t, op)
        for P in (1, 2, 3, 4, 8):
            for N in Ns:
                cases.append(make_case(t, op, P, N, d))
        # edge values (NaN/±0/inf/subnormal/extremes) through the team fold
        for P in (3, 8):
            cases.append(make_case(t, op, P, 4097, "edge", tag="edge"))
        # active-set subsets of an 8-PE job
        for (ps, ls, sz) in ((1, 1, 3), (2, 0, 4), (0, 2, 2), (5, 0, 1)):
            cases.append(make_case(t, op, 8, 1000, d, ps, ls, sz, tag="subset"))
    # BASELINE.json configs at parity-test size
    cases.append(make_case("int", "sum", 2, 1024, "bits", tag="config1"))
    cases.append(make_case("double", "sum", 2, 1 << 20, "unit12", tag="config2"))
    for op in ("and", "or", "xor"):
        cases.append(make_case("long", op, 2, 1 << 20, op if op != "xor" else "bits",
                               tag="config3"))
    cases.append(make_case("double", "sum", 8, 1 << 20, "unit12", tag="config4"))
    for op in ("min", "max"):
        cases.append(make_case("float", op, 8, 1 << 18, "wide", tag="config5"))
    cases.append(make_case("float", "prod", 8, 1 << 18, "prod", tag="config5"))
    # exponent-spread sums where fold order changes the rounding
    for t in ("float", "double", "complexf", "complexd"):
        cases.append(make_case(t, "sum", 8, 1 << 16, "wide", tag="order"))

    with open(os.path.join(OUT, "reduce_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "element_ops": "reference src/shmemu/miscops.c compiled unmodified",
                   "cases": cases}, f, indent=0, sort_keys=True)
    print(f"{len(cases)} reduce cases, {len(O.TYPES)} op grids")


if __name__ == "__main__":
    main()
