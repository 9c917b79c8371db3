"""oracle.py -- Python side of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  The
product (libosgpu_reduce.so and the `osgpu` package) never imports it.

Contents
  * ctypes loaders for oracle/liboracle.so (clean-room restatement of
    src/reductions.c:32-120 + src/shmemu/miscops.c:12-105) and, when present,
    oracle/_ref/libref_ops.so (the reference's own miscops.c, compiled here).
  * the type / op tables of src/reductions.c:248-297
  * deterministic input generators (splitmix64) shared by the golden
    generator, the CPU tests, the GPU parity tests and bench.py
  * the team fold order of src/reductions.c:84-111
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

TYPES = ["short", "int", "long", "longlong", "float", "double",
         "longdouble", "complexf", "complexd"]
OPS = ["sum", "prod", "and", "or", "xor", "max", "min"]
NP_DTYPE = {
    "short": np.int16, "int": np.int32, "long": np.int64, "longlong": np.int64,
    "float": np.float32, "double": np.float64, "longdouble": np.longdouble,
    "complexf": np.complex64, "complexd": np.complex128,
}
INT_TYPES = ("short", "int", "long", "longlong")
REAL_FP = ("float", "double", "longdouble")
CPLX = ("complexf", "complexd")


def has_op(t: str, op: str) -> bool:
    """src/reductions.c:248-297 -- which shmem_<t>_<op>_to_all exist."""
    if op in ("sum", "prod"):
        return True
    if op in ("and", "or", "xor"):
        return t in INT_TYPES
    if op in ("max", "min"):
        return t in INT_TYPES or t in REAL_FP
    return False


ALL_PAIRS = [(t, o) for o in OPS for t in TYPES if has_op(t, o)]
assert len(ALL_PAIRS) == 44


def fold_order(me: int, PE_start: int, logPE_stride: int, PE_size: int):
    """PE order in which PE `me` folds (src/reductions.c:79-111): its own
    source first, then the ascending active set skipping itself."""
    step = 1 << logPE_stride
    return [me] + [PE_start + i * step for i in range(PE_size)
                   if PE_start + i * step != me]


def active_set(PE_start, logPE_stride, PE_size):
    step = 1 << logPE_stride
    return [PE_start + i * step for i in range(PE_size)]


# --------------------------------------------------------------------------
# build + load
# --------------------------------------------------------------------------

def build(ref: bool = True, quiet: bool = True) -> None:
    """make liboracle.so (and oracle/_ref when /root/reference is present)."""
    kw = dict(cwd=HERE, check=True)
    if quiet:
        kw.update(stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-s", "liboracle.so"], **kw)
    if ref and os.path.isdir("/root/reference/src/shmemu"):
        subprocess.run(["make", "-s", "ref"], **kw)


_LIB = None
_REF = None


def lib():
    global _LIB
    if _LIB is None:
        # ORACLE_LIB: another build of the same sources (tests/test_sanitizers.py
        # runs the oracle's tests against an ASan/UBSan build)
        path = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build(ref=False)
        L = ctypes.CDLL(path)
        L.oracle_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_to_all.argtypes = [ctypes.c_int] * 6 + [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_cpu_baseline.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_cpu_baseline.restype = ctypes.c_double
        L.oracle_cpu_baseline_split.argtypes = L.oracle_cpu_baseline.argtypes + [ctypes.c_int]
        L.oracle_cpu_baseline_split.restype = ctypes.c_double
        L.oracle_cpu_baseline_ref.argtypes = L.oracle_cpu_baseline_split.argtypes + [ctypes.c_void_p]
        L.oracle_cpu_baseline_ref.restype = ctypes.c_double
        _LIB = L
    return _LIB


def ref_lib():
    """oracle/_ref/libref_ops.so or None (absent on the GPU box unless built
    in the container and shipped in the snapshot)."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libref_ops.so")
        if not os.path.exists(path):
            return None
        R = ctypes.CDLL(path)
        R.ref_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        _REF = R
    return _REF


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def op_elementwise(t: str, op: str, a: np.ndarray, b: np.ndarray,
                   use_ref: bool = False) -> np.ndarray:
    """out[i] = op(a[i], b[i]) through the restatement (or the reference)."""
    a = np.ascontiguousarray(a, dtype=NP_DTYPE[t])
    b = np.ascontiguousarray(b, dtype=NP_DTYPE[t])
    out = np.empty_like(a)
    L = ref_lib() if use_ref else lib()
    fn = L.ref_op if use_ref else L.oracle_op
    rc = fn(TYPES.index(t), OPS.index(op), _ptr(a), _ptr(b), _ptr(out), a.size)
    if rc != 0:
        raise ValueError(f"no op {t}/{op}")
    return out


def to_all(t: str, op: str, sources: list, PE_start=0, logPE_stride=0,
           PE_size=None) -> list:
    """Team reduce-to-all through the C restatement; returns per-PE targets
    (None for PEs outside the active set)."""
    npes = len(sources)
    if PE_size is None:
        PE_size = npes
    n = sources[0].size
    srcs = [np.ascontiguousarray(s, dtype=NP_DTYPE[t]) for s in sources]
    tgts = [np.zeros_like(srcs[0]) for _ in range(npes)]
    sp = (ctypes.c_void_p * npes)(*[s.ctypes.data for s in srcs])
    tp = (ctypes.c_void_p * npes)(*[x.ctypes.data for x in tgts])
    rc = lib().oracle_to_all(TYPES.index(t), OPS.index(op), npes, PE_start,
                             logPE_stride, PE_size, sp, tp, n)
    if rc != 0:
        raise ValueError("oracle_to_all failed")
    act = set(active_set(PE_start, logPE_stride, PE_size))
    return [tgts[p] if p in act else None for p in range(npes)]


def fold_with(fn, t, op, sources, me, PE_start, logPE_stride, PE_size):
    """fold sources in PE `me`'s order using an elementwise function `fn`
    (used with the reference ops to build goldens)."""
    order = fold_order(me, PE_start, logPE_stride, PE_size)
    acc = np.array(sources[order[0]], dtype=NP_DTYPE[t], copy=True)
    for pe in order[1:]:
        acc = fn(t, op, acc, sources[pe])
    return acc


def ref_elem_fn(t: str, op: str):
    """Address of the reference's own compiled element function
    shmemu_<op>_<t>_func (src/shmemu/miscops.c:12-105, oracle/_ref), or None
    when oracle/_ref is absent."""
    R = ref_lib()
    if R is None:
        return None
    try:
        return ctypes.cast(getattr(R, f"shmemu_{op}_{t}_func"), ctypes.c_void_p).value
    except AttributeError:
        return None


def cpu_baseline(t: str, op: str, sources: list, reps: int = 5,
                 pin: bool = True, threads_per_pe: int = 1, targets: list = None,
                 ref_ops: bool = False) -> float:
    """Median seconds per reduce-to-all call of the reference loop shape,
    one pthread per PE (oracle_reduce.c), or threads_per_pe pthreads per PE
    each running that shape over a contiguous part of the elements.  If
    `targets` is a list, the PEs' result arrays are appended to it.
    ref_ops: call the reference's own compiled element function in the loop
    (oracle/_ref; raises if it is absent)."""
    npes = len(sources)
    srcs = [np.ascontiguousarray(s, dtype=NP_DTYPE[t]) for s in sources]
    tgts = [np.empty_like(srcs[0]) for _ in range(npes)]
    sp = (ctypes.c_void_p * npes)(*[s.ctypes.data for s in srcs])
    tp = (ctypes.c_void_p * npes)(*[x.ctypes.data for x in tgts])
    fn = None
    if ref_ops:
        fn = ref_elem_fn(t, op)
        if fn is None:
            raise ValueError(f"no reference element function for {t}/{op} (oracle/_ref absent?)")
    sec = lib().oracle_cpu_baseline_ref(TYPES.index(t), OPS.index(op), npes, sp, tp,
                                        srcs[0].size, reps, 1 if pin else 0,
                                        threads_per_pe, fn)
    if sec < 0:
        raise ValueError(f"no cpu baseline for {t}/{op}")
    if targets is not None:
        targets.extend(tgts)
    return sec


# --------------------------------------------------------------------------
# deterministic inputs
# --------------------------------------------------------------------------

M64 = (1 << 64) - 1


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of splitmix64 started at `seed` (uint64)."""
    with np.errstate(over="ignore"):
        x = (np.uint64(seed & M64)
             + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def pe_seed(seed: int, pe: int) -> int:
    return (seed ^ (pe * 0x9E37)) & M64


def _fp_from_bits(r: np.ndarray, ebits: int, mbits: int, emin: int, emax: int,
                  signed=True):
    """values sign * 1.m * 2^e with e uniform in [emin, emax] (exact bits)."""
    bias = (1 << (ebits - 1)) - 1
    mant = r & np.uint64((1 << mbits) - 1)
    e = (r >> np.uint64(mbits)) % np.uint64(emax - emin + 1)
    exp = (e.astype(np.int64) + emin + bias).astype(np.uint64)
    sign = (r >> np.uint64(63)) if signed else np.zeros_like(r)
    return (sign << np.uint64(ebits + mbits)) | (exp << np.uint64(mbits)) | mant


def gen_real(t: str, r: np.ndarray, dist: str) -> np.ndarray:
    """Map uint64 draws to values of real FP type t."""
    if dist == "unit12":  # uniform [1, 2): the bench / BASELINE distribution
        if t == "float":
            return ((np.uint64(127) << np.uint64(23)) | (r >> np.uint64(41))).astype(
                np.uint32).view(np.float32)
        d = ((np.uint64(1023) << np.uint64(52)) | (r >> np.uint64(12))).view(np.float64)
        return d.astype(NP_DTYPE[t])
    lo, hi = (-8, 8) if dist in ("mixed", "prod") else (-60, 60)
    signed = dist != "prod"
    if t == "float":
        b = _fp_from_bits(r, 8, 23, lo, hi, signed)
        return b.astype(np.uint32).view(np.float32)
    d = _fp_from_bits(r, 11, 52, lo, hi, signed).view(np.float64)
    if t == "double":
        return d
    # long double: a double plus a perturbation below the double's ulp, so the
    # 64-bit significand is exercised (computed in x87 long double)
    ld = d.astype(np.longdouble)
    frac = (r & np.uint64(0x7FF)).astype(np.longdouble) / np.longdouble(2048.0)
    return ld + ld * frac * np.longdouble(2.0) ** -53


def special_values(t: str) -> np.ndarray:
    """Edge values of type t (NaN payloads, signed zeros, infinities,
    subnormals, extremes)."""
    if t in INT_TYPES:
        info = np.iinfo(NP_DTYPE[t])
        v = [0, 1, -1, 2, -2, 3, info.max, info.min, info.max - 1, info.min + 1,
             info.max // 2, info.min // 2, 0x55, -0x56]
        return np.array(v, dtype=NP_DTYPE[t])
    if t in ("float", "complexf"):
        bits = [0x00000000, 0x80000000, 0x3F800000, 0xBF800000, 0x40200000,
                0xC0A00000, 0x7F7FFFFF, 0xFF7FFFFF, 0x00800000, 0x00000001,
                0x80000003, 0x007FFFFF, 0x7F800000, 0xFF800000, 0x7FC00000,
                0xFFC00000, 0x7FC00123, 0x7F800001, 0xFFA00005, 0x5F000000,
                0x1F000000]
        return np.array(bits, dtype=np.uint32).view(np.float32)
    if t in ("double", "complexd"):
        bits = [0x0, 0x8000000000000000, 0x3FF0000000000000, 0xBFF0000000000000,
                0x4004000000000000, 0xC014000000000000, 0x7FEFFFFFFFFFFFFF,
                0xFFEFFFFFFFFFFFFF, 0x0010000000000000, 0x0000000000000001,
                0x8000000000000003, 0x000FFFFFFFFFFFFF, 0x7FF0000000000000,
                0xFFF0000000000000, 0x7FF8000000000000, 0xFFF8000000000000,
                0x7FF8000000000123, 0x7FF0000000000001, 0xFFF4000000000005,
                0x5FE0000000000000, 0x2000000000000000]
        return np.array(bits, dtype=np.uint64).view(np.float64)
    # long double (x87 80-bit in 16 bytes)
    vals = [0.0, -0.0, 1.0, -1.0, 2.5, -5.0, np.inf, -np.inf]
    ld = [np.longdouble(v) for v in vals]
    fi = np.finfo(np.longdouble)
    ld += [fi.max, -fi.max, fi.tiny, np.longdouble(fi.smallest_subnormal),
           -np.longdouble(fi.smallest_subnormal) * 3, np.longdouble(np.nan),
           -np.longdouble(np.nan), np.longdouble(1e4000) if False else fi.max / 2,
           np.longdouble(1) + fi.eps, np.longdouble(1) - fi.epsneg]
    arr = np.array(ld, dtype=np.longdouble)
    # NaNs with payloads / signalling: craft raw bytes (low 8 = significand,
    # next 2 = sign|exp)
    raw = arr.view(np.uint8).reshape(-1, 16).copy()
    extra = []
    for sig, se in ((0xC000000000000123, 0x7FFF), (0x8000000000000001, 0x7FFF),
                    (0xA000000000000000, 0xFFFF),
                    # x87 encodings with no IEEE counterpart: unnormal,
                    # pseudo-denormal, pseudo-infinity, pseudo-NaN
                    (0x4000000000000000, 0x3FFF), (0x8000000000000001, 0x0000),
                    (0x0000000000000000, 0x7FFF), (0x4000000000000001, 0xFFFF)):
        row = np.zeros(16, dtype=np.uint8)
        row[:8] = np.frombuffer(int(sig).to_bytes(8, "little"), dtype=np.uint8)
        row[8:10] = np.frombuffer(int(se).to_bytes(2, "little"), dtype=np.uint8)
        extra.append(row)
    raw = np.concatenate([raw, np.stack(extra)])
    return raw.reshape(-1).view(np.longdouble)


def gen_input(t: str, n: int, seed: int, dist: str = "mixed") -> np.ndarray:
    """n deterministic values of type t.

    dist: 'mixed' (signed, exponents in [-8, 8]), 'prod' (positive, same
    range), 'wide' (signed, exponents in [-60, 60]), 'unit12' ([1, 2)),
    'bits' (raw random bits for integer types), 'edge' (mixed with ~1/8 of the
    elements replaced by special_values(t)), 'and'/'or' (bit-biased integer
    draws per SURVEY.md 8d config 3: OR / AND of three draws)."""
    dt = NP_DTYPE[t]
    if n == 0:
        return np.zeros(0, dtype=dt)
    r = splitmix64(seed, n)
    if t in INT_TYPES:
        if dist == "and":
            r = r | splitmix64(seed ^ 0xA5A5, n) | splitmix64(seed ^ 0x5A5A, n)
        elif dist == "or":
            r = r & splitmix64(seed ^ 0xA5A5, n) & splitmix64(seed ^ 0x5A5A, n)
        elif dist == "prod":
            # small magnitudes so products stay informative
            r = (r % np.uint64(7)) + np.uint64(1)
        w = np.dtype(dt).itemsize * 8
        v = (r & np.uint64((1 << w) - 1)).astype({16: np.uint16, 32: np.uint32,
                                                  64: np.uint64}[w]).view(dt)
        out = v.copy()
    elif t in REAL_FP:
        out = gen_real(t, r, "mixed" if dist in ("edge", "bits") else dist)
        out = np.ascontiguousarray(out, dtype=dt)
    else:
        base = "float" if t == "complexf" else "double"
        r2 = splitmix64(seed ^ 0xC0FFEE, n)
        d = "mixed" if dist in ("edge", "bits") else dist
        re = gen_real(base, r, d)
        im = gen_real(base, r2, d)
        out = np.empty(n, dtype=dt)
        out.real = re
        out.imag = im
    if dist == "edge":
        sv = special_values(t)
        pick = splitmix64(seed ^ 0xED6E, n)
        mask = (pick & np.uint64(7)) == 0
        idx = ((pick >> np.uint64(8)) % np.uint64(sv.size)).astype(np.int64)
        if t in CPLX:
            comp = "float" if t == "complexf" else "double"
            svr = special_values(comp)
            idx2 = ((pick >> np.uint64(24)) % np.uint64(svr.size)).astype(np.int64)
            re = out.real.copy()
            im = out.imag.copy()
            re[mask] = svr[idx[mask] % svr.size]
            im[mask] = svr[idx2[mask]]
            # write back through views so NaN payloads survive exactly
            fl = out.view(np.float32 if t == "complexf" else np.float64).reshape(-1, 2)
            fl[:, 0] = re
            fl[:, 1] = im
        else:
            out[mask] = sv[idx[mask]]
    return out


def team_inputs(t: str, npes: int, n: int, seed: int, dist: str):
    return [gen_input(t, n, pe_seed(seed, pe), dist) for pe in range(npes)]


def digest(a: np.ndarray) -> str:
    """SHA-256 of the value bytes (long double: the 10 significant bytes of
    each 16-byte slot; padding is not part of the value)."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.longdouble:
        b = a.view(np.uint8).reshape(-1, 16)[:, :10].tobytes()
    else:
        b = a.tobytes()
    return hashlib.sha256(b).hexdigest()


def value_bytes(a: np.ndarray) -> np.ndarray:
    """Bytes that carry the value (for bitwise comparison)."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.longdouble:
        return a.view(np.uint8).reshape(-1, 16)[:, :10].copy()
    return a.view(np.uint8).copy()


def from_value_bytes(t: str, raw: np.ndarray) -> np.ndarray:
    """Inverse of value_bytes (long double slots are zero-padded to 16 B)."""
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    if t == "longdouble":
        rows = raw.reshape(-1, 10)
        full = np.zeros((rows.shape[0], 16), dtype=np.uint8)
        full[:, :10] = rows
        return full.reshape(-1).view(np.longdouble)
    return raw.view(NP_DTYPE[t]).copy()


def load_cases(path=None):
    import json
    if path is None:
        path = os.path.join(os.path.dirname(HERE), "tests", "golden", "reduce_cases.json")
    with open(path) as f:
        return json.load(f)["cases"]


def case_inputs(c: dict):
    return team_inputs(c["type"], c["npes"], c["nreduce"], c["seed"], c["dist"])
