"""osgpu -- Python view of libosgpu_reduce.so (ctypes over the C ABI).

The product is the C-ABI shared library built from ../csrc (declared in
include/osgpu_reduce.h).  This module only loads it and describes its
signatures so tests and bench.py can call the same entry points a C/Fortran
OpenSHMEM application would (shmem_<TYPE>_<OP>_to_all, src/reductions.c:248-297
of the reference).  It never computes anything itself, and it refuses to run
without the compiled library: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# OSGPU_LIB_PATH: load another build of the same library (tuning tools only)
LIB_PATH = os.environ.get("OSGPU_LIB_PATH") or os.path.join(PKG_DIR, "libosgpu_reduce.so")
CSRC = os.path.join(PKG_DIR, "csrc")
REPO = os.path.dirname(PKG_DIR)
HEADER = os.path.join(REPO, "include", "osgpu_reduce.h")

TYPES = ["short", "int", "long", "longlong", "float", "double",
         "longdouble", "complexf", "complexd"]
OPS = ["sum", "prod", "and", "or", "xor", "max", "min"]
CTYPE = {
    "short": ctypes.c_short, "int": ctypes.c_int, "long": ctypes.c_long,
    "longlong": ctypes.c_longlong, "float": ctypes.c_float,
    "double": ctypes.c_double, "longdouble": ctypes.c_longdouble,
    "complexf": ctypes.c_float * 2, "complexd": ctypes.c_double * 2,
}
PATH_AUTO, PATH_P2P, PATH_RCCL, PATH_PULL = 0, 1, 2, 3
# enum osgpu_ran: what osgpu_last_path() reports
RAN = ["none", "team", "pull", "rccl", "staged", "getmem", "fused_team", "fused_pull",
       "barrier_only", "fused_staged", "copy", "fused_copy", "fused_failed", "team_push",
       "host_fold"]


def has_op(t: str, op: str) -> bool:
    if op in ("sum", "prod"):
        return True
    if op in ("and", "or", "xor"):
        return t in ("short", "int", "long", "longlong")
    return op in ("max", "min") and t not in ("complexf", "complexd")


ENTRY_POINTS = [f"shmem_{t}_{o}_to_all" for o in OPS for t in TYPES if has_op(t, o)]
assert len(ENTRY_POINTS) == 44
# data-movement collectives on the same machinery (include/osgpu_reduce.h Part 1b)
COLL_KINDS = ["broadcast", "collect", "fcollect", "alltoall"]
COLL_ENTRY_POINTS = [f"shmem_{k}{b}" for k in COLL_KINDS for b in (32, 64)]


class PeOps(ctypes.Structure):
    """struct osgpu_pe_ops (include/osgpu_reduce.h)"""
    _fields_ = [
        ("my_pe", ctypes.CFUNCTYPE(ctypes.c_int)),
        ("n_pes", ctypes.CFUNCTYPE(ctypes.c_int)),
        ("barrier", ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_long))),
        ("getmem", ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_int)),
    ]


def build(jobs: int = 8, quiet: bool = True) -> str:
    """Compile the gfx950 library in-tree (make in csrc/)."""
    kw = {}
    if quiet:
        kw = dict(stdout=subprocess.DEVNULL)
    subprocess.run(["make", "-s", f"-j{jobs}"], cwd=CSRC, check=True, **kw)
    return LIB_PATH


_LIB = None


def load() -> ctypes.CDLL:
    """Load libosgpu_reduce.so; raises if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() "
                           "(the reduction has no CPU implementation)")
    # One HIP runtime per process: PyTorch ships its own libamdhip64 (same
    # SONAME libamdhip64.so.7, different file name).  Loaded first, our
    # NEEDED entry binds to torch's copy; loaded after us, torch would map a
    # second runtime next to /opt/rocm's and the two corrupt each other's
    # heap at exit.  So when torch is importable, it goes first -- unless
    # OSGPU_NO_TORCH=1: a process that never imports torch (as a C
    # application linking the library) runs on /opt/rocm's runtime.
    if os.environ.get("OSGPU_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    for name in ENTRY_POINTS:
        for pfx in ("", "p"):
            f = getattr(L, pfx + name)
            f.argtypes = [vp, vp, i, i, i, i, vp, vp]
            f.restype = None
    sz_t, lp = ctypes.c_size_t, ctypes.c_void_p
    for name in COLL_ENTRY_POINTS:
        for pfx in ("", "p"):
            f = getattr(L, pfx + name)
            if "broadcast" in name:
                f.argtypes = [vp, vp, sz_t, i, i, i, i, lp]
            else:
                f.argtypes = [vp, vp, sz_t, i, i, i, lp]
            f.restype = None
    L.osgpu_set_pe_ops.argtypes = [vp]
    L.osgpu_heap_register.argtypes = [i, vp, sz]
    L.osgpu_heap_register_segment.argtypes = [i, i, vp, sz]
    L.osgpu_heap_unregister.argtypes = [i]
    L.osgpu_heap_translate.argtypes = [vp, i, i]
    L.osgpu_heap_create.argtypes = [sz, i, i, i, vp, ctypes.POINTER(vp)]
    L.osgpu_heap_destroy.argtypes = [vp]
    L.osgpu_preflight.argtypes = [vp, i, i, i, vp, ctypes.c_char_p, sz]
    L.osgpu_heap_translate.restype = vp
    L.osgpu_ipc_get_handle.argtypes = [vp, vp]
    L.osgpu_ipc_open.argtypes = [vp]
    L.osgpu_ipc_open.restype = vp
    L.osgpu_ipc_close.argtypes = [vp]
    L.osgpu_rccl_unique_id.argtypes = [vp]
    L.osgpu_rccl_init.argtypes = [i, i, vp]
    L.osgpu_rccl_comm_info.argtypes = [ctypes.POINTER(i)] * 3
    L.osgpu_device_identity.argtypes = [ctypes.c_char_p, sz]
    L.osgpu_set_path.argtypes = [i]
    L.osgpu_set_stream.argtypes = [vp]
    L.osgpu_get_stream.restype = vp
    L.osgpu_combine.argtypes = [i, i, vp, vp, i, sz, vp]
    L.osgpu_copy.argtypes = [vp, vp, vp, i, vp]
    L.osgpu_team_combine.argtypes = [i, i, i, vp, vp, sz, vp]
    L.osgpu_team_combine_shape.argtypes = [i, i, i, vp, vp, sz, vp, i]
    L.osgpu_build_id.restype = ctypes.c_char_p
    L.osgpu_has_op.argtypes = [i, i]
    L.osgpu_type_size.argtypes = [i]
    L.osgpu_type_size.restype = sz
    L.osgpu_fold_order.argtypes = [i, i, i, i, ctypes.POINTER(ctypes.c_int)]
    L.osgpu_shard_range.argtypes = [ctypes.c_longlong, i, i, i,
                                    ctypes.POINTER(ctypes.c_longlong),
                                    ctypes.POINTER(ctypes.c_longlong)]
    L.osgpu_host_register.argtypes = [vp, sz]
    L.osgpu_host_unregister.argtypes = [vp]
    L.osgpu_set_fused_max_bytes.argtypes = [ctypes.c_longlong]
    L.osgpu_set_device_barrier.argtypes = [ctypes.c_double, ctypes.c_int]
    L.osgpu_set_team_exchange.argtypes = [ctypes.c_int]
    L.osgpu_set_host_path.argtypes = [ctypes.c_int]
    L.osgpu_set_host_fold_max_bytes.argtypes = [ctypes.c_longlong]
    L.osgpu_set_stage_copy.argtypes = [ctypes.c_int]
    L.osgpu_set_host_chunk_bytes.argtypes = [ctypes.c_longlong]
    L.osgpu_set_stage_bytes.argtypes = [ctypes.c_longlong]
    L.osgpu_checksum.argtypes = [i, i, vp, sz, vp, ctypes.POINTER(ctypes.c_ulonglong)]
    L.osgpu_compare.argtypes = [vp, vp, sz, vp, ctypes.POINTER(ctypes.c_ulonglong),
                                ctypes.POINTER(ctypes.c_ulonglong)]
    L.osgpu_last_path.restype = ctypes.c_int
    L.osgpu_last_coll_path.restype = ctypes.c_int
    L.osgpu_last_error.restype = ctypes.c_char_p
    L.osgpu_version.restype = ctypes.c_char_p
    _LIB = L
    return L


CK_SUM, CK_XOR, CK_HASH = 0, 1, 2

# osgpu_set_host_path modes (include/osgpu_reduce.h enum osgpu_host_path)
HOST_AUTO, HOST_STAGED, HOST_GETMEM = 0, 1, 2
HOST_PATHS = {"auto": HOST_AUTO, "staged": HOST_STAGED, "getmem": HOST_GETMEM}
STAGE_COPY = {"dma": 0, "kout": 1, "kernel": 2}


class host_path:
    """with osgpu.host_path("staged" | "getmem" | "auto" | None): the host
    symmetric-heap path for the block (None: the environment's default),
    restored to the environment's default afterwards."""

    def __init__(self, mode):
        self.mode = -1 if mode is None else HOST_PATHS[mode]

    def __enter__(self):
        assert load().osgpu_set_host_path(self.mode) == 0
        return self

    def __exit__(self, *exc):
        load().osgpu_set_host_path(-1)
        return False


def checksum(t: str, mode: int, ptr: int, n: int, stream: int | None = None) -> int:
    """osgpu_checksum over n elements of type t at device address ptr."""
    out = ctypes.c_ulonglong()
    rc = load().osgpu_checksum(TYPES.index(t), mode, ptr, n, stream, ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(load().osgpu_last_error().decode())
    return out.value


def compare(a: int, b: int, nbytes: int, stream: int | None = None):
    """osgpu_compare: (differing 16-B vectors, first differing byte offset or None)."""
    bad, first = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    rc = load().osgpu_compare(a, b, nbytes, stream, ctypes.byref(bad), ctypes.byref(first))
    if rc != 0:
        raise RuntimeError(load().osgpu_last_error().decode())
    return bad.value, (None if first.value == (1 << 64) - 1 else first.value)


def source_build_id() -> str:
    """The build id the Makefile would stamp on a library built from the
    sources in this tree (csrc/Makefile BUILD_ID)."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp"))
                   + glob.glob(os.path.join(CSRC, "*.hpp")), key=os.path.basename)
    h = hashlib.sha256()
    for f in files + [HEADER]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def device_view(ptr: int, nbytes: int, dtype=None):
    """A torch tensor aliasing `nbytes` of device memory at `ptr` -- e.g. a
    heap made by osgpu_heap_create, whose virtual-memory range no torch
    allocator owns -- through __cuda_array_interface__ (tests/bench only)."""
    import torch

    class _Mem:
        def __init__(self):
            self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                             "data": (ptr, False), "version": 3,
                                             "strides": None}

    t = torch.as_tensor(_Mem(), device="cuda")
    return t.view(dtype) if dtype is not None else t


def heap_create(nbytes: int, PE_start: int, logPE_stride: int, PE_size: int, psync: int) -> int:
    """osgpu_heap_create (collective): this PE's heap base; raises on failure."""
    L = load()
    base = ctypes.c_void_p()
    rc = L.osgpu_heap_create(nbytes, PE_start, logPE_stride, PE_size, psync, ctypes.byref(base))
    if rc != 0:
        raise RuntimeError(f"osgpu_heap_create = {rc}: {L.osgpu_last_error().decode()}")
    return base.value


def preflight(heap_base, PE_start: int, logPE_stride: int, PE_size: int, psync: int):
    """osgpu_preflight (collective): (status code, per-peer report dict)."""
    import json
    L = load()
    buf = ctypes.create_string_buffer(1 << 20)
    rc = L.osgpu_preflight(heap_base, PE_start, logPE_stride, PE_size, psync, buf, len(buf))
    try:
        rep = json.loads(buf.value.decode() or "{}")
    except ValueError:
        rep = {"unparsed": buf.value.decode()[:400]}
    if rc != 0:
        rep["error"] = L.osgpu_last_error().decode()
    return rc, rep


def rccl_comm_info():
    """(nranks, rank, device) of the RCCL communicator (ncclCommCount /
    ncclCommUserRank / ncclCommCuDevice); raises without one."""
    L = load()
    v = [ctypes.c_int(-1) for _ in range(3)]
    rc = L.osgpu_rccl_comm_info(*[ctypes.byref(x) for x in v])
    if rc != 0:
        raise RuntimeError(L.osgpu_last_error().decode())
    return tuple(x.value for x in v)


def device_identity() -> dict:
    """The calling thread's current device: {"device", "pci_bus_id", "uuid"}."""
    import json
    L = load()
    buf = ctypes.create_string_buffer(256)
    if L.osgpu_device_identity(buf, len(buf)) != 0:
        raise RuntimeError(L.osgpu_last_error().decode())
    return json.loads(buf.value.decode())


def last_path() -> str:
    """Name of the path the calling thread's last reduce-to-all call took."""
    return RAN[load().osgpu_last_path()]


def last_coll_path() -> str:
    """Name of the path the calling thread's last data-movement collective took."""
    return RAN[load().osgpu_last_coll_path()]


def to_all(t: str, op: str):
    """The ctypes function shmem_<t>_<op>_to_all."""
    return getattr(load(), f"shmem_{t}_{op}_to_all")


def combine(t: str, op: str, target: int, srcs, n: int, stream: int | None = None):
    """Enqueue the combine kernel: target = fold(op, srcs...) (device ptrs)."""
    L = load()
    arr = (ctypes.c_void_p * len(srcs))(*srcs)
    rc = L.osgpu_combine(TYPES.index(t), OPS.index(op), target, arr, len(srcs), n,
                         stream)
    if rc != 0:
        raise RuntimeError(f"osgpu_combine({t},{op}) = {rc}: "
                           f"{L.osgpu_last_error().decode()}")


def copy(dsts, srcs, nbytes, stream: int | None = None):
    """Enqueue the collectives' copy kernel: dsts[i][:nbytes[i]] = srcs[i][...]."""
    L = load()
    n = len(dsts)
    rc = L.osgpu_copy((ctypes.c_void_p * n)(*dsts), (ctypes.c_void_p * n)(*srcs),
                      (ctypes.c_size_t * n)(*nbytes), n, stream)
    if rc != 0:
        raise RuntimeError(f"osgpu_copy = {rc}: {L.osgpu_last_error().decode()}")


def coll(kind: str, bits: int):
    """The ctypes function shmem_<kind><bits> (broadcast/collect/fcollect/alltoall)."""
    return getattr(load(), f"shmem_{kind}{bits}")


def fold_order(me, PE_start, logPE_stride, PE_size):
    out = (ctypes.c_int * PE_size)()
    rc = load().osgpu_fold_order(me, PE_start, logPE_stride, PE_size, out)
    if rc != 0:
        raise ValueError("PE not in active set")
    return list(out)


def shard_range(nreduce, PE_size, idx, elem_bytes):
    lo, hi = ctypes.c_longlong(), ctypes.c_longlong()
    rc = load().osgpu_shard_range(nreduce, PE_size, idx, elem_bytes,
                                  ctypes.byref(lo), ctypes.byref(hi))
    if rc != 0:
        raise ValueError("bad shard arguments")
    return lo.value, hi.value


def header_symbols(path: str = HEADER):
    """Function names declared in include/osgpu_reduce.h (expanding the
    OSGPU_DECL_ALL macro for both prefixes)."""
    import re
    src = open(path).read()
    names = set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(osgpu_\w+)\s*\(",
                           src, re.M))
    for pfx in ("shmem_", "pshmem_"):
        for e in ENTRY_POINTS + COLL_ENTRY_POINTS:
            names.add(pfx + e[len("shmem_"):])
    return sorted(names)
