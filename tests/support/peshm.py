"""peshm.py -- load/initialise tests/support/pe_shm.c (intra-node PE runtime,
one process per PE).  TEST/BENCH INFRASTRUCTURE."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libpe_shm.so")


def build():
    """(Re)build libpe_shm.so when pe_shm.c is newer.  Several PE processes
    may get here at once: each compiles to its own file and renames it into
    place, so no process ever loads a half-written library."""
    src = os.path.join(HERE, "pe_shm.c")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        tmp = f"{SO}.{os.getpid()}.tmp"
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", tmp, src, "-lrt"], check=True)
        os.replace(tmp, SO)


def load():
    build()
    L = ctypes.CDLL(SO)
    L.pes_init.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                           ctypes.c_ulonglong, ctypes.c_int]
    L.pes_unlink.argtypes = [ctypes.c_char_p]
    L.pes_heap.argtypes = [ctypes.c_int]
    L.pes_heap.restype = ctypes.c_void_p
    L.pes_heap_bytes.restype = ctypes.c_ulonglong
    L.pes_ops.restype = ctypes.c_void_p
    L.pes_set_thread_pe.argtypes = [ctypes.c_int]
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.pes_time_to_all.argtypes = [vp, vp, vp, i, i, i, i, vp, vp, i]
    L.pes_time_to_all.restype = ctypes.c_double
    return L


def init(rank: int, world: int, heap_bytes: int, dist, tag: str = ""):
    """Collective: rank 0 creates the segment, the others map it.  `dist` is
    an initialised torch.distributed (used only for this setup)."""
    L = load()
    name = f"/osgpu_pes_{os.environ.get('MASTER_PORT', '0')}{tag}".encode()
    if rank == 0:
        L.pes_unlink(name)
        assert L.pes_init(name, rank, world, heap_bytes, 1) == 0
    dist.barrier()
    if rank != 0:
        assert L.pes_init(name, rank, world, heap_bytes, 0) == 0
    dist.barrier()
    if rank == 0:
        L.pes_unlink(name)  # mappings stay valid; nothing left in /dev/shm
    return L
