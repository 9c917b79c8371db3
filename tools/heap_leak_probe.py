#!/usr/bin/env python3
"""heap_leak_probe.py -- does device memory come back after
osgpu_heap_destroy / hipMemRelease?  (1) raw HIP VMM in this process:
hipMemCreate + map + unmap + release, with and without a dmabuf export;
(2) osgpu_heap_create / destroy with 1 and 3 threads-as-PEs.  Free HBM
(hipMemGetInfo) before and after each cycle.  Not part of the product."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "test-resilient-osss-ucx_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import osgpu  # noqa: E402

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so")
MiB = 1 << 20


def free():
    torch.cuda.synchronize()
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
    return f.value


class Prop(ctypes.Structure):  # hipMemAllocationProp (enough of it, zeroed)
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int),
                ("loc_type", ctypes.c_int), ("loc_id", ctypes.c_int),
                ("win32", ctypes.c_void_p), ("compressionType", ctypes.c_ubyte),
                ("gpuDirectRDMACapable", ctypes.c_ubyte), ("usage", ctypes.c_ushort),
                ("pad", ctypes.c_ubyte * 64)]


def raw_cycle(export, nbytes=512 * MiB):
    f0 = free()
    p = Prop()
    p.type = 1          # hipMemAllocationTypePinned
    p.requestedHandleType = 1 if export else 0   # hipMemHandleTypePosixFileDescriptor
    p.loc_type = 1      # hipMemLocationTypeDevice
    p.loc_id = 0
    h = ctypes.c_void_p()
    rc = hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(nbytes), ctypes.byref(p),
                          ctypes.c_ulonglong(0))
    assert rc == 0, rc
    fd = ctypes.c_int(-1)
    if export:
        rc = hip.hipMemExportToShareableHandle(ctypes.byref(fd), h, 1, ctypes.c_ulonglong(0))
        assert rc == 0, rc
        os.close(fd.value)
    f1 = free()
    rc = hip.hipMemRelease(h)
    f2 = free()
    return {"raw": True, "export": export, "held_MiB": (f0 - f1) / MiB,
            "after_release_MiB": (f0 - f2) / MiB, "release_rc": rc}


out = []
for e in (False, True):
    out.append(raw_cycle(e))
from support import team as T  # noqa: E402
for P in (1, 3):
    tm = T.Team(P, 1 << 20, device=True)
    tm.activate()
    L = tm.lib
    f0 = free()
    for k in range(3):
        bases = {}

        def create(pe, k=k):
            b = ctypes.c_void_p()
            assert L.osgpu_heap_create(256 * MiB, 0, 0, P, tm.psync_ptr(pe), ctypes.byref(b)) == 0
            bases[pe] = b.value
        tm._on_members(list(range(P)), create)
        fc = free()
        for pe in range(P):
            assert L.osgpu_heap_destroy(ctypes.c_void_p(bases[pe])) == 0
        fd_ = free()
        out.append({"osgpu_heap": True, "P": P, "cycle": k, "held_MiB": (f0 - fc) / MiB,
                    "after_destroy_MiB": (f0 - fd_) / MiB})
for r in out:
    print(json.dumps(r), flush=True)
