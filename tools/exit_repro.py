#!/usr/bin/env python3
"""Bisect an abort at interpreter exit seen after C-thread (pthread) PEs
called the library on device heaps.  usage: exit_repro.py MODE.  Not part
of the product."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("test-resilient-osss-ucx_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import osgpu  # noqa: E402
from support import team as T  # noqa: E402

mode = sys.argv[1]
n = 1024
tm = T.Team(2, 2 * n * 4 + 8192, device=True)
toff = 4096
if mode.startswith("pyth"):
    tm.run("int", "sum", toff, 0, n)
else:
    sig = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
           ctypes.c_int, ctypes.c_int]
    tm.pet.pet_time_to_all.restype = ctypes.c_double
    tm.pet.pet_time_to_all.argtypes = sig
    fn = ctypes.cast(tm.lib.shmem_int_sum_to_all, ctypes.c_void_p)
    tgt = (ctypes.c_void_p * 2)(tm.ptr(0, toff), tm.ptr(1, toff))
    src = (ctypes.c_void_p * 2)(tm.ptr(0, 0), tm.ptr(1, 0))
    tm.pet.pet_time_to_all(fn, 2, tgt, src, None, n, 1)
if "fin" in mode:
    tm.lib.osgpu_finalize()
if "del" in mode:
    del tm
if "exit0" in mode:
    sys.stdout.flush()
    os._exit(0)
print("end of script", flush=True)
