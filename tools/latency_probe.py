#!/usr/bin/env python3
"""Per-call latency of shmem_int_sum_to_all at small nreduce (BASELINE
config 1 shape: 2 PEs), device-resident (team / pull paths) and
host-resident (staged path), timed in C (pet_time_to_all), next to the CPU
reference loop shape.  Not part of the product."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("test-resilient-osss-ucx_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import osgpu  # noqa: E402
import oracle as O  # noqa: E402
from support import team as T  # noqa: E402

sig = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
       ctypes.c_int, ctypes.c_int]
out = {}
mode = os.environ.get("PROBE_TAG", "")
KINDS = [k == "1" for k in os.environ.get("PROBE_KINDS", "10").split(",")] if os.environ.get("PROBE_KINDS") else (True, False)
FIN = os.environ.get("PROBE_FINALIZE", "1") == "1"
SIZES = [int(x) for x in os.environ.get("PROBE_SIZES", "1024,65536,1048576").split(",")]
for n in SIZES:
    row = {}
    for device in KINDS:
        tm = T.Team(2, 2 * n * 4 + 8192, device=device)
        tm.pet.pet_time_to_all.restype = ctypes.c_double
        tm.pet.pet_time_to_all.argtypes = sig
        toff = (n * 4 + 4095) // 4096 * 4096
        fn = ctypes.cast(tm.lib.shmem_int_sum_to_all, ctypes.c_void_p)
        tgt = (ctypes.c_void_p * 2)(tm.ptr(0, toff), tm.ptr(1, toff))
        src = (ctypes.c_void_p * 2)(tm.ptr(0, 0), tm.ptr(1, 0))
        if device:
            # host barriers (fused off) vs one launch with device barriers
            paths = (("team", osgpu.PATH_AUTO, 0), ("pull", osgpu.PATH_PULL, 0),
                     ("fused_team", osgpu.PATH_AUTO, 1 << 30),
                     ("fused_pull", osgpu.PATH_PULL, 1 << 30))
            sel = os.environ.get("PROBE_PATHS")
            if sel:
                paths = [p for p in paths if p[0] in sel.split(",")]
            ps = (ctypes.c_void_p * 2)(tm.psync_ptr(0), tm.psync_ptr(1))
            for name, path, lim in paths:
                tm.lib.osgpu_set_path(path)
                tm.lib.osgpu_set_fused_max_bytes(lim)
                row[name + "_us"] = tm.pet.pet_time_to_all(
                    fn, 2, tgt, src, ps, n, int(os.environ.get("PROBE_REPS", "200"))) * 1e6
            tm.lib.osgpu_set_path(osgpu.PATH_AUTO)
            tm.lib.osgpu_set_fused_max_bytes(-1)
        else:
            ps = (ctypes.c_void_p * 2)(tm.ptr(0, tm.psync_off), tm.ptr(1, tm.psync_off))
            row["host_staged_us"] = tm.pet.pet_time_to_all(fn, 2, tgt, src, ps, n, 200) * 1e6
        if FIN:
            tm.lib.osgpu_finalize()
        del tm
    srcs = O.team_inputs("int", 2, n, 5, "bits")
    row["cpu_reference_loop_us"] = O.cpu_baseline("int", "sum", srcs, reps=200, pin=True) * 1e6
    out[n] = row
    print(json.dumps({"tag": mode, "nreduce": n, **row}), flush=True)
