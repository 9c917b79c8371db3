#!/usr/bin/env python3
"""team_offsets.py -- does the relative placement of the P sources and P
targets change the team kernel's rate (DRAM bank/row correlation of the
2P streams one wave touches at the same index)?  The arrays are carved
from one allocation at base + k*(n*8 + k*delta) for a sweep of delta; the
team kernel (osgpu_team_combine, double sum) and, as the same-mix
reference, the copy kernel with P ranges (osgpu_copy) are timed with one
HIP-event span over REPS launches.  JSON lines on stdout.  Not part of the
product."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
REPS = int(os.environ.get("REPS", "20"))
N = int(os.environ.get("TO_N", str(64 << 20)))
PS = [int(x) for x in os.environ.get("TO_P", "2,4").split(",")]
DELTAS = [int(x) for x in os.environ.get(
    "TO_DELTAS", "0,256,4096,65536,1048576,2097152,3145728").split(",")]


def span(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(REPS):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / REPS


for P in PS:
    nb = N * 8
    maxd = max(DELTAS)
    buf = torch.empty(2 * P * (nb + 2 * P * maxd) + (1 << 21), dtype=torch.uint8, device="cuda")
    base = (buf.data_ptr() + (1 << 21) - 1) // (1 << 21) * (1 << 21)
    for d in DELTAS:
        addr = [base + k * nb + (k * (k + 1) // 2) * d for k in range(2 * P)]
        srcs = (ctypes.c_void_p * P)(*addr[:P])
        dsts = (ctypes.c_void_p * P)(*addr[P:])
        for a in addr[:P]:
            osgpu.device_view(a, nb).view(torch.float64).fill_(1.25)
        torch.cuda.synchronize()
        N_ = (ctypes.c_size_t * P)(*([nb] * P))

        def team():
            assert L.osgpu_team_combine(5, 0, P, dsts, srcs, N, sp) == 0

        def copy():
            assert L.osgpu_copy(dsts, srcs, N_, P, sp) == 0

        B = 2 * P * nb
        tt, tc = span(team), span(copy)
        print(json.dumps({"P": P, "delta": d, "team_us": tt * 1e6, "team_frac": B / tt / 8e12,
                          "copy_us": tc * 1e6, "copy_frac": B / tc / 8e12,
                          "team_of_copy": tc / tt}), flush=True)
    del buf
    torch.cuda.empty_cache()
