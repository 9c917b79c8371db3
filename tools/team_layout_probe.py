#!/usr/bin/env python3
"""team_layout_probe.py -- how much of the team kernel's rate at P members
is the placement of its 2P arrays?  (round 3: at P = 4 the same kernel ran
at 0.71-0.74 or 0.81-0.82 of 8 TB/s depending on which torch allocations it
got, profiles/r03_team_variants_interleaved.jsonl.)  Layouts:
  torch      P sources + P targets as separate torch allocations, made again
             for each of TL_REPEATS trials (allocator / driver placement)
  carved:S   one allocation, array k at k * (n*8 + S) (stride padding S)
For each: the team kernel (double sum, osgpu_team_combine) and the copy
kernel with P ranges on the same arrays, HIP-event span over REPS launches.
JSON lines on stdout.  Not part of the product."""
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
N = int(os.environ.get("TL_N", str(64 << 20)))
P = int(os.environ.get("TL_P", "4"))
nb = N * 8


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


def measure(layout, addrs):
    S = (ctypes.c_void_p * P)(*addrs[:P])
    D = (ctypes.c_void_p * P)(*addrs[P:])
    Nb = (ctypes.c_size_t * P)(*([nb] * P))

    def team():
        assert L.osgpu_team_combine(5, 0, P, D, S, N, sp) == 0

    def copy():
        assert L.osgpu_copy(D, S, Nb, P, sp) == 0

    B = 2 * P * nb
    tt, tc = span(team), span(copy)
    tt2 = span(team)
    t = min(tt, tt2)
    print(json.dumps({"P": P, "layout": layout, "team_us": t * 1e6, "team_frac": B / t / 8e12,
                      "copy_us": tc * 1e6, "copy_frac": B / tc / 8e12, "team_of_copy": tc / t,
                      "addr_mod_1GiB_MiB": [round((a % (1 << 30)) / (1 << 20), 1) for a in addrs]}),
          flush=True)


for trial in range(int(os.environ.get("TL_REPEATS", "4"))):
    arrs = [torch.empty(N, dtype=torch.float64, device="cuda").uniform_(1, 2) for _ in range(2 * P)]
    torch.cuda.synchronize()
    measure(f"torch#{trial}", [a.data_ptr() for a in arrs])
    del arrs
    torch.cuda.empty_cache()
for pad in [int(x) for x in os.environ.get("TL_PADS", "0,2097152,67108864,268435456").split(",")]:
    buf = torch.empty(2 * P * (nb + pad) + (2 << 20), dtype=torch.uint8, device="cuda")
    base = (buf.data_ptr() + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    addrs = [base + k * (nb + pad) for k in range(2 * P)]
    for a in addrs[:P]:
        osgpu.device_view(a, nb).view(torch.float64).uniform_(1, 2)
    torch.cuda.synchronize()
    measure(f"carved:{pad}", addrs)
    del buf
    torch.cuda.empty_cache()
