#!/usr/bin/env python3
"""team_type_sweep.py -- the owner-computes team kernel (osgpu_team_combine:
one launch = every member's shard of a P-PE call) for every (type, op) at
P = 2, 4, 8 co-resident PEs, 128 MiB per array: HBM bytes per launch
2 * P * n * s (P source reads + P target writes).  HIP events on the launch
stream, median of 10.  One JSON line per kernel on stdout and in
gpurun_out/team_type_sweep.jsonl.  Not part of the product."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import osgpu  # noqa: E402

L = osgpu.load()
BYTES = int(os.environ.get("TT_BYTES", str(128 << 20)))
SIZE = {"short": 2, "int": 4, "long": 8, "longlong": 8, "float": 4, "double": 8,
        "longdouble": 16, "complexf": 8, "complexd": 16}
out = open(os.path.join(ROOT, "gpurun_out", "team_type_sweep.jsonl"), "a")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    torch.cuda.synchronize()
    for e0, e1 in ev:
        e0.record(st)
        fn()
        e1.record(st)
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev)
    return ts[len(ts) // 2]


srcs = [torch.empty(BYTES, dtype=torch.uint8, device="cuda") for _ in range(8)]
dsts = [torch.empty(BYTES, dtype=torch.uint8, device="cuda") for _ in range(8)]
g = torch.Generator(device="cuda").manual_seed(9)
for b in srcs:   # finite values of either sign in every type's encoding
    b.view(torch.float32).uniform_(-1.5, 1.5, generator=g)
PS = [int(p) for p in os.environ.get("TT_PS", "2,4,8").split(",")]
TS = os.environ.get("TT_TYPES", ",".join(osgpu.TYPES)).split(",")
for t in TS:
    n = BYTES // SIZE[t]
    if t == "longdouble":   # normal x87 values near 1 with random signs
        for b in srcs:
            v = b.view(torch.int64).view(-1, 2)
            v[:, 0] |= -(1 << 63)
            v[:, 1] = 0x3fff + (v[:, 1] & 3) - 1 + ((v[:, 1] >> 20) & 1) * 0x8000
    for op in osgpu.OPS:
        if not osgpu.has_op(t, op):
            continue
        for P in PS:
            S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs[:P]])
            D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts[:P]])
            ti, oi = osgpu.TYPES.index(t), osgpu.OPS.index(op)

            def f(S=S, D=D, ti=ti, oi=oi, P=P):
                assert L.osgpu_team_combine(ti, oi, P, D, S, n, sp) == 0

            sec = timeit(f)
            B = 2 * P * n * SIZE[t]
            rec = {"kernel": "team", "type": t, "op": op, "P": P, "us": sec * 1e6,
                   "GBs": B / sec / 1e9, "frac": B / sec / 8e12}
            print(json.dumps(rec), flush=True)
            out.write(json.dumps(rec) + "\n")
