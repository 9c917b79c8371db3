#!/usr/bin/env python3
"""Roofline of every (type, op) combine kernel on one MI355X: K = 2 and 8
inputs, 512 MiB per input array; and the owner-computes team kernel for
P = 2, 4, 8 co-resident PEs (double sum).  HIP events on the launch stream,
median of 10.  One JSON line per kernel.  Not part of the product."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import osgpu  # noqa: E402

L = osgpu.load()
BYTES = 512 << 20
SIZE = {"short": 2, "int": 4, "long": 8, "longlong": 8, "float": 4, "double": 8,
        "longdouble": 16, "complexf": 8, "complexd": 16}


def timeit(fn, reps=10):
    s = torch.cuda.Stream()
    for _ in range(3):
        fn(s.cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn(s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2]


bufs = [torch.empty(BYTES, dtype=torch.uint8, device="cuda") for _ in range(9)]
for b in bufs:
    b.view(torch.float32).uniform_(0.5, 1.5)   # finite, non-NaN bit patterns for every type
out = bufs[8]
KS = [int(k) for k in os.environ.get("TS_KS", "2,8").split(",")]
TS = os.environ.get("TS_TYPES", ",".join(osgpu.TYPES)).split(",")
for K in KS:
    for t in TS:
        for op in osgpu.OPS:
            if not osgpu.has_op(t, op):
                continue
            n = BYTES // SIZE[t]
            srcs = (ctypes.c_void_p * K)(*[bufs[j].data_ptr() for j in range(K)])
            ti, oi = osgpu.TYPES.index(t), osgpu.OPS.index(op)

            def f(stream, srcs=srcs, ti=ti, oi=oi, n=n):
                rc = L.osgpu_combine(ti, oi, out.data_ptr(), srcs, K, n, ctypes.c_void_p(stream))
                assert rc == 0

            sec = timeit(f)
            B = (K + 1) * BYTES
            print(json.dumps({"kernel": "combine", "type": t, "op": op, "K": K,
                              "us": sec * 1e6, "GBs": B / sec / 1e9,
                              "frac": B / sec / 8e12}), flush=True)
torch.cuda.synchronize()
