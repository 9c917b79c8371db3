#!/usr/bin/env python3
"""Does the relative placement of the combine's three streams (two inputs,
one output) in HBM change its rate?  Carves a, b, out from one allocation
at offsets 0, S + da, 2S + db and times osgpu_combine (double sum, K = 2,
64 Mi elements) with HIP events on its stream.  Not part of the product."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
n = 64 << 20
S = n * 8
buf = torch.empty(3 * S + (64 << 20), dtype=torch.uint8, device="cuda:0")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
for da, db in ((0, 0), (4096, 8192), (1 << 20, 2 << 20), (256, 512), (2048, 4096),
               (64 << 10, 128 << 10), (3 << 20, 7 << 20), (12288, 20480)):
    base = buf.data_ptr()
    a, b, o = base, base + S + da, base + 2 * S + db
    srcs = (ctypes.c_void_p * 2)(a, b)
    torch.cuda.synchronize()
    for _ in range(5):
        L.osgpu_combine(5, 0, o, srcs, 2, n, sp)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(30)]
    for e0, e1 in ev:
        e0.record(st)
        L.osgpu_combine(5, 0, o, srcs, 2, n, sp)
        e1.record(st)
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    med = ts[len(ts) // 2] * 1e-3
    print(json.dumps({"da": da, "db": db, "us_median": med * 1e6,
                      "TBps": 3 * S / med / 1e12, "frac": 3 * S / med / 8e12}), flush=True)
