#!/usr/bin/env python3
"""graph_probe.py -- back-to-back combine launches (config 2: double sum,
K = 2, 64 Mi) submitted one by one vs as one captured HIP graph of the same
launches: wall time per launch over 50, and the kernel time (HIP events
around single launches).  Not part of the product."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
n = 64 << 20
a = torch.empty(n, dtype=torch.float64, device="cuda").uniform_(1, 2)
b = torch.empty(n, dtype=torch.float64, device="cuda").uniform_(1, 2)
o = torch.empty(n, dtype=torch.float64, device="cuda")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
K = 50
B = 3 * n * 8


def launch():
    assert L.osgpu_combine(5, 0, o.data_ptr(), srcs, 2, n, sp) == 0


torch.cuda.synchronize()
for _ in range(5):
    launch()
torch.cuda.synchronize()
res = {}
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(K):
        launch()
    torch.cuda.synchronize()
    res.setdefault("loop_us_per_launch", []).append((time.perf_counter() - t0) / K * 1e6)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    for _ in range(K):
        launch()
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    res.setdefault("graph_us_per_launch", []).append((time.perf_counter() - t0) / K * 1e6)
assert torch.equal(o, a + b)
res["frac_loop"] = [B / (u * 1e-6) / 8e12 for u in res["loop_us_per_launch"]]
res["frac_graph"] = [B / (u * 1e-6) / 8e12 for u in res["graph_us_per_launch"]]
print(json.dumps(res), flush=True)
