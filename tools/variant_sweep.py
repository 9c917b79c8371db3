#!/usr/bin/env python3
"""Time double-sum combines (K = 2..8 inputs, 512 MiB each) for every
library variant in tools/variants/ (each in its own process).  Not part of
the product."""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import ctypes, json, sys, torch
sys.path.insert(0, %r)
import osgpu
L = osgpu.load()
BYTES = 512 << 20
bufs = [torch.empty(BYTES, dtype=torch.uint8, device="cuda") for _ in range(9)]
for b in bufs: b.view(torch.float64).uniform_(1, 2)
s = torch.cuda.Stream()
res = {}
for K in (2, 3, 4, 6, 8):
    srcs = (ctypes.c_void_p * K)(*[bufs[j].data_ptr() for j in range(K)])
    n = BYTES // 8
    f = lambda: L.osgpu_combine(5, 0, bufs[8].data_ptr(), srcs, K, n, ctypes.c_void_p(s.cuda_stream))
    for _ in range(3): f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s); f(); e1.record(s); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    ts.sort()
    res["K%%d" %% K] = round((K + 1) * BYTES / ts[len(ts) // 2] / 1e9, 1)
print("RESULT " + json.dumps(res))
''' % os.path.join(ROOT, "test-resilient-osss-ucx_amd")
for so in sorted(glob.glob(os.path.join(ROOT, "tools", "variants", "*", "libosgpu_reduce.so"))):
    env = dict(os.environ, OSGPU_LIB_PATH=so)
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True,
                       timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    print(os.path.basename(os.path.dirname(so)), line[0][7:] if line else r.stderr[-300:],
          flush=True)
