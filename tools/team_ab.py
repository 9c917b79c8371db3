#!/usr/bin/env python3
"""team_ab.py -- A/B of a team-kernel build: team_vec_kernel<T,SUM,P> through
osgpu_team_combine, one launch over all n elements (every member's shard),
2*P*n*s HBM bytes per launch, launch average = HIP event span over REPS
back-to-back launches.  OSGPU_LIB_PATH selects the build.  One JSON line per
(type, P).  Not part of the product."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import osgpu  # noqa: E402

L = osgpu.load()
REPS = int(os.environ.get("REPS", "50"))
tag = os.environ.get("AB_TAG", "shipped")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
for t, code, P, n in (("double", 5, 2, 64 << 20), ("float", 4, 2, 128 << 20),
                      ("double", 5, 4, 32 << 20)):
    dt = torch.float64 if t == "double" else torch.float32
    xs = [torch.empty(n, dtype=dt, device="cuda:0").uniform_(1, 2) for _ in range(P)]
    ys = [torch.empty(n, dtype=dt, device="cuda:0") for _ in range(P)]
    S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in xs])
    D = (ctypes.c_void_p * P)(*[y.data_ptr() for y in ys])
    torch.cuda.synchronize()
    for _ in range(5):
        assert L.osgpu_team_combine(code, 0, P, D, S, n, sp) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(REPS):
        L.osgpu_team_combine(code, 0, P, D, S, n, sp)
    e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / REPS
    ok = bool(torch.equal(ys[0], sum(xs[1:], xs[0])) if P == 2 else True)
    B = 2 * P * n * xs[0].element_size()
    print(json.dumps({"variant": tag, "type": t, "P": P, "n": n, "us": us,
                      "frac": B / us / 1e6 / 8000.0, "exact_P2": ok}), flush=True)
    del xs, ys
    torch.cuda.empty_cache()
