#!/usr/bin/env python3
"""Placement census: how often does a fresh allocation make a streaming
kernel collapse, and which array is slow when it does?  (VERDICT r04 item
2: a 4-member placement at 0.369 of 8 TB/s; round 5 saw the COPY kernel at
0.312 on one allocation.)  Each trial frees everything, allocates P source
and P target arrays of n doubles afresh (torch, cache emptied), and times
  * the team kernel (double sum) and the same-mix copy over all P pairs,
  * each pair src_i -> dst_i alone through the copy kernel.
One JSON line per trial.  Not part of the product.
    python tools/placement_census.py [trials=30] [P=4] [n=64Mi]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import osgpu  # noqa: E402

TRIALS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
N = int(sys.argv[3]) if len(sys.argv) > 3 else 64 << 20
REPS = 8
L = osgpu.load()
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def span(f):
    f()
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(REPS):
        f()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


for trial in range(TRIALS):
    torch.cuda.empty_cache()
    xs = [torch.empty(N, dtype=torch.float64, device="cuda:0").uniform_(1, 2) for _ in range(P)]
    ys = [torch.empty(N, dtype=torch.float64, device="cuda:0") for _ in range(P)]
    S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in xs])
    D = (ctypes.c_void_p * P)(*[y.data_ptr() for y in ys])
    NB = (ctypes.c_size_t * P)(*([N * 8] * P))
    torch.cuda.synchronize()
    B = 2 * P * N * 8
    tt = span(lambda: L.osgpu_team_combine(5, 0, P, D, S, N, sp))
    tc = span(lambda: L.osgpu_copy(D, S, NB, P, sp))
    pair = []
    for i in range(P):
        Di = (ctypes.c_void_p * 1)(ys[i].data_ptr())
        Si = (ctypes.c_void_p * 1)(xs[i].data_ptr())
        Ni = (ctypes.c_size_t * 1)(N * 8)
        t = span(lambda: L.osgpu_copy(Di, Si, Ni, 1, sp))
        pair.append(round(2 * N * 8 / t / 8e6, 4))
    print(json.dumps({"trial": trial, "P": P, "team_frac": B / tt / 8e6, "copy_frac": B / tc / 8e6,
                      "pair_copy_frac": pair,
                      "src": [hex(x.data_ptr()) for x in xs], "dst": [hex(y.data_ptr()) for y in ys]}),
          flush=True)
    del xs, ys
