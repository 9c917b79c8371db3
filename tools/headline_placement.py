#!/usr/bin/env python3
"""headline_placement.py -- the headline combine (double sum, K = 2,
64 Mi elements) on fresh allocations: each trial allocates a spacer of a
different size, then a, b and out (so their physical pages differ from
trial to trial), times 50 launches with one HIP event pair, and frees
everything.  The spread over trials
on one box, against the spread between leases of the bench line (236.7 to
251.4 us, profiles/r06_bench_run8..11.log), says whether the lease-to-lease
spread is placement.  Not part of the product; JSON lines on stdout and in
gpurun_out/headline_placement.jsonl."""
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
trials = int(os.environ.get("HP_TRIALS", "10"))
reps = 50
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
out_f = open(os.path.join(ROOT, "gpurun_out", "headline_placement.jsonl"), "a")
B = 3 * n * 8


def span(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


for trial in range(trials):
    spacer = torch.empty((trial * 37 + 1) << 20, dtype=torch.uint8, device=dev)
    a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
    b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
    o = torch.empty(n, dtype=torch.float64, device=dev)
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    torch.cuda.synchronize()

    def comb():
        assert L.osgpu_combine(5, 0, o.data_ptr(), srcs, 2, n, sp) == 0

    for _ in range(20):
        comb()
    t = span(comb)
    rec = {"trial": trial, "us": t * 1e6, "frac": B / t / 8e12,
           "a_mod_2MiB": a.data_ptr() % (2 << 20), "b_minus_a": b.data_ptr() - a.data_ptr(),
           "o_minus_a": o.data_ptr() - a.data_ptr()}
    print(json.dumps(rec), flush=True)
    out_f.write(json.dumps(rec) + "\n")
    del a, b, o, spacer
    torch.cuda.empty_cache()
