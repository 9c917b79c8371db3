#!/usr/bin/env python3
"""PCIe ceiling of this MI355X host link, to read the host-staged path's
rate against: pinned H2D alone, D2H alone, and both at once on two streams
(1 GiB each).  Not part of the product."""
import json
import time

import torch

GB = 1e9
n = 1 << 30
h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def h2d():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)


def both():
    h2d()
    d2h()


r = {"h2d_GBs": n / timed(h2d) / GB, "d2h_GBs": n / timed(d2h) / GB}
t = timed(both)
r["bidir_each_way_GBs"] = n / t / GB
print(json.dumps(r))
