#!/usr/bin/env python3
"""copy_ceiling.py -- is the library's copy kernel the box's streaming
ceiling?  Same bytes (1.5 GiB read + 1.5 GiB written, the 128 Mi combine's
footprint; and 768 MiB each, config 2's) through osgpu_copy, hipMemcpyAsync
device-to-device (the runtime's blit), and torch's copy_.  HIP events, median
of 20.  Not part of the product; JSON lines on stdout."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
hip = ctypes.CDLL("libamdhip64.so")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)


def timed(fn, reps=20):
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


for nb in (768 << 20, 1536 << 20):
    a = torch.empty(nb, dtype=torch.uint8, device="cuda").fill_(1)
    o = torch.empty(nb, dtype=torch.uint8, device="cuda")
    D = (ctypes.c_void_p * 1)(o.data_ptr())
    S = (ctypes.c_void_p * 1)(a.data_ptr())
    N = (ctypes.c_size_t * 1)(nb)

    def k():
        assert L.osgpu_copy(D, S, N, 1, sp) == 0

    def m():
        assert hip.hipMemcpyAsync(ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(a.data_ptr()),
                                  ctypes.c_size_t(nb), 3, sp) == 0

    def t():
        with torch.cuda.stream(st):
            o.copy_(a)

    for name, fn in (("osgpu_copy", k), ("hipMemcpyAsync_D2D", m), ("torch_copy_", t)):
        sec = timed(fn)
        print(json.dumps({"copy": name, "bytes_each_way": nb, "us": sec * 1e6,
                          "frac_of_8TBs": 2 * nb / sec / 8e12}), flush=True)
    del a, o
    torch.cuda.empty_cache()
