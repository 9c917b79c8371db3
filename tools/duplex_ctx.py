#!/usr/bin/env python3
"""Duplex H2D + D2H rate in THIS process after a bench step (argv[1], as in
tools/host_staged_context.py): 64 MiB copies on two streams created the way
the STAGED path creates its copy streams, from three kinds of host memory --
torch pinned, numpy registered with hipHostRegister (the bench's pinned
heap), hipHostMalloc.  Separates "the copies are slow" from "the staged
path's schedule is slow".  One JSON line.  Not part of the product."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "test-resilient-osss-ucx_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import osgpu  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
import host_staged_context as H  # noqa: E402

N = 64 << 20
prefix = sys.argv[1].split("+") if len(sys.argv) > 1 else ["none"]
g = {"bench": bench, "torch": torch, "osgpu": osgpu, "ctypes": ctypes, "N": N}
for p in prefix:
    exec(H.STEPS[p], g)
torch.cuda.synchronize()

hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
vp = ctypes.c_void_p


def ck(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


least, greatest = ctypes.c_int(), ctypes.c_int()
ck(hip.hipDeviceGetStreamPriorityRange(ctypes.byref(least), ctypes.byref(greatest)), "range")
s_in, s_out = vp(), vp()
ck(hip.hipStreamCreateWithPriority(ctypes.byref(s_in), 1, least), "stream in")
ck(hip.hipStreamCreateWithPriority(ctypes.byref(s_out), 1, greatest), "stream out")
d_in = torch.empty(N, dtype=torch.uint8, device="cuda")
d_out = torch.empty(N, dtype=torch.uint8, device="cuda").fill_(3)
torch.cuda.synchronize()
H2D, D2H = 1, 2


def rates(h_in, h_out):
    def run(pairs):
        best = 1e9
        for _ in range(4):
            t0 = time.perf_counter()
            for dst, src, kind, st in pairs:
                ck(hip.hipMemcpyAsync(vp(dst), vp(src), ctypes.c_size_t(N), kind, st), "copy")
            for *_, st in pairs:
                ck(hip.hipStreamSynchronize(st), "sync")
            best = min(best, time.perf_counter() - t0)
        return N / best / 1e9
    up = (d_in.data_ptr(), h_in, H2D, s_in)
    down = (h_out, d_out.data_ptr(), D2H, s_out)
    return {"h2d": run([up]), "d2h": run([down]), "duplex_each_way": run([up, down])}


out = {"prefix": prefix, "priorities": [least.value, greatest.value]}
tp_in = torch.empty(N, dtype=torch.uint8, pin_memory=True)
tp_out = torch.empty(N, dtype=torch.uint8, pin_memory=True)
out["torch_pinned"] = rates(tp_in.data_ptr(), tp_out.data_ptr())
a = np.ones(2 * N + 4096, dtype=np.uint8)
base = (a.ctypes.data + 4095) // 4096 * 4096
ck(hip.hipHostRegister(vp(base), ctypes.c_size_t(2 * N), 2), "register")  # mapped
out["numpy_registered"] = rates(base, base + N)
ck(hip.hipHostUnregister(vp(base)), "unregister")
hm_in, hm_out = vp(), vp()
ck(hip.hipHostMalloc(ctypes.byref(hm_in), ctypes.c_size_t(N), 0), "hostmalloc")
ck(hip.hipHostMalloc(ctypes.byref(hm_out), ctypes.c_size_t(N), 0), "hostmalloc")
out["hip_host_malloc"] = rates(hm_in.value, hm_out.value)
print(json.dumps(out), flush=True)
