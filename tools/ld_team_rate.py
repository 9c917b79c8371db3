#!/usr/bin/env python3
"""ld_team_rate.py -- the long double (x87 soft-float) team kernel alone:
osgpu_team_combine(longdouble, sum|prod, P) over n elements (one launch =
every member's shard of a P-PE call), HIP events on its stream, median of
REPS.  HBM bytes per launch 2 * P * n * 16 (P 16-B reads + P 16-B writes per
element).  Data: "ones" (every element 1.0: exponent difference 0), "random" (random
64-bit significands, exponents 2^-3..2^3, random signs) or "positive" (the
same, all positive: sums of one sign take the addition-only fast add).
Not part of the product; JSON lines on stdout and gpurun_out/ld_team_rate.jsonl."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
n = int(os.environ.get("LD_N", str(8 << 20)))
REPS = int(os.environ.get("REPS", "20"))
out = open(os.path.join(ROOT, "gpurun_out", "ld_team_rate.jsonl"), "a")
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
g = torch.Generator(device=dev).manual_seed(5)
# LD_ONLY="sum/random/8": one case (e.g. for a PMC pass)
only = os.environ.get("LD_ONLY")
for op_name, op in (("sum", 0), ("prod", 1)):
    for dist in ("ones", "random", "positive"):
        for P in (2, 4, 8):
            if only and only != f"{op_name}/{dist}/{P}":
                continue
            srcs = []
            for p in range(P):
                v = torch.empty((n, 2), dtype=torch.int64, device=dev)
                if dist == "ones":
                    v[:, 0] = -(1 << 63)
                    v[:, 1] = 0x3fff
                else:
                    v[:, 0] = torch.randint(-(1 << 62), 1 << 62, (n,), device=dev, generator=g) | (-(1 << 63))
                    e = 0x3fff + torch.randint(-3, 4, (n,), device=dev, generator=g)
                    sgn = torch.randint(0, 2, (n,), device=dev, generator=g) << 15
                    v[:, 1] = e | (sgn if dist == "random" else 0)
                srcs.append(v)
            dsts = [torch.empty((n, 2), dtype=torch.int64, device=dev) for _ in range(P)]
            S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs])
            D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts])
            torch.cuda.synchronize()
            for _ in range(2):
                assert L.osgpu_team_combine(6, op, P, D, S, n, sp) == 0
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(REPS)]
            for e0, e1 in ev:
                e0.record(st)
                L.osgpu_team_combine(6, op, P, D, S, n, sp)
                e1.record(st)
            torch.cuda.synchronize()
            ts = sorted(e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev)
            med = ts[len(ts) // 2]
            B = 2 * P * n * 16
            rec = {"type": "longdouble", "op": op_name, "dist": dist, "P": P, "nreduce": n,
                   "kernel_us": med * 1e6, "GBs": B / med / 1e9, "frac_of_8TBs": B / med / 8e12,
                   "pe0_equals_pe1": bool(torch.equal(dsts[0], dsts[1]))}
            print(json.dumps(rec), flush=True)
            out.write(json.dumps(rec) + "\n")
            del srcs, dsts
            torch.cuda.empty_cache()
