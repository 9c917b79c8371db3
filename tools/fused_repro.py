#!/usr/bin/env python3
"""Minimal fused-path call (2..3 PEs as threads on cuda:0) with the debug
trace on; prints the path taken and checks the result against the oracle.
Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("test-resilient-osss-ucx_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import numpy as np  # noqa: E402
import oracle as O  # noqa: E402
from support import team as T  # noqa: E402

P = int(os.environ.get("P", "2"))
n = int(os.environ.get("N", "1000"))
t, op = os.environ.get("T", "double"), os.environ.get("OP", "sum")
tm = T.Team(P, 2 * n * 16 + 8192, device=True)
src = O.team_inputs(t, P, n, 0x5EED, "wide")
s = src[0].dtype.itemsize
toff = (n * s + 4095) // 4096 * 4096
for pe in range(P):
    tm.write(pe, 0, src[pe])
tm.run(t, op, toff, 0, n)
print("paths", tm.last_paths, flush=True)
want = O.to_all(t, op, src)
for pe in range(P):
    got = tm.read(pe, toff, n * s).view(want[pe].dtype)
    print("PE", pe, "bit-exact", np.array_equal(got.view(np.uint8), want[pe].view(np.uint8)),
          flush=True)
