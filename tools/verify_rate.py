#!/usr/bin/env python3
"""Rate of the verification kernels (csrc/verify.hip) against the HBM
roofline: checksum of 1 GiB (one read stream) and compare of 2 x 1 GiB (two
read streams), median of 10 synchronous calls.  Not part of the product."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

nb = 1 << 30
a = torch.randint(0, 1 << 62, (nb // 8,), dtype=torch.int64, device="cuda")
b = a.clone()
torch.cuda.synchronize()
out = {}
for name, fn, bytes_ in (
        ("checksum_sum_long", lambda: osgpu.checksum("long", osgpu.CK_SUM, a.data_ptr(), nb // 8), nb),
        ("checksum_hash_long", lambda: osgpu.checksum("long", osgpu.CK_HASH, a.data_ptr(), nb // 8), nb),
        ("compare", lambda: osgpu.compare(a.data_ptr(), b.data_ptr(), nb), 2 * nb)):
    fn()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    out[name] = {"ms": t * 1e3, "GBs": bytes_ / t / 1e9, "frac_of_8TBs": bytes_ / t / 8e12}
# kernel-only: an empty call's fixed cost (memset + launch + read-back + sync)
e = torch.empty(16, dtype=torch.int64, device="cuda")
ts = []
for _ in range(20):
    t0 = time.perf_counter()
    osgpu.checksum("long", osgpu.CK_SUM, e.data_ptr(), 1)
    ts.append(time.perf_counter() - t0)
fixed = sorted(ts)[len(ts) // 2]
out["fixed_call_ms"] = fixed * 1e3
for k, v in list(out.items()):
    if isinstance(v, dict):
        b = nb * (2 if k == "compare" else 1)
        v["kernel_frac_of_8TBs_est"] = b / max(v["ms"] * 1e-3 - fixed, 1e-9) / 8e12
print(json.dumps(out))
