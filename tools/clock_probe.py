#!/usr/bin/env python3
"""clock_probe.py -- does a VALU-bound kernel run at the clock a memory-bound
one does?  Runs (1) the x87 team kernel (8-member long double sum, random
signs, 8 Mi elements: VALU-bound) and (2) the headline combine (double sum,
K = 2, 64 Mi: HBM-bound), each back to back for CP_SECONDS, timing every
launch with HIP events, while a thread samples `rocm-smi --showclocks
--showpower --json` every ~0.5 s.  One JSON line per phase: launch-time
percentiles and the sampled shader clock / socket power.  Not part of the
product."""
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
SECS = float(os.environ.get("CP_SECONDS", "8"))
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)
out = open(os.path.join(ROOT, "gpurun_out", "clock_probe.jsonl"), "a")


def smi_sampler(samples, stop):
    while not stop.is_set():
        t = time.time()
        try:
            r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--json"],
                               capture_output=True, text=True, timeout=10)
            d = json.loads(r.stdout)
            card = d[sorted(d)[0]]
            samples.append({"t": t, **{k: v for k, v in card.items()
                                       if "sclk" in k.lower() or "power" in k.lower()
                                       or "mclk" in k.lower() or "fclk" in k.lower()}})
        except Exception as e:  # keep sampling
            samples.append({"t": t, "error": repr(e)[:200]})
        time.sleep(0.5)


def run_phase(name, launch, nbytes):
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    samples, stop = [], threading.Event()
    th = threading.Thread(target=smi_sampler, args=(samples, stop), daemon=True)
    th.start()
    times = []
    t_end = time.time() + SECS
    while time.time() < t_end:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        launch()
        e1.record(st)
        e1.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3)
    stop.set()
    th.join(timeout=15)
    ts = sorted(times)
    pct = {p: ts[min(len(ts) - 1, int(p / 100 * len(ts)))] for p in (5, 50, 95)}
    rec = {"phase": name, "launches": len(ts), "us_p5": pct[5], "us_median": pct[50],
           "us_p95": pct[95], "frac_of_8TBs_median": nbytes / pct[50] / 8e6,
           "first_10_us": times[:10], "last_10_us": times[-10:], "smi": samples}
    line = json.dumps(rec)
    print(line, flush=True)
    out.write(line + "\n")


# (1) the x87 team kernel, 8 members, random signs
n, P = 8 << 20, 8
g = torch.Generator(device=dev).manual_seed(5)
srcs = []
for _ in range(P):
    v = torch.empty((n, 2), dtype=torch.int64, device=dev)
    v[:, 0] = torch.randint(-(1 << 62), 1 << 62, (n,), device=dev, generator=g) | (-(1 << 63))
    e = 0x3fff + torch.randint(-3, 4, (n,), device=dev, generator=g)
    v[:, 1] = e | (torch.randint(0, 2, (n,), device=dev, generator=g) << 15)
    srcs.append(v)
dsts = [torch.empty((n, 2), dtype=torch.int64, device=dev) for _ in range(P)]
S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs])
D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts])
torch.cuda.synchronize()
run_phase("x87_team_sum_8_random", lambda: L.osgpu_team_combine(6, 0, P, D, S, n, sp),
          2 * P * n * 16)
del srcs, dsts
torch.cuda.empty_cache()

# (2) the headline combine
n = 64 << 20
a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
o = torch.empty(n, dtype=torch.float64, device=dev)
AB = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
torch.cuda.synchronize()
run_phase("combine_double_sum_64Mi", lambda: L.osgpu_combine(5, 0, o.data_ptr(), AB, 2, n, sp),
          3 * n * 8)
