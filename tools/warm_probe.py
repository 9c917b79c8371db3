#!/usr/bin/env python3
"""warm_probe.py -- does the headline combine run slower at the start of a
process (clock / power-state ramp) and what separates back-to-back launches?
Not part of the product; one MI355X.

  trend   from a cold process: 400 launches of combine_vec_kernel<double,SUM,2>
          at 64 Mi, HIP events around every launch; per-launch times reported
          as medians over windows of launches (1-10, 11-50, 51-100, ...), with
          the wall clock of each window
  gap     the same launches with events only at the two ends (wall per launch
          and event span per launch) vs with events around every launch
JSON lines on stdout and in gpurun_out/warm_probe.jsonl."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
OUT = open(os.path.join(ROOT, "gpurun_out", "warm_probe.jsonl"), "a")
dev = torch.device("cuda:0")
n = int(os.environ.get("WP_N", str(64 << 20)))
B = 3 * n * 8


def emit(d):
    line = json.dumps(d)
    print(line, flush=True)
    OUT.write(line + "\n")
    OUT.flush()


a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
o = torch.empty(n, dtype=torch.float64, device=dev)
st = torch.cuda.Stream(device=dev)
sp = ctypes.c_void_p(st.cuda_stream)
srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
torch.cuda.synchronize()


def launch():
    assert L.osgpu_combine(5, 0, o.data_ptr(), srcs, 2, n, sp) == 0


def trend(total=400):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(total)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record(st)
        launch()
        e1.record(st)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ks = [e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev]
    starts = [ev[0][0].elapsed_time(e0) * 1e-3 for e0, _ in ev]
    wins = [(0, 10), (10, 50), (50, 100), (100, 200), (200, 300), (300, 400)]
    rows = []
    for lo, hi in wins:
        w = sorted(ks[lo:hi])
        span = (starts[hi - 1] + ks[hi - 1] - starts[lo]) / (hi - lo)
        rows.append({"launches": f"{lo + 1}-{hi}", "median_us": w[len(w) // 2] * 1e6,
                     "min_us": w[0] * 1e6, "frac_median": B / w[len(w) // 2] / 8e12,
                     "span_per_launch_us": span * 1e6})
    emit({"probe": "trend", "n": n, "total_wall_ms": wall * 1e3, "windows": rows})


def gap(reps=100):
    out = {"probe": "gap", "n": n}
    for mode in ("ends", "every"):
        torch.cuda.synchronize()
        if mode == "ends":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(reps):
                launch()
            e1.record(st)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            out[mode] = {"wall_per_launch_us": wall / reps * 1e6,
                         "event_span_per_launch_us": e0.elapsed_time(e1) * 1e3 / reps}
        else:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(reps)]
            t0 = time.perf_counter()
            for x0, x1 in ev:
                x0.record(st)
                launch()
                x1.record(st)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            ks = [x0.elapsed_time(x1) * 1e-3 for x0, x1 in ev]
            out[mode] = {"wall_per_launch_us": wall / reps * 1e6,
                         "kernel_avg_us": sum(ks) / reps * 1e6,
                         "event_span_per_launch_us": ev[0][0].elapsed_time(ev[-1][1]) * 1e3 / reps}
    emit(out)


if __name__ == "__main__":
    for p in (sys.argv[1:] or ["trend", "gap", "trend"]):
        globals()[p]()
