#!/usr/bin/env python3
"""ld_rocprof.py -- the long double team kernel's figure, rocprof-backed.

  run    (under rocprofv3 --kernel-trace --stats):  bench.py's own
         longdouble_team_rate (x87 soft-float team kernel, 8 members,
         4 Mi elements, 1.5 s warm-up by time, then 20 launches in one HIP
         event span -- random signs, then one sign), its JSON on stdout;
  parse  <rocprof dir> <bench json> <out json>: the dispatches of
         ld_team_kernel<0, 8, true> from the kernel trace, split into the
         two data sets by time; for each, the average over (a) every launch
         (what --stats averages: warm-up and ramp included) and (b) the 20
         launches of the timed window (the last 20 of the set), next to the
         bench's event-timed average from the same run.

Not part of the product.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "test-resilient-osss-ucx_amd")]
KERNEL = "ld_team_kernel<0, 8, true>"


def run():
    import torch
    import bench
    import osgpu
    L = osgpu.load()
    print(json.dumps(bench.longdouble_team_rate(L, torch)), flush=True)


def parse(d, bench_json, out_json):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    assert f, f"no kernel trace under {d}"
    rows = []
    for fn in f:
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                if KERNEL in r.get("Kernel_Name", ""):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    # the two data sets: split at the largest gap between dispatches (the
    # second set's input generation and synchronisation sit between them)
    gaps = [(rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
    cut = max(gaps)[1] + 1
    b = json.loads([l for l in open(bench_json) if l.startswith("{")][-1])
    out = {"kernel": "osgpu::x87::ld_team_kernel<SUM, 8>", "members": b["members"],
           "nreduce": b["nreduce"], "algorithmic_bytes_per_launch": b["algorithmic_bytes_per_launch"],
           "how": "rocprofv3 --kernel-trace of bench.py longdouble_team_rate (1.5 s warm-up, then "
                  "20 launches timed by one HIP event pair); rocprof averages over every launch "
                  "and over the last 20 (the timed window)"}
    B = b["algorithmic_bytes_per_launch"]
    for name, sel in (("random_signs", rows[:cut]), ("one_sign", rows[cut:])):
        durs = [(e - s) / 1e3 for s, e in sel]
        last = durs[-20:]
        ev = b[name]["kernel_avg_us"]
        span = (sel[-1][1] - sel[-20][0]) / 1e3 / 20
        rec = {"launches": len(durs), "rocprof_avg_all_us": sum(durs) / len(durs),
               "rocprof_avg_timed_window_us": sum(last) / len(last),
               "rocprof_span_timed_window_us_per_launch": span,
               "rocprof_min_us": min(durs), "event_avg_us": ev,
               "frac_event": B / (ev * 1e-6) / 8e12,
               "frac_rocprof_timed_window": B / (span * 1e-6) / 8e12,
               "frac_rocprof_all": B / (sum(durs) / len(durs) * 1e-6) / 8e12}
        rec["event_vs_rocprof_timed_window"] = ev / span
        out[name] = rec
    with open(out_json, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(*sys.argv[2:5])
