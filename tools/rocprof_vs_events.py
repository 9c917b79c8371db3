#!/usr/bin/env python3
"""rocprof_vs_events.py -- the headline kernel's average duration in a
rocprofv3 kernel trace of the driver's own N=1 command against the line's
HIP-event figure (`roofline.kernel_avg_us`), plus every team kernel's rocprof
average.  Not part of the product.

  python tools/rocprof_vs_events.py PROF_DIR BENCH_LOG OUT_JSON

PROF_DIR holds run_kernel_trace.csv / run_kernel_stats.csv from
`rocprofv3 --kernel-trace --stats -d PROF_DIR -o run --output-format csv --
python3 bench.py --gpus 1 --steps K --warmup W` (tools/gpu_round.sh step
`proffull`).  Bursts: launches of the headline kernel at the full grid less
than 1 ms apart; the timed region is the first burst of at least K launches (the W warm-up
launches form a shorter burst before it)."""
import collections
import csv
import json
import os
import statistics
import sys


def main(prof, bench_log, out_path):
    line = None
    for text in open(bench_log):
        if text.startswith("{"):
            line = json.loads(text)
    steps, warmup = line["steps"], line["warmup"]
    rows = list(csv.DictReader(open(os.path.join(prof, "run_kernel_trace.csv"))))
    head = [r for r in rows if "combine_lds_kernel<double, 0, 2, 2>" in r["Kernel_Name"]]
    # the headline shape is the most launched one (the 128 Mi north-star
    # launches come later, fewer)
    grid = collections.Counter(int(r["Grid_Size_X"]) for r in head).most_common(1)[0][0]
    head = sorted((r for r in head if int(r["Grid_Size_X"]) == grid),
                  key=lambda r: int(r["Start_Timestamp"]))
    bursts, cur = [], [head[0]]
    for a, b in zip(head, head[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) < 1_000_000:
            cur.append(b)
        else:
            bursts.append(cur)
            cur = [b]
    bursts.append(cur)
    # the warm-up launches are a burst of their own (bench.py synchronises and
    # sets the timed region up after them)
    burst = next(b for b in bursts if len(b) >= steps)
    timed = burst[:steps]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in timed]
    span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e3 / steps
    stats = list(csv.DictReader(open(os.path.join(prof, "run_kernel_stats.csv"))))
    team = {r["Name"].split("(")[0].replace("void osgpu::", ""):
            {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
            for r in stats if "team_" in r["Name"]}
    out = {"kernel": "combine_lds_kernel<double, 0, 2, 2>", "grid": grid,
           "command": f"rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 "
                      f"--steps {steps} --warmup {warmup}",
           "timed_region_launches": len(timed),
           "avg_duration_us_timed": statistics.mean(dur),
           "span_per_launch_us_timed": span,
           "all_full_grid_launches": len(head),
           "median_us_all": statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                                              for r in head),
           "bench_line_kernel_avg_us": line["roofline"].get("kernel_avg_us"),
           "bench_line_frac": line["roofline"]["frac"],
           "team_kernels_rocprof": team}
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
