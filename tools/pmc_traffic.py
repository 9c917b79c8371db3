#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py into HBM
bytes per launch of the combine kernel (profiles/<round>_traffic.json).

Corrections (MI355X_MICROARCH.md, section HBM / rocprofv3 PMC):
  * FETCH_SIZE and WRITE_SIZE are in KiB;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
    streaming read (16 B/lane) -> doubled;
  * WRITE_SIZE is exact for 16-B-per-lane streaming stores.
The two counters come from separate passes (FETCH_SIZE needs 3 TCC slots,
WRITE_SIZE 2; they do not fit one pass).

usage: pmc_traffic.py FETCH_DIR WRITE_DIR NREDUCE OUT.json [KERNEL [BYTES_PER_ELEM]]
  KERNEL          substring of the kernel name (default the K=2 double-sum
                  combine); BYTES_PER_ELEM algorithmic bytes per element per
                  launch (default 24 = 2 reads + 1 write of 8 B; the team
                  kernel at P = 2: 32)
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = "combine_vec_kernel<double, 0, 2>"


def values(d, counter):
    global KERNEL
    vals = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for row in csv.DictReader(f):
                if KERNEL in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    global KERNEL
    fdir, wdir, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    if len(sys.argv) > 5:
        KERNEL = sys.argv[5]
    per_elem = int(sys.argv[6]) if len(sys.argv) > 6 else 24
    f = values(fdir, "FETCH_SIZE")
    w = values(wdir, "WRITE_SIZE")
    if not f or not w:
        sys.exit(f"no counter rows for {KERNEL} (fetch {len(f)}, write {len(w)})")
    fk, wk = statistics.median(f), statistics.median(w)
    read_b = 2.0 * fk * 1024.0
    write_b = wk * 1024.0
    alg = per_elem * n
    res = {
        "kernel": KERNEL, "nreduce": n, "launches": [len(f), len(w)],
        "FETCH_SIZE_KiB_median": fk, "WRITE_SIZE_KiB_median": wk,
        "read_bytes": read_b, "write_bytes": write_b,
        "bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                  "bench.py; FETCH_SIZE x2 (gfx950 half-count on 16-B streaming reads), "
                  "KiB -> bytes",
    }
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
