#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into HBM bytes per
launch of one kernel (profiles/<round>_traffic*.json; bench.py's live
traffic uses traffic() on its own passes over tools/pmc_probe.py).

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
                  kernel at P members: 16 * P)
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL = "combine_lds_kernel<double, 0, 2, 2>"  # bench.COMBINE_KERNEL
METHOD = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 "
          "(gfx950 half-count on 16-B streaming reads), KiB -> bytes, median over launches")


def values(d, counter, kernel=KERNEL):
    vals = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for row in csv.DictReader(f):
                if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def traffic(fdir, wdir, n, kernel=KERNEL, per_elem=24):
    """dict of the per-launch HBM bytes of `kernel`, or None without rows"""
    f = values(fdir, "FETCH_SIZE", kernel)
    w = values(wdir, "WRITE_SIZE", kernel)
    if not f or not w:
        return None
    fk, wk = statistics.median(f), statistics.median(w)
    read_b = 2.0 * fk * 1024.0
    write_b = wk * 1024.0
    alg = per_elem * n
    return {
        "kernel": kernel, "nreduce": n, "launches": [len(f), len(w)],
        "FETCH_SIZE_KiB_median": fk, "WRITE_SIZE_KiB_median": wk,
        "read_bytes": read_b, "write_bytes": write_b,
        "bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "method": METHOD,
    }


def main():
    fdir, wdir, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    kernel = sys.argv[5] if len(sys.argv) > 5 else KERNEL
    per_elem = int(sys.argv[6]) if len(sys.argv) > 6 else 24
    res = traffic(fdir, wdir, n, kernel, per_elem)
    if res is None:
        sys.exit(f"no counter rows for {kernel}")
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
