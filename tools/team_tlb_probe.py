#!/usr/bin/env python3
"""team_tlb_probe.py -- is the 8-member team kernel's placement spread
(0.90-0.98 of the same-mix copy across fresh allocations, bench.py
roofline_team_by_members["8"]) address translation?

`run` (under rocprofv3 --pmc TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_MISS
TCP_UTCL1_THRASHING_STALL): TRIALS fresh placements of the 16 arrays
(8 sources + 8 targets of 64 Mi doubles); per placement 5 launches of the
team kernel (osgpu_team_combine, double sum, P = 8) and 5 of the
round-robin copy over the same arrays, each timed with HIP events; one JSON
line per placement.  `parse DIR LOG OUT`: the counters per launch, joined to
the placements in launch order, one JSON line per placement with the rate
beside the translation misses and thrashing stalls.  Not part of the
product.
"""
import csv
import ctypes
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "test-resilient-osss-ucx_amd")]
P, N, REPS = 8, 64 << 20, 5
TRIALS = int(os.environ.get("TT_TRIALS", "6"))
# the counters of the pass (TT_COUNTERS=a,b,... for another set, e.g. the
# L2's fabric requests TCC_EA0_RDREQ,TCC_EA0_WRREQ: step `teamea`)
COUNTERS = tuple(os.environ.get(
    "TT_COUNTERS", "TCP_UTCL1_REQUEST,TCP_UTCL1_TRANSLATION_MISS,TCP_UTCL1_THRASHING_STALL").split(","))


def run():
    import torch
    import osgpu
    L = osgpu.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    for trial in range(TRIALS):
        srcs_t = [torch.empty(N, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
                  for _ in range(P)]
        dsts_t = [torch.empty(N, dtype=torch.float64, device=dev) for _ in range(P)]
        S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in srcs_t])
        D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in dsts_t])
        NB = (ctypes.c_size_t * P)(*([N * 8] * P))
        torch.cuda.synchronize()
        out = {"trial": trial, "src_va_mod_2MiB": [x.data_ptr() % (2 << 20) for x in srcs_t]}
        for name, fn in (("team", lambda: L.osgpu_team_combine(5, 0, P, D, S, N, sp)),
                         ("copy", lambda: L.osgpu_copy(D, S, NB, P, sp))):
            ts = []
            for _ in range(REPS):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                assert fn() == 0
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            out[name + "_us_median"] = statistics.median(ts)
        out["team_over_copy"] = out["copy_us_median"] / out["team_us_median"]
        print(json.dumps(out), flush=True)
        del srcs_t, dsts_t
        torch.cuda.empty_cache()


def parse(d, log, dst):
    rows = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "")
                kind = "team" if "team_vec_kernel<double, 0, 8" in k else (
                    "copy" if "copy_vec_kernel" in k else None)
                if kind and r.get("Counter_Name") in COUNTERS:
                    rows.setdefault((kind, int(r["Dispatch_Id"])), {})[r["Counter_Name"]] = \
                        rows.get((kind, int(r["Dispatch_Id"])), {}).get(r["Counter_Name"], 0.0) + \
                        float(r["Counter_Value"])
    trials = [json.loads(l) for l in open(log) if l.startswith("{")]
    with open(dst, "w") as fo:
        for kind in ("team", "copy"):
            ids = sorted(i for (k, i) in rows if k == kind)
            for t in trials:
                mine = ids[t["trial"] * REPS:(t["trial"] + 1) * REPS]
                for c in COUNTERS:
                    v = [rows[(kind, i)].get(c, 0.0) for i in mine]
                    t[f"{kind}_{c}_median"] = statistics.median(v) if v else None
        for t in trials:
            fo.write(json.dumps(t) + "\n")
            print(json.dumps({k: t[k] for k in t if k != "src_va_mod_2MiB"}))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(*sys.argv[2:5])
