#!/usr/bin/env python3
"""reg_table.py -- per-kernel register use and occupancy from a gfx950 .s
(hipcc --save-temps).  Not part of the product.

  python tools/isa/reg_table.py team-hip-amdgcn-amd-amdhsa-gfx950.s [filter] [--json out]

For every kernel in the code object's metadata: VGPRs, AGPRs, SGPRs,
scratch bytes, spills and the waves per SIMD those registers allow.  On
CDNA3/4 the unified register file holds 512 registers per lane per SIMD;
a wave's allocation is VGPRs rounded up to the accumulation offset (4),
plus AGPRs, in granules of 8 -- waves/SIMD = min(8, 512 // alloc).
"""
import json
import re
import subprocess
import sys


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def parse(path):
    text = open(path).read()
    md = text[text.index("amdhsa.kernels:"):]
    recs = []
    for item in re.split(r"\n  - ", md)[1:]:
        f = dict(re.findall(r"\.(\w+):\s+(\S+)", item))
        if "name" not in f or f["name"].endswith(".kd"):
            continue
        recs.append(f)
    names = demangle([r["name"] for r in recs])
    rows = []
    for r, nm in zip(recs, names):
        v = int(r.get("vgpr_count", 0))
        a = int(r.get("agpr_count", 0))
        # vgpr_count already includes the AGPRs on gfx90a+ (unified file)
        # when agpr_count > 0; compute the allocation both ways and keep the
        # larger (conservative)
        alloc = max(v, ((v - a + 3) // 4) * 4 + a) if a else v
        alloc = ((alloc + 7) // 8) * 8
        rows.append({"kernel": nm, "vgpr": v, "agpr": a, "sgpr": int(r.get("sgpr_count", 0)),
                     "scratch": int(r.get("private_segment_fixed_size", 0)),
                     "vgpr_spill": int(r.get("vgpr_spill_count", 0)),
                     "waves_per_simd": min(8, 512 // max(alloc, 1))})
    return rows


def main():
    path = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    rows = [r for r in parse(path) if not flt or flt in r["kernel"]]
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    for r in rows:
        print(f"{r['vgpr']:4d} {r['agpr']:3d} {r['scratch']:5d} {r['waves_per_simd']}  {r['kernel']}")


if __name__ == "__main__":
    main()
