#!/usr/bin/env python3
"""Sweep the host-staged path's knobs on one GPU (each setting in its own
process: HSA_* variables are read at runtime start).  Prints one JSON line
per setting.  Not part of the product."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
PES = int(os.environ.get("SWEEP_PES", "2"))

SETTINGS = json.loads(os.environ["SWEEP_SETTINGS"]) if os.environ.get("SWEEP_SETTINGS") else \
    [{}, {"OSGPU_HOST_BOUNCE": "0"}] if os.environ.get("SWEEP_BOUNCE") else [
    {},
    {"OSGPU_STAGE_BYTES": str(8 << 20)},
    {"OSGPU_STAGE_BYTES": str(128 << 20)},
    {"HSA_ENABLE_SDMA": "0"},
    {"HSA_ENABLE_SDMA": "0", "OSGPU_STAGE_BYTES": str(128 << 20)},
]

CODE = ("import sys, json; sys.path.insert(0, %r); import bench; "
        "print('RESULT ' + json.dumps(bench.host_staged_time(%d, pes=%d)))") % (ROOT, N, PES)

for s in SETTINGS:
    env = dict(os.environ, **s)
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    out = json.loads(line[0][7:]) if line else {"error": r.stderr[-500:]}
    out.pop("note", None)
    print(json.dumps({"env": s, "pes": PES, **out}), flush=True)
