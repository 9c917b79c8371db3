#!/usr/bin/env python3
"""Per-call latency of shmem_int_sum_to_all with one PROCESS per PE sharing
cuda:0 (IPC device heaps, shared-memory runtime barrier): fused one-launch
path (device-side barriers) vs host barriers, team and pull form.  Launches
tests/support/mp_worker.py in `latency` mode; prints one JSON line per world
size.  Not part of the product."""
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "support", "mp_worker.py")


def run(world):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tempfile.mkdtemp()
    mode = os.environ.get("MP_MODE", "latency")  # another worker mode: debugging runs
    procs = [subprocess.Popen([sys.executable, WORKER, mode, out],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(world),
                                       LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=str(port)))
             for r in range(world)]
    rcs = [p.wait(timeout=600) for p in procs]
    assert rcs == [0] * world, rcs
    if mode != "latency":
        return mode + " ok"
    return json.load(open(os.path.join(out, "rank0.json")))["latency"]


if __name__ == "__main__":
    for world in [int(w) for w in os.environ.get("MP_WORLDS", "2,4").split(",")]:
        print(json.dumps({"probe": "mp_latency", "pes": world, "processes": world,
                          "gpus": 1, "latency": run(world)}), flush=True)
