#!/usr/bin/env python3
"""crossover.py -- where the drop-in starts beating the reference's loop for
small calls (BASELINE config 1's shape: shmem_int_sum_to_all, 2 PEs).
GPU: 2 PE processes sharing cuda:0 (IPC device heaps, shared-memory runtime;
tools/mp_latency.py): median per call barrier to barrier of the fused
one-launch path and of the host-barrier team path, device heaps, and the
fused staged path on a pinned host heap (config 1's own placement).  CPU:
the reference's loop shape (oracle/oracle_reduce.c) on 2 pinned cores, same
sizes.  One JSON line per size on stdout and gpurun_out/crossover.jsonl.
Not part of the product."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle")]
SIZES = [int(x) for x in os.environ.get(
    "XO_SIZES", "256,1024,2048,4096,8192,16384,32768,65536").split(",")]


def main():
    import oracle as O
    env = dict(os.environ, MP_WORLDS="2", MP_SIZES=",".join(map(str, SIZES)),
               MP_REPS=os.environ.get("XO_REPS", "300"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mp_latency.py")], env=env,
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        sys.exit(r.stdout[-2000:] + r.stderr[-2000:])
    lat = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["latency"]
    out = open(os.path.join(ROOT, "gpurun_out", "crossover.jsonl"), "w")
    for n in SIZES:
        src = O.team_inputs("int", 2, n, 5, "bits")
        reps = max(50, min(20000, int(2e7 / max(n, 1))))
        cpu = O.cpu_baseline("int", "sum", src, reps=reps, pin=True) * 1e6
        rec = {"nreduce": n, "cpu_reference_loop_us": cpu,
               "fused_team_us": lat[f"{n}/fused_team"]["us_median"],
               "host_barrier_team_us": lat[f"{n}/team"]["us_median"],
               "host_fused_staged_us": lat[f"{n}/host_fused_staged"]["us_median"],
               "correct": all(lat[f"{n}/{k}"]["correct"]
                              for k in ("fused_team", "team", "host_fused_staged"))}
        rec["gpu_faster"] = rec["fused_team_us"] < cpu
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
