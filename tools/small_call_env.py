#!/usr/bin/env python3
"""small_call_env.py -- BASELINE config 1's shape (shmem_int_sum_to_all,
nreduce = 1 Ki, 2 PE processes on one GPU, device heaps) through
tools/mp_latency.py under environment variants: the fused one-launch path's
call time (timed in C, barrier to barrier) and, with OSGPU_FUSED_TRACE=1,
its in-kernel phase clocks (PE 0, median over the calls).  One JSON line per
variant on stdout and in gpurun_out/small_call_env.jsonl.  Not part of the
product.

  SC_VARIANTS="base;trace:OSGPU_FUSED_TRACE=1;devkarg:HIP_FORCE_DEV_KERNARG=1"
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = open(os.path.join(ROOT, "gpurun_out", "small_call_env.jsonl"), "a")
    spec = os.environ.get("SC_VARIANTS",
                          "base;trace:OSGPU_FUSED_TRACE=1;devkarg:HIP_FORCE_DEV_KERNARG=1")
    for item in spec.split(";"):
        name, _, envs = item.partition(":")
        env = dict(os.environ, MP_WORLDS="2", MP_SIZES=os.environ.get("SC_SIZES", "1024"),
                   MP_REPS=os.environ.get("SC_REPS", "300"))
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mp_latency.py")], env=env,
                           capture_output=True, text=True, timeout=500)
        if r.returncode != 0:
            print(json.dumps({"variant": name, "error": (r.stdout + r.stderr)[-800:]}), flush=True)
            sys.exit(1)
        lat = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["latency"]
        rec = {"variant": name, "env": envs}
        for k, v in lat.items():
            if k.endswith(("/fused_team", "/team", "/host_fused_staged")):
                rec[k] = {"us": v["us_median"], "us_c": v.get("us_median_timed_in_c"),
                          "correct": v["correct"]}
        phases = {}
        for m in re.finditer(r"\[osgpu fused PE 0 epoch \d+\] (.*) us", r.stderr):
            f = m.group(1).replace("ticket+fence", "ticket_fence").split()
            for key, val in zip(f[0::2], f[1::2]):
                phases.setdefault(key, []).append(float(val))
        if phases:
            rec["phases_us_median"] = {k: sorted(v)[len(v) // 2] for k, v in phases.items()}
            rec["phases_calls"] = max(len(v) for v in phases.values())
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
        out.flush()


if __name__ == "__main__":
    main()
