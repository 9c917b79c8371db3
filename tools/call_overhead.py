#!/usr/bin/env python3
"""call_overhead.py -- where the whole-call time of the TEAM path goes
(bench.py roofline_call: shmem_double_sum_to_all, 2 PEs as pthreads on one
GPU, nreduce = 64 Mi, src/reductions.c:82,113 barriers), per completion-wait
mode (OSGPU_SYNC block / spin / word, runtime.cpp stream_wait) and flags:
+contig / +tiles / +merge (OSGPU_TEAM_LOCAL=shards / tiles / merge:
contiguous shards, interleaved tiles, or one grid launched by the first PE
thread, for co-resident PE threads, shmem_reduce.cpp run_team; merge is the
default since r04_call_overhead_6), +sleep
(PET_SLEEP_BARRIER=1: the PE-thread runtime's barrier sleeps instead of
polling, tests/support/pe_threads.c).  (Round-4 files _1.._5 also compare a
merged launch of co-resident PE threads and one shared stream, since
removed: neither was faster.)  Each mode
runs in its own process (the mode is read once) with OSGPU_CALL_TRACE=1:
PE 0's host clock at entry sync, barrier 1, launch, completion wait,
barrier 2; the median of every phase over the calls, beside the call time
timed in C and the team kernel alone (one launch over both shards, HIP
events).  One JSON line per mode on stdout and in
gpurun_out/call_overhead.jsonl.  Not part of the product.

  python tools/call_overhead.py            (on the GPU box)
  python tools/call_overhead.py child MODE (one mode; used by the above)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "test-resilient-osss-ucx_amd")]


def child(mode):
    import torch
    import bench
    import osgpu
    n = int(os.environ.get("CO_N", str(64 << 20)))
    reps = int(os.environ.get("CO_REPS", "30"))
    L = osgpu.load()
    k = bench.team_kernel_rate(L, torch, n, 20, P=2)
    api = bench.api_call_time(n, reps=reps)
    # the team kernel alone over the very arrays the call uses (the call's
    # heap layout: both PEs' slices of one allocation, target at the next
    # 4 KiB past the source), one launch over both shards, HIP events
    import ctypes
    from support import team as T
    tm = T.Team(2, 2 * n * 8 + 8192, device=True)
    toff = (n * 8 + 4095) // 4096 * 4096
    for pe in range(2):
        tm.buf[pe * tm.H: pe * tm.H + n * 8].view(torch.float64).uniform_(1, 2)
    S = (ctypes.c_void_p * 2)(tm.ptr(0, 0), tm.ptr(1, 0))
    D = (ctypes.c_void_p * 2)(tm.ptr(0, toff), tm.ptr(1, toff))
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    torch.cuda.synchronize()

    def launch():
        assert L.osgpu_team_combine(5, 0, 2, D, S, n, sp) == 0
    for _ in range(3):
        launch()
    k_layout = bench.span_per_launch(torch, st, launch, 20)
    print(json.dumps({"mode": mode, "n": n, "ms_per_call": api["team"]["ms_per_call"],
                      "kernel_us": k["kernel_avg_us"], "kernel_us_call_layout": k_layout * 1e6,
                      "pull_ms_per_call": api["pull"]["ms_per_call"]}), flush=True)


def main():
    out = open(os.path.join(ROOT, "gpurun_out", "call_overhead.jsonl"), "a")
    # MODE = <OSGPU_SYNC>[+contig|+tiles|+merge][+sleep]
    default = "block+contig+sleep,block+contig,block+tiles,block+merge,word+merge"
    for mode in os.environ.get("CO_MODES", default + "," + default).split(","):
        sync, *flags = mode.split("+")
        env = dict(os.environ, OSGPU_SYNC=sync, OSGPU_CALL_TRACE="1")
        if "contig" in flags:
            env["OSGPU_TEAM_LOCAL"] = "shards"
        if "tiles" in flags:
            env["OSGPU_TEAM_LOCAL"] = "tiles"
        if "merge" in flags:
            env["OSGPU_TEAM_LOCAL"] = "merge"
        if "sleep" in flags:
            env["PET_SLEEP_BARRIER"] = "1"
        r = subprocess.run([sys.executable, __file__, "child", mode], env=env, capture_output=True,
                           text=True, timeout=600)
        if r.returncode != 0:
            print(json.dumps({"mode": mode, "error": (r.stdout + r.stderr)[-800:]}), flush=True)
            sys.exit(r.returncode if r.returncode > 0 else 1)
        rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        # trace lines of the team-path calls (the pull path prints none)
        phases = {}
        for line in r.stderr.splitlines():
            if not line.startswith("[osgpu call]"):
                continue
            f = line.split()[2:-1]
            for name, v in zip(f[0::2], f[1::2]):
                phases.setdefault(name, []).append(float(v))
        rec["phases_us_median"] = {k: sorted(v)[len(v) // 2] for k, v in phases.items()}
        rec["phases_calls"] = max((len(v) for v in phases.values()), default=0)
        call_us = rec["ms_per_call"] * 1e3
        rec["frac_call"] = 4 * rec["n"] * 8 / (call_us * 1e-6) / 8e12
        rec["frac_kernel"] = 4 * rec["n"] * 8 / (rec["kernel_us"] * 1e-6) / 8e12
        rec["frac_kernel_call_layout"] = 4 * rec["n"] * 8 / (rec["kernel_us_call_layout"] * 1e-6) / 8e12
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
        out.flush()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(sys.argv[2])
    else:
        main()
