#!/usr/bin/env python3
"""Deterministic layout sweep of the shipped team kernel (VERDICT r04 item 2:
a 4-member placement ran at 0.369 of 8 TB/s against 0.80 on others).

The P sources and P targets of osgpu_team_combine (double sum, n elements
each) are carved out of ONE allocation at controlled relative offsets:
array i (sources 0..P-1, then targets) starts at base + i * (n*8 + skew(i)),
for skew families that align the arrays on large powers of two, stagger
them by small steps, or scatter them pseudo-randomly.  Every layout times
the team kernel and, on the very same ranges, the copy kernel moving P
read + P write streams (osgpu_copy, one segment per member): the ratio
team/copy isolates the kernel's own sensitivity to the layout from the
memory's.  One JSON line per (P, layout), with every array's address.

    python tools/team_layout_sweep.py [n=64Mi] [members=3,4] [reps=10]
Not part of the product."""
import ctypes
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "test-resilient-osss-ucx_amd")]

import torch  # noqa: E402
import osgpu  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
MEMBERS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "3,4").split(",")]
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 10

KiB, MiB = 1 << 10, 1 << 20


def families(P):
    rnd = random.Random(1234 + P)
    fam = {
        "gap0": lambda i: 0,       # arrays n*8 + 4 MiB apart: equal low 22 address bits
        "gap256B": lambda i: 256 * i,
        "gap4K": lambda i: 4 * KiB * i,
        "gap64K": lambda i: 64 * KiB * i,
        "gap1M": lambda i: 1 * MiB * i,
        "gap2M": lambda i: 2 * MiB * i,
        "gap2M+4K": lambda i: 2 * MiB * i + 4 * KiB * i,
    }
    for r in range(3):
        offs = [rnd.randrange(0, 512) * 4 * KiB for _ in range(2 * P)]
        fam[f"rand4K_{r}"] = (lambda o: (lambda i: o[i]))(offs)
    for k in ("symheap", "symheap+4K", "symheap+64K", "symheap+1M"):
        fam[k] = None
    if os.environ.get("SWEEP_ONLY"):
        fam = {k: v for k, v in fam.items() if k in os.environ["SWEEP_ONLY"].split(",")}
    return fam


def main():
    L = osgpu.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    P_max = max(MEMBERS)
    slack = 2 * P_max * (4 * MiB + 4 * MiB) + P_max * MiB + 32 * MiB
    buf = torch.empty(2 * P_max * N * 8 + slack, dtype=torch.uint8, device=dev)
    base = (buf.data_ptr() + 2 * MiB - 1) // (2 * MiB) * (2 * MiB)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def span(launch):
        for _ in range(2):
            launch()
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(REPS):
            launch()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / REPS  # us

    for P in MEMBERS:
        for name, skew in families(P).items():
            if name.startswith("symheap"):
                # a symmetric heap per member: source at 0, target at n*8 +
                # 2 MiB of heap p; heaps back to back (+ an optional skew per heap)
                H = 2 * N * 8 + 4 * MiB
                d = {"symheap": 0, "symheap+4K": 4 * KiB, "symheap+64K": 64 * KiB,
                     "symheap+1M": MiB}[name]
                addr = [base + p * (H + d) for p in range(P)] + \
                       [base + p * (H + d) + N * 8 + 2 * MiB for p in range(P)]
            else:
                # array i; the 4 MiB spacing beyond n*8 keeps skewed arrays apart
                addr = [base + i * (N * 8 + 4 * MiB) + skew(i) for i in range(2 * P)]
            assert addr[-1] + N * 8 <= buf.data_ptr() + buf.numel()
            for i in range(P):  # sources: a known value per member
                tmp = torch.full((N,), 1.0 + i / 8, dtype=torch.float64, device=dev)
                osgpu.copy([addr[i]], [tmp.data_ptr()], [N * 8])
                torch.cuda.synchronize()
                del tmp
            torch.cuda.synchronize()
            srcs = (ctypes.c_void_p * P)(*addr[:P])
            dsts = (ctypes.c_void_p * P)(*addr[P:])

            def team():
                if L.osgpu_team_combine(5, 0, P, dsts, srcs, N, sp) != 0:
                    raise RuntimeError(L.osgpu_last_error().decode())

            D = (ctypes.c_void_p * P)(*addr[P:])
            S = (ctypes.c_void_p * P)(*addr[:P])
            NB = (ctypes.c_size_t * P)(*([N * 8] * P))

            def copy():
                assert L.osgpu_copy(D, S, NB, P, sp) == 0

            t_team = span(team)
            t_copy = span(copy)
            t_team2 = span(team)
            # check one element of every target against member q's fold
            ok = True
            x = [1.0 + i / 8 for i in range(P)]
            for q in range(P):
                acc = x[q]
                for k in range(P):
                    if k != q:
                        acc = acc + x[k]
                got = torch.empty(1, dtype=torch.float64, device=dev)
                osgpu.copy([got.data_ptr()], [addr[P + q] + 8 * 12345], [8])
                torch.cuda.synchronize()
                ok = ok and float(got.item()) == acc
            B = 2 * P * N * 8
            tt = min(t_team, t_team2)
            print(json.dumps({
                "P": P, "layout": name, "team_us": tt, "team_us_runs": [t_team, t_team2],
                "copy_us": t_copy, "team_frac": B / tt / 8e6, "copy_frac": B / t_copy / 8e6,
                "team_of_copy": t_copy / tt, "ok": ok,
                "offsets_MiB": [round((a - base) / MiB, 4) for a in addr]}), flush=True)


if __name__ == "__main__":
    main()
