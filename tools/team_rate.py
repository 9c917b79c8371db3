#!/usr/bin/env python3
"""Owner-computes team kernel rate on one GPU: shmem_double_sum_to_all over
P threads-as-PEs with device heaps (TEAM path), timed in C from the common
start barrier to PE 0's return (tests/support/pe_threads.c:pet_time_to_all),
median of `reps`.  Team HBM traffic per call = 2 * P * N * 8 bytes (every
shard read from P sources and written to P targets).  Not part of the
product; prints one JSON line per P."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "test-resilient-osss-ucx_amd"), os.path.join(ROOT, "tests"),
                ROOT]


def main():
    import torch
    import osgpu
    import bench
    from support import team as T
    L = osgpu.load()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32 << 20
    t = os.environ.get("TR_TYPE", "double")   # double | longdouble (x87, 16-B slots)
    s = 16 if t == "longdouble" else 8
    reps = 20
    for P in (2, 4, 8):
        toff = (n * s + 4095) // 4096 * 4096
        tm = T.Team(P, toff + n * s, device=True)
        for pe in range(P):
            if t == "longdouble":  # x87 1.0: significand 0x8000.., exponent 0x3fff
                v = tm.buf[pe * tm.H: pe * tm.H + n * s].view(torch.int64).view(n, 2)
                v[:, 0] = -(1 << 63)
                v[:, 1] = 0x3fff
            else:
                tm.buf[pe * tm.H: pe * tm.H + n * s].view(torch.float64).fill_(1.0 + pe)
        torch.cuda.synchronize()
        fn = ctypes.cast(getattr(L, f"shmem_{t}_sum_to_all"), ctypes.c_void_p)
        tgt = (ctypes.c_void_p * P)(*[tm.ptr(pe, toff) for pe in range(P)])
        src = (ctypes.c_void_p * P)(*[tm.ptr(pe, 0) for pe in range(P)])
        ps = (ctypes.c_void_p * P)(*[tm.psync_ptr(pe) for pe in range(P)])
        bench._timer_sig(tm.pet)
        sec = tm.pet.pet_time_to_all(fn, P, tgt, src, ps, n, reps)
        if t == "longdouble":  # P * 1.0: exponent 0x3fff + log2(P) for P = 2, 4, 8
            got = tm.buf[toff: toff + n * s].view(torch.int64).view(n, 2)
            e = 0x3fff + (P.bit_length() - 1)
            ok = bool((got[:, 0] == -(1 << 63)).all()) and bool(((got[:, 1] & 0xffff) == e).all())
        else:
            want = float(sum(1.0 + pe for pe in range(P)))
            ok = all(bool((tm.buf[pe * tm.H + toff: pe * tm.H + toff + n * 8]
                           .view(torch.float64) == want).all()) for pe in range(P))
        print(json.dumps({"type": t, "P": P, "nreduce": n, "ms_per_call": sec * 1e3,
                          "team_hbm_GBs": 2 * P * n * s / sec / 1e9,
                          "frac_of_8TBs": 2 * P * n * s / sec / 8e12,
                          "correct": ok}), flush=True)
        del tm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
