#!/usr/bin/env python3
"""Measure the data-movement collectives on one MI355X.

  kernel   the copy kernel alone (osgpu_copy, HIP events on its own stream):
           P ranges of NB bytes in one launch, local HBM; traffic 2*P*NB per
           launch (read + write) vs 8 TB/s.  Also with the source at a 4-byte
           phase (collect32's block offsets).
  device   shmem_<kind>64 through the C ABI, P threads-as-PEs on one GPU
           (COPY path), median call time in C (pet_time_coll); all-PE bytes
           moved: broadcast 2(P-1)NB, others 2*P*P*NB.
  host     the same call on host symmetric heaps: STAGED (PCIe-bound; the
           P PEs share one GPU's link here) and GETMEM (runtime memcpy).
  cpu      the reference's loop shape on the host cores (oracle_coll.c).

usage: coll_bench.py [--pes 4] [--nbytes 64Mi] [--reps 10] [--out FILE]
Not part of the product; prints one JSON line per measurement."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("test-resilient-osss-ucx_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import osgpu  # noqa: E402  (imports torch first: one HIP runtime)
import torch  # noqa: E402
import oracle_coll as OC  # noqa: E402
from support import team as T  # noqa: E402

HBM_PEAK = 8.0e12
KINDS = ["broadcast", "collect", "fcollect", "alltoall"]


def emit(out, rec):
    line = json.dumps(rec)
    print(line, flush=True)
    if out:
        with open(out, "a") as f:
            f.write(line + "\n")


def kernel_rate(P, nb, reps, phase=0):
    src = torch.empty(P * nb + 64, dtype=torch.uint8, device="cuda:0")
    dst = torch.empty(P * nb + 64, dtype=torch.uint8, device="cuda:0")
    src.random_(0, 256)
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    dsts = [dst.data_ptr() + i * nb for i in range(P)]
    srcs = [src.data_ptr() + phase + i * nb for i in range(P)]
    ts = []
    with torch.cuda.stream(st):
        for r in range(reps + 3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            osgpu.copy(dsts, srcs, [nb] * P, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            if r >= 3:
                ts.append(e0.elapsed_time(e1) * 1e-3)
    assert torch.equal(dst[:P * nb], src[phase:phase + P * nb])
    ts.sort()
    t = ts[len(ts) // 2]
    return t, 2 * P * nb / t


def api_time(kind, P, nb, reps, device):
    esz = 8
    n = nb // esz
    sb = P * nb if kind == "alltoall" else nb
    tgt_off = T._align(sb)
    tm = T.Team(P, tgt_off + P * nb, device=device)
    if device:
        tm.buf.random_(0, 256)
        torch.cuda.synchronize()
    else:
        # every page written: untouched calloc pages all map the shared zero
        # page, and memcpy from it is a cache hit, not a DRAM read
        tm.hbuf.fill(0x5A)
    fn = ctypes.cast(osgpu.coll(kind, 64), ctypes.c_void_p)
    tgt = (ctypes.c_void_p * P)(*[tm.ptr(pe, tgt_off) for pe in range(P)])
    src = (ctypes.c_void_p * P)(*[tm.ptr(pe, 0) for pe in range(P)])
    ps = (ctypes.c_void_p * P)(*[tm.psync_ptr(pe) for pe in range(P)])
    f = tm.pet.pet_time_coll
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
    t = f(fn, P, tgt, src, ps, n, 1 if kind == "broadcast" else -1, reps)
    if not device:
        tm.lib.osgpu_finalize()
    del tm
    return t


def moved(kind, P, nb):
    return 2 * (P - 1) * nb if kind == "broadcast" else 2 * P * P * nb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pes", type=int, default=4)
    ap.add_argument("--nbytes", type=int, default=64 << 20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--skip", default="", help="comma list of: kernel,device,host,cpu")
    a = ap.parse_args()
    skip = set(a.skip.split(",")) if a.skip else set()
    P, nb = a.pes, a.nbytes
    if "kernel" not in skip:
        for phase in (0, 4):
            t, bw = kernel_rate(P, nb, a.reps, phase)
            emit(a.out, {"what": "copy_kernel", "ranges": P, "bytes_per_range": nb,
                         "src_phase": phase, "us": t * 1e6, "GBps": bw / 1e9,
                         "frac_of_8TBps": bw / HBM_PEAK})
    for kind in KINDS:
        rec = {"what": f"shmem_{kind}64", "pes": P, "bytes_per_pe": nb,
               "bytes_moved_all_pes": moved(kind, P, nb)}
        if "device" not in skip:
            t = api_time(kind, P, nb, a.reps, True)
            rec["device_ms"] = t * 1e3
            rec["device_GBps"] = moved(kind, P, nb) / t / 1e9
            rec["device_frac_of_8TBps"] = moved(kind, P, nb) / t / HBM_PEAK
        if "host" not in skip:
            for hp in ("staged", "getmem"):
                with osgpu.host_path(hp):
                    t = api_time(kind, P, nb, max(3, a.reps // 3), False)
                rec[f"host_{hp}_ms"] = t * 1e3
        if "cpu" not in skip:
            t = OC.cpu_baseline(kind, P, nb, root=1, reps=5)
            rec["cpu_reference_loop_ms"] = t * 1e3
            rec["cpu_cores"] = P
        emit(a.out, rec)


if __name__ == "__main__":
    main()
