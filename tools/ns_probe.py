#!/usr/bin/env python3
"""ns_probe.py -- where the combine's HBM rate goes at the north-star size.
Not part of the product; one MI355X.

  alloc   double sum K = 2 at 128 Mi (1 GiB per array) on fresh torch
          allocations, several placements (a decoy allocation shifts them)
  carve   the three arrays carved from one allocation at relative offsets
  flush   back-to-back launches vs launches behind a 1 GiB write to another
          buffer (what the 256 MiB Infinity Cache keeps between launches), at
          2^24..2^28 elements
  team    the TEAM path's kernel (team_vec_kernel<double,SUM,2>) over all n,
          one launch, and as the 2-PE call issues it (two launches of n/2 on
          two streams), vs the combine; bytes 4*n*8 vs 3*n*8
  split   the 128 Mi combine as k back-to-back launches over n/k chunks
          (k = 1..16) on one stream, timed as a group
  alt     2^26 / 2^27 combines alternating between two array sets per launch
          (no chance of reuse from the previous launch's arrays)
Every figure: median of REPS launches timed with HIP events on the launch
stream; JSON lines on stdout and in gpurun_out/ns_probe.jsonl.
usage: python tools/ns_probe.py [alloc carve flush team]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "test-resilient-osss-ucx_amd"))
import torch  # noqa: E402
import osgpu  # noqa: E402

L = osgpu.load()
REPS = int(os.environ.get("REPS", "20"))
OUT = open(os.path.join(ROOT, "gpurun_out", "ns_probe.jsonl"), "a")
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
sp = ctypes.c_void_p(st.cuda_stream)


def emit(d):
    line = json.dumps(d)
    print(line, flush=True)
    OUT.write(line + "\n")
    OUT.flush()


def time_launches(launch, reps=REPS, between=None):
    for _ in range(3):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    torch.cuda.synchronize()
    for e0, e1 in ev:
        if between is not None:
            between()
        e0.record(st)
        launch()
        e1.record(st)
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) * 1e-3 for e0, e1 in ev)
    return ts[len(ts) // 2], ts[0]


def combine_launcher(a, b, o, n):
    srcs = (ctypes.c_void_p * 2)(a, b)

    def go():
        rc = L.osgpu_combine(5, 0, o, srcs, 2, n, sp)
        assert rc == 0
    return go


def alloc():
    n = 128 << 20
    for trial, decoy in enumerate((0, 2 << 20, 64 << 20, 300 << 20, 1 << 30)):
        d = torch.empty(decoy, dtype=torch.uint8, device=dev) if decoy else None
        a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
        b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
        o = torch.empty(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        med, best = time_launches(combine_launcher(a.data_ptr(), b.data_ptr(), o.data_ptr(), n))
        assert torch.equal(o[:1 << 20], a[:1 << 20] + b[:1 << 20])
        emit({"probe": "alloc", "n": n, "decoy": decoy, "us": med * 1e6,
              "frac": 3 * n * 8 / med / 8e12, "best_frac": 3 * n * 8 / best / 8e12,
              "addr_mod_1g": [p.data_ptr() % (1 << 30) for p in (a, b, o)]})
        del a, b, o, d
        torch.cuda.empty_cache()


def carve():
    n = 128 << 20
    S = n * 8
    buf = torch.empty(3 * S + (80 << 20), dtype=torch.uint8, device=dev)
    buf.view(torch.float64)[: 3 * n].uniform_(1, 2)
    for da, db in ((0, 0), (4096, 8192), (64 << 10, 128 << 10), (1 << 20, 2 << 20),
                   (256 << 10, 768 << 10), (2 << 20, 6 << 20), (32 << 20, 64 << 20)):
        base = buf.data_ptr()
        med, best = time_launches(combine_launcher(base, base + S + da, base + 2 * S + db, n))
        emit({"probe": "carve", "n": n, "da": da, "db": db, "us": med * 1e6,
              "frac": 3 * S / med / 8e12, "best_frac": 3 * S / best / 8e12})
    del buf
    torch.cuda.empty_cache()


def flush():
    junk = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    for lg in (24, 25, 26, 27, 28):
        n = 1 << lg
        a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
        b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
        o = torch.empty(n, dtype=torch.float64, device=dev)
        go = combine_launcher(a.data_ptr(), b.data_ptr(), o.data_ptr(), n)
        hot, _ = time_launches(go)
        cold, _ = time_launches(go, between=lambda: junk.fill_(1))
        emit({"probe": "flush", "n": n, "us_back_to_back": hot * 1e6,
              "us_after_1GiB_write": cold * 1e6, "frac_back_to_back": 3 * n * 8 / hot / 8e12,
              "frac_after_flush": 3 * n * 8 / cold / 8e12})
        del a, b, o
        torch.cuda.empty_cache()


def team():
    n = 64 << 20
    a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
    b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
    o0 = torch.empty(n, dtype=torch.float64, device=dev)
    o1 = torch.empty(n, dtype=torch.float64, device=dev)
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    dsts = (ctypes.c_void_p * 2)(o0.data_ptr(), o1.data_ptr())

    def one():
        assert L.osgpu_team_combine(5, 0, 2, dsts, srcs, n, sp) == 0

    med, best = time_launches(one)
    assert torch.equal(o0, a + b) and torch.equal(o1, b + a)
    emit({"probe": "team_one_launch", "n": n, "us": med * 1e6, "frac": 4 * n * 8 / med / 8e12,
          "best_frac": 4 * n * 8 / best / 8e12})
    # as the 2-PE call issues it: PE g launches shard g on its own stream
    st2 = torch.cuda.Stream()
    sp2 = ctypes.c_void_p(st2.cuda_stream)
    h = n // 2
    halves = []
    for g, s_ in ((0, sp), (1, sp2)):
        off = g * h * 8
        halves.append(((ctypes.c_void_p * 2)(a.data_ptr() + off, b.data_ptr() + off),
                       (ctypes.c_void_p * 2)(o0.data_ptr() + off, o1.data_ptr() + off), s_))

    def split():
        ev = torch.cuda.Event()
        ev.record(st)
        st2.wait_event(ev)
        for sr, ds, s_ in halves:
            assert L.osgpu_team_combine(5, 0, 2, ds, sr, h, s_) == 0
        ev2 = torch.cuda.Event()
        ev2.record(st2)
        st.wait_event(ev2)

    med, best = time_launches(split)
    emit({"probe": "team_two_shards", "n": n, "us": med * 1e6, "frac": 4 * n * 8 / med / 8e12,
          "best_frac": 4 * n * 8 / best / 8e12})
    med, best = time_launches(combine_launcher(a.data_ptr(), b.data_ptr(), o0.data_ptr(), n))
    emit({"probe": "combine_same_arrays", "n": n, "us": med * 1e6,
          "frac": 3 * n * 8 / med / 8e12, "best_frac": 3 * n * 8 / best / 8e12})


def split():
    n = 128 << 20
    a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
    b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
    o = torch.empty(n, dtype=torch.float64, device=dev)
    for k in (1, 2, 4, 8, 16):
        c = n // k
        gos = [combine_launcher(a.data_ptr() + i * c * 8, b.data_ptr() + i * c * 8,
                                o.data_ptr() + i * c * 8, c) for i in range(k)]

        def group():
            for g in gos:
                g()
        o.zero_()
        med, best = time_launches(group)
        assert torch.equal(o, a + b)
        emit({"probe": "split", "n": n, "k": k, "us": med * 1e6,
              "frac": 3 * n * 8 / med / 8e12, "best_frac": 3 * n * 8 / best / 8e12})
    del a, b, o
    torch.cuda.empty_cache()


def alt():
    for lg in (26, 27):
        n = 1 << lg
        sets = []
        for _ in range(2):
            sets.append([torch.empty(n, dtype=torch.float64, device=dev).uniform_(1, 2)
                         for _ in range(3)])
        gos = [combine_launcher(x.data_ptr(), y.data_ptr(), z.data_ptr(), n) for x, y, z in sets]
        flip = [0]

        def go():
            gos[flip[0]]()
            flip[0] ^= 1
        med, best = time_launches(go)
        emit({"probe": "alt", "n": n, "us": med * 1e6,
              "frac": 3 * n * 8 / med / 8e12, "best_frac": 3 * n * 8 / best / 8e12})
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    for name in (sys.argv[1:] or ["alloc", "carve", "flush", "team"]):
        globals()[name]()
