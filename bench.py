#!/usr/bin/env python3
"""bench.py -- device-resident shmem_double_sum_to_all combine on MI355X.

Metric (BASELINE.json): GiB/s of the device-resident shmem_double_sum_to_all
combine + fraction of the HBM roofline, at 1/2/4/8 GPUs.

N = 1 (default) -- BASELINE config 2: nreduce = 64 Mi doubles, 1 MI355X,
  "device-resident combine kernel only".  One step = one launch of the
  combine kernel that shmem_double_sum_to_all runs on the P2P path for a
  2-PE active set (K = 2 inputs: the PE's own source and its peer's, both in
  HBM) through the C ABI (osgpu_combine).  Algorithmic bytes per step
  B = (K + 1) * nreduce * 8 (2 reads + 1 write), value = K_steps * B / t.

N > 1 (torchrun, one process per GPU) -- one PE per GPU, every PE calls
  shmem_double_sum_to_all(nreduce = 64 Mi per PE) over all N PEs (weak
  scaling: per-GPU data fixed).  Path: RCCL allreduce over xGMI (default) or
  the exact-order peer-read kernel over IPC-mapped heaps (--path p2p).  Per
  step the job combines N sources into N targets; value counts the same
  algorithmic bytes as N=1, (N + 1) * nreduce * 8 per PE result summed over
  the N PEs, divided by the max-over-ranks time.

Also printed (same JSON line): roofline of the dominant kernel from HIP
events on the launch stream, the reference's CPU loop shape timed on this
host (oracle, rank 0, N = 1 only), and the full C-API call time of a 2-PE
threads-as-PEs team on the GPU (barriers + syncs included).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for sub in ("test-resilient-osss-ucx_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec, MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--nreduce", type=int, default=64 << 20)
    ap.add_argument("--path", choices=["rccl", "p2p"], default="rccl")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-api", action="store_true")
    ap.add_argument("--cpu-n", type=int, default=64 << 20,
                    help="nreduce of the CPU-baseline sample")
    return ap.parse_args()


def load_traffic():
    """HBM bytes per launch of the combine kernel measured with rocprofv3
    PMC counters (profiles/*traffic*.json, written by tools/pmc_traffic.py)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json"))):
        try:
            with open(p) as f:
                best = json.load(f)
        except Exception:
            pass
    return best


def cpu_baseline(n):
    """The reference's loop shape (oracle_reduce.c: copy, barrier, 64-element
    getmem chunks, per-element function-pointer op, barrier) with 2 pthreads
    as PEs on this host's cores."""
    import numpy as np
    import oracle as O
    src = O.team_inputs("double", 2, n, 0x5EED, "unit12")
    # size the repetition count for ~10 s of CPU work (bounded sample)
    probe = O.cpu_baseline("double", "sum", src, reps=1, pin=True)
    reps = max(3, min(200, int(10.0 / max(probe, 1e-3))))
    t0 = time.time()
    sec = O.cpu_baseline("double", "sum", src, reps=reps, pin=True)
    wall = time.time() - t0
    B = 2 * 3 * n * 8  # two PE results, each (K+1)*n*8
    return {"value": B / sec / GIB, "unit": "GiB/s", "cores": 2, "kind": "port",
            "sample": (f"oracle/oracle_reduce.c reference loop shape, double sum, "
                       f"2 PEs (pthreads pinned to cores 0-1), nreduce={n}, median of "
                       f"{reps} after 1 warm-up ({sec*1e3:.1f} ms/call, {wall:.1f} s total); "
                       f"bytes = 2 PE results x 3*n*8; host nproc={os.cpu_count()}")}


def api_call_time(n, reps=10):
    """Full shmem_double_sum_to_all through the C ABI: 2 threads-as-PEs on
    cuda:0 (P2P path, barriers + stream syncs included)."""
    import numpy as np
    from support import team as T
    tm = T.Team(2, 2 * n * 8 + 8192, device=True)
    toff = (n * 8 + 4095) // 4096 * 4096
    for pe in range(2):
        tm.buf[pe * tm.H: pe * tm.H + n * 8].view(__import__("torch").float64).uniform_(1, 2)
    tm.run("double", "sum", toff, 0, n)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        tm.run("double", "sum", toff, 0, n)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    return {"ms_per_call": med * 1e3, "GiB_s": 2 * 3 * n * 8 / med / GIB,
            "note": "2 PEs (threads) on one GPU, both PEs' calls, barrier-to-barrier"}


def bench_single(args):
    import torch
    import osgpu
    L = osgpu.load()
    n = args.nreduce
    dev = torch.device("cuda:0")
    a = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
    b = torch.empty(n, dtype=torch.float64, device=dev).uniform_(1.0, 2.0)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    stream = torch.cuda.Stream(device=dev)
    srcs = (ctypes.c_void_p * 2)(a.data_ptr(), b.data_ptr())
    sp = ctypes.c_void_p(stream.cuda_stream)
    torch.cuda.synchronize()  # inputs were written on torch's default stream

    def step():
        rc = L.osgpu_combine(5, 0, out.data_ptr(), srcs, 2, n, sp)
        if rc != 0:
            raise RuntimeError(L.osgpu_last_error().decode())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness spot check of the timed kernel
    idx = torch.randint(0, n, (4096,), device=dev)
    assert torch.equal(out[idx], a[idx] + b[idx])

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    kms = [s.elapsed_time(e) for s, e in ev]
    kavg = sum(kms) / len(kms) * 1e-3
    B = 3 * n * 8
    res = {
        "metric": "GiB/s device-resident shmem_double_sum_to_all combine + %HBM peak, 1/2/4/8 GPU",
        "value": args.steps * B / t / GIB,
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: uniform [1,2) doubles resident in HBM",
        "config": {"workload": "BASELINE config 2: shmem_double_sum_to_all combine, "
                               "nreduce=64Mi, K=2 inputs (source + peer source), 1 MI355X, "
                               "device-resident combine kernel",
                   "nreduce": n, "K": 2, "bytes_per_step": B},
    }
    tr = load_traffic()
    res["roofline"] = {
        "bound": "hbm", "achieved": B / kavg / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": B / kavg / 1e9 / HBM_PEAK_GBS,
        "traffic": tr.get("bytes_per_launch") if tr and tr.get("nreduce") == n else None,
        "kernel": "osgpu::combine_vec_kernel<double, SUM, 2>",
        "kernel_avg_us": kavg * 1e6,
        "algorithmic_bytes_per_launch": B,
    }
    if not args.no_api:
        try:
            res["api"] = api_call_time(n)
        except Exception as e:  # report, never hide
            res["api"] = {"error": repr(e)}
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.cpu_n)
    print(json.dumps(res), flush=True)


def bench_multi(args):
    import torch
    import torch.distributed as dist
    import osgpu
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    L = osgpu.load()
    n = args.nreduce
    dev = torch.device("cuda", local)

    @ctypes.CFUNCTYPE(ctypes.c_int)
    def my_pe():
        return rank

    @ctypes.CFUNCTYPE(ctypes.c_int)
    def n_pes():
        return world

    @ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                      ctypes.POINTER(ctypes.c_long))
    def barrier(a, b, c, p):
        dist.barrier()

    ops = osgpu.PeOps(my_pe, n_pes, barrier,
                      ctypes.cast(None, osgpu.PeOps._fields_[3][1]))
    assert L.osgpu_set_pe_ops(ctypes.byref(ops)) == 0

    heap = torch.empty(2 * n * 8 + 4096, dtype=torch.uint8, device=dev)
    src = heap[: n * 8].view(torch.float64)
    tgt = heap[n * 8 + 4096: n * 8 + 4096 + n * 8].view(torch.float64)
    src.uniform_(1.0, 2.0)
    if args.path == "rccl":
        uid = (ctypes.c_char * 128)()
        if rank == 0:
            assert L.osgpu_rccl_unique_id(uid) == 0
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_char * 128).from_buffer_copy(obj[0])
        assert L.osgpu_rccl_init(world, rank, uid) == 0
        L.osgpu_set_path(osgpu.PATH_RCCL)
    else:
        h = (ctypes.c_char * 64)()
        assert L.osgpu_ipc_get_handle(ctypes.c_void_p(heap.data_ptr()), h) == 0
        hs = [None] * world
        dist.all_gather_object(hs, bytes(h))
        for pe in range(world):
            if pe == rank:
                base = heap.data_ptr()
            else:
                hb = (ctypes.c_char * 64).from_buffer_copy(hs[pe])
                base = L.osgpu_ipc_open(hb)
                assert base, L.osgpu_last_error().decode()
            assert L.osgpu_heap_register(pe, ctypes.c_void_p(base), heap.numel()) == 0
        L.osgpu_set_path(osgpu.PATH_P2P)
    psync = (ctypes.c_long * 128)()
    wrk = (ctypes.c_double * 64)()
    fn = L.shmem_double_sum_to_all

    def step():
        fn(tgt.data_ptr(), src.data_ptr(), n, 0, 0, world, wrk, psync)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    tt = torch.tensor([t], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt.item())
    B = world * (world + 1) * n * 8
    if rank == 0:
        res = {
            "metric": "GiB/s device-resident shmem_double_sum_to_all combine + %HBM peak, 1/2/4/8 GPU",
            "value": args.steps * B / t / GIB,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: uniform [1,2) doubles resident in HBM",
            "config": {"workload": f"shmem_double_sum_to_all over {world} PEs, one per "
                                   f"MI355X, nreduce=64Mi per PE ({args.path} path)",
                       "nreduce": n, "path": args.path,
                       "bytes_per_step": B,
                       "parallelism": f"pe{world}"},
        }
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        bench_multi(args)
    else:
        bench_single(args)


if __name__ == "__main__":
    main()
