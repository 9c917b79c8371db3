#!/usr/bin/env python3
"""Probe HIP IPC export/import of device allocations between two processes
(sizes, torch vs hipMalloc allocations).  Not part of the product.
usage: python tools/ipc_probe.py   (spawns its two ranks itself)"""
import ctypes
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "test-resilient-osss-ucx_amd")]
SIZES = [256 << 20, 512 << 20, (1 << 30) - (2 << 20), 1 << 30, (1 << 30) + 4096,
         (1 << 31) - (2 << 20), 1 << 31]


def worker():
    import torch
    import torch.distributed as dist
    import osgpu
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    L = osgpu.load()
    hip = ctypes.CDLL("libamdhip64.so")
    for kind in ("hipMalloc", "torch"):
        for sz in SIZES:
            if kind == "torch":
                t = torch.empty(sz, dtype=torch.uint8, device="cuda:0")
                ptr = t.data_ptr()
            else:
                p = ctypes.c_void_p()
                assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(sz)) == 0
                ptr = p.value
            h = (ctypes.c_char * 64)()
            rc = L.osgpu_ipc_get_handle(ctypes.c_void_p(ptr), h)
            hs = [None, None]
            dist.all_gather_object(hs, bytes(h))
            t0 = time.time()
            print(f"[rank {rank}] {kind} {sz} get={rc} opening...", flush=True)
            m = L.osgpu_ipc_open((ctypes.c_char * 64).from_buffer_copy(hs[1 - rank]))
            print(f"[rank {rank}] {kind} {sz} open={'ok' if m else 'FAIL'} "
                  f"{time.time() - t0:.3f}s", flush=True)
            dist.barrier()
            if m:
                L.osgpu_ipc_close(ctypes.c_void_p(m))
            dist.barrier()
            if kind == "torch":
                del t
                torch.cuda.empty_cache()
            else:
                hip.hipFree(ctypes.c_void_p(ptr))
    dist.destroy_process_group()


def main():
    if os.environ.get("RANK") is not None:
        return worker()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, __file__],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
             for r in range(2)]
    for p in procs:
        p.wait()


if __name__ == "__main__":
    main()
