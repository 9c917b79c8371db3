"""vmm_probe.py -- step-by-step probe of osgpu_heap_create with N processes on
cuda:0 (PE services: the shared-memory runtime).  Each rank logs every step
to gpurun_out/vmm_probe_rank<r>.log as it happens (OSGPU_DEBUG=1), creates a
heap of each size in VMM_SIZES, writes a pattern into its heap, reads every
peer's heap through the mapping (one launch of the copy kernel per peer) and
checks the bytes.  usage: python tools/vmm_probe.py [nprocs]"""
import ctypes
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "test-resilient-osss-ucx_amd"), os.path.join(ROOT, "tests")]


def worker():
    import torch
    import torch.distributed as dist
    import osgpu
    from support import peshm
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    log = lambda m: print(f"[rank {rank} {time.strftime('%H:%M:%S')}] {m}", flush=True)  # noqa
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    L = osgpu.load()
    PES = peshm.init(rank, world, 1 << 24, dist, tag="v")
    assert L.osgpu_set_pe_ops(PES.pes_ops()) == 0
    psync = PES.pes_heap(rank) + (1 << 24) - 8192
    log("ready")
    for size in [int(x) for x in os.environ.get("VMM_SIZES", str(64 << 20)).split(",")]:
        base = ctypes.c_void_p()
        t0 = time.time()
        rc = L.osgpu_heap_create(size, 0, 0, world, psync, ctypes.byref(base))
        log(f"heap_create({size}) rc={rc} {L.osgpu_last_error().decode()!r} "
            f"{time.time() - t0:.2f}s base={base.value}")
        if rc != 0:
            break
        pat = torch.full((1 << 20,), rank + 1, dtype=torch.uint8, device="cuda:0")
        ends = [0, size - (1 << 20)]
        for off in ends:
            osgpu.copy([base.value + off], [pat.data_ptr()], [1 << 20])
        torch.cuda.synchronize()
        dist.barrier()
        buf = torch.empty(1 << 20, dtype=torch.uint8, device="cuda:0")
        for pe in range(world):
            for off in ends:
                p = L.osgpu_heap_translate(base.value + off, rank, pe)
                osgpu.copy([buf.data_ptr()], [p], [1 << 20])
                torch.cuda.synchronize()
                ok = bool((buf == pe + 1).all())
                log(f"read PE {pe} @+{off}: {'ok' if ok else 'WRONG'}")
        # a torch view of the heap through __cuda_array_interface__
        class _View:
            def __init__(self, ptr, nb):
                self.__cuda_array_interface__ = {"shape": (nb,), "typestr": "|u1",
                                                 "data": (ptr, False), "version": 3,
                                                 "strides": None}
        try:
            t = torch.as_tensor(_View(base.value, size), device="cuda:0")
            t[: 1 << 20].fill_(7)
            torch.cuda.synchronize()
            osgpu.copy([buf.data_ptr()], [base.value], [1 << 20])
            torch.cuda.synchronize()
            log(f"torch view: device={t.device} ok={bool((buf == 7).all())} "
                f"sum={int(t[:1 << 20].sum())}")
            del t
        except Exception as e:
            log(f"torch view failed: {e!r}")
        dist.barrier()
        log(f"destroy rc={L.osgpu_heap_destroy(base)}")
        dist.barrier()
    dist.destroy_process_group()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OSGPU_DEBUG="1", VMM_WORKER="1")
        f = open(os.path.join(out, f"vmm_probe_rank{r}.log"), "w")
        procs.append((subprocess.Popen([sys.executable, "-u", __file__], env=env, stdout=f,
                                       stderr=subprocess.STDOUT), f))
    rc = 0
    for p, f in procs:
        try:
            rc |= p.wait(timeout=float(os.environ.get("VMM_TIMEOUT", "150")))
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            rc = 124
        f.close()
    print("vmm_probe rc", rc)
    sys.exit(rc)


if __name__ == "__main__":
    worker() if os.environ.get("VMM_WORKER") else main()
