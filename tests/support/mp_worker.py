"""mp_worker.py -- TEST INFRASTRUCTURE: one rank (= one PE = one process) of a
multi-process run of libosgpu_reduce.so, the way an OpenSHMEM job runs one
process per PE.  PE services come from torch.distributed (gloo): my_pe =
rank, shmem_barrier = dist.barrier.

modes
  host  no GPU: fold order, shard partition and the nreduce = 0 collective
        (two barriers through the Python callback) -- checked across ranks
  hostcoll  no GPU, shared-memory PE runtime: every data-movement
        collective with nelems = 0 (synchronises only, pSync left zeroed)
  ipc   GPU: each rank allocates its device symmetric heap, exports it with
        osgpu_ipc_get_handle, opens every peer's (osgpu_ipc_open) and
        registers them; then shmem_<T>_<op>_to_all runs on the team path,
        the pull path and in place, and the collectives (broadcast / collect /
        fcollect / alltoall) on the COPY path; results written for the
        parent to check
  hoststaged  GPU, host heaps in shared memory: reductions and collectives
        on the STAGED and GETMEM paths
usage: RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. \
       python mp_worker.py MODE OUTDIR
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "test-resilient-osss-ucx_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import osgpu  # noqa: E402


def pe_ops(rank, world, counter):
    @ctypes.CFUNCTYPE(ctypes.c_int)
    def my_pe():
        return rank

    @ctypes.CFUNCTYPE(ctypes.c_int)
    def n_pes():
        return world

    @ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                      ctypes.POINTER(ctypes.c_long))
    def barrier(a, b, c, p):
        counter[0] += 1
        dist.barrier()

    getmem_t = osgpu.PeOps._fields_[3][1]
    ops = osgpu.PeOps(my_pe, n_pes, barrier, ctypes.cast(None, getmem_t))
    return ops, (my_pe, n_pes, barrier)


def run_colls(L, rank, world, src_addr, tgt_addr, psync, out, tag, write, read):
    """Every case of support/coll_cases.py: source at src_addr, target
    (sentinel-filled) at tgt_addr, both symmetric; target bytes to `out`."""
    from support import coll_cases as CC
    for kind, bits, counts, root in CC.cases(world):
        raw = CC.source(kind, bits, counts, rank, world)
        tb = CC.target_bytes(kind, bits, counts, world)
        if raw.size:
            write(src_addr, raw)
        write(tgt_addr, np.full(tb, CC.SENTINEL, np.uint8))
        dist.barrier()
        f = osgpu.coll(kind, bits)
        if kind == "broadcast":
            f(tgt_addr, src_addr, counts[rank], root, 0, 0, world, psync)
        else:
            f(tgt_addr, src_addr, counts[rank], 0, 0, world, psync)
        out[CC.key(kind, bits, tag)] = bytes(read(tgt_addr, tb)).hex()
        assert not any(ctypes.string_at(psync, 1024)), "pSync not reset"
        dist.barrier()


def main():
    mode, outdir = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    L = osgpu.load()
    counter = [0]
    PES = None
    if os.environ.get("OSGPU_TEST_PES", "gloo") == "shm" or mode in ("hoststaged", "hostcoll"):
        from support import peshm
        PES = peshm.init(rank, world, 1 << 24, dist)
        assert L.osgpu_set_pe_ops(PES.pes_ops()) == 0
    else:
        ops, keep = pe_ops(rank, world, counter)
        assert L.osgpu_set_pe_ops(ctypes.byref(ops)) == 0
    res = {"rank": rank}
    if mode == "hoststaged":
        import oracle as O
        base = PES.pes_heap(rank)
        out = {}
        for t, op, n, dist_ in (("double", "sum", 300_007, "wide"), ("float", "max", 4097, "edge"),
                                ("long", "or", 65, "or"), ("complexf", "prod", 1000, "edge"),
                                ("longdouble", "min", 333, "edge")):
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            src = np.ascontiguousarray(O.gen_input(t, n, O.pe_seed(0xDEF, rank), dist_))
            raw = src.view(np.uint8).reshape(-1)
            toff = (n * s + 4095) // 4096 * 4096
            # symmetric pSync at the top of the shared heap (the staged path
            # exchanges its staging-buffer handles through spare pSync words)
            psync = base + (1 << 24) - 4096
            for hp, inplace in (("staged", False), ("staged", True), ("getmem", False)):
                os.environ["OSGPU_HOST_PATH"] = hp
                ctypes.memmove(base, raw.ctypes.data, raw.size)
                tgt = base + (0 if inplace else toff)
                wrk = (ctypes.c_byte * 4096)()
                getattr(L, f"shmem_{t}_{op}_to_all")(tgt, base, n, 0, 0, world, wrk, psync)
                got = np.frombuffer(ctypes.string_at(tgt, n * s), dtype=np.uint8)
                if t == "longdouble":
                    got = got.reshape(-1, 16)[:, :10].reshape(-1)
                out[f"{t}/{op}/{hp}/{int(inplace)}"] = got.tobytes().hex()
                assert not any(ctypes.string_at(psync, 1024)), "pSync not reset"
                dist.barrier()
        for hp in ("staged", "getmem"):
            os.environ["OSGPU_HOST_PATH"] = hp
            run_colls(L, rank, world, base, base + (1 << 22), psync, out, hp,
                      lambda off, raw: ctypes.memmove(off, raw.ctypes.data, raw.size),
                      lambda off, nb: np.frombuffer(ctypes.string_at(off, nb), np.uint8))
        os.environ.pop("OSGPU_HOST_PATH", None)
        res["out"] = out
    if mode == "hostcoll":
        psync = PES.pes_heap(rank) + (1 << 24) - 4096
        buf = PES.pes_heap(rank)
        for kind in ("broadcast", "collect", "fcollect", "alltoall"):
            for bits in (32, 64):
                f = osgpu.coll(kind, bits)
                if kind == "broadcast":
                    f(buf, buf, 0, world - 1, 0, 0, world, psync)
                else:
                    f(buf, buf, 0, 0, 0, world, psync)
                assert not any(ctypes.string_at(psync, 512)), "pSync not reset"
        res["zero_byte_collectives"] = "ok"
    if mode == "host":
        res["order"] = osgpu.fold_order(rank, 0, 0, world)
        res["shards"] = {str(eb): [osgpu.shard_range(n, world, rank, eb)
                                   for n in (0, 1, 63, 1000, 4097, 1 << 20)]
                         for eb in (2, 4, 8, 16)}
        psync = (ctypes.c_long * 128)()
        buf = (ctypes.c_double * 8)()
        L.shmem_double_sum_to_all(buf, buf, 0, 0, 0, world, buf, psync)
        res["barriers"] = counter[0]
    elif mode == "ipc":
        import torch
        import oracle as O
        torch.cuda.set_device(0)
        H = 1 << 22
        heap = torch.zeros(H, dtype=torch.uint8, device="cuda:0")
        h = (ctypes.c_char * 64)()
        assert L.osgpu_ipc_get_handle(ctypes.c_void_p(heap.data_ptr()), h) == 0
        hs = [None] * world
        dist.all_gather_object(hs, bytes(h))
        mapped = []
        for pe in range(world):
            if pe == rank:
                base = heap.data_ptr()
            else:
                base = L.osgpu_ipc_open((ctypes.c_char * 64).from_buffer_copy(hs[pe]))
                assert base, L.osgpu_last_error().decode()
                mapped.append(base)
            assert L.osgpu_heap_register(pe, ctypes.c_void_p(base), H) == 0
        out = {}
        for t, op, n, dist_ in (("double", "sum", 100_003, "wide"), ("float", "min", 4097, "edge"),
                                ("int", "prod", 1000, "bits"), ("complexd", "prod", 999, "edge"),
                                ("longdouble", "sum", 517, "wide"), ("short", "xor", 4096, "bits")):
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            src = O.gen_input(t, n, O.pe_seed(0xABC, rank), dist_)
            toff = (n * s + 4095) // 4096 * 4096
            raw = np.ascontiguousarray(src).view(np.uint8).reshape(-1)
            for path, inplace in ((osgpu.PATH_AUTO, False), (osgpu.PATH_PULL, False),
                                  (osgpu.PATH_AUTO, True)):
                heap[: raw.size].copy_(torch.from_numpy(raw.copy()).cuda())
                torch.cuda.synchronize()
                L.osgpu_set_path(path)
                psync = (ctypes.c_long * 128)()
                wrk = (ctypes.c_byte * 4096)()
                tgt = heap.data_ptr() + (0 if inplace else toff)
                dist.barrier()
                getattr(L, f"shmem_{t}_{op}_to_all")(tgt, heap.data_ptr(), n, 0, 0, world,
                                                     wrk, psync)
                torch.cuda.synchronize()
                got = heap[(0 if inplace else toff):(0 if inplace else toff) + n * s].cpu().numpy()
                if t == "longdouble":
                    got = got.reshape(-1, 16)[:, :10].reshape(-1)
                out[f"{t}/{op}/{path}/{int(inplace)}"] = got.tobytes().hex()
                dist.barrier()
        L.osgpu_set_path(osgpu.PATH_AUTO)
        if PES is not None:  # collect needs the runtime's getmem (pSync words)
            psync = PES.pes_heap(rank) + (1 << 24) - 4096

            def wr(off, raw):
                lo = off - heap.data_ptr()
                heap[lo:lo + raw.size].copy_(torch.from_numpy(raw.copy()).cuda())
                torch.cuda.synchronize()

            def rd(off, nb):
                torch.cuda.synchronize()
                lo = off - heap.data_ptr()
                return heap[lo:lo + nb].cpu().numpy()

            run_colls(L, rank, world, heap.data_ptr(), heap.data_ptr() + (1 << 21), psync, out,
                      "device", wr, rd)
        res["out"] = out
        dist.barrier()
        for p in mapped:
            L.osgpu_ipc_close(ctypes.c_void_p(p))
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
