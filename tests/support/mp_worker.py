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
  golden  GPU, IPC device heaps + shared-memory runtime: every golden case
        whose PEs fit in the job (tests/golden/reduce_cases.json), team and
        pull form, so small calls run the fused one-launch path with its
        device-side barriers between processes; per-PE SHA-256 and the path
        taken are written for the parent; then calls around a 64 KiB fused
        limit are checked against the oracle
  goldenhost  the same golden cases on host heaps (the shared-memory
        symmetric heap, pinned on every PE): small calls take the fused staged
        path (H2D, exchange and D2H in one launch), larger ones STAGED
  collgolden  GPU, IPC device heaps: broadcast / collect / fcollect /
        alltoall cases of support/coll_cases.py fused_cases (active subsets,
        roots, odd sizes, source == target); small calls run the fused
        one-launch copy; SHA-256 of every target region (margins included)
  latency  GPU, same setup: per-call time of shmem_int_sum_to_all, fused
        path vs host barriers (bench/tool use)
usage: RANK=.. WORLD_SIZE=.. MASTER_ADDR=127.0.0.1 MASTER_PORT=.. \
       python mp_worker.py MODE OUTDIR
"""
import ctypes
import json
import os
import sys
import time

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


def finalize_cycle_mode(L, PES, rank, world, cycles=4):
    """osgpu_finalize between rounds of calls, 2 processes: every round
    re-creates the staging sets, the device-barrier flag areas and their
    HIP IPC mappings (the previous ones closed), then runs a host-staged
    reduce, a fused small device call and a team device call on an
    osgpu_heap_create heap -- each checked bit for bit."""
    import torch
    import oracle as O
    torch.cuda.set_device(0)
    PES.pes_barrier.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    hsync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 4096
    bp = ctypes.c_void_p()
    assert L.osgpu_heap_create(64 << 20, 0, 0, world, hsync, ctypes.byref(bp)) == 0
    base = bp.value
    hbase = PES.pes_heap(rank)
    wrk = (ctypes.c_byte * 4096)()
    bad = []
    paths = set()
    for k in range(cycles):
        for what, n, dev in (("staged", 300_007, False), ("fused", 1000, True),
                             ("team", 1 << 20, True)):
            srcs = [O.gen_input("double", n, O.pe_seed(0xF0 + 3 * k + len(what), r), "wide")
                    for r in range(world)]
            want = O.value_bytes(O.to_all("double", "sum", srcs)[rank]).reshape(-1)
            raw = np.ascontiguousarray(srcs[rank]).view(np.uint8).reshape(-1)
            if dev:
                stage = torch.from_numpy(raw.copy()).cuda()
                torch.cuda.synchronize()
                osgpu.copy([base], [stage.data_ptr()], [raw.size])
                torch.cuda.synchronize()
                src, tgt = base, base + (32 << 20)
            else:
                ctypes.memmove(hbase, raw.ctypes.data, raw.size)
                src, tgt = hbase, hbase + (4 << 20)
                L.osgpu_set_host_path(osgpu.HOST_STAGED)
            PES.pes_barrier(0, 0, world, None)
            L.shmem_double_sum_to_all(tgt, src, n, 0, 0, world, wrk, psync)
            ran = osgpu.last_path()
            L.osgpu_set_host_path(-1)
            if dev:
                out_t = torch.empty(n * 8, dtype=torch.uint8, device="cuda:0")
                osgpu.copy([out_t.data_ptr()], [tgt], [n * 8])
                torch.cuda.synchronize()
                got = out_t.cpu().numpy()
            else:
                got = np.frombuffer(ctypes.string_at(tgt, n * 8), np.uint8)
            if not np.array_equal(got, want):
                bad.append((k, what, ran))
            paths.add(ran)
            PES.pes_barrier(0, 0, world, None)
        assert L.osgpu_finalize() == 0
        PES.pes_barrier(0, 0, world, None)
    PES.pes_barrier(0, 0, world, None)
    assert L.osgpu_heap_destroy(ctypes.c_void_p(base)) == 0
    return {"finalize_cycles": cycles, "finalize_bad": bad, "finalize_paths": sorted(paths)}


def heap_leak_mode(L, PES, rank, world):
    """create / destroy heaps of MP_LEAK_GIB GiB per PE (a comma list is
    cycled: "16,8,16,4") MP_LEAK_CYCLES times, a reduction at the far end of
    each heap checked against the oracle.  Destroyed heaps that another
    process imported keep their HBM on this ROCm; heap.cpp's pool hands one
    back (as a prefix) to every later create of the same member set up to
    its size, so the cycles must never run out of HBM.  Then a create larger
    than the device fails with OSGPU_ENOMEM on every member, at once."""
    import torch
    torch.cuda.set_device(0)
    PES.pes_barrier.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192
    import oracle as O
    gibs = [int(x) for x in os.environ.get("MP_LEAK_GIB", "16").split(",")]
    cycles = int(os.environ.get("MP_LEAK_CYCLES", "20"))
    wrk = (ctypes.c_byte * 4096)()
    rsync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 4096
    done, bases, bad, free_gib = 0, [], 0, []
    for k in range(cycles):
        gib = gibs[k % len(gibs)]
        bp = ctypes.c_void_p()
        rc = L.osgpu_heap_create(gib << 30, 0, 0, world, psync, ctypes.byref(bp))
        if rc != 0:
            return {"leak_cycles_done": done, "leak_fail": L.osgpu_last_error().decode(),
                    "leak_gib": gibs, "leak_bases": bases, "leak_bad": bad,
                    "leak_free_gib": free_gib}
        base = bp.value
        bases.append(hex(base))
        # a reduction at the far end of the heap
        n = 1 << 20
        off = (gib << 30) - 2 * n * 8
        srcs = [O.gen_input("double", n, O.pe_seed(0x1EA + k, r), "wide") for r in range(world)]
        want = O.value_bytes(O.to_all("double", "sum", srcs)[rank]).reshape(-1)
        stage = torch.from_numpy(np.ascontiguousarray(srcs[rank]).view(np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        osgpu.copy([base + off], [stage.data_ptr()], [n * 8])
        torch.cuda.synchronize()
        PES.pes_barrier(0, 0, world, None)
        L.shmem_double_sum_to_all(base + off + n * 8, base + off, n, 0, 0, world, wrk, rsync)
        out_t = torch.empty(n * 8, dtype=torch.uint8, device="cuda:0")
        osgpu.copy([out_t.data_ptr()], [base + off + n * 8], [n * 8])
        torch.cuda.synchronize()
        bad += int(not np.array_equal(out_t.cpu().numpy(), want))
        # the registered size is the requested one: beyond it is not symmetric
        past = L.osgpu_heap_translate(ctypes.c_void_p(base + (gib << 30) + 4096), rank,
                                      (rank + 1) % world)
        bad += int(past is not None)
        del stage, out_t
        PES.pes_barrier(0, 0, world, None)
        assert L.osgpu_heap_destroy(ctypes.c_void_p(base)) == 0
        PES.pes_barrier(0, 0, world, None)
        done += 1
        free_gib.append(torch.cuda.mem_get_info()[0] / (1 << 30))
        print(f"heapleak rank {rank} cycle {k} ({gib} GiB) ok, free {free_gib[-1]:.1f} GiB",
              flush=True)
    # more than the device holds: OSGPU_ENOMEM (-6) on every member, quickly
    t0 = time.time()
    bp = ctypes.c_void_p()
    rc = L.osgpu_heap_create(1 << 50, 0, 0, world, psync, ctypes.byref(bp))
    enomem = {"rc": rc, "error": L.osgpu_last_error().decode(), "seconds": time.time() - t0}
    return {"leak_cycles_done": done, "leak_fail": None, "leak_gib": gibs, "leak_bases": bases,
            "leak_bad": bad, "leak_free_gib": free_gib, "enomem": enomem}


def preflight_mode(L, PES, rank, world):
    """osgpu_preflight over a 3-chunk heap (OSGPU_HEAP_CHUNK_BYTES = 64 MiB),
    the STAGED staging areas and the device-barrier flag areas: every probe
    of every peer passes; then a team reduction on the same heap is
    bit-exact (the probes' patterns do not disturb later use)."""
    import torch
    import oracle as O
    torch.cuda.set_device(0)
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192
    bp = ctypes.c_void_p()
    assert L.osgpu_heap_create(3 * (64 << 20), 0, 0, world, psync, ctypes.byref(bp)) == 0, \
        L.osgpu_last_error().decode()
    base = bp.value
    rc, rep = osgpu.preflight(base, 0, 0, world, psync)
    rc_none, rep_none = osgpu.preflight(None, 0, 0, world, psync)   # staging + flags only
    assert not any(ctypes.string_at(psync, 512)), "pSync not reset"
    n = 1 << 20
    srcs = [O.gen_input("double", n, O.pe_seed(0x9F, r), "wide") for r in range(world)]
    want = O.value_bytes(O.to_all("double", "sum", srcs)[rank]).reshape(-1)
    stage = torch.from_numpy(np.ascontiguousarray(srcs[rank]).view(np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    off = (64 << 20) - n * 4            # straddles chunks 0 and 1
    osgpu.copy([base + off], [stage.data_ptr()], [n * 8])
    torch.cuda.synchronize()
    dist.barrier()
    wrk = (ctypes.c_byte * 4096)()
    L.shmem_double_sum_to_all(base + off + n * 8, base + off, n, 0, 0, world, wrk,
                              PES.pes_heap(rank) + PES.pes_heap_bytes() - 4096)
    out_t = torch.empty(n * 8, dtype=torch.uint8, device="cuda:0")
    osgpu.copy([out_t.data_ptr()], [base + off + n * 8], [n * 8])
    torch.cuda.synchronize()
    exact = bool(np.array_equal(out_t.cpu().numpy(), want))
    ran = osgpu.last_path()
    dist.barrier()
    # a planted wrong mapping (heap.cpp test hook): PE 0 reaches PE 1's heap
    # chunks and staging through PE 2's ranges
    os.environ["OSGPU_TEST_HOOKS"] = "1"   # tests/support/osgpu_test_hooks.h
    assert L.osgpu_test_preflight_fault(0, 1) == 0
    rc_fault, rep_fault = osgpu.preflight(base, 0, 0, world, psync)
    assert L.osgpu_test_preflight_fault(-1, -1) == 0
    os.environ.pop("OSGPU_TEST_HOOKS", None)
    dist.barrier()
    assert L.osgpu_heap_destroy(ctypes.c_void_p(base)) == 0
    return {"preflight_rc": rc, "preflight": rep, "preflight_none_rc": rc_none,
            "preflight_none": rep_none, "after_exact": exact, "after_path": ran,
            "fault_rc": rc_fault, "fault": rep_fault}


def preflight_wide_mode(L, PES, rank, world):
    """osgpu_preflight over an active set larger than the team kernel's 8
    members (the remote-write blocks were sized for 8 writers):
    a 2-chunk heap, the staging areas and the flag areas; every probe of
    every peer must pass, and the heap's chunk ends outside the written
    blocks must keep their bytes (nothing written past a block)."""
    import torch
    torch.cuda.set_device(0)
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192
    bp = ctypes.c_void_p()
    chunk = 64 << 20
    assert L.osgpu_heap_create(2 * chunk, 0, 0, world, psync, ctypes.byref(bp)) == 0, \
        L.osgpu_last_error().decode()
    base = bp.value
    # a guard band next to each block: 4 KiB below every high-end block and
    # above every low-end block, filled with a known byte
    wb = (16 * world + 127) // 128 * 128
    guard = torch.full((4096,), 0xA5, dtype=torch.uint8, device="cuda:0")
    spots = [base + wb, base + chunk - wb - 4096, base + chunk + wb,
             base + 2 * chunk - wb - 4096]
    for a in spots:
        osgpu.copy([a], [guard.data_ptr()], [4096])
    torch.cuda.synchronize()
    dist.barrier()
    rc, rep = osgpu.preflight(base, 0, 0, world, psync)
    rc_none, rep_none = osgpu.preflight(None, 0, 0, world, psync)
    torch.cuda.synchronize()
    back = torch.empty(4096, dtype=torch.uint8, device="cuda:0")
    intact = True
    for a in spots:
        osgpu.copy([back.data_ptr()], [a], [4096])
        torch.cuda.synchronize()
        intact = intact and bool(torch.equal(back, guard))
    dist.barrier()
    assert L.osgpu_heap_destroy(ctypes.c_void_p(base)) == 0
    return {"preflight_rc": rc, "preflight": rep, "preflight_none_rc": rc_none,
            "preflight_none": rep_none, "guards_intact": intact}


def mixed_topology_mode(L, rank, world):
    """2 processes x 2 PE threads (4 PEs): osgpu_heap_create must refuse the
    topology on every member (OSGPU_EINVAL, a message naming it) instead of
    importing each remote heap once per thread into ranges only that
    thread's device may access (heap.cpp)."""
    import threading
    import torch
    from support import peshm
    torch.cuda.set_device(0)
    P = peshm.load()
    npes, hb = 2 * world, 1 << 20
    name = f"/osgpu_pes_{os.environ.get('MASTER_PORT', '0')}mx".encode()
    if rank == 0:
        P.pes_unlink(name)
        assert P.pes_init(name, 2 * rank, npes, hb, 1) == 0
    dist.barrier()
    if rank != 0:
        assert P.pes_init(name, 2 * rank, npes, hb, 0) == 0
    dist.barrier()
    if rank == 0:
        P.pes_unlink(name)
    assert L.osgpu_set_pe_ops(P.pes_ops()) == 0
    out = {}

    def pe_thread(pe):
        P.pes_set_thread_pe(pe)
        torch.cuda.set_device(0)
        bp = ctypes.c_void_p()
        rc = L.osgpu_heap_create(64 << 20, 0, 0, npes, P.pes_heap(pe) + hb - 8192,
                                 ctypes.byref(bp))
        out[str(pe)] = {"rc": rc, "error": L.osgpu_last_error().decode()}
        if rc == 0:
            L.osgpu_heap_destroy(bp)

    th = [threading.Thread(target=pe_thread, args=(2 * rank + t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dist.barrier()
    return {"mixed": out}


def heap_cycle_mode(L, PES, rank, world, cycles=6):
    """osgpu_heap_create / osgpu_heap_destroy repeated with growing sizes,
    and two heaps alive at once: each heap gets its own registry segment,
    a reduction inside each is bit-exact, destroying frees the HBM (free
    memory returns to its starting level) and unregisters the ranges."""
    import torch
    import oracle as O
    torch.cuda.set_device(0)
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192
    PES.pes_barrier.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    wrk = (ctypes.c_byte * 4096)()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    segs, bad = [], 0
    for k in range(cycles):
        bases = []
        for h in range(2):                     # two heaps alive at once
            nbytes = (64 << 20) * (k + 1) + (h << 21)
            bp = ctypes.c_void_p()
            rc = L.osgpu_heap_create(nbytes, 0, 0, world, psync, ctypes.byref(bp))
            assert rc == 0, (rc, L.osgpu_last_error().decode())
            bases.append((bp.value, nbytes))
        for base, nbytes in bases:
            n = min(nbytes // 16, 1 << 20)
            src = O.gen_input("double", n, O.pe_seed(0xC0 + k, rank), "wide")
            raw = np.ascontiguousarray(src).view(np.uint8)
            stage = torch.from_numpy(raw.copy()).cuda()
            torch.cuda.synchronize()   # osgpu.copy's default stream does not wait for torch's
            osgpu.copy([base], [stage.data_ptr()], [raw.size])
            torch.cuda.synchronize()
            PES.pes_barrier(0, 0, world, None)
            L.shmem_double_sum_to_all(base + nbytes // 2, base, n, 0, 0, world, wrk, psync)
            got = np.empty(n * 8, np.uint8)
            torch.cuda.synchronize()
            got_t = torch.empty(n * 8, dtype=torch.uint8, device="cuda:0")
            osgpu.copy([got_t.data_ptr()], [base + nbytes // 2], [n * 8])
            torch.cuda.synchronize()
            got[:] = got_t.cpu().numpy()
            allsrc = [O.gen_input("double", n, O.pe_seed(0xC0 + k, r), "wide")
                      for r in range(world)]
            want = O.value_bytes(O.to_all("double", "sum", allsrc)[rank]).reshape(-1)
            ok_ = bool(np.array_equal(got, want))
            bad += int(not ok_)
            if not ok_:
                diff = np.nonzero(got != want)[0]
                print(f"heapcycle rank {rank} cycle {k} heap {bases.index((base, nbytes))}: "
                      f"{diff.size} bytes differ, first {diff[:4].tolist()}, base {base:#x}, "
                      f"path {osgpu.last_path()}", flush=True)
            segs.append(int(L.osgpu_heap_translate(base, rank, rank) == base))
            PES.pes_barrier(0, 0, world, None)
        print(f"heapcycle rank {rank} cycle {k}: bases {[hex(b_) for b_, _ in bases]} "
              f"free {torch.cuda.mem_get_info()[0] >> 20} MiB", flush=True)
        for base, _ in bases:
            assert L.osgpu_heap_destroy(ctypes.c_void_p(base)) == 0
            # the range is no longer a registered heap
            assert L.osgpu_heap_translate(base, rank, rank) in (0, None)
        PES.pes_barrier(0, 0, world, None)
        print(f"heapcycle rank {rank} cycle {k} destroyed: free "
              f"{torch.cuda.mem_get_info()[0] >> 20} MiB", flush=True)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    return {"heap_cycles": cycles, "heap_cycle_bad": bad, "heap_translated": segs,
            "free_drop_MiB": (free0 - free1) / 2**20}


def vmm_heap_mode(L, PES, rank, world):
    """osgpu_heap_create: one contiguous device heap per PE (virtual-memory
    chunks exported as dmabuf descriptors), every member's mapped here.
    A symmetric double array of MP_VMM_BYTES (default 2.5 GiB) per PE --
    beyond what one HIP IPC export can carry -- reduced on the team path
    (owner-computes, host barriers) and on the pull path; the two 2.5 GiB
    targets must be identical bit for bit (osgpu_compare, full size), a
    sample must match the oracle's per-PE fold, and a long xor over the same
    arrays must satisfy checksum(target) == xor of checksum(source_p) at
    full size.  Then a small call (fused one-launch path) on the same heap."""
    import numpy as np
    import torch
    import oracle as O
    torch.cuda.set_device(0)
    nbytes = int(os.environ.get("MP_VMM_BYTES", str(5 << 29)))
    n = nbytes // 8
    nbytes = n * 8
    al = 2 << 20
    slot = (nbytes + al - 1) // al * al
    off_t, off_p, off_s = slot, 2 * slot, 3 * slot      # team target, pull target, small
    heap_bytes = 3 * slot + (16 << 20)
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192
    PES.pes_barrier.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    base_p = ctypes.c_void_p()
    # a member that cannot make its heap (1 PiB): every member gets the same
    # failure, promptly, and nothing is left registered
    import time as _time
    t0 = _time.perf_counter()
    rc = L.osgpu_heap_create(1 << 50 if rank == 1 else 64 << 20, 0, 0, world, psync,
                             ctypes.byref(base_p))
    fail_s = _time.perf_counter() - t0
    assert rc != 0, "a heap of 1 PiB on one member must fail everywhere"
    assert not any(ctypes.string_at(psync, 512)), "pSync not reset"
    rc = L.osgpu_heap_create(heap_bytes, 0, 0, world, psync, ctypes.byref(base_p))
    assert rc == 0, (rc, L.osgpu_last_error().decode())
    assert not any(ctypes.string_at(psync, 512)), "pSync not reset"
    base = base_p.value
    res = {"heap_bytes": heap_bytes, "nbytes": nbytes, "failed_create_s": fail_s}
    # every member's heap is reachable at base + offset on every PE
    for pe in range(world):
        peer = L.osgpu_heap_translate(base + off_t, rank, pe)
        assert peer, f"PE {pe}'s heap not registered"
    wrk = (ctypes.c_byte * 4096)()
    g = torch.Generator(device="cuda:0").manual_seed(0x7A5 + rank)
    stage = torch.empty(n, dtype=torch.float64, device="cuda:0")
    # signed values spread over 2^-20..2^20: FP sums depend on the fold order
    stage.uniform_(-1.0, 1.0, generator=g)
    stage.mul_(torch.exp2(torch.randint(-20, 21, (n,), device="cuda:0", generator=g,
                                        dtype=torch.int32).to(torch.float64)))
    osgpu.copy([base], [stage.data_ptr()], [nbytes])
    torch.cuda.synchronize()
    sync = lambda: PES.pes_barrier(0, 0, world, None)  # noqa: E731
    sync()
    paths = {}
    for name, path, off in (("team", osgpu.PATH_AUTO, off_t), ("pull", osgpu.PATH_PULL, off_p)):
        L.osgpu_set_path(path)
        sync()
        L.shmem_double_sum_to_all(base + off, base, n, 0, 0, world, wrk, psync)
        paths[name] = osgpu.last_path()
        sync()
    L.osgpu_set_path(osgpu.PATH_AUTO)
    res["paths"] = paths
    res["team_vs_pull_mismatch"], _ = osgpu.compare(base + off_t, base + off_p, nbytes)
    res["hash_team"] = osgpu.checksum("double", osgpu.CK_HASH, base + off_t, n)
    # sampled oracle parity: every rank's source at the sampled indices
    idx = torch.randint(0, n, (1 << 15,), generator=torch.Generator().manual_seed(99))
    osgpu.copy([stage.data_ptr()], [base + off_t], [nbytes])
    torch.cuda.synchronize()
    got = stage[idx.cuda()].cpu().numpy()
    osgpu.copy([stage.data_ptr()], [base], [nbytes])
    torch.cuda.synchronize()
    mine = stage[idx.cuda()].cpu()
    allv = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    want = O.fold_with(O.op_elementwise, "double", "sum", [a.numpy() for a in allv], rank, 0, 0,
                       world)
    res["sample_mismatch"] = int(np.count_nonzero(got.view(np.uint64) != want.view(np.uint64)))
    res["sample_checked"] = int(idx.numel())
    # full-size checksum of checksums: long xor on the team path
    L.shmem_long_xor_to_all(base + off_t, base, n, 0, 0, world, wrk, psync)
    paths["xor"] = osgpu.last_path()
    sync()
    cks = [None] * world
    dist.all_gather_object(cks, osgpu.checksum("long", osgpu.CK_XOR, base, n))
    want_x = 0
    for v in cks:
        want_x ^= v
    res["xor_checksum_ok"] = osgpu.checksum("long", osgpu.CK_XOR, base + off_t, n) == want_x
    # a small object on the same heap: the fused one-launch path
    m = 1000
    small = torch.arange(m, dtype=torch.int32, device="cuda:0") + rank
    osgpu.copy([base + off_s], [small.data_ptr()], [m * 4])
    torch.cuda.synchronize()
    sync()
    L.shmem_int_sum_to_all(base + off_s + 8192, base + off_s, m, 0, 0, world, wrk, psync)
    paths["small"] = osgpu.last_path()
    osgpu.copy([small.data_ptr()], [base + off_s + 8192], [m * 4])
    torch.cuda.synchronize()
    want_s = world * np.arange(m, dtype=np.int32) + world * (world - 1) // 2
    res["small_ok"] = bool(np.array_equal(small.cpu().numpy(), want_s))
    del stage
    sync()
    L.osgpu_finalize()
    assert L.osgpu_heap_destroy(ctypes.c_void_p(base)) == 0
    return res


def fuzz_case(k, world):
    """Case k of the multi-process random sweep (the same on every rank)."""
    import oracle as O
    rng = np.random.default_rng(0xF0F0 + k)
    t = O.TYPES[rng.integers(len(O.TYPES))]
    ops = [op for op in O.OPS if O.has_op(t, op)]
    op = ops[rng.integers(len(ops))]
    stride = int(rng.choice([0, 0, 1])) if world >= 2 else 0
    step = 1 << stride
    size = int(rng.integers(1, (world - 1) // step + 2))
    start = int(rng.integers(0, world - (size - 1) * step))
    r = rng.random()
    n = int(rng.choice([0, 1, 2, 15, 63, 64, 65, 257, 1023, 4097])) if r < 0.35 \
        else int(rng.integers(1, 8192)) if r < 0.8 else int(rng.integers(8192, 70000))
    s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
    ph = lambda: s * int(rng.integers(0, 16 // s if s < 16 else 2))  # noqa: E731
    soff = 4096 + ph()
    in_place = bool(rng.random() < 0.15)
    toff = soff if in_place else (soff + n * s + 4095) // 4096 * 4096 + 4096 + ph()
    dists = ["bits", "mixed", "edge"] if t in O.INT_TYPES else \
        (["prod", "edge"] if op == "prod" else ["mixed", "edge", "wide"])
    return dict(t=t, op=op, start=start, stride=stride, size=size, n=n, soff=soff, toff=toff,
                in_place=in_place, dist=dists[rng.integers(len(dists))],
                host=bool(rng.random() < 0.35),
                path=int(rng.choice([osgpu.PATH_AUTO, osgpu.PATH_AUTO, osgpu.PATH_PULL])),
                seed=int(rng.integers(1 << 40)))


def device_heap_modes(L, PES, mode, rank, world):
    import time
    import torch
    import oracle as O
    torch.cuda.set_device(0)
    H = 40 << 20
    heap = torch.zeros(H, dtype=torch.uint8, device="cuda:0")
    h = (ctypes.c_char * 64)()
    assert L.osgpu_ipc_get_handle(ctypes.c_void_p(heap.data_ptr()), h) == 0
    hs = [None] * world
    dist.all_gather_object(hs, bytes(h))
    mapped = []
    for pe in range(world):
        base = heap.data_ptr()
        if pe != rank:
            base = L.osgpu_ipc_open((ctypes.c_char * 64).from_buffer_copy(hs[pe]))
            assert base, L.osgpu_last_error().decode()
            mapped.append(base)
        assert L.osgpu_heap_register(pe, ctypes.c_void_p(base), H) == 0
    psync = PES.pes_heap(rank) + PES.pes_heap_bytes() - 8192  # top of the shm heap
    PES.pes_barrier.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    sync = lambda: PES.pes_barrier(0, 0, world, None)  # noqa: E731
    wrk = (ctypes.c_byte * 4096)()
    dev0 = heap.data_ptr()
    res = {}

    def put(off, arr):
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        if raw.size:
            heap[off:off + raw.size].copy_(torch.from_numpy(raw.copy()).cuda())

    if mode in ("golden", "goldenhost"):
        digests, paths = {}, {}
        host = mode == "goldenhost"
        if host:  # the shared-memory symmetric heap, pinned on every PE
            hbase = PES.pes_heap(rank)
            hbytes = (1 << 26) - (1 << 16)
            assert L.osgpu_host_register(ctypes.c_void_p(hbase), hbytes) == 0
        for ci, c in enumerate(O.load_cases()):
            if c["npes"] > world:
                continue
            t, op, n = c["type"], c["op"], c["nreduce"]
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            act = O.active_set(c["PE_start"], c["logPE_stride"], c["PE_size"])
            toff = max(4096, (n * s + 4095) // 4096 * 4096)
            if host and 2 * toff > hbytes:
                continue
            if rank < c["npes"]:
                if host:
                    raw = np.ascontiguousarray(O.case_inputs(c)[rank]).view(np.uint8).reshape(-1)
                    ctypes.memmove(hbase, raw.ctypes.data, raw.size)
                else:
                    put(0, O.case_inputs(c)[rank])
            fn = getattr(L, f"shmem_{t}_{op}_to_all")
            for path in ((osgpu.PATH_AUTO,) if host else (osgpu.PATH_AUTO, osgpu.PATH_PULL)):
                L.osgpu_set_path(path)
                if host:
                    ctypes.memset(hbase + toff, 0xA5, max(n * s, 16))
                else:
                    heap[toff:toff + max(n * s, 16)].fill_(0xA5)
                    torch.cuda.synchronize()
                sync()
                if rank in act:
                    b0 = hbase if host else dev0
                    fn(b0 + toff, b0, n, c["PE_start"], c["logPE_stride"], c["PE_size"],
                       wrk, psync)
                    paths[f"{ci}/{path}"] = osgpu.last_path()
                    if host:
                        got = np.frombuffer(ctypes.string_at(hbase + toff, n * s), np.uint8)
                    else:
                        got = heap[toff:toff + n * s].cpu().numpy()
                    if t == "longdouble":
                        got = got.reshape(-1, 16)[:, :10].reshape(-1)
                    digests[f"{ci}/{path}"] = O.digest(O.from_value_bytes(t, got))
                    assert not any(ctypes.string_at(psync, 1024)), "pSync not reset"
                sync()
        L.osgpu_set_path(osgpu.PATH_AUTO)
        res["digests"], res["paths"] = digests, paths
        if host:
            # misaligned host arrays: the kernel's PCIe copies fall back to
            # dword / byte accesses
            mis = {}
            for t, op, so, to in (("int", "sum", 4, 4), ("short", "prod", 2, 6),
                                  ("double", "sum", 8, 12), ("complexf", "prod", 3, 5)):
                s = np.dtype(O.NP_DTYPE[t]).itemsize
                for n in (1, 1000, 4099):
                    src = O.team_inputs(t, world, n, 0x77 + n, "wide")
                    want = O.to_all(t, op, src)[rank]
                    raw = np.ascontiguousarray(src[rank]).view(np.uint8).reshape(-1)
                    toff = (n * s + 8192 + 4095) // 4096 * 4096 + to
                    ctypes.memmove(hbase + so, raw.ctypes.data, raw.size)
                    ctypes.memset(hbase + toff, 0x5A, n * s)
                    sync()
                    getattr(L, f"shmem_{t}_{op}_to_all")(hbase + toff, hbase + so, n, 0, 0,
                                                         world, wrk, psync)
                    got = np.frombuffer(ctypes.string_at(hbase + toff, n * s), np.uint8)
                    mis[f"{t}/{op}/{n}/{so}/{to}"] = [
                        bool(np.array_equal(got, want.view(np.uint8).reshape(-1))),
                        osgpu.last_path()]
                    sync()
            res["misaligned"] = mis
            assert L.osgpu_host_unregister(ctypes.c_void_p(hbase)) == 0
    if mode == "fuzz":
        # seeded random calls, the same draw on every rank: (type, op), an
        # active subset of the job at any start and stride, nreduce mostly
        # inside the fused one-launch range, 16-B phases of source and
        # target, in-place, device heaps (team / pull) or the pinned host heap
        # (fused staged / staged); every member's target against the oracle's
        # fold in its order, non-members' targets untouched, pSync back at 0
        hbase = PES.pes_heap(rank)
        hbytes = (1 << 24) - (1 << 16)
        assert L.osgpu_host_register(ctypes.c_void_p(hbase), hbytes) == 0
        bad, paths = [], {}
        for k in range(int(os.environ.get("MP_FUZZ_CASES", "600"))):
            c = fuzz_case(k, world)
            t, op, n = c["t"], c["op"], c["n"]
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            nb = n * s
            src = O.team_inputs(t, world, n, c["seed"], c["dist"])
            act = O.active_set(c["start"], c["stride"], c["size"])
            raw = np.ascontiguousarray(src[rank]).view(np.uint8).reshape(-1)
            soff, toff, host = c["soff"], c["toff"], c["host"]
            b0 = hbase if host else dev0
            if host:
                if raw.size:
                    ctypes.memmove(hbase + soff, raw.ctypes.data, raw.size)
                if not c["in_place"]:
                    ctypes.memset(hbase + toff, 0x5A, max(nb, 16))
            else:
                put(soff, src[rank])
                if not c["in_place"]:
                    heap[toff:toff + max(nb, 16)].fill_(0x5A)
                torch.cuda.synchronize()
            L.osgpu_set_path(c["path"])
            sync()
            if rank in act:
                getattr(L, f"shmem_{t}_{op}_to_all")(b0 + toff, b0 + soff, n, c["start"],
                                                     c["stride"], c["size"], wrk, psync)
                ran = osgpu.last_path()
                paths[ran] = paths.get(ran, 0) + 1
                got = (np.frombuffer(ctypes.string_at(hbase + toff, nb), np.uint8) if host
                       else heap[toff:toff + nb].cpu().numpy())
                if t == "longdouble":
                    got = got.reshape(-1, 16)[:, :10].reshape(-1)
                want = O.to_all(t, op, src, c["start"], c["stride"], c["size"])[rank]
                if not np.array_equal(O.value_bytes(O.from_value_bytes(t, got)),
                                      O.value_bytes(want)):
                    bad.append([k, "target", ran])
                if any(ctypes.string_at(psync, 1024)):
                    bad.append([k, "pSync"])
            elif not c["in_place"]:
                tg = (np.frombuffer(ctypes.string_at(hbase + toff, max(nb, 16)), np.uint8)
                      if host else heap[toff:toff + max(nb, 16)].cpu().numpy())
                if not (tg == 0x5A).all():
                    bad.append([k, "non-member target"])
            sync()
        L.osgpu_set_path(osgpu.PATH_AUTO)
        assert L.osgpu_host_unregister(ctypes.c_void_p(hbase)) == 0
        res["fuzz_bad"], res["fuzz_paths"] = bad, paths
    if mode == "timeout":
        # a member that never enters the call: after one good fused call,
        # rank 0 calls alone; the device barrier must time out and be
        # reported (MP_FATAL=0) or abort the process with a message (=1)
        n = 1024
        put(0, np.arange(n, dtype=np.int32))
        torch.cuda.synchronize()
        sync()
        L.shmem_int_sum_to_all(dev0 + 8192, dev0, n, 0, 0, world, wrk, psync)
        res["first"] = osgpu.last_path()
        sync()
        fatal = int(os.environ.get("MP_FATAL", "0"))
        L.osgpu_set_device_barrier(0.5, fatal)
        if rank == 0:
            t0 = time.perf_counter()
            L.shmem_int_sum_to_all(dev0 + 8192, dev0, n, 0, 0, world, wrk, psync)
            res["alone"] = osgpu.last_path()
            res["seconds"] = time.perf_counter() - t0
            res["error"] = L.osgpu_last_error().decode()
        dist.barrier()
        L.osgpu_set_device_barrier(-1, 1)
    if mode == "late":
        # The last member enters every call MP_LATE_S seconds after the
        # others (entry barrier), on the team and pull forms of the fused
        # reduce, a fused fcollect and a fused collect; then MP_JITTER_CALLS
        # calls whose members enter with random delays of up to 2 ms.  With a
        # short wait slice (OSGPU_DEVICE_BARRIER_SLICE_MS from the test)
        # these go through many continuations at both barriers.  Every
        # result must be bit-exact and nothing may abort: the device barrier
        # waits without bound, like the reference's.
        import random
        late = float(os.environ.get("MP_LATE_S", "1.5"))
        lat = {}
        L.osgpu_last_continuations.restype = ctypes.c_int
        n = 4099
        # the set's flag areas are made by the first fused call (a collective
        # setup with host barriers): make them before anyone is late
        put(0, np.arange(n, dtype=np.int32))
        torch.cuda.synchronize()
        sync()
        L.shmem_int_sum_to_all(dev0 + 65536, dev0, n, 0, 0, world, wrk, psync)
        sync()
        for ci, (t, op, path) in enumerate((("int", "sum", osgpu.PATH_AUTO),
                                            ("double", "sum", osgpu.PATH_AUTO),
                                            ("float", "prod", osgpu.PATH_PULL),
                                            ("complexd", "prod", osgpu.PATH_AUTO))):
            s_ = np.dtype(O.NP_DTYPE[t]).itemsize
            src = O.team_inputs(t, world, n, 0x1A7E + ci, "wide")
            want = O.to_all(t, op, src)[rank]
            toff = (n * s_ + 4095) // 4096 * 4096
            L.osgpu_set_path(path)
            put(0, src[rank])
            heap[toff:toff + n * s_].fill_(0x5A)
            torch.cuda.synchronize()
            sync()
            if rank == world - 1:
                time.sleep(late)
            t0 = time.perf_counter()
            getattr(L, f"shmem_{t}_{op}_to_all")(dev0 + toff, dev0, n, 0, 0, world, wrk, psync)
            dt = time.perf_counter() - t0
            got = heap[toff:toff + n * s_].cpu().numpy()
            lat[f"{t}/{op}/{path}"] = [bool(np.array_equal(got, want.view(np.uint8).reshape(-1))),
                                       osgpu.last_path(), dt, L.osgpu_last_continuations()]
            sync()
        L.osgpu_set_path(osgpu.PATH_AUTO)
        # fused fcollect64 and collect32 with the last member late
        for kind, bits in (("fcollect", 64), ("collect", 32)):
            cnt = 300 + 7 * rank if kind == "collect" else 300
            esz = bits // 8
            raw = np.arange(cnt * esz, dtype=np.uint8) + rank
            counts = [300 + 7 * r if kind == "collect" else 300 for r in range(world)]
            want = np.concatenate([np.arange(c * esz, dtype=np.uint8) + r
                                   for r, c in enumerate(counts)])
            coff = 1 << 20
            put(0, raw)
            heap[coff:coff + want.size].fill_(0x5A)
            torch.cuda.synchronize()
            sync()
            if rank == world - 1:
                time.sleep(late)
            t0 = time.perf_counter()
            osgpu.coll(kind, bits)(dev0 + coff, dev0, cnt, 0, 0, world, psync)
            dt = time.perf_counter() - t0
            got = heap[coff:coff + want.size].cpu().numpy()
            lat[f"{kind}{bits}"] = [bool(np.array_equal(got, want)), osgpu.last_coll_path(), dt,
                                    L.osgpu_last_continuations()]
            sync()
        # random entry delays on every member
        rng = random.Random(77 + rank)
        jit = {"calls": 0, "exact": 0, "paths": [], "continuations": 0}
        for k in range(int(os.environ.get("MP_JITTER_CALLS", "120"))):
            t, op = (("int", "sum"), ("double", "sum"), ("float", "min"))[k % 3]
            m = (1000, 65536, 4099)[k % 3]
            s_ = np.dtype(O.NP_DTYPE[t]).itemsize
            src = O.team_inputs(t, world, m, 0x7700 + k, "wide")
            want = O.to_all(t, op, src)[rank]
            toff = (m * s_ + 4095) // 4096 * 4096
            put(0, src[rank])
            torch.cuda.synchronize()
            sync()
            time.sleep(rng.random() * 0.002)
            getattr(L, f"shmem_{t}_{op}_to_all")(dev0 + toff, dev0, m, 0, 0, world, wrk, psync)
            got = heap[toff:toff + m * s_].cpu().numpy()
            jit["calls"] += 1
            jit["exact"] += bool(np.array_equal(got, want.view(np.uint8).reshape(-1)))
            if osgpu.last_path() not in jit["paths"]:
                jit["paths"].append(osgpu.last_path())
            jit["continuations"] += L.osgpu_last_continuations()
        res["late"], res["jitter"] = lat, jit
    if mode == "collgolden":
        import hashlib
        from support import coll_cases as CC
        import oracle_coll as OC
        digests, paths = {}, {}
        # second pass: collect again under a 256-B fused limit -- the launch
        # then only exchanges the counts when the gathered total is larger
        runs = [(str(ci), c, -1) for ci, c in enumerate(CC.fused_cases())]
        runs += [(f"{ci}/big", c, 256) for ci, c in enumerate(CC.fused_cases())
                 if c["kind"] == "collect"]
        # third pass: every case on the host heap (the shared-memory symmetric
        # heap, pinned on every PE) with staging forced: fused staged copies
        runs += [(f"{ci}/host", c, -1) for ci, c in enumerate(CC.fused_cases())]
        hbase = PES.pes_heap(rank)
        hbytes = 1 << 24
        assert L.osgpu_host_register(ctypes.c_void_p(hbase), hbytes) == 0

        def hput(off, arr):
            raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
            ctypes.memmove(hbase + off, raw.ctypes.data, raw.size)

        for ci, c, lim in runs:
            L.osgpu_set_fused_max_bytes(lim)
            host = ci.endswith("/host")
            # host heaps: forced staging (small calls stay on getmem otherwise)
            if host:
                L.osgpu_set_host_path(osgpu.HOST_STAGED)
            else:
                L.osgpu_set_host_path(-1)
            b0 = hbase if host else dev0
            npes, start, log, size = c["set"]
            if npes > world:
                continue
            per_src, tgt_off, tgt_bytes, src_off = CC.fused_layout(c)
            pes = OC.active_set(start, log, size)
            if rank < npes:
                src, tgt = CC.fused_inputs(c, rank)
                (hput if host else put)(tgt_off - CC.MARGIN, tgt)
                if not c["same"] and src.size:
                    (hput if host else put)(0, src)
            torch.cuda.synchronize()
            sync()
            if rank in pes:
                f = osgpu.coll(c["kind"], c["bits"])
                cnt = CC.fused_counts(c)[rank]
                if c["kind"] == "broadcast":
                    f(b0 + tgt_off, b0 + src_off, cnt, c["root"], start, log, size, psync)
                else:
                    f(b0 + tgt_off, b0 + src_off, cnt, start, log, size, psync)
                paths[ci] = osgpu.last_coll_path()
                assert not any(ctypes.string_at(psync, 1024)), "pSync not reset"
            if rank < npes:
                lo, hi = tgt_off - CC.MARGIN, tgt_off + tgt_bytes + CC.MARGIN
                got = (np.frombuffer(ctypes.string_at(hbase + lo, hi - lo), np.uint8) if host
                       else heap[lo:hi].cpu().numpy())
                digests[ci] = hashlib.sha256(got.tobytes()).hexdigest()
            sync()
        L.osgpu_set_fused_max_bytes(-1)
        L.osgpu_set_host_path(-1)
        assert L.osgpu_host_unregister(ctypes.c_void_p(hbase)) == 0
        res["digests"], res["paths"] = digests, paths
    if mode == "golden":
        # around a 64 KiB fused limit: under, at, just over
        lim = 64 << 10
        L.osgpu_set_fused_max_bytes(lim)
        bound = {}
        for t, op in (("double", "sum"), ("float", "prod"), ("int", "sum")):
            s = np.dtype(O.NP_DTYPE[t]).itemsize
            for n in (lim // s - 5, lim // s, lim // s + 1, lim // 4 // s, lim // 4 // s + 1):
                src = O.team_inputs(t, world, n, 0x77 + n, "wide")
                want = O.to_all(t, op, src)[rank]
                toff = (n * s + 4095) // 4096 * 4096
                for path in (osgpu.PATH_AUTO, osgpu.PATH_PULL):
                    L.osgpu_set_path(path)
                    put(0, src[rank])
                    heap[toff:toff + n * s].fill_(0x5A)
                    torch.cuda.synchronize()
                    sync()
                    getattr(L, f"shmem_{t}_{op}_to_all")(dev0 + toff, dev0, n, 0, 0, world,
                                                         wrk, psync)
                    got = heap[toff:toff + n * s].cpu().numpy()
                    bound[f"{t}/{op}/{n}/{path}"] = [
                        bool(np.array_equal(got, want.view(np.uint8).reshape(-1))),
                        osgpu.last_path(),
                        n * s <= (lim if path == osgpu.PATH_AUTO else lim // 4)]
                    sync()
        L.osgpu_set_fused_max_bytes(-1)
        L.osgpu_set_path(osgpu.PATH_AUTO)
        res["boundary"] = bound
        # misaligned arrays: a shared 16-B phase (vector body + scalar head
        # and tail edges) and differing phases (element-wise body)
        mis = {}
        for t, op in (("short", "sum"), ("int", "prod"), ("float", "sum"), ("double", "prod"),
                      ("complexf", "sum"), ("complexd", "prod"), ("long", "xor")):
            s = np.dtype(O.NP_DTYPE[t]).itemsize
            for n in (1, 17, 1000, 4099):
                src = O.team_inputs(t, world, n, 0x99 + n, "wide" if t != "long" else "bits")
                want = O.to_all(t, op, src)[rank]
                for so, to in ((s, s), (s, 2 * s), (0, s), (8, 8)):
                    if so % s or to % s:
                        continue
                    toff = (n * s + 8192 + 4095) // 4096 * 4096 + to
                    for path in (osgpu.PATH_AUTO, osgpu.PATH_PULL):
                        L.osgpu_set_path(path)
                        put(so, src[rank])
                        heap[toff:toff + n * s].fill_(0x5A)
                        torch.cuda.synchronize()
                        sync()
                        getattr(L, f"shmem_{t}_{op}_to_all")(dev0 + toff, dev0 + so, n, 0, 0,
                                                             world, wrk, psync)
                        got = heap[toff:toff + n * s].cpu().numpy()
                        mis[f"{t}/{op}/{n}/{so}/{to}/{path}"] = [
                            bool(np.array_equal(got, want.view(np.uint8).reshape(-1))),
                            osgpu.last_path()]
                        sync()
        L.osgpu_set_path(osgpu.PATH_AUTO)
        res["misaligned"] = mis
    if mode == "latency":
        reps = int(os.environ.get("MP_REPS", "300"))
        lat = {}
        for n in [int(x) for x in os.environ.get("MP_SIZES", "1024,65536,1048576").split(",")]:
            put(0, np.arange(n, dtype=np.int32) + rank)
            toff = (n * 4 + 4095) // 4096 * 4096
            torch.cuda.synchronize()
            for name, path, lim in (("team", osgpu.PATH_AUTO, 0), ("pull", osgpu.PATH_PULL, 0),
                                    ("fused_team", osgpu.PATH_AUTO, 1 << 30),
                                    ("fused_pull", osgpu.PATH_PULL, 1 << 30)):
                L.osgpu_set_path(path)
                L.osgpu_set_fused_max_bytes(lim)
                ts, evs = [], []
                events = os.environ.get("MP_EVENTS") == "1"  # GPU-side span (own stream)
                if events:
                    st = torch.cuda.Stream()
                    L.osgpu_set_stream(ctypes.c_void_p(st.cuda_stream))
                for r in range(reps + 5):
                    if events:
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                    sync()
                    t0 = time.perf_counter()
                    if events:
                        e0.record(st)
                    L.shmem_int_sum_to_all(dev0 + toff, dev0, n, 0, 0, world, wrk, psync)
                    if events:
                        e1.record(st)
                    sync()
                    ts.append(time.perf_counter() - t0)
                    if events:
                        evs.append((e0, e1))
                torch.cuda.synchronize()
                gpu = [a.elapsed_time(b) * 1e3 for a, b in evs[5:]] or [float("nan")]
                if events:
                    L.osgpu_set_stream(None)
                ran = osgpu.last_path()
                got = heap[toff:toff + n * 4].view(torch.int32).cpu().numpy()
                ok = bool(np.array_equal(got, world * np.arange(n, dtype=np.int32)
                                         + world * (world - 1) // 2))
                # the same call timed in C between the runtime's barriers (as
                # the CPU baseline is timed): no Python in the loop
                fnp = ctypes.cast(L.shmem_int_sum_to_all, ctypes.c_void_p)
                tc = PES.pes_time_to_all(fnp, ctypes.c_void_p(dev0 + toff), ctypes.c_void_p(dev0),
                                         n, 0, 0, world, ctypes.c_void_p(ctypes.addressof(wrk)),
                                         ctypes.c_void_p(psync), reps)
                lat[f"{n}/{name}"] = {"us_median": float(np.median(ts[5:]) * 1e6),
                                      "us_median_timed_in_c": tc * 1e6,
                                      "gpu_us_median": float(np.median(gpu)),
                                      "us_p10": float(np.percentile(ts[5:], 10) * 1e6),
                                      "path": ran, "correct": ok}
            # data-movement collectives on the same device heaps: fused copy
            # (one launch) vs the copy kernel between host barriers
            for kind in ("fcollect", "collect", "broadcast", "alltoall"):
                f = osgpu.coll(kind, 32)
                ne = n // world if kind == "alltoall" else n
                coff = (world * n * 4 + 4095) // 4096 * 4096 + (8 << 20)
                for name, lim in (("host_barriers", 0), ("fused", 1 << 30)):
                    L.osgpu_set_fused_max_bytes(lim)
                    ts = []
                    for r in range(reps + 5):
                        sync()
                        t0 = time.perf_counter()
                        if kind == "broadcast":
                            f(dev0 + coff, dev0, ne, 0, 0, 0, world, psync)
                        else:
                            f(dev0 + coff, dev0, ne, 0, 0, world, psync)
                        sync()
                        ts.append(time.perf_counter() - t0)
                    lat[f"{n}/{kind}32_{name}"] = {"us_median": float(np.median(ts[5:]) * 1e6),
                                                   "us_p10": float(np.percentile(ts[5:], 10) * 1e6),
                                                   "path": osgpu.last_coll_path(),
                                                   "correct": True}
            # host symmetric heap (the shared-memory heap, pinned): pipelined
            # STAGED path vs the fused one-launch staged path
            hbase = PES.pes_heap(rank)
            src_h = np.ctypeslib.as_array((ctypes.c_int32 * n).from_address(hbase))
            src_h[:] = np.arange(n, dtype=np.int32) + rank
            assert L.osgpu_host_register(ctypes.c_void_p(hbase), 1 << 23) == 0
            # host_fold: the library's default for host-heap calls of at most
            # its limit (64 KiB per PE), forced on at every size here
            for name, lim, fold in (("host_staged", 0, 0), ("host_fused_staged", 1 << 30, 0),
                                    ("host_fold", 0, 1 << 30)):
                L.osgpu_set_fused_max_bytes(lim)
                L.osgpu_set_host_fold_max_bytes(fold)
                ts = []
                for r in range(reps + 5):
                    sync()
                    t0 = time.perf_counter()
                    L.shmem_int_sum_to_all(hbase + toff, hbase, n, 0, 0, world, wrk, psync)
                    sync()
                    ts.append(time.perf_counter() - t0)
                got = np.ctypeslib.as_array((ctypes.c_int32 * n).from_address(hbase + toff))
                ok = bool(np.array_equal(got, world * np.arange(n, dtype=np.int32)
                                         + world * (world - 1) // 2))
                ran = osgpu.last_path()
                fnp = ctypes.cast(L.shmem_int_sum_to_all, ctypes.c_void_p)
                tc = PES.pes_time_to_all(fnp, ctypes.c_void_p(hbase + toff), ctypes.c_void_p(hbase),
                                         n, 0, 0, world, ctypes.c_void_p(ctypes.addressof(wrk)),
                                         ctypes.c_void_p(psync), reps)
                lat[f"{n}/{name}"] = {"us_median": float(np.median(ts[5:]) * 1e6),
                                      "us_median_timed_in_c": tc * 1e6,
                                      "us_p10": float(np.percentile(ts[5:], 10) * 1e6),
                                      "path": ran, "correct": ok}
            L.osgpu_set_host_fold_max_bytes(0)
            # the collectives on the same pinned host heap: the runtime's
            # getmem (the default for small calls) vs the forced one-launch
            # staged copy
            if n <= 1 << 16:
                coff = 1 << 22
                for kind in ("fcollect", "broadcast", "alltoall"):
                    f = osgpu.coll(kind, 32)
                    ne = n // world if kind == "alltoall" else n
                    for name, lim in (("host_getmem", 0), ("host_fused_staged", 1 << 30)):
                        L.osgpu_set_fused_max_bytes(lim)
                        if lim:  # the one-launch staged form needs staging forced
                            L.osgpu_set_host_path(osgpu.HOST_STAGED)
                        ts = []
                        for r in range(reps + 5):
                            sync()
                            t0 = time.perf_counter()
                            if kind == "broadcast":
                                f(hbase + coff, hbase, ne, 0, 0, 0, world, psync)
                            else:
                                f(hbase + coff, hbase, ne, 0, 0, world, psync)
                            sync()
                            ts.append(time.perf_counter() - t0)
                        L.osgpu_set_host_path(-1)
                        lat[f"{n}/{kind}32_{name}"] = {
                            "us_median": float(np.median(ts[5:]) * 1e6),
                            "us_p10": float(np.percentile(ts[5:], 10) * 1e6),
                            "path": osgpu.last_coll_path(), "correct": True}
            assert L.osgpu_host_unregister(ctypes.c_void_p(hbase)) == 0
        L.osgpu_set_fused_max_bytes(-1)
        L.osgpu_set_path(osgpu.PATH_AUTO)
        res["latency"] = lat
    dist.barrier()
    L.osgpu_finalize()
    for p in mapped:
        L.osgpu_ipc_close(ctypes.c_void_p(p))
    return res


def mixpush_mode(L, PES, rank, world, iters=24):
    """Host-heap calls (STAGED path through the set's staging buffers)
    alternating with device-heap calls on the push form of the team
    exchange, which scatters into the same staging buffers: a PE that
    leaves the staged call early must not overwrite slots a slower peer is
    still draining into its host target (run_team_push barriers before its
    first scatter).  Arrival order is jittered per call; every result is
    compared bit for bit with the oracle."""
    import random
    import torch
    import oracle as O
    torch.cuda.set_device(0)
    H = 1 << 23
    heap = torch.zeros(H, dtype=torch.uint8, device="cuda:0")
    h = (ctypes.c_char * 64)()
    assert L.osgpu_ipc_get_handle(ctypes.c_void_p(heap.data_ptr()), h) == 0
    hs = [None] * world
    dist.all_gather_object(hs, bytes(h))
    mapped = []
    for pe in range(world):
        if pe == rank:
            b = heap.data_ptr()
        else:
            b = L.osgpu_ipc_open((ctypes.c_char * 64).from_buffer_copy(hs[pe]))
            assert b, L.osgpu_last_error().decode()
            mapped.append(b)
        assert L.osgpu_heap_register(pe, ctypes.c_void_p(b), H) == 0
    base = PES.pes_heap(rank)
    psync = base + (1 << 24) - 4096
    nh, nd = 300_007, 200_003
    hsrc = [O.gen_input("double", nh, O.pe_seed(0x51, r), "wide") for r in range(world)]
    dsrc = [O.gen_input("double", nd, O.pe_seed(0x52, r), "wide") for r in range(world)]
    want_h = O.value_bytes(O.to_all("double", "sum", hsrc)[rank]).reshape(-1).tobytes()
    want_d = O.value_bytes(O.to_all("double", "sum", dsrc)[rank]).reshape(-1).tobytes()
    raw_h = np.ascontiguousarray(hsrc[rank]).view(np.uint8).reshape(-1)
    ctypes.memmove(base, raw_h.ctypes.data, raw_h.size)
    htgt = base + (1 << 23)
    heap[: nd * 8].copy_(torch.from_numpy(np.ascontiguousarray(dsrc[rank]).view(np.uint8).copy()))
    dtoff = 4 << 20
    torch.cuda.synchronize()
    L.osgpu_set_host_path(osgpu.HOST_STAGED)
    L.osgpu_set_fused_max_bytes(0)          # host barriers: the staged pipeline
    rng = random.Random(rank * 7919 + 1)
    bad = {"host": 0, "device": 0}
    paths = set()
    wrk = (ctypes.c_byte * 4096)()
    dist.barrier()
    for it in range(iters):
        ctypes.memset(htgt, 0, nh * 8)
        time.sleep(rng.random() * 0.004)
        L.osgpu_set_team_exchange(0)
        L.shmem_double_sum_to_all(htgt, base, nh, 0, 0, world, wrk, psync)
        paths.add(osgpu.last_path())
        if ctypes.string_at(htgt, nh * 8) != want_h:
            bad["host"] += 1
        time.sleep(rng.random() * 0.004)
        L.osgpu_set_team_exchange(1)
        L.shmem_double_sum_to_all(heap.data_ptr() + dtoff, heap.data_ptr(), nd, 0, 0, world,
                                  wrk, psync)
        paths.add(osgpu.last_path())
        torch.cuda.synchronize()
        if heap[dtoff:dtoff + nd * 8].cpu().numpy().tobytes() != want_d:
            bad["device"] += 1
        heap[dtoff:dtoff + nd * 8].zero_()
        torch.cuda.synchronize()
    L.osgpu_set_team_exchange(-1)
    L.osgpu_set_fused_max_bytes(-1)
    L.osgpu_set_host_path(-1)
    dist.barrier()
    L.osgpu_finalize()
    for p in mapped:
        L.osgpu_ipc_close(ctypes.c_void_p(p))
    return {"mixpush_bad": bad, "mixpush_paths": sorted(paths)}


def main():
    mode, outdir = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    L = osgpu.load()
    # small host-heap calls on the GPU paths (the host fold off) unless the
    # mode measures or checks the host fold itself
    L.osgpu_set_host_fold_max_bytes(-1 if os.environ.get("MP_HOST_FOLD") == "1" else 0)
    counter = [0]
    PES = None
    if os.environ.get("OSGPU_TEST_PES", "gloo") == "shm" or mode in (
            "hoststaged", "hostcoll", "golden", "goldenhost", "collgolden", "latency",
            "timeout", "vmm", "late", "mixpush", "heapcycle", "finalizecycle", "heapleak",
            "fuzz", "preflight", "preflightwide"):
        from support import peshm
        PES = peshm.init(rank, world, (1 << 26) if mode == "goldenhost" else (1 << 24), dist)
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
            # pinned: the heap registered on every PE (osgpu_host_register) --
            # small calls then run the fused one-launch staged path
            for pinned in (False, True):
                if pinned:
                    assert L.osgpu_host_register(ctypes.c_void_p(base), 1 << 24) == 0
                for hp, inplace, fused in (("staged", False, -1), ("staged", True, -1),
                                           ("staged", False, 0), ("getmem", False, -1),
                                           ("fold", False, -1), ("fold", True, -1)):
                    # fold: the automatic path with the host fold on (the
                    # library's default for small host-heap calls)
                    L.osgpu_set_host_path(osgpu.HOST_PATHS.get(hp, osgpu.HOST_AUTO))
                    L.osgpu_set_host_fold_max_bytes(-1 if hp == "fold" else 0)
                    L.osgpu_set_fused_max_bytes(fused)
                    ctypes.memmove(base, raw.ctypes.data, raw.size)
                    tgt = base + (0 if inplace else toff)
                    wrk = (ctypes.c_byte * 4096)()
                    getattr(L, f"shmem_{t}_{op}_to_all")(tgt, base, n, 0, 0, world, wrk, psync)
                    key = f"{t}/{op}/{hp}/{int(inplace)}/{fused}/{int(pinned)}"
                    res.setdefault("paths", {})[key] = osgpu.last_path()
                    got = np.frombuffer(ctypes.string_at(tgt, n * s), dtype=np.uint8)
                    if t == "longdouble":
                        got = got.reshape(-1, 16)[:, :10].reshape(-1)
                    out[key] = got.tobytes().hex()
                    assert not any(ctypes.string_at(psync, 1024)), "pSync not reset"
                    dist.barrier()
                if pinned:
                    assert L.osgpu_host_unregister(ctypes.c_void_p(base)) == 0
            L.osgpu_set_fused_max_bytes(-1)
            L.osgpu_set_host_fold_max_bytes(0)
        for hp in ("staged", "getmem"):
            L.osgpu_set_host_path(osgpu.HOST_PATHS[hp])
            run_colls(L, rank, world, base, base + (1 << 22), psync, out, hp,
                      lambda off, raw: ctypes.memmove(off, raw.ctypes.data, raw.size),
                      lambda off, nb: np.frombuffer(ctypes.string_at(off, nb), np.uint8))
        L.osgpu_set_host_path(-1)
        res["out"] = out
    if mode == "mixpush":
        res.update(mixpush_mode(L, PES, rank, world))
    if mode in ("golden", "goldenhost", "collgolden", "latency", "timeout", "late", "fuzz"):
        res.update(device_heap_modes(L, PES, mode, rank, world))
    if mode == "vmm":
        res.update(vmm_heap_mode(L, PES, rank, world))
    if mode == "heapcycle":
        res.update(heap_cycle_mode(L, PES, rank, world))
    if mode == "heapleak":
        res.update(heap_leak_mode(L, PES, rank, world))
    if mode == "preflight":
        res.update(preflight_mode(L, PES, rank, world))
    if mode == "preflightwide":
        res.update(preflight_wide_mode(L, PES, rank, world))
    if mode == "mixedtopo":
        res.update(mixed_topology_mode(L, rank, world))
    if mode == "finalizecycle":
        res.update(finalize_cycle_mode(L, PES, rank, world))
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
            # fused: -1 = default (one launch, device barriers, when the
            # runtime has getmem for the flag-area exchange), 0 = host barriers
            for path, inplace, fused in ((osgpu.PATH_AUTO, False, -1), (osgpu.PATH_AUTO, False, 0),
                                         (osgpu.PATH_PULL, False, -1), (osgpu.PATH_PULL, False, 0),
                                         (osgpu.PATH_AUTO, True, -1), (osgpu.PATH_AUTO, False, 9)):
                # fused 9: host barriers with the push form of the team exchange
                L.osgpu_set_team_exchange(1 if fused == 9 else 0)
                heap[: raw.size].copy_(torch.from_numpy(raw.copy()).cuda())
                torch.cuda.synchronize()
                L.osgpu_set_path(path)
                L.osgpu_set_fused_max_bytes(0 if fused == 9 else fused)
                # pSync must be symmetric (getmem-able) when the runtime has getmem
                psync = (PES.pes_heap(rank) + (1 << 24) - 8192 if PES is not None
                         else ctypes.addressof((ctypes.c_long * 128)()))
                wrk = (ctypes.c_byte * 4096)()
                tgt = heap.data_ptr() + (0 if inplace else toff)
                dist.barrier()
                getattr(L, f"shmem_{t}_{op}_to_all")(tgt, heap.data_ptr(), n, 0, 0, world,
                                                     wrk, psync)
                ran = osgpu.last_path()
                torch.cuda.synchronize()
                got = heap[(0 if inplace else toff):(0 if inplace else toff) + n * s].cpu().numpy()
                if t == "longdouble":
                    got = got.reshape(-1, 16)[:, :10].reshape(-1)
                out[f"{t}/{op}/{path}/{int(inplace)}/{fused}"] = got.tobytes().hex()
                res.setdefault("paths", {})[f"{t}/{op}/{path}/{int(inplace)}/{fused}"] = ran
                dist.barrier()
        L.osgpu_set_path(osgpu.PATH_AUTO)
        L.osgpu_set_fused_max_bytes(-1)
        L.osgpu_set_team_exchange(-1)
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
