"""Multi-process (one process per PE) runs of libosgpu_reduce.so, world size 2.

* CPU (gloo, no GPU): PE services supplied through Python callbacks
  (my_pe = rank, shmem_barrier = dist.barrier) as bench.py does at N > 1;
  fold orders and shard partitions agree across ranks; the nreduce = 0
  collective performs exactly the reference's two barriers
  (src/reductions.c:82,113).
* GPU: two processes share cuda:0, export/import their device heaps over HIP
  IPC (the multi-GPU path's mechanism) and run shmem_*_to_all on the team
  path, the pull path and in place; every PE's target must equal the oracle
  bit for bit.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "support", "mp_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(mode, world, tmp_path, timeout=600):
    """Run `world` worker processes; each one's output goes to a log file as
    it is written (under $MP_LOG_DIR when set, e.g. gpurun_out/, so a stalled
    rank shows where it stopped), and its tail is reported on failure."""
    port = _free_port()
    logdir = os.environ.get("MP_LOG_DIR") or str(tmp_path)
    os.makedirs(logdir, exist_ok=True)
    procs = []
    extra = {}
    # PE processes sharing one GPU: at most 16 hardware queues between them
    # (HIP's default is four per process; more than 16 on the GPU and its
    # scheduler time-slices the queues in milliseconds, INTEGRATION.md,
    # profiles/r02_mp_latency_hwq.jsonl).  MP_HWQ=default keeps HIP's default.
    # (the box exports HIP's default, 4: lowered here, never raised)
    if world > 4 and os.environ.get("MP_HWQ") != "default":
        extra["GPU_MAX_HW_QUEUES"] = str(min(max(1, 16 // world),
                                             int(os.environ.get("GPU_MAX_HW_QUEUES", "16"))))
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1",
                   **extra)
        log = os.path.join(logdir, f"{mode}_w{world}_rank{r}.log")
        f = open(log, "w")
        procs.append((subprocess.Popen([sys.executable, WORKER, mode, str(tmp_path)], env=env,
                                       stdout=f, stderr=subprocess.STDOUT), f, log))
    try:
        for p, f, _ in procs:
            p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        for q, _, _ in procs:
            q.kill()
        raise
    finally:
        for _, f, _ in procs:
            f.close()
    for p, _, log in procs:
        assert p.returncode == 0, open(log).read()[-3000:]
    return [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]


def test_host_logic_world2(tmp_path):
    res = launch("host", 2, tmp_path)
    assert [r["order"] for r in res] == [O.fold_order(0, 0, 0, 2), O.fold_order(1, 0, 0, 2)]
    for eb in ("2", "4", "8", "16"):
        for k, n in enumerate((0, 1, 63, 1000, 4097, 1 << 20)):
            lo0, hi0 = res[0]["shards"][eb][k]
            lo1, hi1 = res[1]["shards"][eb][k]
            assert lo0 == 0 and hi0 == lo1 and hi1 == n
    assert [r["barriers"] for r in res] == [2, 2]


def test_zero_byte_collectives_processes(tmp_path):
    """broadcast/collect/fcollect/alltoall with nelems = 0, one process per
    PE over the shared-memory runtime, no GPU: only synchronisation."""
    res = launch("hostcoll", 2, tmp_path)
    assert [r["zero_byte_collectives"] for r in res] == ["ok", "ok"]


def _check_colls(res, tag):
    from support import coll_cases as CC
    world = len(res)
    n = 0
    for kind, bits, counts, root in CC.cases(world):
        want = CC.expected(kind, bits, counts, root, world)
        for r in range(world):
            assert res[r]["out"][CC.key(kind, bits, tag)] == want[r].tobytes().hex(), \
                (kind, bits, tag, r)
            n += 1
    assert n == 8 * world


def _check_specs(res, specs, seed):
    for t, op, n, d in specs:
        src = [O.gen_input(t, n, O.pe_seed(seed, r), d) for r in range(len(res))]
        want = O.to_all(t, op, src)
        for r in range(len(res)):
            wb = O.value_bytes(want[r]).reshape(-1).tobytes().hex()
            keys = [k for k in res[r]["out"] if k.startswith(f"{t}/{op}/")]
            assert keys
            for key in keys:
                assert res[r]["out"][key] == wb, (key, r)


@pytest.mark.gpu
@pytest.mark.parametrize("pes", ["gloo", "shm"])
def test_ipc_heaps_two_processes(tmp_path, monkeypatch, pes):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OSGPU_TEST_PES", pes)
    res = launch("ipc", 2, tmp_path)
    specs = (("double", "sum", 100_003, "wide"), ("float", "min", 4097, "edge"),
             ("int", "prod", 1000, "bits"), ("complexd", "prod", 999, "edge"),
             ("longdouble", "sum", 517, "wide"), ("short", "xor", 4096, "bits"))
    _check_specs(res, specs, 0xABC)
    # which path ran: with the shm runtime (getmem available) calls of at most
    # 1 MiB per PE (team form; 256 KiB pull form) take the fused one-launch
    # path unless it is switched off (suffix /0); long double and the gloo
    # runtime keep host barriers
    for t, op, n, _ in specs:
        for r in range(2):
            for key, ran in res[r]["paths"].items():
                if not key.startswith(f"{t}/{op}/"):
                    continue
                path, inplace, fused = key.split("/")[2:]
                team = path == "0" and inplace == "0"
                s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
                fusable = (pes == "shm" and fused == "-1" and t != "longdouble" and
                           n * s <= (1 << 20) // (1 if team else 4))
                want = ("fused_" if fusable else "") + ("team" if team else "pull")
                if fused == "9":  # push form: needs the staging exchange (getmem)
                    want = "team_push" if pes == "shm" else "team"
                assert ran == want, (key, r, ran)
    if pes == "shm":  # collect needs getmem: the shm runtime has it
        _check_colls(res, "device")


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_staged_then_push_processes(tmp_path, world, monkeypatch):
    """A host-heap call (STAGED, 64 KiB chunks) followed by a device-heap call
    on the push form of the team exchange, 24 times with jittered arrivals:
    both scatter through the set's staging buffers, and every result stays
    bit-exact (the push exchange barriers before its first scatter)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OSGPU_STAGE_BYTES", "65536")
    res = launch("mixpush", world, tmp_path)
    for r in res:
        assert r["mixpush_bad"] == {"host": 0, "device": 0}, r
        assert r["mixpush_paths"] == ["staged", "team_push"], r


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_host_staged_processes(tmp_path, world, monkeypatch):
    """Host symmetric heaps (shared memory), one process per PE -- the
    reference's own data placement.  STAGED: H2D -> exchange through the
    IPC-mapped staging buffers -> D2H (64 KiB chunks: many pipeline turns);
    GETMEM: peers' sources pulled through the runtime's getmem; fold: the
    default automatic path, whose calls pulling at most 256 KiB per PE are
    folded on the host (shmem_reduce.cpp run_host_fold) -- bit-exact against the same
    golden vectors."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OSGPU_STAGE_BYTES", "65536")
    res = launch("hoststaged", world, tmp_path)
    specs = (("double", "sum", 300_007, "wide"), ("float", "max", 4097, "edge"),
             ("long", "or", 65, "or"), ("complexf", "prod", 1000, "edge"),
             ("longdouble", "min", 333, "edge"))
    _check_specs(res, specs, 0xDEF)
    # small calls on a pinned heap: the fused one-launch staged path
    for r in range(world):
        for key, ran in res[r]["paths"].items():
            t, op, hp, inplace, fused, pinned = key.split("/")
            n = next(sp[2] for sp in specs if sp[0] == t and sp[1] == op)
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            small = fused == "-1" and t != "longdouble" and n * s <= (1 << 20)
            want = ("getmem" if hp == "getmem" else
                    "host_fold" if hp == "fold" and (world - 1) * n * s <= (256 << 10) else
                    "fused_staged" if pinned == "1" and small else "staged")
            assert ran == want, (key, r, ran)
    _check_colls(res, "staged")
    _check_colls(res, "getmem")



@pytest.mark.gpu
def test_fused_path_golden_processes(tmp_path):
    """Eight processes share cuda:0 (IPC device heaps, shared-memory runtime):
    every golden case (up to 8 PEs, active subsets included), team and pull
    form.  Calls of at
    most 1 MiB per PE (all types but long double) run as ONE launch whose
    barriers are device flags written across processes; the rest keep host
    barriers.  Per-PE results bit-exact against the reference digests, and
    calls around a 64 KiB fused limit bit-exact against the oracle."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 8
    res = launch("golden", world, tmp_path)
    cases = O.load_cases()
    nfused = nchecked = 0
    for r in range(world):
        for key, dg in res[r]["digests"].items():
            ci, path = key.split("/")
            c = cases[int(ci)]
            assert dg == c["digests"][str(r)], (c["type"], c["op"], c["npes"], c["nreduce"],
                                                c["tag"], path, r)
            nchecked += 1
            s = 16 if c["type"] == "longdouble" else np.dtype(O.NP_DTYPE[c["type"]]).itemsize
            ran = res[r]["paths"][key]
            if c["nreduce"] == 0:
                want = "barrier_only"
            else:
                team = path == "0" and c["PE_size"] >= 2
                fused = (c["type"] != "longdouble" and c["PE_size"] >= 2 and
                         c["nreduce"] * s <= (1 << 20) // (1 if team else 4))
                want = ("fused_" if fused else "") + ("team" if team else "pull")
            assert ran == want, (key, r, ran, want)
            nfused += ran.startswith("fused_")
    assert nchecked > 8000 and nfused > 6000, (nchecked, nfused)
    for r in range(world):
        for key, (exact, ran, fused) in res[r]["boundary"].items():
            assert exact, (key, r)
            assert ran.startswith("fused_") == fused, (key, r, ran)
    # misaligned sources/targets (shared and differing 16-B phases), fused
    for r in range(world):
        assert len(res[r]["misaligned"]) > 100
        for key, (exact, ran) in res[r]["misaligned"].items():
            assert exact, (key, r)
            assert ran.startswith("fused_"), (key, r, ran)


@pytest.mark.gpu
def test_random_calls_processes(tmp_path):
    """Four processes on cuda:0, 600 seeded random calls drawn the same on
    every rank (tests/support/mp_worker.py fuzz_case): any (type, op), active
    subsets at any start and stride, nreduce mostly inside the one-launch
    range, 16-B phases, in-place, device heaps and the pinned host heap.
    Every member's target bit-exact against the oracle's fold in its order,
    non-members untouched, pSync reset; the one-launch paths (device
    barriers) and the host-barrier paths are both exercised."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = launch("fuzz", 4, tmp_path)
    paths = {}
    for r in res:
        assert r["fuzz_bad"] == [], (r["rank"], r["fuzz_bad"][:5])
        for k, v in r["fuzz_paths"].items():
            paths[k] = paths.get(k, 0) + v
    for p in ("fused_team", "fused_pull", "fused_staged", "team", "pull"):
        assert paths.get(p, 0) > 0, paths


@pytest.mark.gpu
def test_fused_staged_golden_processes(tmp_path):
    """The golden cases with at most 4 PEs on HOST symmetric heaps (the
    reference's placement: a shared-memory heap, pinned on every PE), four
    processes on cuda:0.  Calls of at most 1 MiB per PE (not long double)
    run as one launch that copies the source in over PCIe, exchanges on the
    GPU and copies the target out; larger ones take the pipelined STAGED
    path.  Every member's target bit-exact against the reference digests."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 4
    res = launch("goldenhost", world, tmp_path)
    cases = O.load_cases()
    nfused = nchecked = 0
    for r in range(world):
        for key, dg in res[r]["digests"].items():
            c = cases[int(key.split("/")[0])]
            assert dg == c["digests"][str(r)], (c["type"], c["op"], c["npes"], c["nreduce"],
                                                c["tag"], r)
            nchecked += 1
            s = 16 if c["type"] == "longdouble" else np.dtype(O.NP_DTYPE[c["type"]]).itemsize
            ran = res[r]["paths"][key]
            if c["nreduce"] == 0:
                want = "barrier_only"
            elif c["type"] != "longdouble" and c["PE_size"] >= 2 and c["nreduce"] * s <= 1 << 20:
                want = "fused_staged"
            else:
                want = "staged"
            assert ran == want, (key, r, ran, want)
            nfused += ran == "fused_staged"
    assert nchecked > 1000 and nfused > 700, (nchecked, nfused)
    for r in range(world):  # misaligned host arrays (dword / byte PCIe copies)
        for key, (exact, ran) in res[r]["misaligned"].items():
            assert exact and ran == "fused_staged", (key, r, ran)


@pytest.mark.gpu
def test_fused_collectives_processes(tmp_path):
    """broadcast / collect / fcollect / alltoall (32/64) with one process per
    PE (8 on cuda:0, IPC device heaps): small calls run as one launch with
    the device-side barriers (fused copy; collect's counts ride on the device
    arrival).  collect again under a 256-B limit: the launch exchanges the
    counts and the COPY path moves the larger totals.  Every member's target
    region, margins included, must equal the restatement's
    (oracle/oracle_coll.py)."""
    import hashlib
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from support import coll_cases as CC
    world = 8
    res = launch("collgolden", world, tmp_path)
    nfused = nbig = nhost = 0
    for ci, c in enumerate(CC.fused_cases()):
        if c["set"][0] > world:
            continue
        exp = CC.fused_expected(c)
        keys = [str(ci), f"{ci}/host"] + ([f"{ci}/big"] if c["kind"] == "collect" else [])
        total = sum(CC.fused_counts(c).values()) * c["bits"] // 8
        for key in keys:
            for r in range(c["set"][0]):
                want = hashlib.sha256(exp[r].tobytes()).hexdigest()
                assert res[r]["digests"][key] == want, (c, key, r)
                ran = res[r]["paths"].get(key)
                if ran is None:
                    continue
                if key.endswith("/host"):
                    # staging forced (OSGPU_HOST_PATH=staged); collect keeps
                    # its count exchange and the chunked STAGED copy
                    want = ("fused_staged" if c["kind"] != "collect" else
                            "staged" if total else "barrier_only")
                    assert ran == want, (c, key, r, ran)
                    nhost += ran == "fused_staged"
                elif key.endswith("/big") and total > 256:
                    assert ran == "copy", (c, key, r, ran)
                    nbig += 1
                else:
                    assert ran == "fused_copy", (c, key, r, ran)
                    nfused += 1
    assert nfused > 800 and nbig > 100 and nhost > 600, (nfused, nbig, nhost)


@pytest.mark.gpu
def test_finalize_cycles_processes(tmp_path):
    """osgpu_finalize between rounds, 2 processes: the staging sets, flag
    areas and their IPC mappings are made again each round, and a
    host-staged reduce, a fused small call and a team call stay bit-exact."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = launch("finalizecycle", 2, tmp_path, timeout=300)
    for r in res:
        assert r["finalize_bad"] == [], r
        assert r["finalize_paths"] == ["fused_team", "staged", "team"], r


@pytest.mark.gpu
def test_heap_reuse_processes(tmp_path, monkeypatch):
    """Twelve rounds of heaps of 16, 8, 16 and 4 GiB per PE made and
    destroyed by 2 processes (144 GiB per PE in all).  A destroyed heap with
    imported chunks keeps its HBM on this ROCm; heap.cpp's pool hands it
    back, as a prefix of its range, to every later create of the same member
    set up to its size -- same base every round, free HBM flat after the
    first, a reduction at each heap's far end bit-exact against the oracle,
    nothing registered past the requested size.  Then a create larger than
    the device fails with OSGPU_ENOMEM (-6) on every member within seconds."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if torch.cuda.mem_get_info()[1] < (100 << 30):
        pytest.skip("needs a GPU of at least 100 GiB")
    monkeypatch.setenv("MP_LEAK_GIB", "16,8,16,4")
    monkeypatch.setenv("MP_LEAK_CYCLES", "12")
    res = launch("heapleak", 2, tmp_path, timeout=400)
    for r in res:
        assert r["leak_fail"] is None and r["leak_cycles_done"] == 12, r
        assert r["leak_bad"] == 0, r
        assert len(set(r["leak_bases"])) == 1, r
        assert min(r["leak_free_gib"]) > r["leak_free_gib"][0] - 1.0, r["leak_free_gib"]
        e = r["enomem"]
        assert e["rc"] == -6 and e["seconds"] < 10, e
        assert "out of device memory" in e["error"], e


@pytest.mark.gpu
def test_preflight_processes(tmp_path, monkeypatch):
    """osgpu_preflight with 3 processes on cuda:0 over a heap of three
    64-MiB chunks: every chunk end, staging area and flag word of every peer
    reads back its owner's pattern through this process's mapping (host copy
    and copy kernel), and every peer's remote writes into this process's
    chunk ends and staging area (host copy, then copy kernel) reach it; a
    reduction on the same heap afterwards is bit-exact.  A planted wrong
    mapping (osgpu_test_preflight_fault(0, 1): PE 0 reaches PE 1 through PE 2's
    ranges) fails PE 0's reads of PE 1 and PE 1's check of PE 0's writes."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OSGPU_HEAP_CHUNK_BYTES", str(64 << 20))
    world = 3
    res = launch("preflight", world, tmp_path, timeout=300)
    for r in range(world):
        x = res[r]
        assert x["preflight_rc"] == 0, x["preflight"]
        peers = sorted(x["preflight"])
        assert peers == sorted(str(p) for p in range(world) if p != r), x["preflight"]
        for p in peers:
            e = x["preflight"][p]
            assert e == {"chunks": 3, "staging": True, "flags": True, "status": "ok",
                         "remote_write": "ok"}, (r, p, e)
            f = x["preflight_none"][p]
            assert f["chunks"] == 0 and f["staging"] and f["status"] == "ok", (r, p, f)
            assert f["remote_write"] == "ok", (r, p, f)
        assert x["after_exact"] and x["after_path"] == "team", x
    # the planted fault: PE 0's reads of PE 1 read PE 2's data; PE 1 never
    # sees PE 0's writes (they went to PE 2); both calls fail
    f0, f1 = res[0]["fault"], res[1]["fault"]
    assert res[0]["fault_rc"] != 0 and res[1]["fault_rc"] != 0, (f0, f1)
    assert "read other data" in f0["1"]["status"], f0
    assert f0["2"]["status"] == "ok", f0
    rw = f1["0"]["remote_write"]
    assert "not seen by the owner" in rw and "heap chunk 2 high" in rw and "staging" in rw, f1
    assert f1["2"]["remote_write"] == "ok", f1


@pytest.mark.gpu
def test_preflight_more_than_8_members(tmp_path, monkeypatch):
    """osgpu_preflight with 10 processes on cuda:0 (more than the team
    kernel's 8): every probe and remote write of every peer passes, and the
    bytes next to every written block are untouched (the blocks are sized
    by the active set)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OSGPU_HEAP_CHUNK_BYTES", str(64 << 20))
    world = 10
    res = launch("preflightwide", world, tmp_path, timeout=300)
    for r in range(world):
        x = res[r]
        assert x["preflight_rc"] == 0 and x["preflight_none_rc"] == 0, x
        assert sorted(x["preflight"]) == sorted(str(p) for p in range(world) if p != r)
        for p, e in x["preflight"].items():
            assert e["chunks"] == 2 and e["status"] == "ok" and e["remote_write"] == "ok", (r, p, e)
        assert x["guards_intact"], x


@pytest.mark.gpu
def test_heap_refuses_mixed_topology(tmp_path):
    """2 processes x 2 PE threads: osgpu_heap_create refuses the topology
    on all 4 PEs (OSGPU_EINVAL with a message) -- never per-thread imports
    registered process-wide (the last writer would win)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = launch("mixedtopo", 2, tmp_path, timeout=200)
    got = {}
    for r in res:
        got.update(r["mixed"])
    assert sorted(got) == ["0", "1", "2", "3"], got
    for pe, x in got.items():
        assert x["rc"] == -1 and "unsupported topology" in x["error"], (pe, x)


@pytest.mark.gpu
def test_heap_create_destroy_cycles_processes(tmp_path):
    """osgpu_heap_create / osgpu_heap_destroy six times over, two heaps
    alive at once, 2 processes: every reduction inside every heap bit-exact
    (a new heap's range must not reach an old heap's memory: heap.cpp keeps
    imported ranges reserved), ranges registered while alive and
    unregistered after destroy.  The HBM of heaps that another process
    imported does not come back before the processes exit on this ROCm
    (every unmap / release call succeeds): the drop is
    recorded and bounded by the bytes of all heaps made."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = launch("heapcycle", 2, tmp_path, timeout=300)
    made_MiB = 2 * sum(2 * 64 * (k + 1) + 2 for k in range(6))   # both processes
    for r in res:
        assert r["heap_cycle_bad"] == 0, r
        assert all(r["heap_translated"]), r
        assert r["free_drop_MiB"] < made_MiB + 512, r


@pytest.mark.gpu
def test_vmm_heap_large_objects_processes(tmp_path):
    """osgpu_heap_create with three processes on cuda:0: each PE's device heap
    is ONE contiguous virtual range of dmabuf-exported chunks, mapped whole
    into every member, so a 2.5 GiB symmetric array per PE (more than one HIP
    IPC export carries) is base + offset on every PE like the
    reference's heap (src/shmemc/comms.c:89-105).  shmem_double_sum_to_all
    runs on the exact team kernel: its full 2.5 GiB target equals the pull
    path's bit for bit on every PE (GPU compare), a 32 Ki sample equals the
    oracle's per-PE fold, long xor satisfies checksum-of-checksums at full
    size, and a small call on the same heap takes the fused path.  First, a
    heap one member cannot make (1 PiB) fails on every member within
    seconds."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 3
    res = launch("vmm", world, tmp_path, timeout=300)
    for r in range(world):
        x = res[r]
        assert x["nbytes"] >= 5 << 29
        assert x["failed_create_s"] < 10, x["failed_create_s"]  # no wait for absent peers
        assert x["paths"] == {"team": "team", "pull": "pull", "xor": "team",
                              "small": "fused_team"}, x["paths"]
        assert x["team_vs_pull_mismatch"] == 0, (r, x)
        assert x["sample_mismatch"] == 0 and x["sample_checked"] == 1 << 15, (r, x)
        assert x["xor_checksum_ok"], r
        assert x["small_ok"], r
    # fold orders differ per PE (PE 0 == PE 1 by a + b == b + a; PE 2 differs)
    assert res[0]["hash_team"] == res[1]["hash_team"] != res[2]["hash_team"]


@pytest.mark.gpu
@pytest.mark.parametrize("slice_ms", ["100", "0.05"])
def test_late_member_fused_processes(tmp_path, monkeypatch, slice_ms):
    """A member that enters a fused call 1.5 s after the others (beyond the
    old 0.5 s bound and many wait slices) -- team and pull reduce, fused
    fcollect, fused collect -- and 120 calls entered with random delays:
    every result bit-exact, every call on the fused path, no abort.  The
    device barrier waits without bound like the reference's
    (src/shmemc/waituntil.c:57-71); the GPU is released every slice and the
    call continues by relaunch (runtime.cpp fused_complete).  With 50 us
    slices the jittered calls run through continuations at both barriers."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("OSGPU_DEVICE_BARRIER_SLICE_MS", slice_ms)
    world = 3
    res = launch("late", world, tmp_path, timeout=300)
    for r in range(world):
        for key, (exact, ran, dt, cont) in res[r]["late"].items():
            assert exact, (key, r)
            assert ran in ("fused_team", "fused_pull", "fused_copy"), (key, r, ran)
            if r < world - 1:   # the punctual members waited for the late one
                assert dt > 1.3 and cont >= 5, (key, r, dt, cont)
        j = res[r]["jitter"]
        assert j["exact"] == j["calls"] == 120, (r, j)
        assert set(j["paths"]) <= {"fused_team"}, (r, j)
    if slice_ms == "0.05":
        assert sum(res[r]["jitter"]["continuations"] for r in range(world)) > 50


@pytest.mark.gpu
@pytest.mark.parametrize("fatal", [0, 1])
def test_device_barrier_timeout(tmp_path, monkeypatch, fatal):
    """A member that never enters a fused call, under an explicit 0.5 s
    device-barrier bound (the default is none, like the reference's barrier):
    the others' call fails once the member has been away that long --
    reported through osgpu_last_error / last_path == fused_failed under the
    non-fatal policy, an abort with a message under the fatal one."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("MP_FATAL", str(fatal))
    if not fatal:
        res = launch("timeout", 2, tmp_path)
        assert res[0]["first"] == "fused_team" and res[1]["first"] == "fused_team"
        assert res[0]["alone"] == "fused_failed", res[0]
        assert "device barrier (entry): a member of the active set stayed away" in res[0]["error"]
        assert 0.4 < res[0]["seconds"] < 5.0, res[0]["seconds"]
        return
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, WORKER, "timeout", str(tmp_path)],
                                      env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    out0, _ = procs[0].communicate(timeout=120)
    procs[1].kill()   # waits in dist.barrier for the aborted rank 0
    procs[1].communicate()
    assert procs[0].returncode != 0
    assert "device barrier (entry): a member of the active set stayed away" in out0, out0[-2000:]
