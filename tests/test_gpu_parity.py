"""GPU parity: libosgpu_reduce.so on an MI355X against the reference.

Every case of tests/golden/reduce_cases.json (per-PE SHA-256 digests of
targets folded with the reference's compiled element ops in the order of
src/reductions.c:79-111) is replayed through the real C entry point
shmem_<T>_<op>_to_all by a team of threads-as-PEs whose symmetric heaps live
in HBM (P2P path).  Bar: bit-exact, including floating point, NaN payloads,
signed zeros and subnormals -- the kernels reproduce each PE's own fold
order, so no tolerance is needed.  Host-heap (staged) runs, in-place calls,
ragged/misaligned spans and the raw combine launcher are checked against the
oracle on the same inputs.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
import osgpu

pytestmark = pytest.mark.gpu

# x87 80-bit long double runs on the GPU through the soft-float in x87.hpp
LD_ON_GPU = True
CASES = [c for c in O.load_cases() if LD_ON_GPU or c["type"] != "longdouble"]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


_TEAMS = {}


def team(device=True, host_fold=False):
    from support import team as T
    key = device
    if key not in _TEAMS:
        _TEAMS[key] = T.Team(8, 20 << 20, device=device)
    tm = _TEAMS[key]
    tm.host_fold = host_fold   # the library default (True) or the GPU paths
    tm.activate()
    return tm


def tgt_off(nbytes):
    return max(4096, (nbytes + 4095) // 4096 * 4096)


def run_case(tm, c, in_place=False):
    t, op, n = c["type"], c["op"], c["nreduce"]
    s = O.NP_DTYPE[t]().itemsize if t != "longdouble" else 16
    nbytes = n * s
    src = O.case_inputs(c)
    toff = 0 if in_place else tgt_off(nbytes)
    for pe in range(c["npes"]):
        tm.write(pe, 0, src[pe])
        if not in_place:
            tm.fill(pe, toff, max(nbytes, 16), 0xA5)
    tm.run(t, op, toff, 0, n, c["PE_start"], c["logPE_stride"], c["PE_size"])
    act = O.active_set(c["PE_start"], c["logPE_stride"], c["PE_size"])
    out = {}
    for pe in range(c["npes"]):
        raw = tm.read(pe, toff, nbytes)
        if pe in act:
            out[pe] = O.from_value_bytes(t, raw if t != "longdouble" else
                                         raw.reshape(-1, 16)[:, :10].reshape(-1))
        elif not in_place:
            assert (tm.read(pe, toff, max(nbytes, 16)) == 0xA5).all(), \
                f"non-member PE {pe} target was written"
    return out


def check(c, out):
    for pe, dg in c["digests"].items():
        got = O.digest(out[int(pe)])
        assert got == dg, (f"{c['type']}/{c['op']} P={c['npes']} N={c['nreduce']} "
                           f"{c['tag']} start={c['PE_start']} PE {pe}")


def _by_pair():
    pairs = {}
    for c in CASES:
        pairs.setdefault((c["type"], c["op"]), []).append(c)
    return sorted(pairs.items())


def _expected_path(c, team_form):
    """Path the library must have taken.  PEs here are threads of one
    process: the fused one-launch path needs every member in its own process
    (tests/test_multiproc.py covers it), so these calls keep host barriers."""
    if c["nreduce"] == 0:
        return "barrier_only"
    return "team" if team_form and c["PE_size"] >= 2 else "pull"


@pytest.mark.parametrize("pair,cases", _by_pair(), ids=lambda x: "%s" % (x,) if isinstance(x, tuple) else "")
def test_device_resident_matches_golden(torch_cuda, pair, cases):
    tm = team(device=True)
    for c in cases:
        check(c, run_case(tm, c))
        act = O.active_set(c["PE_start"], c["logPE_stride"], c["PE_size"])
        want = _expected_path(c, True)
        assert all(tm.last_paths[pe] == want for pe in act), (tm.last_paths, want)


def test_team_push_matches_golden(torch_cuda):
    """Every golden case through the push form of the team exchange
    (osgpu_set_team_exchange(1)): sources scattered into the owners'
    staging inboxes, folded there, results written to every target -- the
    fabric sees remote writes only.  Small staging slots force many chunks."""
    tm = team(device=True)
    L = tm.lib
    L.osgpu_finalize()
    L.osgpu_set_stage_bytes(65536)
    L.osgpu_set_team_exchange(1)
    try:
        for c in CASES:
            check(c, run_case(tm, c))
            act = O.active_set(c["PE_start"], c["logPE_stride"], c["PE_size"])
            want = ("barrier_only" if c["nreduce"] == 0 else
                    "team_push" if c["PE_size"] >= 2 else "pull")
            assert all(tm.last_paths[pe] == want for pe in act), (tm.last_paths, want)
    finally:
        L.osgpu_set_team_exchange(-1)
        L.osgpu_finalize()
        L.osgpu_set_stage_bytes(-1)


def test_pull_path_matches_golden(torch_cuda):
    """The same cases forced onto the pull form (every PE reads every source,
    the reference's own schedule) instead of the owner-computes team kernel."""
    tm = team(device=True)
    tm.lib.osgpu_set_path(osgpu.PATH_PULL)
    try:
        for c in CASES:
            if c["nreduce"] <= 4097 and c["npes"] in (2, 3, 8) and c["tag"] != "subset":
                check(c, run_case(tm, c))
                assert tm.last_paths[c["PE_start"]] == _expected_path(c, False)
    finally:
        tm.lib.osgpu_set_path(osgpu.PATH_AUTO)


@pytest.mark.parametrize("t,op", [("double", "sum"), ("float", "prod"), ("int", "xor"),
                                  ("complexd", "prod"), ("short", "min"),
                                  ("complexf", "sum"), ("longdouble", "sum")])
def test_in_place_target_equals_source(torch_cuda, t, op):
    tm = team(device=True)
    for c in CASES:
        if c["type"] == t and c["op"] == op and c["tag"] in ("grid", "edge") and \
                c["npes"] in (2, 3, 8):
            check(c, run_case(tm, c, in_place=True))


@pytest.mark.parametrize("t,op", [("int", "sum"), ("double", "sum"), ("long", "and"),
                                  ("float", "min"), ("complexd", "prod"),
                                  ("short", "prod"), ("longdouble", "prod")])
@pytest.mark.parametrize("host_path", ["staged", "getmem"])
def test_host_staged_matches_golden(torch_cuda, t, op, host_path, monkeypatch):
    """Host symmetric heaps.  staged: H2D own source -> team exchange on the
    GPU through the staging buffers -> D2H, 4 KiB chunks so the two-slot
    pipeline turns over many times; getmem: every peer's source pulled
    through the runtime's shmem_getmem (the reference's transport)."""
    L = osgpu.load()
    L.osgpu_set_host_chunk_bytes(4096)  # many chunks
    L.osgpu_set_stage_bytes(4096)
    L.osgpu_finalize()  # staging is sized at set-up
    try:
        with osgpu.host_path(host_path):
            tm = team(device=False)
            n = 0
            for c in CASES:
                if c["type"] == t and c["op"] == op and c["nreduce"] <= 4097 and \
                        c["npes"] in (1, 2, 3, 8):
                    check(c, run_case(tm, c))
                    if c["nreduce"] > 0 and c["npes"] > 1:
                        assert set(tm.last_paths.values()) <= {host_path, "fused_staged"}, \
                            tm.last_paths
                    n += 1
            assert n > 10
            c = next(c for c in CASES if c["type"] == t and c["op"] == op and c["npes"] == 3
                     and c["nreduce"] == 4097 and c["tag"] == "grid")
            check(c, run_case(tm, c, in_place=True))
    finally:
        L.osgpu_set_host_chunk_bytes(-1)
        L.osgpu_set_stage_bytes(-1)
        L.osgpu_finalize()


@pytest.mark.parametrize("t,op", sorted({(c["type"], c["op"]) for c in CASES}))
def test_host_fold_matches_golden(torch_cuda, t, op):
    """The library's default for small HOST symmetric-heap calls (each PE
    pulling at most 256 KiB from its peers): the host fold (shmem_reduce.cpp run_host_fold, host_fold.hip)
    -- the reference's algorithm on each PE's thread with the kernels'
    element ops compiled for the host.  Bit-exact on the golden cases (NaN
    payloads, signed zeros, wrap-around, x87 long double included), in
    place too; above the limit the same calls take the GPU (STAGED).  Every
    one of the 44 (type, op) pairs."""
    tm = team(device=False, host_fold=True)
    lim = 256 << 10   # on (PE_size - 1) * nreduce * size
    n = nfold = 0
    for c in CASES:
        if c["type"] == t and c["op"] == op and c["nreduce"] <= 4097 and \
                c["npes"] in (1, 2, 3, 8):
            check(c, run_case(tm, c))
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            if c["nreduce"] > 0:
                want = "host_fold" if (c["PE_size"] - 1) * c["nreduce"] * s <= lim else "staged"
                assert set(tm.last_paths.values()) <= {want, "fused_staged"}, tm.last_paths
                nfold += want == "host_fold"
            n += 1
    assert n > 10 and nfold > 5
    c = next(c for c in CASES if c["type"] == t and c["op"] == op and c["npes"] == 3
             and c["nreduce"] == 4097 and c["tag"] == "grid")
    check(c, run_case(tm, c, in_place=True))


@pytest.mark.parametrize("stage_copy", ["kout", "kernel", "dma"])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_staged_copy_modes(torch_cuda, stage_copy, pinned, monkeypatch):
    """The STAGED path's PCIe legs by DMA engine or by kernel
    (OSGPU_STAGE_COPY, shmem_reduce.cpp stage_leg), on pageable heaps (the
    pinned bounce buffers' device view) and on heaps pinned with
    osgpu_host_register (the heap's own device view), 4 KiB chunks, odd
    lengths and offsets: bit-exact on the golden cases."""
    L = osgpu.load()
    L.osgpu_set_stage_bytes(4096)
    L.osgpu_set_host_path(osgpu.HOST_STAGED)
    L.osgpu_set_stage_copy(osgpu.STAGE_COPY[stage_copy])
    L.osgpu_finalize()
    tm = team(device=False)
    if pinned:
        assert L.osgpu_host_register(ctypes.c_void_p(tm.base), tm.npes * tm.H) == 0
        L.osgpu_set_fused_max_bytes(0)   # small calls too: the staged path
    try:
        n = 0
        for c in CASES:
            if (c["type"], c["op"]) in (("double", "sum"), ("int", "xor"), ("complexd", "prod"),
                                        ("short", "min"), ("longdouble", "max")) and \
                    c["nreduce"] <= 4097 and c["npes"] in (2, 3, 8):
                check(c, run_case(tm, c))
                if c["nreduce"] > 0:
                    assert tm.last_paths[c["PE_start"]] == "staged", tm.last_paths
                n += 1
        assert n > 20
    finally:
        if pinned:
            L.osgpu_set_fused_max_bytes(-1)
            L.osgpu_host_unregister(ctypes.c_void_p(tm.base))
        L.osgpu_set_stage_bytes(-1)
        L.osgpu_set_host_path(-1)
        L.osgpu_set_stage_copy(-1)
        L.osgpu_finalize()


def test_staged_copy_streams_survive_extra_streams(torch_cuda):
    """With more streams in the process than the staging set expects (a
    torch side stream and the thread's osgpu stream, created first), the
    H2D and D2H copy streams still come from different priority pools, and
    a 64 Mi-double pinned STAGED call keeps both directions moving at once:
    more than 36 GB/s each way (27.7 when they shared a queue and took
    turns), unless the GPU's DMA engine was in its low power state before
    or after the timed calls (then its D2H alone is below 40 GB/s and the
    rate is only reported).  The hard assertion is the priorities'."""
    import torch
    import bench
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.ones(1 << 20, device="cuda").add_(1)
    osgpu.load().osgpu_get_stream()
    torch.cuda.synchronize()
    res = bench.host_staged_time(64 << 20, reps=3)
    L = osgpu.load()
    dev = torch.cuda.current_device()
    assert res["pinned"]["correct"] and res["pageable"]["correct"], res
    # (host_staged_time finalizes at its end: set the streams up again)
    tm = team(device=False)
    c = next(c for c in CASES if c["type"] == "double" and c["op"] == "sum" and c["npes"] == 2
             and c["nreduce"] > 1000)
    check(c, run_case(tm, c))
    pi, po = ctypes.c_int(), ctypes.c_int()
    assert L.osgpu_copy_stream_info(dev, ctypes.byref(pi), ctypes.byref(po)) == 0
    assert pi.value != po.value, (pi.value, po.value)
    # the rate is reported, and asserted only when the DMA engine was in its
    # high power state both before and after the timed calls (ADVICE r05:
    # a state drop during them must not fail a test about stream priorities)
    print("pinned STAGED each way GB/s", res["pinned"]["pcie_GBs_each_way"],
          "dma before/after", res["dma_state"], res["dma_state_after"])
    if not res["dma_state"]["low_state"] and not res["dma_state_after"]["low_state"]:
        assert res["pinned"]["pcie_GBs_each_way"] > 36, res
    del side


_S = []


def _stream(torch):
    """A non-default torch stream, after draining the device: torch's default
    stream has handle 0, and a NULL stream means "the calling thread's
    stream" to osgpu_combine, which would not be ordered after torch's work."""
    torch.cuda.synchronize()
    if not _S:
        _S.append(torch.cuda.Stream())
    return _S[0].cuda_stream


def _dev(torch, arr):
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    return torch.from_numpy(raw.copy()).to("cuda:0")


@pytest.mark.parametrize("t", ["short", "int", "long", "float", "double", "complexf",
                               "complexd"] + (["longdouble"] if LD_ON_GPU else []))
@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 9, 17])
def test_combine_ragged_and_misaligned(torch_cuda, t, k):
    """Raw combine launcher: any element offset (16-byte phase), any n, K up
    to 17 (chunked into launches of <= 8 inputs, order preserved)."""
    torch = torch_cuda
    op = "sum" if t != "longdouble" else "max"
    s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
    for n in (1, 7, 255, 1000, 4099):
        for shift_in, shift_out in ((0, 0), (1, 1), (1, 0), (3, 2)):
            if s >= 16 and (shift_in or shift_out):
                continue
            ins = [O.gen_input(t, n, 1000 + 7 * j + n, "edge") for j in range(k)]
            want = ins[0]
            for x in ins[1:]:
                want = O.op_elementwise(t, op, want, x)
            bufs = [_dev(torch, np.concatenate([O.gen_input(t, shift_in, 5, "mixed"), x]))
                    for x in ins]
            out = torch.zeros((n + shift_out) * s, dtype=torch.uint8, device="cuda:0")
            # osgpu_combine is asynchronous: enqueue it on torch's stream so
            # it is ordered after the uploads and the zero fill
            osgpu.combine(t, op, out.data_ptr() + shift_out * s,
                          [b.data_ptr() + shift_in * s for b in bufs], n, _stream(torch))
            torch.cuda.synchronize()
            got = out.cpu().numpy()[shift_out * s:]
            if t == "longdouble":
                got = got.reshape(-1, 16)[:, :10].reshape(-1)
            want_b = O.value_bytes(want).reshape(-1)
            bad = np.nonzero(got.reshape(-1) != want_b)[0]
            assert bad.size == 0, (t, k, n, shift_in, shift_out, bad[:8] // s)


@pytest.mark.parametrize("op", ["sum", "prod", "max", "min"])
def test_longdouble_8byte_aligned_arrays(torch_cuda, op):
    """long double arrays that are only 8-byte aligned take the scalar
    soft-float kernel (the usual 16-byte-aligned ones the vector kernel)."""
    torch = torch_cuda
    n, k = 1001, 3
    ins = [O.gen_input("longdouble", n, 77 + j, "edge") for j in range(k)]
    want = ins[0]
    for x in ins[1:]:
        want = O.op_elementwise("longdouble", op, want, x)
    bufs = [_dev(torch, np.concatenate([np.zeros(8, np.uint8), x.view(np.uint8)]))
            for x in ins]
    out = torch.zeros(n * 16 + 8, dtype=torch.uint8, device="cuda:0")
    osgpu.combine("longdouble", op, out.data_ptr() + 8, [b.data_ptr() + 8 for b in bufs], n,
                  _stream(torch))
    torch.cuda.synchronize()
    got = out.cpu().numpy()[8:].reshape(-1, 16)[:, :10].reshape(-1)
    assert np.array_equal(got, O.value_bytes(want).reshape(-1))


@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_active_sets_beyond_eight_pes(torch_cuda, device):
    """12 PEs (threads), the whole job and a 10-PE subset: past the team
    kernel's 8 members the device path is the pull form with the fold
    chained over launches of at most 8 inputs (combine.hip launch_op), the
    host path every PE folding its own staged chunk.  Bit-exact per PE."""
    from support import team as T
    npes = 12
    tm = T.Team(npes, 2 * 4097 * 16 + 8192, device=device)
    try:
        for t, op, dist_ in (("double", "sum", "wide"), ("float", "prod", "wide"),
                             ("int", "xor", "bits"), ("complexd", "prod", "edge"),
                             ("longdouble", "max", "edge"), ("short", "sum", "bits")):
            s = 16 if t == "longdouble" else O.NP_DTYPE[t]().itemsize
            for n in (1000, 4097):
                for start, size in ((0, 12), (2, 10)):
                    src = O.team_inputs(t, npes, n, 0x1200 + n + start, dist_)
                    want = O.to_all(t, op, src, start, 0, size)
                    toff = tgt_off(n * s)
                    for pe in range(npes):
                        tm.write(pe, 0, src[pe])
                        tm.fill(pe, toff, n * s, 0x3C)
                    tm.run(t, op, toff, 0, n, start, 0, size)
                    for pe in range(npes):
                        raw = tm.read(pe, toff, n * s)
                        if want[pe] is None:
                            assert (raw == 0x3C).all(), (t, op, n, start, pe)
                            continue
                        if t == "longdouble":
                            raw = raw.reshape(-1, 16)[:, :10].reshape(-1)
                        assert np.array_equal(raw, O.value_bytes(want[pe]).reshape(-1)), \
                            (t, op, n, start, size, pe)
    finally:
        tm.lib.osgpu_finalize()
        team(device)  # restore the shared 8-PE team for the other tests


def test_large_config2_shape_properties(torch_cuda):
    """BASELINE config 2 at full size (nreduce = 64 Mi doubles, 2 inputs):
    checked against the oracle on a strided sample and through the exact
    identity sum(a)+sum(b) = sum(out) for values in [1, 2) (every a+b is exact
    in binary64 only up to one rounding, so the check is sample-exact plus a
    relative bound on the total)."""
    torch = torch_cuda
    n = 64 << 20
    a = torch.rand(n, dtype=torch.float64, device="cuda:0") + 1.0
    b = torch.rand(n, dtype=torch.float64, device="cuda:0") + 1.0
    out = torch.empty_like(a)
    osgpu.combine("double", "sum", out.data_ptr(), [a.data_ptr(), b.data_ptr()], n,
                  _stream(torch))
    torch.cuda.synchronize()
    idx = torch.randint(0, n, (1 << 16,), device="cuda:0")
    sa, sb, so = a[idx].cpu().numpy(), b[idx].cpu().numpy(), out[idx].cpu().numpy()
    assert np.array_equal(so.view(np.uint64),
                          O.op_elementwise("double", "sum", sa, sb).view(np.uint64))
    # tail elements (ragged end) too
    assert torch.equal(out[-1000:], a[-1000:] + b[-1000:])
    assert torch.equal(out, a + b)   # torch's own add is IEEE RNE on these values


def test_config3_bitwise_full_size(torch_cuda):
    """BASELINE config 3: long and/or/xor, 256 MiB per array (32 Mi int64)."""
    torch = torch_cuda
    n = 32 << 20
    g = torch.Generator(device="cuda:0").manual_seed(3)
    a = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda:0", generator=g)
    b = torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device="cuda:0", generator=g)
    out = torch.empty_like(a)
    for op, ref in (("and", torch.bitwise_and), ("or", torch.bitwise_or),
                    ("xor", torch.bitwise_xor)):
        osgpu.combine("long", op, out.data_ptr(), [a.data_ptr(), b.data_ptr()], n,
                      _stream(torch))
        torch.cuda.synchronize()
        assert torch.equal(out, ref(a, b)), op
    # xor is its own inverse: (a ^ b) ^ b == a
    osgpu.combine("long", "xor", out.data_ptr(), [out.data_ptr(), b.data_ptr()], n,
                  _stream(torch))
    torch.cuda.synchronize()
    assert torch.equal(out, a)


def test_heap_create_threads_as_pes(torch_cuda):
    """osgpu_heap_create when the members are threads of one process (they
    share each other's range directly, no descriptors): three PEs each make
    a 24 MiB device heap in the same collective call; double sum (team and
    pull form), int xor and long double sum run on objects inside the heaps,
    bit-exact against the oracle's per-PE folds; pSync comes back zeroed
    (the helper asserts it), and the heaps are destroyed again."""
    tm = team(True)
    L = tm.lib
    P = 3
    nbytes = 24 << 20
    bases = {}

    def create(pe):
        b = ctypes.c_void_p()
        rc = L.osgpu_heap_create(nbytes, 0, 0, P, tm.psync_ptr(pe), ctypes.byref(b))
        assert rc == 0, L.osgpu_last_error().decode()
        bases[pe] = b.value

    tm._on_members(list(range(P)), create)
    assert len(set(bases.values())) == P
    views = {pe: osgpu.device_view(bases[pe], nbytes) for pe in range(P)}
    try:
        for t, op, n, dist, path in (("double", "sum", 100_003, "wide", osgpu.PATH_AUTO),
                                     ("double", "sum", 100_003, "wide", osgpu.PATH_PULL),
                                     ("int", "xor", 777_777, "bits", osgpu.PATH_AUTO),
                                     ("longdouble", "sum", 4099, "wide", osgpu.PATH_AUTO)):
            s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
            src = O.team_inputs(t, P, n, 0x4EA9, dist)
            toff = (n * s + 4095) // 4096 * 4096
            for pe in range(P):
                raw = np.ascontiguousarray(src[pe]).view(np.uint8).reshape(-1)
                views[pe][:raw.size].copy_(torch_cuda.from_numpy(raw.copy()).cuda())
                views[pe][toff:toff + n * s].fill_(0xA5)
            torch_cuda.cuda.synchronize()
            L.osgpu_set_path(path)
            fn = osgpu.to_all(t, op)
            pwrk = (ctypes.c_byte * 4096)()
            tm._on_members(list(range(P)), lambda pe: fn(
                bases[pe] + toff, bases[pe], n, 0, 0, P, ctypes.addressof(pwrk),
                tm.psync_ptr(pe)))
            L.osgpu_set_path(osgpu.PATH_AUTO)
            want = O.to_all(t, op, src)
            for pe in range(P):
                torch_cuda.cuda.synchronize()
                got = views[pe][toff:toff + n * s].cpu().numpy()
                if t == "longdouble":
                    got = got.reshape(-1, 16)[:, :10].reshape(-1)
                assert np.array_equal(got, O.value_bytes(want[pe]).reshape(-1)), (t, op, path, pe)
                assert tm.last_paths[pe] == ("pull" if path == osgpu.PATH_PULL else "team")
    finally:
        torch_cuda.cuda.synchronize()
        views.clear()
        for pe in range(P):
            assert L.osgpu_heap_destroy(ctypes.c_void_p(bases[pe])) == 0


@pytest.mark.parametrize("t,op,P", [("double", "sum", 2), ("float", "min", 5), ("int", "prod", 8),
                                    ("complexd", "prod", 3), ("longdouble", "sum", 8),
                                    ("longdouble", "prod", 4)])
@pytest.mark.parametrize("shift", [0, 1])
def test_team_combine_launcher(torch_cuda, t, op, P, shift):
    """osgpu_team_combine, the TEAM path's kernel through the C ABI: output q
    is member q's fold order (src/reductions.c:79-111), bit-exact against
    the oracle; shift 1 starts every array one element past a 16-B boundary
    (scalar head and tail around the vector body)."""
    s = 16 if t == "longdouble" else np.dtype(O.NP_DTYPE[t]).itemsize
    n = 70_001
    src = O.team_inputs(t, P, n, 0x7EA0 + P, "wide")
    want = O.to_all(t, op, src)
    nb = n * s + 64
    dev = torch_cuda.device("cuda:0")
    ins = [torch_cuda.empty(nb, dtype=torch_cuda.uint8, device=dev) for _ in range(P)]
    outs = [torch_cuda.full((nb,), 0x5A, dtype=torch_cuda.uint8, device=dev) for _ in range(P)]
    off = shift * s if t != "longdouble" else 0
    for p in range(P):
        raw = np.ascontiguousarray(src[p]).view(np.uint8).reshape(-1)
        ins[p][off:off + raw.size].copy_(torch_cuda.from_numpy(raw.copy()).to(dev))
    S = (ctypes.c_void_p * P)(*[x.data_ptr() + off for x in ins])
    D = (ctypes.c_void_p * P)(*[x.data_ptr() + off for x in outs])
    torch_cuda.cuda.synchronize()
    L = osgpu.load()
    assert L.osgpu_team_combine(osgpu.TYPES.index(t), osgpu.OPS.index(op), P, D, S, n, None) == 0
    torch_cuda.cuda.synchronize()
    for q in range(P):
        got = outs[q][off:off + n * s].cpu().numpy()
        if t == "longdouble":
            got = got.reshape(-1, 16)[:, :10].reshape(-1)
        assert np.array_equal(got, O.value_bytes(want[q]).reshape(-1)), (t, op, P, q)
        assert (outs[q][:off].cpu().numpy() == 0x5A).all()
        assert (outs[q][off + n * s:].cpu().numpy() == 0x5A).all()


REMOTE_CASES = [(t, op, P) for P in (2, 5, 8)
                for t, op in (("double", "sum"), ("float", "prod"), ("double", "min"),
                              ("float", "max"), ("int", "sum"), ("long", "xor"),
                              ("short", "prod"), ("complexf", "sum"), ("complexd", "prod"))]


@pytest.mark.parametrize("t,op,P", REMOTE_CASES)
def test_team_remote_shapes_match_golden(torch_cuda, t, op, P):
    """The team kernel's REMOTE launch shapes (team.hip TeamShape<..., true>:
    the register form at 2 members, rounds of 2 vectors at 5-8 -- what a
    call whose members' heaps sit on other GPUs launches) run on
    one GPU through osgpu_team_combine_shape: every member's output
    bit-exact against the oracle on edge-value inputs (NaN payloads, ±0,
    infinities, wrap-around), with a scalar head and tail."""
    s = np.dtype(O.NP_DTYPE[t]).itemsize
    n = 50_003
    src = O.team_inputs(t, P, n, 0x3E70 + P, "edge")
    want = O.to_all(t, op, src)
    nb = n * s + 64
    dev = torch_cuda.device("cuda:0")
    ins = [torch_cuda.empty(nb, dtype=torch_cuda.uint8, device=dev) for _ in range(P)]
    outs = [torch_cuda.full((nb,), 0x5A, dtype=torch_cuda.uint8, device=dev) for _ in range(P)]
    off = s
    for p in range(P):
        raw = np.ascontiguousarray(src[p]).view(np.uint8).reshape(-1)
        ins[p][off:off + raw.size].copy_(torch_cuda.from_numpy(raw.copy()).to(dev))
    S = (ctypes.c_void_p * P)(*[x.data_ptr() + off for x in ins])
    D = (ctypes.c_void_p * P)(*[x.data_ptr() + off for x in outs])
    torch_cuda.cuda.synchronize()
    L = osgpu.load()
    assert L.osgpu_team_combine_shape(osgpu.TYPES.index(t), osgpu.OPS.index(op), P, D, S, n,
                                      None, 1) == 0
    torch_cuda.cuda.synchronize()
    for q in range(P):
        got = outs[q][off:off + n * s].cpu().numpy()
        assert np.array_equal(got, O.value_bytes(want[q]).reshape(-1)), (t, op, P, q)
        assert (outs[q][:off].cpu().numpy() == 0x5A).all()
        assert (outs[q][off + n * s:].cpu().numpy() == 0x5A).all()


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("sign", [0, 1])
def test_longdouble_same_sign_sums(torch_cuda, P, sign):
    """long double sums whose inputs all carry one sign take the
    addition-only fast add in every round (x87.hpp add_same_fast, a
    wave-uniform choice per element): whole waves of same-sign elements
    (wide exponents, carries out of the significand), then the same arrays
    with a NaN, an infinity and denormals in a few elements -- those lanes'
    folds leave the fast path while the rest of their wave stays on it.
    Every member's target bit-exact against the oracle's per-PE fold."""
    n = 65_537
    src = O.team_inputs("longdouble", P, n, 0x5A5E + P, "wide")
    raws = [O.value_bytes(s).reshape(-1, 10).copy() for s in src]
    for r in raws:
        r[:, 9] = (r[:, 9] & 0x7F) | (0x80 if sign else 0)
    for spoil in (False, True):
        if spoil:   # a few special elements in otherwise same-sign waves
            k = np.arange(0, n, 997)
            raws[0][k[::3], :] = 0
            raws[0][k[::3], 7] = 0xC0       # quiet NaN significand
            raws[0][k[::3], 8] = 0xFF
            raws[0][k[::3], 9] = 0x7F | (0x80 if sign else 0)
            raws[P - 1][k[1::3], :8] = 0
            raws[P - 1][k[1::3], 7] = 0x80  # infinity: J bit only
            raws[P - 1][k[1::3], 8] = 0xFF
            raws[P - 1][k[1::3], 9] = 0x7F | (0x80 if sign else 0)
            raws[1][k[2::3], 8] = 0         # denormals (exponent 0)
            raws[1][k[2::3], 9] = 0x80 if sign else 0
            raws[1][k[2::3], 7] &= 0x7F
        ins_np = [np.ascontiguousarray(O.from_value_bytes("longdouble", r.reshape(-1)))
                  for r in raws]
        want = O.to_all("longdouble", "sum", ins_np)
        dev = torch_cuda.device("cuda:0")
        ins = [torch_cuda.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy())
               .to(dev) for x in ins_np]
        outs = [torch_cuda.empty(n * 16, dtype=torch_cuda.uint8, device=dev) for _ in range(P)]
        S = (ctypes.c_void_p * P)(*[x.data_ptr() for x in ins])
        D = (ctypes.c_void_p * P)(*[x.data_ptr() for x in outs])
        torch_cuda.cuda.synchronize()
        L = osgpu.load()
        assert L.osgpu_team_combine(osgpu.TYPES.index("longdouble"), 0, P, D, S, n, None) == 0
        torch_cuda.cuda.synchronize()
        for q in range(P):
            got = outs[q].cpu().numpy().reshape(-1, 16)[:, :10].reshape(-1)
            assert np.array_equal(got, O.value_bytes(want[q]).reshape(-1)), (P, sign, spoil, q)


@pytest.fixture
def small_launches(monkeypatch):
    """At most 2048 threads per launch for the test (osgpu_test_max_launch_
    threads, a test hook): every combine and team call of more than a few
    tiles takes the multi-launch path that calls of 2^31+ threads take (an
    8-member team call of 1 Gi doubles), at small sizes; restored after."""
    monkeypatch.setenv("OSGPU_TEST_HOOKS", "1")
    L = osgpu.load()
    L.osgpu_test_max_launch_threads.argtypes = [ctypes.c_longlong]
    assert L.osgpu_test_max_launch_threads(2048) == 0, L.osgpu_last_error()
    yield
    assert L.osgpu_test_max_launch_threads(0) == 0


@pytest.mark.parametrize("t", ["short", "float", "double", "complexd"])
@pytest.mark.parametrize("k", [1, 2, 5, 8])
def test_combine_multi_launch(torch_cuda, small_launches, t, k):
    """The combine kernels over many launches (combine.hip launch_k: the
    first launch takes the unaligned head and the tail, the others run on
    shifted pointers): ragged n, 16-byte phases, every element bit-exact."""
    torch = torch_cuda
    s = np.dtype(O.NP_DTYPE[t]).itemsize
    for n in (4099, 100_003):
        for shift in (0, 1):
            if s >= 16 and shift:
                continue
            ins = [O.gen_input(t, n, 3000 + 7 * j + n, "edge") for j in range(k)]
            want = ins[0]
            for x in ins[1:]:
                want = O.op_elementwise(t, "sum", want, x)
            bufs = [_dev(torch, np.concatenate([O.gen_input(t, shift, 5, "mixed"), x])) for x in ins]
            out = torch.zeros((n + shift) * s, dtype=torch.uint8, device="cuda:0")
            osgpu.combine(t, "sum", out.data_ptr() + shift * s,
                          [b.data_ptr() + shift * s for b in bufs], n, _stream(torch))
            torch.cuda.synchronize()
            got = out.cpu().numpy()[shift * s:]
            bad = np.nonzero(got.reshape(-1) != O.value_bytes(want).reshape(-1))[0]
            assert bad.size == 0, (t, k, n, shift, bad[:8] // s)


@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("t,op", [("double", "sum"), ("int", "xor"), ("float", "max"),
                                  ("complexf", "prod"), ("short", "min")])
def test_team_multi_launch(torch_cuda, small_launches, P, t, op):
    """The team kernels (LDS form at 2-4 and, real types, 8 members; register
    form otherwise) over many launches (team.hip team_launch_p): ragged n,
    one 16-byte phase for every array, every member's result bit-exact
    against its own fold order."""
    torch = torch_cuda
    s = np.dtype(O.NP_DTYPE[t]).itemsize
    L = osgpu.load()
    for n in (5_001, 100_003):
        for shift in (0, 1):
            if s >= 16 and shift:
                continue
            srcs = [O.gen_input(t, n, 4000 + 11 * p + n, "edge") for p in range(P)]
            want = O.to_all(t, op, srcs)
            pad = O.gen_input(t, shift, 5, "mixed")
            ins = [_dev(torch, np.concatenate([pad, x])) for x in srcs]
            outs = [torch.zeros((n + shift) * s, dtype=torch.uint8, device="cuda:0")
                    for _ in range(P)]
            S = (ctypes.c_void_p * P)(*[x.data_ptr() + shift * s for x in ins])
            D = (ctypes.c_void_p * P)(*[y.data_ptr() + shift * s for y in outs])
            torch.cuda.synchronize()
            assert L.osgpu_team_combine(osgpu.TYPES.index(t), osgpu.OPS.index(op), P, D, S, n,
                                        None) == 0, L.osgpu_last_error()
            torch.cuda.synchronize()
            for q in range(P):
                got = outs[q].cpu().numpy()[shift * s:]
                bad = np.nonzero(got.reshape(-1) != O.value_bytes(want[q]).reshape(-1))[0]
                assert bad.size == 0, (t, op, P, n, shift, q, bad[:8] // s)
